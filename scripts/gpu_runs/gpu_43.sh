#!/bin/bash
# Fused-SGD master-weight L2 warm-up: correctness + A/B (on/off) x (persistent 2 / 1 tile per block), same box.
source scripts/gpu_steps.sh
step tests 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "sgd or persistent or engine or optimizers or splitk"
grep -q " passed" gpurun_out/tests.log && ! grep -q -E "[0-9]+ failed" gpurun_out/tests.log || exit 1
step on_t2 300 python bench.py --steps 20 --warmup 5
step off_t2 300 python bench.py --steps 20 --warmup 5 --no_sgd_prefetch
step on_t1 300 python bench.py --steps 20 --warmup 5 --tpb 1
step off_t1 300 python bench.py --steps 20 --warmup 5 --tpb 1 --no_sgd_prefetch
step on_t2b 300 python bench.py --steps 20 --warmup 5
step off_t2b 300 python bench.py --steps 20 --warmup 5 --no_sgd_prefetch
