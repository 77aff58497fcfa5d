#!/bin/bash
# ReLU 1-bit activation masks: bitwise tests, flagship step with / without.
source scripts/gpu_steps.sh
step mask_tests 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -k "mask or persistent or epilogues or engine"
grep -q " passed" gpurun_out/mask_tests.log && ! grep -q -E "[0-9]+ failed" gpurun_out/mask_tests.log || exit 1
step bench_nomask 300 python bench.py --steps 20 --warmup 5 --no_relu_mask
step bench_mask 300 python bench.py --steps 20 --warmup 5
step bench_nomask2 300 python bench.py --steps 20 --warmup 5 --no_relu_mask
step bench_mask2 300 python bench.py --steps 20 --warmup 5
step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o p -- python3 bench.py --steps 5 --warmup 2
