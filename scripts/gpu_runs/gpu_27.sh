#!/bin/bash
# 32-bit LDS-DMA offsets + unified ReLU mask epilogue: tests, flagship step, kernel stats, BASELINE configs.
source scripts/gpu_steps.sh
step tests 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_engine_gpu.py tests/test_graph_gpu.py -x -q --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/tests.log && ! grep -q -E "[0-9]+ failed" gpurun_out/tests.log || exit 1
step bench1 300 python bench.py --steps 20 --warmup 5
step bench2 300 python bench.py --steps 20 --warmup 5
step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o p -- python3 bench.py --steps 5 --warmup 2
bash scripts/bench_configs.sh > gpurun_out/bench_configs.log 2>&1
