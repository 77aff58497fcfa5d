#!/bin/bash
source scripts/gpu_steps.sh
step gemm_tests 900 python -m pytest tests/test_gemm_gpu.py -x -q -m gpu
step gemm_bench 600 python scripts/bench_gemm.py --json gpurun_out/gemm_bench.json
step engine_tests 600 python -m pytest tests/test_engine_gpu.py -q -m gpu
step bench 600 python bench.py --steps 10 --warmup 3
