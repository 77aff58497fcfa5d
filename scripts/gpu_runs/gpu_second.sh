#!/bin/bash
source scripts/gpu_steps.sh
step gpu_tests 900 python -m pytest tests -q -m gpu
step gemm_bench 600 python scripts/bench_gemm.py --json gpurun_out/gemm_bench.json
step bench 600 python bench.py --steps 10 --warmup 3
step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run -- python bench.py --steps 5 --warmup 2
