#!/bin/bash
# Batched GEMM epilogues + compile-time activation: numerics, then the flagship profile.
source scripts/gpu_steps.sh
step gemm_tests 900 python -m pytest tests/test_gemm_gpu.py -q -m gpu -x
step engine_tests 900 python -m pytest tests/test_engine_gpu.py tests/test_graph_gpu.py -q -m gpu -x
step bench_default 600 python bench.py --steps 10 --warmup 3
step prof_default 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_default -o k -- python3 bench.py --steps 5 --warmup 2
step gemm_bench 600 python scripts/bench_gemm.py --variants 8phase_stagger --rounds 2
