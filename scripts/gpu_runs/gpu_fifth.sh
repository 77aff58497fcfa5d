#!/bin/bash
source scripts/gpu_steps.sh
step gemm_tests 900 python -m pytest tests/test_gemm_gpu.py -x -q -m gpu
step ablation 300 python scripts/ablation_tn.py
step gemm_bench 600 python scripts/bench_gemm.py --variants 8phase,8phase_stagger --json gpurun_out/gemm_bench.json
step engine_tests 600 python -m pytest tests/test_engine_gpu.py -q -m gpu
step bench 600 python bench.py --steps 10 --warmup 3
