#!/bin/bash
# 4-phase (half-tile) schedule: numerics across variants, then per-GEMM throughput vs the 8-phase kernel.
source scripts/gpu_steps.sh
step gemm_tests 900 python -m pytest tests/test_gemm_gpu.py -q -m gpu -x
step gemm_bench 600 python scripts/bench_gemm.py --variants 8phase_stagger,4phase_stagger --rounds 3 --no_torch
