#!/bin/bash
source scripts/gpu_steps.sh
step counters 120 rocprofv3 -L
step prof_bench 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- python bench.py --steps 5 --warmup 2
step gm2 300 python scripts/bench_gemm.py --variants 8phase_stagger --group_m 2 --rounds 2
step gm8 300 python scripts/bench_gemm.py --variants 8phase_stagger --group_m 8 --rounds 2
step gm16 300 python scripts/bench_gemm.py --variants 8phase_stagger --group_m 16 --rounds 2
