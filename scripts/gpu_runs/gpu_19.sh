#!/bin/bash
# 4-phase default: full GEMM/engine numerics, then flagship A/B against the 8-phase schedule.
source scripts/gpu_steps.sh
step gemm_tests 900 python -m pytest tests/test_gemm_gpu.py tests/test_engine_gpu.py tests/test_graph_gpu.py -q -m gpu -x
step b_4ph 600 python bench.py --steps 20 --warmup 3
step b_8ph 600 python bench.py --steps 20 --warmup 3 --gemm_variant 8phase_stagger
step b_4ph2 600 python bench.py --steps 20 --warmup 3
step b_8ph2 600 python bench.py --steps 20 --warmup 3 --gemm_variant 8phase_stagger
step prof_4ph 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_4ph -o k -- python3 bench.py --steps 5 --warmup 2
