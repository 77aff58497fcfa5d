#!/bin/bash
# Round 3 (session 2): the side-optimizer test (fp32 master pinned) and every BASELINE.json configuration on one GPU
# with split fp32 masters (scripts/bench_configs.sh).
source scripts/gpu_steps.sh
step pytest_sideopt 300 python -u -m pytest tests/test_side_opt_gpu.py -x -q --timeout 120 --timeout-method thread
bash scripts/bench_configs.sh
