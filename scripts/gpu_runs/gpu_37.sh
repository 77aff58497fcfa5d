#!/bin/bash
# Stability under sustained load: long flagship run (persistent blocks + masks), repeated race screens.
source scripts/gpu_steps.sh
step long_bench 600 python bench.py --steps 300 --warmup 5
step race_x5 600 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 300 --timeout-method thread -k "race_screen or persistent or relu_mask"
for i in 2 3; do step race_r$i 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -k "race_screen"; done
