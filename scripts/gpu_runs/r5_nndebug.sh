#!/bin/bash
source scripts/gpu_steps.sh
step nn_debug 200 python -u scripts/debug_nn_engine.py 512 1024 3 1024
step nn_debug2 200 python -u scripts/debug_nn_engine.py 2048 8192 3 1024
step nn_tests2 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_nnwgrad_gpu.py -k engine
