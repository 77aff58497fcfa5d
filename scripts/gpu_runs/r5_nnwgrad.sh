#!/bin/bash
# Round 5: the NN weight-gradient layout's kernels -- GPU numerics tests, then per-GEMM timing against the TN layout.
source scripts/gpu_steps.sh
step nn_tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_nnwgrad_gpu.py
step nn_bench 300 python -u scripts/bench_nn_wgrad.py --json gpurun_out/nn_wgrad.json
