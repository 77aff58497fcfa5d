#!/bin/bash
# Round 5: NN weight-gradient layout -- engine tests, then the flagship step A/B (interleaved) against the TN layout.
source scripts/gpu_steps.sh
step nn_tests 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_nnwgrad_gpu.py
for i in 1 2; do
  step ab_tn_$i 200 python -u bench.py --steps 20 --warmup 5 --methods none --wgrad_layout tn
  step ab_nn_$i 200 python -u bench.py --steps 20 --warmup 5 --methods none --wgrad_layout nn
done
