#!/bin/bash
# Round 5: headline candidates interleaved -- TN on the weight-gradient stream (round-5 default so far), NN serial
# (new default), TN serial; plus the engine tests.
source scripts/gpu_steps.sh
step nn_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_nnwgrad_gpu.py
for i in 1 2 3; do
  step c_tn_$i 200 python -u bench.py --steps 20 --warmup 5 --methods none --wgrad_layout tn
  step d_nn_$i 200 python -u bench.py --steps 20 --warmup 5 --methods none
  step s_tn_$i 200 python -u bench.py --steps 20 --warmup 5 --methods none --wgrad_layout tn --no-wgrad_stream
done
