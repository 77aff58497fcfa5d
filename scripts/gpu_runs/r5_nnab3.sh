#!/bin/bash
# Round 5: NN weight-gradient modes interleaved (serial backward): tn, nn (dW1 + dW2), nn_w1 (dW1 only); TN on the
# weight-gradient stream for reference; engine tests first.
source scripts/gpu_steps.sh
step nn_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_nnwgrad_gpu.py
for i in 1 2 3; do
  step s_tn_$i 200 python -u bench.py --steps 20 --warmup 5 --methods none --wgrad_layout tn --no-wgrad_stream
  step s_nn_$i 200 python -u bench.py --steps 20 --warmup 5 --methods none --wgrad_layout nn
  step s_w1_$i 200 python -u bench.py --steps 20 --warmup 5 --methods none --wgrad_layout nn_w1
  step c_tn_$i 200 python -u bench.py --steps 20 --warmup 5 --methods none --wgrad_layout tn
done
