#!/bin/bash
# Round 5, finite data (fan-in init): weight-gradient layouts and the concurrent weight-gradient stream, interleaved.
source scripts/gpu_steps.sh
H="--steps 20 --warmup 5 --methods none --no_reference_init"
for i in 1 2; do
  step f_nn_$i 200 python -u bench.py $H
  step f_tn_s_$i 200 python -u bench.py $H --wgrad_layout tn --no-wgrad_stream
  step f_tn_c_$i 200 python -u bench.py $H --wgrad_layout tn
  step f_nn_c_$i 200 env DLLM_NN_CONCURRENT=1 python -u bench.py $H
  step f_nnw1_$i 200 python -u bench.py $H --wgrad_layout nn_w1
done
