#!/bin/bash
# Round 5: NN vs TN weight-gradient layout on one box -- isolated GEMMs, then interleaved step pairs with the
# weight-gradient stream (headline) and serial.
source scripts/gpu_steps.sh
step nn_bench 300 python -u scripts/bench_nn_wgrad.py --json gpurun_out/nn_wgrad_ab.json
for i in 1 2 3; do
  step c_tn_$i 200 python -u bench.py --steps 20 --warmup 5 --methods none --wgrad_layout tn
  step c_nn_$i 200 python -u bench.py --steps 20 --warmup 5 --methods none --wgrad_layout nn
done
for i in 1 2; do
  step s_tn_$i 200 python -u bench.py --steps 20 --warmup 5 --methods none --wgrad_layout tn --no-wgrad_stream
  step s_nn_$i 200 python -u bench.py --steps 20 --warmup 5 --methods none --wgrad_layout nn --no-wgrad_stream
done
