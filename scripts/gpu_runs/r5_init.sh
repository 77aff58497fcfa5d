#!/bin/bash
# Round 5: the flagship step with the reference's 2e-2 init (the stack diverges to inf / NaN after the first update:
# the reference's own hyper-parameters) vs a variance-preserving fan-in init (finite, dense data throughout).
source scripts/gpu_steps.sh
for i in 1 2; do
  step init_ref_$i 200 python -u bench.py --steps 20 --warmup 5 --methods none
  step init_fanin_$i 200 python -u bench.py --steps 20 --warmup 5 --methods none --init_scale fan_in
  step init_fanin_tn_$i 200 python -u bench.py --steps 20 --warmup 5 --methods none --init_scale fan_in --wgrad_layout tn --no-wgrad_stream
done
