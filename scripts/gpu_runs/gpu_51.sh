#!/bin/bash
# dL/dy drawn when the backward starts (--lazy_dy 1: hot in L2/MALL for the first dgrad) vs before the forward; interleaved.
source scripts/gpu_steps.sh
for i in 1 2 3; do
  step d$i 300 python bench.py --steps 20 --warmup 5
  step l$i 300 python bench.py --steps 20 --warmup 5 --lazy_dy 1
done
