#!/bin/bash
# Concurrent weight-gradient stream (whole-chip grids) vs the serial backward, 5 interleaved pairs
source scripts/gpu_steps.sh
for i in 1 2 3 4 5; do
  step serial_$i 120 python bench.py --steps 30 --warmup 5 --methods none
  step wgs_$i 120 python bench.py --steps 30 --warmup 5 --methods none --wgrad_stream
done
