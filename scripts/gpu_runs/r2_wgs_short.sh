#!/bin/bash
# Concurrent weight-gradient stream vs serial at the bench's default step counts (10 timed, 3 warmup), 4 pairs
source scripts/gpu_steps.sh
for i in 1 2 3 4; do
  step wgs_$i 120 python bench.py --methods none
  step serial_$i 120 python bench.py --methods none --no-wgrad_stream
done
