#!/bin/bash
# Round 3 (session 2): forward (NT) raster band 8 vs 4 in the flagship step, interleaved.
source scripts/gpu_steps.sh
for r in 1 2 3; do
  step head_gm8_$r 300 python -u bench.py --methods none --steps 20 --warmup 5
  step head_gm4_$r 300 python -u bench.py --methods none --steps 20 --warmup 5 --group_m_nt 4
done
