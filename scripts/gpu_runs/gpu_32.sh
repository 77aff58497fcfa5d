#!/bin/bash
# Raster group size (group_m) sweep of the six FFN GEMMs (persistent 2 tiles/block).
source scripts/gpu_steps.sh
for g in 2 4 8 16; do
  step gm$g 300 python scripts/bench_gemm.py --variants tpb2 --no_torch --rounds 3 --group_m $g
done
