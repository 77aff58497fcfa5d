#!/bin/bash
# Round 3: raster group size (group_m) of the persistent 8-phase GEMMs on the flagship FFN shapes.
source scripts/gpu_steps.sh
export PYTHONUNBUFFERED=1
for gm in 2 4 8 16; do
  step gm$gm 200 python -u scripts/bench_gemm.py --variants tpb8 --group_m $gm --rounds 3 --iters 10 --no_torch
done
