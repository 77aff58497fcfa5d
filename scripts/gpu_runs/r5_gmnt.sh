#!/bin/bash
# Round 5, finite data: raster band of the NT GEMMs (fwd-1, dgrad) with the NN band at 8, interleaved.
source scripts/gpu_steps.sh
export PYTHONUNBUFFERED=1
for i in 1 2 3; do
  for g in 4 8 2; do
    step gmnt_${g}_$i 240 python3 bench.py --steps 20 --warmup 5 --methods none --no_reference_init --group_m_nt $g --json_out gpurun_out/gmnt_${g}_$i.json
  done
done
