#!/bin/bash
# Round 5, finite data: tiles per persistent block and the NT raster band, interleaved.
source scripts/gpu_steps.sh
H="--steps 20 --warmup 5 --methods none --no_reference_init"
for i in 1 2 3; do
  step t_def_$i 200 python -u bench.py $H
  step t_tpb4_$i 200 python -u bench.py $H --tpb 4
  step t_tpb2_$i 200 python -u bench.py $H --tpb 2
  step t_nt8_$i 200 python -u bench.py $H --group_m_nt 8
done
