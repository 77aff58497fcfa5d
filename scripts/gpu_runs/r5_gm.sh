#!/bin/bash
# Round 5, finite data: NN raster band 4 vs 8 (and 16), interleaved.
source scripts/gpu_steps.sh
H="--steps 20 --warmup 5 --methods none --no_reference_init"
for i in 1 2 3; do
  step gm_44_$i 200 python -u bench.py $H
  step gm_48_$i 200 python -u bench.py $H --group_m_nn 8
  step gm_416_$i 200 python -u bench.py $H --group_m_nn 16
done
