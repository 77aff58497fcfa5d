#!/bin/bash
# Round 5: raster bands of the MP (TP8) shard's GEMMs (NT 224-row fwd-1 / dgrad, TN fwd-2), 100 steps, interleaved.
source scripts/gpu_steps.sh
export PYTHONUNBUFFERED=1
T="--method tp --ffn_dim 1792 --layers 1 --steps 100 --warmup 20 --methods none --no_reference_init"
for i in 1 2; do
  for c in "4 4" "4 2" "4 8" "4 16" "8 4" "2 4"; do
    set -- $c
    step tp8r_nt$1_tn$2_$i 120 python3 bench.py $T --group_m_nt $1 --group_m_tn $2 --json_out gpurun_out/tp8r_nt$1_tn$2_$i.json
  done
done
