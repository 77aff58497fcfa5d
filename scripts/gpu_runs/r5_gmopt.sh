#!/bin/bash
# Round 5, finite data: raster band of the NN fused-SGD weight gradients (--group_m_nn_opt) with the NN stores at 8.
source scripts/gpu_steps.sh
export PYTHONUNBUFFERED=1
for i in 1 2 3; do
  for g in 8 4 2; do
    step gmopt_${g}_$i 240 python3 bench.py --steps 20 --warmup 5 --methods none --group_m_nn_opt $g --json_out gpurun_out/gmopt_${g}_$i.json
  done
done
