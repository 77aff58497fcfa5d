#!/bin/bash
# Round 5: the MP (TP8) shard over 100 steps -- default, HIP-graph capture, data pipeline overlap; interleaved.
source scripts/gpu_steps.sh
TP="--method tp --ffn_dim 1792 --layers 1 --steps 100 --warmup 20 --methods none"
for i in 1 2; do
  step tp8_$i 200 python3 bench.py $TP --json_out gpurun_out/tp8_$i.json
  step tp8_graph_$i 200 python3 bench.py $TP --graph --json_out gpurun_out/tp8_graph_$i.json
  step tp8_ovl_$i 200 python3 bench.py $TP --data_overlap --json_out gpurun_out/tp8_ovl_$i.json
done
