#!/bin/bash
# Round 4: TP8-shard MP step captured in a HIP graph (bench.py --graph: every step one graph replay, device-seeded
# RNG) vs eager launches, interleaved.
source scripts/gpu_steps.sh
TP="python -u bench.py --methods none --method tp --ffn_dim 1792 --layers 1 --steps 50 --warmup 10"
for r in 1 2; do
  step tp8_eager_$r 300 $TP --json_out gpurun_out/tp8_eager_$r.json
  step tp8_graph_$r 300 $TP --graph --json_out gpurun_out/tp8_graph_$r.json
done
