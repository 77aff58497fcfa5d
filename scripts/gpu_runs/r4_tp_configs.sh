#!/bin/bash
# Round 4: the two MP configs with the longer timed windows of scripts/bench_configs.sh, twice.
source scripts/gpu_steps.sh
for r in 1 2; do
  step tp8_100_$r 300 python bench.py --methods none --method tp --ffn_dim 1792 --layers 1 --steps 100 --warmup 20 --json_out gpurun_out/tp8_100_$r.json
  step tpfull_50_$r 300 python bench.py --methods none --method tp --ffn_dim 14336 --layers 1 --steps 50 --warmup 10 --json_out gpurun_out/tpfull_50_$r.json
done
