#!/bin/bash
# Round 4: fewer hardware queues for the forced-communicator methods: 4 (box default) vs 2 vs 3, interleaved.
source scripts/gpu_steps.sh
B="python3 bench.py --steps 10 --warmup 3 --methods zero,fsdp,hybrid"
for r in 1 2; do
  step q4_$r 600 $B --json_out gpurun_out/q4_$r.json
  step q2_$r 600 $B --hw_queues 2 --json_out gpurun_out/q2_$r.json
  step q3_$r 600 $B --hw_queues 3 --json_out gpurun_out/q3_$r.json
done
