#!/bin/bash
# Round 4: are the size-1 collectives' idle gaps hardware-queue sharing?  The forced-communicator methods (zero, fsdp,
# hybrid) at the box's 4 HW queues vs 8, interleaved, with exposed_ms_diff.
source scripts/gpu_steps.sh
B="python3 bench.py --steps 5 --warmup 2 --methods zero,fsdp,hybrid"
for r in 1 2; do
  step q4_$r 600 $B --json_out gpurun_out/q4_$r.json
  step q8_$r 600 $B --hw_queues 8 --json_out gpurun_out/q8_$r.json
done
