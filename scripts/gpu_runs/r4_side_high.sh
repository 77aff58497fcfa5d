#!/bin/bash
# Round 4: do the forced-comm methods' idle gaps come from side streams sharing a hardware queue with the collective
# streams?  Engine side streams at high priority (DLLM_SIDE_STREAMS=high: their own queue set) vs the pool default.
source scripts/gpu_steps.sh
B="python3 bench.py --steps 5 --warmup 2 --methods zero,fsdp,hybrid"
for r in 1 2; do
  step pool_$r 600 $B --json_out gpurun_out/pool_$r.json
  step high_$r 600 env DLLM_SIDE_STREAMS=high $B --json_out gpurun_out/high_$r.json
done
