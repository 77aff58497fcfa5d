#!/bin/bash
# Round 4: persistent-grid policy of the forced-communicator methods at N=1: min 2 blocks per CU (the policy of every
# run with collectives) vs 1 (size-1 in-place collectives launch no RCCL kernel that would need CUs), interleaved.
source scripts/gpu_steps.sh
B="python3 bench.py --steps 10 --warmup 3 --methods ddp,zero,fsdp,hybrid"
for r in 1 2; do
  step bpc2_$r 600 $B --json_out gpurun_out/bpc2_$r.json
  step bpc1_$r 600 $B --min_bpc 1 --json_out gpurun_out/bpc1_$r.json
done
