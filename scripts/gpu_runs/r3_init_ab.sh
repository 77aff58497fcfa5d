#!/bin/bash
# Round 3: the N=1 headline with the side methods' process group created before it (eager RCCL communicator, lazy
# communicator via DLLM_NCCL_EAGER=0) or after it (the fix), against no process group at all; interleaved.
# Regenerates profiles/r3/headline_rccl_init_order_r3.txt.
source scripts/gpu_steps.sh
B="python -u bench.py --gpus 1 --steps 20 --warmup 5"
for r in 1 2 3; do
  step none_$r 300 $B --methods none
  step after_$r 300 $B --methods ddp
  step eager_$r 300 $B --methods ddp --dist_first
  step lazy_$r 300 env DLLM_NCCL_EAGER=0 $B --methods ddp --dist_first
done
