#!/bin/bash
# Round 3 diagnostic: do idle extra streams (as an RCCL communicator creates) slow the N=1 headline's GEMMs?
source scripts/gpu_steps.sh
B="python -u bench.py --gpus 1 --steps 20 --warmup 5 --methods none"
for r in 1 2; do
  step base_$r 300 $B
  step s4_$r 300 env DLLM_DIAG_STREAMS=4:0 $B
  step s2hi_$r 300 env DLLM_DIAG_STREAMS=2:-1 $B
  step comm_$r 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --methods ddp --dist_first
done
