#!/bin/bash
# Round 3: is the live-communicator GEMM penalty also there with the N>1 grid policy (2 persistent blocks per CU)?
source scripts/gpu_steps.sh
B="python -u bench.py --gpus 1 --steps 20 --warmup 5"
for r in 1 2; do
  step bpc2_nocomm_$r 300 $B --methods none --min_bpc 2
  step bpc2_comm_$r 300 $B --methods ddp --dist_first --min_bpc 2
  step bpc2_comm_q8_$r 300 env GPU_MAX_HW_QUEUES=8 $B --methods ddp --dist_first --min_bpc 2
  step bpc1_nocomm_$r 300 $B --methods none
done
