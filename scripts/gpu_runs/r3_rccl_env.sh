#!/bin/bash
# Round 3: what an existing RCCL communicator costs the GEMMs, by environment -- eager communicator before the N=1
# headline with the default settings, without torch's NCCL watchdog monitoring, and with 8 instead of 16 HW queues.
source scripts/gpu_steps.sh
B="python -u bench.py --gpus 1 --steps 20 --warmup 5 --methods ddp --dist_first"
for r in 1 2; do
  step base_$r 300 $B
  step nomon_$r 300 env TORCH_NCCL_ENABLE_MONITORING=0 TORCH_NCCL_ASYNC_ERROR_HANDLING=0 TORCH_NCCL_DUMP_ON_TIMEOUT=0 $B
  step q8_$r 300 env GPU_MAX_HW_QUEUES=8 $B
  step none_$r 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --methods none
done
