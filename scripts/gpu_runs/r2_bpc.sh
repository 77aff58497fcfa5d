#!/bin/bash
# Persistent-grid policy under overlapping collectives: min blocks per CU 1 vs 2 (ZeRO-2 / DDP / FSDP over size-1
# RCCL communicators, whose copy kernels run next to the GEMMs)
source scripts/gpu_steps.sh
for i in 1 2 3; do
  for m in zero ddp fsdp; do
    step ${m}_b2_$i 150 python bench.py --steps 20 --warmup 5 --methods none --method $m --force_comm --min_bpc 2
    step ${m}_b1_$i 150 python bench.py --steps 20 --warmup 5 --methods none --method $m --force_comm --min_bpc 1
  done
done
