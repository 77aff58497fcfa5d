#!/bin/bash
# Round 4: the TP-shard forward's TN GEMM (K = F/tp) native vs hipBLASLt.
source scripts/gpu_steps.sh
step tn_small_k 180 python -u scripts/bench_tn_small_k.py
