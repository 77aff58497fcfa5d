#!/bin/bash
# Round 4: the forward's second GEMM (plain NT store, K = F) through hipBLASLt (DLLM_NT_STORE_LIB=1) vs the native
# persistent kernel, in the flagship step, interleaved.
source scripts/gpu_steps.sh
H="python -u bench.py --methods none --steps 20 --warmup 5"
for r in 1 2 3; do
  step head_nat_$r 300 $H --json_out gpurun_out/head_nat_$r.json
  step head_lib_$r 300 env DLLM_NT_STORE_LIB=1 $H --json_out gpurun_out/head_lib_$r.json
done
