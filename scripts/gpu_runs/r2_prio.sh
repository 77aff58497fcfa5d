#!/bin/bash
# MFMA-cluster priority variants of the 8-phase GEMM (build-time DLLM_PRIO_MODE, alternate builds loaded via
# DLLM_NATIVE_LIB): 0 = per-cluster setprio (default), 1 = static prio for waves 4-7, 2 = none; plus tpb 4.
source scripts/gpu_steps.sh
L=distributed-llm-code-samples_amd
for i in 1 2; do
  step p0_$i 300 python bench.py --steps 20 --warmup 5 --methods none
  step p1_$i 300 env DLLM_NATIVE_LIB=$L/_dllm_native_prio1.so python bench.py --steps 20 --warmup 5 --methods none
  step p2_$i 300 env DLLM_NATIVE_LIB=$L/_dllm_native_prio2.so python bench.py --steps 20 --warmup 5 --methods none
  step t4_$i 300 python bench.py --steps 20 --warmup 5 --methods none --tpb 4
done
