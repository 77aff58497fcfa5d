#!/bin/bash
# Fused-SGD epilogue batch size: 8 row groups per load batch (default) vs 4 vs 2; plus the full default bench timing
source scripts/gpu_steps.sh
L=distributed-llm-code-samples_amd
for i in 1 2 3; do
  step c8_$i 120 python bench.py --steps 20 --warmup 5 --methods none
  step c16_$i 120 env DLLM_NATIVE_LIB=$L/_dllm_native_sgdc16.so python bench.py --steps 20 --warmup 5 --methods none
  step c32_$i 120 env DLLM_NATIVE_LIB=$L/_dllm_native_sgdc32.so python bench.py --steps 20 --warmup 5 --methods none
done
step default_bench 600 bash -c 'time python bench.py'
