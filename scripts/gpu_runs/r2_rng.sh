#!/bin/bash
# Philox with one 32x32->64 multiply per product and raw v_sqrt in Box-Muller: RNG throughput and step A/B
source scripts/gpu_steps.sh
OLD=distributed-llm-code-samples_amd/ab/_dllm_native_oldrng.so
step tests 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_graph_gpu.py -q -x -k "rng or devseed or graph" --timeout 120 --timeout-method thread
step rng_new 120 python scripts/bench_rng.py
step rng_old 120 env DLLM_NATIVE_LIB=$OLD python scripts/bench_rng.py
for i in 1 2; do
  step tp_new_$i 120 python bench.py --method tp --methods none --steps 50 --warmup 10
  step tp_old_$i 120 env DLLM_NATIVE_LIB=$OLD python bench.py --method tp --methods none --steps 50 --warmup 10
  step flag_new_$i 120 python bench.py --methods none --steps 20 --warmup 5
  step flag_old_$i 120 env DLLM_NATIVE_LIB=$OLD python bench.py --methods none --steps 20 --warmup 5
done
