#!/bin/bash
# Fused-SGD epilogue with non-temporal master / working-copy traffic (build with -DDLLM_SGD_NT=1): tests, then step A/B.
source scripts/gpu_steps.sh
export NTLIB=$PWD/distributed-llm-code-samples_amd/_dllm_native_sgdnt.so
step nt_tests 300 env DLLM_NATIVE_LIB=$NTLIB python -u -m pytest tests/test_gemm_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "sgd or persistent or engine"
step d1 300 python bench.py --steps 20 --warmup 5
step n1 300 env DLLM_NATIVE_LIB=$NTLIB python bench.py --steps 20 --warmup 5
step d2 300 python bench.py --steps 20 --warmup 5
step n2 300 env DLLM_NATIVE_LIB=$NTLIB python bench.py --steps 20 --warmup 5
step d3 300 python bench.py --steps 20 --warmup 5
step n3 300 env DLLM_NATIVE_LIB=$NTLIB python bench.py --steps 20 --warmup 5
