#!/bin/bash
# Software-pipelined fused-SGD epilogue (next batch's master loads issued before this batch's stores) vs baseline
source scripts/gpu_steps.sh
L=distributed-llm-code-samples_amd
step test_pipe4 300 env DLLM_NATIVE_LIB=$L/_dllm_native_sgdpipe4.so python -u -m pytest tests/test_gemm_gpu.py tests/test_engine_gpu.py -q -x -k "sgd or engine or epilog" --timeout 120 --timeout-method thread
step test_pipe2 300 env DLLM_NATIVE_LIB=$L/_dllm_native_sgdpipe2.so python -u -m pytest tests/test_gemm_gpu.py -q -x -k "sgd or epilog" --timeout 120 --timeout-method thread
for i in 1 2 3; do
  step base_$i 120 python bench.py --steps 20 --warmup 5 --methods none
  step pipe4_$i 120 env DLLM_NATIVE_LIB=$L/_dllm_native_sgdpipe4.so python bench.py --steps 20 --warmup 5 --methods none
  step pipe2_$i 120 env DLLM_NATIVE_LIB=$L/_dllm_native_sgdpipe2.so python bench.py --steps 20 --warmup 5 --methods none
done
step test_adam1 300 env DLLM_NATIVE_LIB=$L/_dllm_native_adampipe1.so python -u -m pytest tests/test_gemm_gpu.py tests/test_engine_gpu.py -q -x -k "adam" --timeout 120 --timeout-method thread
for i in 1 2 3; do
  step abase_$i 120 python bench.py --steps 10 --warmup 3 --methods none --layers 8 --ffn_dim 14336 --gated --optimizer adam
  step adam1_$i 120 env DLLM_NATIVE_LIB=$L/_dllm_native_adampipe1.so python bench.py --steps 10 --warmup 3 --methods none --layers 8 --ffn_dim 14336 --gated --optimizer adam
done
