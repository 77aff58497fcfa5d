#!/bin/bash
# Round 5: config 5 (fused AdamW through the transposed map) with one tile per block vs persistent blocks (alternate
# build DLLM_ADAMS_T_PERS=1), interleaved; plus config 5 with SGD for the AdamW gap.
source scripts/gpu_steps.sh
C5="--methods none --optimizer adam --gated --act silu --ffn_dim 14336 --layers 32 --steps 6 --warmup 2"
ALT=$PWD/distributed-llm-code-samples_amd/_dllm_native_adamspers.so
for i in 1 2; do
  step c5_base_$i 300 python -u bench.py $C5
  step c5_pers_$i 300 env DLLM_NATIVE_LIB=$ALT python -u bench.py $C5
done
step c5_sgd 300 python -u bench.py --methods none --gated --act silu --ffn_dim 14336 --layers 32 --steps 6 --warmup 2
