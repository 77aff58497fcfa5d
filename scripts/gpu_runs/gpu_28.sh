#!/bin/bash
# Llama-dims gated stack with / without persistent blocks (after excluding DGLU/AdamW), flagship recheck.
source scripts/gpu_steps.sh
L="--steps 4 --warmup 2 --method hybrid --tp 1 --gated --act silu --ffn_dim 14336 --layers 32"
step llama_tpb2 600 python bench.py $L
step llama_tpb1 600 python bench.py $L --tpb 1
step llama_adam_tpb2 600 python bench.py $L --optimizer adam
step flag 300 python bench.py --steps 20 --warmup 5
step gelu_tpb2 300 python bench.py --steps 10 --warmup 3 --act gelu
step gelu_tpb1 300 python bench.py --steps 10 --warmup 3 --act gelu --tpb 1
step tests 600 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread
