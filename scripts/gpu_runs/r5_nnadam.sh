#!/bin/bash
# Round 5: NN weight-gradient layout for gated stacks with fused AdamW (EPI_ADAMS_T, NT DGLU): tests, then the
# Llama-3-8B-dims stack (L32 SwiGLU AdamW, config 5) tn vs auto, interleaved.
source scripts/gpu_steps.sh
step nn_tests 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_nnwgrad_gpu.py
C5="--methods none --optimizer adam --gated --act silu --ffn_dim 14336 --layers 32 --steps 6 --warmup 2"
for i in 1 2; do
  step c5_tn_$i 300 python -u bench.py $C5 --wgrad_layout tn
  step c5_nn_$i 300 python -u bench.py $C5
done
