#!/bin/bash
# Round 5: whole-chip side-stream optimizer (side_optimizer -1) vs the fused AdamW epilogue on config 5; tests first.
source scripts/gpu_steps.sh
step side_tests 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_side_opt_gpu.py
C5="--methods none --optimizer adam --gated --act silu --ffn_dim 14336 --layers 32 --steps 6 --warmup 2"
for i in 1 2; do
  step c5_fused_$i 300 python -u bench.py $C5
  step c5_side_$i 300 python -u bench.py $C5 --side_opt -1
done
step flag_side 200 python -u bench.py --methods none --steps 20 --warmup 5 --side_opt -1
