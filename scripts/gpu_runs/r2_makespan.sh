#!/bin/bash
# makespan-optimal tiles per persistent block: GEMM tests, flagship bench, MP F=14336 (1792-tile GEMMs) A/B vs cap 4
source scripts/gpu_steps.sh
step test_gemm 600 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread
for i in 1 2; do
  step flag_$i 300 python bench.py --steps 20 --warmup 5 --methods none
  step tp14k_new_$i 300 python bench.py --steps 20 --warmup 5 --methods none --method tp --ffn_dim 14336 --layers 1
  step tp14k_cap4_$i 300 python bench.py --steps 20 --warmup 5 --methods none --method tp --ffn_dim 14336 --layers 1 --tpb 4
  step tp14k_cap2_$i 300 python bench.py --steps 20 --warmup 5 --methods none --method tp --ffn_dim 14336 --layers 1 --tpb 2
done
