#!/bin/bash
# Epilogue skew of the persistent GEMMs: correctness tests, then interleaved benches skew 0 / 4 / 2, then a
# kernel trace with the default (skew 4).
source scripts/gpu_steps.sh
step test_gemm 600 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread
for i in 1 2; do
  step b_s0_$i 300 python bench.py --steps 20 --warmup 5 --methods none --skew 0
  step b_s4_$i 300 python bench.py --steps 20 --warmup 5 --methods none --skew 4
  step b_s2_$i 300 python bench.py --steps 20 --warmup 5 --methods none --skew 2
done
step prof_skew 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_skew -o run -- python3 bench.py --steps 10 --warmup 3 --methods none
