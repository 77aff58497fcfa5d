#!/bin/bash
# Epilogue skew with small K offsets per group (skew = groups + 256*k_tiles_per_group): keeps the groups within
# the L2 reuse window of their shared operand panels (skew by 1/4 tile was 12% slower: panel reuse lost)
source scripts/gpu_steps.sh
for i in 1 2; do
  step c_s0_$i 300 python bench.py --steps 20 --warmup 5 --methods none --skew 0
  step c_s4x2_$i 300 python bench.py --steps 20 --warmup 5 --methods none --skew $((4 + 256*2))
  step c_s4x4_$i 300 python bench.py --steps 20 --warmup 5 --methods none --skew $((4 + 256*4))
  step c_s2x8_$i 300 python bench.py --steps 20 --warmup 5 --methods none --skew $((2 + 256*8))
done
