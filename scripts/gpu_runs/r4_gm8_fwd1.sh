#!/bin/bash
# Round 4: with the forward's second GEMM on hipBLASLt at N=1, the raster band of the remaining native NT GEMM (fwd1):
# --group_m_nt 8 vs 4 in the flagship step, interleaved.
source scripts/gpu_steps.sh
H="python -u bench.py --methods none --steps 20 --warmup 5"
for r in 1 2 3; do
  step gm4_$r 300 $H --json_out gpurun_out/gm4_$r.json
  step gm8_$r 300 $H --group_m_nt 8 --json_out gpurun_out/gm8_$r.json
done
