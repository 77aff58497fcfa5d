#!/bin/bash
# Round 3 (session 2): split fp32 master (bf16 working copy + 16-bit residual) in the fused-SGD weight-gradient
# GEMM: numerics vs the fp32-master form and interleaved timing; the default bench line on the same box.
source scripts/gpu_steps.sh
step sgd_split 300 python -u scripts/bench_sgd_split.py --rounds 7 --iters 10
step bench_default 300 python -u bench.py --methods none
