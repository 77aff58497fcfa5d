#!/bin/bash
# TN (weight-gradient) main-loop variants: 8-phase (one tile / persistent 2) vs 4-phase, random operands.
source scripts/gpu_steps.sh
step tn_variants 300 python scripts/bench_gemm.py --variants tpb1,tpb2,4phase_stagger --no_torch --rounds 3 --cases dW
