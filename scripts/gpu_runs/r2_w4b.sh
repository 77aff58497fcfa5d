#!/bin/bash
# 4-wave / 4-stage NT GEMM prototype vs 8-phase vs hipBLASLt (random operands)
source scripts/gpu_steps.sh
step w4b 300 python experiments/bench_w4b.py
