#!/bin/bash
# Round 4: the weight-gradient product [16384, 4096] K=8192 as TN (the step's layout), NN and NT: the layout's cost.
source scripts/gpu_steps.sh
step tn_layout 180 python -u scripts/bench_sgd_epilogue.py --layouts
