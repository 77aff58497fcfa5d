#!/bin/bash
# Round 4 final tree: rocprofv3 kernel stats of the flagship step and of the TP8-shard MP step (no splitk_reduce).
source scripts/gpu_steps.sh
step prof_head_final 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_head_final -o run -- python3 bench.py --gpus 1 --steps 10 --warmup 3 --methods none
step prof_tp8_final 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tp8_final -o run -- python3 bench.py --steps 20 --warmup 3 --methods none --method tp --ffn_dim 1792 --layers 1
