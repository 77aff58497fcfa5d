#!/bin/bash
# Round-2 end-state profiles: flagship step (defaults: 4 tiles per persistent block), ZeRO-2 force_comm step
source scripts/gpu_steps.sh
step prof_dp1 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dp1 -o run -- python3 bench.py --steps 10 --warmup 3 --methods none
step prof_zero 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_zero -o run -- python3 bench.py --steps 10 --warmup 3 --methods none --method zero --force_comm
