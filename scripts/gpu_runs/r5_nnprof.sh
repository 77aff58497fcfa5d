#!/bin/bash
# Round 5: NN weight-gradient layout -- transposes on the compute vs the weight-gradient stream (interleaved), and the
# step's kernel trace.
source scripts/gpu_steps.sh
for i in 1 2; do
  step side0_$i 200 env DLLM_NN_TRANSPOSE_SIDE=0 python -u bench.py --steps 20 --warmup 5 --methods none
  step side1_$i 200 python -u bench.py --steps 20 --warmup 5 --methods none
  step tn_$i 200 python -u bench.py --steps 20 --warmup 5 --methods none --wgrad_layout tn
done
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_nn -o run -- python3 bench.py --steps 20 --warmup 5 --methods none
