#!/bin/bash
# Round 5: serial backward, NN vs TN weight gradients -- per-kernel traces, then interleaved step pairs.
source scripts/gpu_steps.sh
step prof_s_tn 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s_tn -o run -- python3 bench.py --steps 20 --warmup 5 --methods none --no-wgrad_stream --wgrad_layout tn
step prof_s_nn 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s_nn -o run -- python3 bench.py --steps 20 --warmup 5 --methods none --no-wgrad_stream --wgrad_layout nn
for i in 1 2 3; do
  step s_tn_$i 200 python -u bench.py --steps 20 --warmup 5 --methods none --wgrad_layout tn --no-wgrad_stream
  step s_nn_$i 200 python -u bench.py --steps 20 --warmup 5 --methods none --wgrad_layout nn --no-wgrad_stream
  step c_tn_$i 200 python -u bench.py --steps 20 --warmup 5 --methods none --wgrad_layout tn
done
