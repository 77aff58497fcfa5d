#!/bin/bash
# Fresh per-kernel breakdown of the flagship step (N=1 fused path) and of the ZeRO path at world 1.
source scripts/gpu_steps.sh
step prof_default 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_default -o k -- python3 bench.py --steps 5 --warmup 2
step prof_zero1 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_zero1 -o k -- python3 bench.py --steps 5 --warmup 2 --force_comm --method zero
