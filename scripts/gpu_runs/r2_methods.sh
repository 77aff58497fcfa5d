#!/bin/bash
# bench.py with the side-by-side methods (driver default command), plus a kernel trace of the ZeRO-2
# size-1-communicator path (where do the per-step fills/copies come from?)
source scripts/gpu_steps.sh
step bench_methods 400 python bench.py --steps 20 --warmup 5
step prof_zero 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_zero -o run -- python3 bench.py --steps 5 --warmup 2 --method zero --force_comm --methods none --observe_steps 0
