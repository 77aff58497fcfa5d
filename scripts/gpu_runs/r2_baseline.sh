#!/bin/bash
# Round-2 baseline: default bench (driver contract), ddp/fsdp force_comm, and a rocprofv3 kernel-stats run.
source scripts/gpu_steps.sh
step bench 300 python bench.py --steps 20 --warmup 5
step bench2 300 python bench.py --steps 20 --warmup 5
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 10 --warmup 3
