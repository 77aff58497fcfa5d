#!/bin/bash
# Round 3 end (session 3): smoke, the driver's exact N=1 command twice, and a kernel-stats profile of the headline.
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step driver_1 900 python3 bench.py --gpus 1 --steps 20 --warmup 5
step driver_2 900 python3 bench.py --gpus 1 --steps 20 --warmup 5
step head_stats 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o head -- python3 bench.py --methods none --steps 10 --warmup 3
