#!/bin/bash
# Round 4: the driver's N=1 command once more on the final tree (another box).
source scripts/gpu_steps.sh
step driver_g 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json_out gpurun_out/driver_g.json
