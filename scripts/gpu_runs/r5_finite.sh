#!/bin/bash
# Round 5: the driver's N=1 command after switching the bench to finite data (fan-in init; reference_init alongside).
source scripts/gpu_steps.sh
step driver_finite 700 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json_out gpurun_out/r5_driver_finite.json
