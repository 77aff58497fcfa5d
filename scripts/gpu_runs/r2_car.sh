#!/bin/bash
# custom all-reduce protocol timing, 2 and 4 ranks as processes sharing one GPU (not xGMI)
source scripts/gpu_steps.sh
step bench_car 300 python scripts/bench_car.py --ranks 2,4
