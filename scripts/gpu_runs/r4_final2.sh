#!/bin/bash
# Round 4, after the side-stream policy change: the driver's N=1 command and the N=2 / N=4 rehearsals (torchrun and
# bench.py's own launcher over gloo on one GPU).
source scripts/gpu_steps.sh
step driver_e 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json_out gpurun_out/driver_e.json
bash scripts/gpu_runs/rehearsal.sh || exit $?
