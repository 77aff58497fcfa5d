#!/bin/bash
# Round 3 end: the driver's exact N=1 command (headline + side-by-side methods), twice, plus smoke.
source scripts/gpu_steps.sh
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step driver_1 900 python3 bench.py --gpus 1 --steps 20 --warmup 5
step driver_2 900 python3 bench.py --gpus 1 --steps 20 --warmup 5
