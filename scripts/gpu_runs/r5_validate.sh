#!/bin/bash
# Round 5 (after the NN weight-gradient layout): the whole GPU suite, smoke(), the driver's full N=1 command with
# every side method, and a second headline run.
source scripts/gpu_steps.sh
step pytest_gpu 1000 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step driver_full 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json_out gpurun_out/r5_driver_full_nn.json
step headline2 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --methods none
