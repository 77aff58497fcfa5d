#!/bin/bash
# Round 5, final tree: the whole GPU suite, smoke(), and the driver's N=1 command (headline + reference_init + methods).
source scripts/gpu_steps.sh
step pytest_gpu 1100 python -u -m pytest tests -m gpu -q --timeout 500 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step driver_final 700 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json_out gpurun_out/r5_driver_final.json
