#!/bin/bash
# Round 4 round-end rehearsal on one box: the whole GPU suite, smoke(), and the driver's N=1 command twice
# (exposed_ms_diff reproducibility within a box; compare with profiles/r4/driver_command_*_r4.json for across boxes).
source scripts/gpu_steps.sh
step pytest_gpu 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step driver_a 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json_out gpurun_out/driver_a.json
step driver_b 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json_out gpurun_out/driver_b.json
