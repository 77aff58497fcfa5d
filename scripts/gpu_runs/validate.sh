#!/bin/bash
# Validation: the whole GPU test suite, smoke(), the driver's N=1 bench command (driver contract), the MP (TP8) shard.
source scripts/gpu_steps.sh
step pytest_gpu 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step driver 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 --json_out gpurun_out/driver.json
step tp8 200 python -u bench.py --method tp --ffn_dim 1792 --layers 1 --methods none --steps 100 --warmup 20 --json_out gpurun_out/tp8.json
