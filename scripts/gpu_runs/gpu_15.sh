#!/bin/bash
# Full GPU suite on the current build, then every BASELINE.json config on this box's one GPU.
source scripts/gpu_steps.sh
step gpu_tests 1200 python -m pytest tests -q -m gpu -x
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
bash scripts/bench_configs.sh
