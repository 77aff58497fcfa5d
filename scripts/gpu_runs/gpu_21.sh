#!/bin/bash
# Session re-entry check: full GPU test suite, smoke(), flagship bench (N=1), kernel stats.
source scripts/gpu_steps.sh
step gputests 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 20 --warmup 5
step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o p -- python3 bench.py --steps 5 --warmup 2
