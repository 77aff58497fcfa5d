#!/bin/bash
# Full validation of the current tree: GPU test suite, smoke(), default bench.
source scripts/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py --steps 20 --warmup 5
