#!/bin/bash
# Re-entry validation of the restored tree: GPU suite, smoke, default bench (driver contract).
source scripts/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python bench.py
step bench_fp32 300 python scripts/bench_fp32.py
