#!/bin/bash
# Validation: the whole GPU test suite, smoke(), the default bench line (driver contract).
source scripts/gpu_steps.sh
step pytest_gpu 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python bench.py
