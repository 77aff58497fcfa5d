#!/bin/bash
# Round 5, last tree: the whole GPU suite and smoke().
source scripts/gpu_steps.sh
step pytest_gpu_last 1000 python -u -m pytest tests -m gpu -q --timeout 500 --timeout-method thread
step smoke_last 200 python -c "import __graft_entry__ as g; g.smoke()"
