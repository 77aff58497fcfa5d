#!/bin/bash
# Final tree: the GPU suite (port fixture change) and smoke
source scripts/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
