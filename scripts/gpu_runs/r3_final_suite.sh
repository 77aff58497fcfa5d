#!/bin/bash
# Round 3 end (session 3): the whole GPU suite and smoke on the final tree.
source scripts/gpu_steps.sh
step pytest_gpu 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
