#!/bin/bash
# Round 5: the whole GPU suite (incl. the 2-rank NN layout test) and smoke after decoupling W2 storage; headline.
source scripts/gpu_steps.sh
step pytest_gpu 1100 python -u -m pytest tests -m gpu -q --timeout 500 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step headline 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --methods none
