#!/bin/bash
# Round 5: the whole GPU suite after the NN weight-gradient default.
source scripts/gpu_steps.sh
step pytest_gpu 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
