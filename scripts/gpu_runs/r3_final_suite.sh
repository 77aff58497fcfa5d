#!/bin/bash
# Round 3 end (session 3): the whole GPU suite on the final tree.
source scripts/gpu_steps.sh
step pytest_gpu 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
