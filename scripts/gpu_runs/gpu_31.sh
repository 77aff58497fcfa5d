#!/bin/bash
# Full-size numerics of the current kernels (persistent blocks + ReLU masks) vs an independent torch step.
source scripts/gpu_steps.sh
step validate_full 600 python scripts/validate_full.py
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
