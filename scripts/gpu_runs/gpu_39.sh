#!/bin/bash
# GEMM library split into per-layout translation units: full GPU suite + flagship bench.
source scripts/gpu_steps.sh
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench 300 python bench.py --steps 20 --warmup 5
