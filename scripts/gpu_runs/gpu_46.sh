#!/bin/bash
# Launch-gap check: eager step vs HIP-graph-captured step (same kernels), interleaved.
source scripts/gpu_steps.sh
step eager1 300 python bench.py --steps 30 --warmup 5
step graph1 300 python bench.py --steps 30 --warmup 5 --graph
step eager2 300 python bench.py --steps 30 --warmup 5
step graph2 300 python bench.py --steps 30 --warmup 5 --graph
