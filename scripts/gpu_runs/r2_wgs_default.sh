#!/bin/bash
# Default bench with the concurrent weight-gradient stream on (N=1 headline), its bitwise test, and the graph path
source scripts/gpu_steps.sh
step tests 300 python -u -m pytest tests/test_engine_gpu.py tests/test_graph_gpu.py -q -x --timeout 120 --timeout-method thread
step bench 300 python bench.py
step bench_graph 120 python bench.py --graph --methods none --steps 10 --warmup 3
