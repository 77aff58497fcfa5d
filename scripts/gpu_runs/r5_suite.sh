#!/bin/bash
# Round 5: the whole GPU suite and smoke() on the current tree, then the 8-phase (persistent, balanced reads) vs
# 4-phase main loops on the FFN shapes (interleaved, one process).
source scripts/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step gemm_var 300 python3 scripts/bench_gemm.py --variants tpb8,8phase_stagger,4phase_stagger --rounds 3 --iters 10 --no_torch
