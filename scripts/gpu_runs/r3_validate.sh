#!/bin/bash
# Round 3: whole GPU suite (FSDP per-weight chains, zero-copy custom all-reduce, observer, full-size wgrad-stream race
# screen), then the 256x128 family's co-residency skew experiment on the two slowest-vs-8ph shapes.
source scripts/gpu_steps.sh
export PYTHONUNBUFFERED=1
step pytest_gpu 1000 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
step pp_skew 300 python -u scripts/bench_gemm.py --variants tpb8,pp1,pp1s2,pp1s4,pp1s8 --cases fwd2,sgd --rounds 3 --iters 10 --no_torch
