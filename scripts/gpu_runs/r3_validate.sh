#!/bin/bash
# Round 3: whole GPU suite (FSDP per-weight chains, zero-copy custom all-reduce, observer, full-size wgrad-stream race
# screen), smoke(); the comm observer with the native RCCL layer (execution spans) against a trace of the same
# process; the 256x128 family's co-residency skew experiment on the two slowest-vs-8ph shapes.
source scripts/gpu_steps.sh
export PYTHONUNBUFFERED=1
step pytest_gpu 700 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread
step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
step obsn_zero_traced 300 rocprofv3 --kernel-trace -d gpurun_out/obsn_zero -o run -- python3 -u scripts/observe_diag.py --method zero --steps 3 --comm native
step obsn_fsdp_traced 300 rocprofv3 --kernel-trace -d gpurun_out/obsn_fsdp -o run -- python3 -u scripts/observe_diag.py --method fsdp --steps 3 --comm native
step pp_skew 300 python -u scripts/bench_gemm.py --variants tpb8,pp1,pp1s2,pp1s4,pp1s8 --cases fwd2,sgd --rounds 3 --iters 10 --no_torch
