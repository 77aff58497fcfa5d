#!/bin/bash
# Round 3: (1) GEMM grid policies under a collective-like CU footprint (scripts/bench_occupancy.py);
# (2) the comm observer and a rocprofv3 kernel trace of the SAME process (observe_diag under rocprofv3), for ZeRO
# and FSDP at N=1 over size-1 communicators, to compare overlap_frac with the trace's own.
source scripts/gpu_steps.sh
export PYTHONUNBUFFERED=1
step occupancy 400 python -u scripts/bench_occupancy.py
step obs_zero_traced 300 rocprofv3 --kernel-trace -d gpurun_out/obs_zero -o run -- python3 -u scripts/observe_diag.py --method zero --steps 3
step obs_fsdp_traced 300 rocprofv3 --kernel-trace -d gpurun_out/obs_fsdp -o run -- python3 -u scripts/observe_diag.py --method fsdp --steps 3
