#!/bin/bash
# Round 3: comm observer vs a kernel trace of the same process (ZeRO, FSDP at N=1 over size-1 communicators),
# the observer GPU tests, the occupancy bench under a trace (is the stand-in resident next to the GEMM?), and the
# gated (Llama-dims) stack with / without the wgrad stream at 16 HW queues plus its kernel stats.
source scripts/gpu_steps.sh
export PYTHONUNBUFFERED=1
step obs_test 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_observe_gpu.py
step obs_zero_traced 300 rocprofv3 --kernel-trace -d gpurun_out/obs_zero -o run -- python3 -u scripts/observe_diag.py --method zero --steps 3
step obs_fsdp_traced 300 rocprofv3 --kernel-trace -d gpurun_out/obs_fsdp -o run -- python3 -u scripts/observe_diag.py --method fsdp --steps 3
step occ_traced 300 rocprofv3 --kernel-trace -d gpurun_out/occ -o run -- python3 -u scripts/bench_occupancy.py --cases dx --policies tpb8,tpb8b2 --blocks 0,64 --rounds 1 --iters 4
L="--methods none --layers 32 --ffn_dim 14336 --gated --act silu --steps 4 --warmup 2"
step gated_ws 600 python -u bench.py $L --json_out gpurun_out/gated_ws.json
step gated_nows 600 python -u bench.py $L --no-wgrad_stream --json_out gpurun_out/gated_nows.json
step gated_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/gated_prof -o run -- python3 bench.py $L --no-wgrad_stream --steps 2 --warmup 1
