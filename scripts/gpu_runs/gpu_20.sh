#!/bin/bash
# Phase breakdown (HIP events) of the flagship step and of the ZeRO path; roctx ranges in a marker trace.
source scripts/gpu_steps.sh
step phases_default 600 python bench.py --steps 10 --warmup 3 --phases
step phases_zero1 600 python bench.py --steps 10 --warmup 3 --phases --force_comm --method zero
export DLLM_ROCTX=1
step marker_trace 600 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv -d gpurun_out/marker -o m -- python3 bench.py --steps 3 --warmup 1
