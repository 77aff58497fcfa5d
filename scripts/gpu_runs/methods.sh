#!/bin/bash
# The reference's methods side by side at N=1 over size-1 communicators (ddp, zero, fsdp, tp, hybrid), with the
# comm observer's per-role collective time and hidden fraction; the BASELINE.json configurations (bench_configs.sh).
source scripts/gpu_steps.sh
step methods 900 python bench.py --steps 10 --warmup 3 --json_out gpurun_out/methods.json
step configs 900 bash scripts/bench_configs.sh
