#!/bin/bash
# Round 4 start: box environment (HW queue setting), the driver's N=1 command, headline kernel stats.
source scripts/gpu_steps.sh
{ echo "GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES-<unset>}"; env | grep -E '^(HIP|HSA|GPU|NCCL|RCCL|OMP)_' | sort; rocm-smi --showclocks 2>/dev/null | head -20; } > gpurun_out/env.txt 2>&1
step driver_1 600 python3 bench.py --gpus 1 --steps 20 --warmup 5
step headline_stats 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_head -o run -- python3 bench.py --gpus 1 --steps 10 --warmup 3 --methods none
