#!/bin/bash
# Round 5, finite data: the headline's kernel trace and serial-step MFMA busy per GEMM family.
source scripts/gpu_steps.sh
step prof_finite 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_finite -o run -- python3 bench.py --steps 20 --warmup 5 --methods none --no_reference_init
step pmc_finite 120 timeout -s KILL 110 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_finite -o p -- python3 bench.py --steps 2 --warmup 1 --methods none --no_reference_init
