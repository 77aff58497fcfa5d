#!/bin/bash
# Round 5: MFMA busy per GEMM family in the NN-layout flagship step (PMC, its own pass).
source scripts/gpu_steps.sh
step pmc_nn 120 timeout -s KILL 110 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_nn -o p -- python3 bench.py --steps 2 --warmup 1 --methods none
