#!/bin/bash
# MFMA utilisation of the flagship step's kernels (PMC, own pass; no tracing domains combined with --pmc).
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step pmc_step 120 timeout -s KILL 110 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/pmc_step -o p -- python3 bench.py --steps 2 --warmup 1
