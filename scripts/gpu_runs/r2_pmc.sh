#!/bin/bash
# PMC: L2 hit rate, effective clock and MFMA busy per GEMM of the flagship step (own passes, --pmc only)
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step pmc_l2 120 timeout -s KILL 110 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_l2 -o p -- python3 bench.py --steps 2 --warmup 1 --methods none
