#!/bin/bash
# PMC passes (own runs, --pmc only): L2 hit rate, effective clock, MFMA busy; HBM requests per GEMM of the step.
source scripts/gpu_steps.sh
step pmc_l2 120 timeout -s KILL 110 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_l2 -o p -- python3 bench.py --steps 2 --warmup 1 --methods none
step pmc_hbm 120 timeout -s KILL 110 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d gpurun_out/pmc_hbm -o p -- python3 bench.py --steps 2 --warmup 1 --methods none
