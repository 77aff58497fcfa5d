#!/bin/bash
# Round 5, final tree (NN weight-gradient layout, finite data): LDS conflicts, wait/issue-stall split, L2 hit rate and
# HBM requests per GEMM family of the headline step (each pass its own run, --pmc only).
source scripts/gpu_steps.sh
S="python3 bench.py --steps 2 --warmup 1 --methods none --no_reference_init"
step pmc_sq 120 timeout -s KILL 110 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_sq -o p -- $S
step pmc_tcc 120 timeout -s KILL 110 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_tcc -o p -- $S
