#!/bin/bash
# PMC passes over the fp32 NT GEMM (native vs torch): MFMA busy, LDS bank conflicts / waits, VALU, clock
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step pmc_f32_a 120 timeout -s KILL 110 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_f32_a -o p -- python3 scripts/pmc_fp32.py nt
step pmc_f32_b 120 timeout -s KILL 110 rocprofv3 --pmc SQ_INSTS_MFMA SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES GRBM_COUNT --output-format csv -d gpurun_out/pmc_f32_b -o p -- python3 scripts/pmc_fp32.py nt
