#!/bin/bash
source scripts/gpu_steps.sh
step w4 300 python scripts/bench_w4.py
step w4_pmc 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/w4_pmc -o p -- python3 scripts/bench_w4.py
step w4_pmc2 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS TCC_HIT TCC_MISS --output-format csv -d gpurun_out/w4_pmc2 -o p -- python3 scripts/bench_w4.py
