#!/bin/bash
source scripts/gpu_steps.sh
ARGS="python3 scripts/bench_gemm.py --variants 8phase_stagger --rounds 1 --iters 3 --no_torch"
step pmc_a 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_a -o p -- $ARGS
step pmc_b 600 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS TCC_HIT TCC_MISS --output-format csv -d gpurun_out/pmc_b -o p -- $ARGS
step pmc_c 600 rocprofv3 --pmc TA_BUSY_ TCP_PENDING_STALL_CYCLES_ TCC_EA0_RDREQ_ SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM --output-format csv -d gpurun_out/pmc_c -o p -- $ARGS
