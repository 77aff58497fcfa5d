#!/bin/bash
# fp32 kernel with the XOR-2-safe K-contiguous swizzle: numerics, throughput vs torch, bank-conflict PMC (fp32 NT
# and the flagship bf16 step)
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step test_fp32 600 python -u -m pytest tests/test_gemm_gpu.py -x -q -k "fp32" --timeout 120 --timeout-method thread
step bench_fp32 300 python scripts/bench_fp32.py
step pmc_f32_c 120 timeout -s KILL 110 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_f32_c -o p -- python3 scripts/pmc_fp32.py nt
step pmc_bf16 120 timeout -s KILL 110 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_bf16 -o p -- python3 bench.py --steps 2 --warmup 1 --methods none
