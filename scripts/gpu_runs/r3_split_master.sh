#!/bin/bash
# Round 3: split fp32 masters -- numerics (GPU tests), the fused-SGD wgrad GEMMs in both forms (bench_sgd_split.py),
# per-GEMM time and MFMA-busy of the serial step in both forms (kernel trace + one PMC pass each).
# Regenerates profiles/r3/sgd_split_gemm_r3.log, pmc_mfma_serial_split_vs_fp32_r3.txt (see profiles/README.md).
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step pytest_split 300 python -u -m pytest tests/test_split_master_gpu.py tests/test_side_opt_gpu.py -x -v --timeout 120 --timeout-method thread
step sgd_split 300 python -u scripts/bench_sgd_split.py --rounds 7 --iters 10
step trace_split 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ser_split -o s -- python3 bench.py --methods none --steps 6 --warmup 2 --no-wgrad_stream
step trace_fp32 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ser_fp32 -o s -- python3 bench.py --methods none --steps 6 --warmup 2 --no-wgrad_stream --master fp32
step pmc_split 120 timeout -s KILL 110 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_split -o p -- python3 bench.py --steps 2 --warmup 1 --methods none --no-wgrad_stream
step pmc_fp32 120 timeout -s KILL 110 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_fp32 -o p -- python3 bench.py --steps 2 --warmup 1 --methods none --no-wgrad_stream --master fp32
