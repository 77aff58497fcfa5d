#!/bin/bash
# Round 3 (session 2): per-kernel time and PMC of the serial flagship step (no wgrad stream, so each GEMM runs alone)
# with split vs fp32 masters: kernel trace stats, then one PMC pass each (MFMA busy, GRBM clock, L2 hits).
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step trace_split 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ser_split -o s -- python3 bench.py --methods none --steps 6 --warmup 2 --no-wgrad_stream
step trace_fp32 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ser_fp32 -o s -- python3 bench.py --methods none --steps 6 --warmup 2 --no-wgrad_stream --master fp32
step pmc_split 120 timeout -s KILL 110 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_split -o p -- python3 bench.py --steps 2 --warmup 1 --methods none --no-wgrad_stream
step pmc_fp32 120 timeout -s KILL 110 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_fp32 -o p -- python3 bench.py --steps 2 --warmup 1 --methods none --no-wgrad_stream --master fp32
