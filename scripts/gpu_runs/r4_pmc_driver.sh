#!/bin/bash
# Round 4: serial-step MFMA busy per GEMM family (--pmc pass of its own; VERDICT item 3's metric), then the driver's
# N=1 command with the round-4 tree (forced-comm methods on one block per CU).
source scripts/gpu_steps.sh
step pmc_mfma 120 timeout -s KILL 110 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_mfma -o p -- python3 bench.py --steps 2 --warmup 1 --methods none --no-wgrad_stream
step driver_d 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json_out gpurun_out/driver_d.json
