#!/bin/bash
# PMC: HBM read / write requests per GEMM of the flagship step (fused-SGD wgrad vs bf16-storing wgrad via --side_opt)
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step pmc_fused 120 timeout -s KILL 110 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_fused -o p -- python3 bench.py --steps 2 --warmup 1 --methods none
step pmc_side 120 timeout -s KILL 110 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_side -o p -- python3 bench.py --steps 2 --warmup 1 --methods none --side_opt 32
