#!/bin/bash
# Round 5 evidence on the final kernels: serial-step MFMA busy per GEMM family (PMC), the weight-gradient product as
# TN / NN / NT (bf16 store, isolated), and the driver's N=2 / N=4 invocations rehearsed over gloo on one GPU.
source scripts/gpu_steps.sh
step pmc_mfma 120 timeout -s KILL 110 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_mfma -o p -- python3 bench.py --steps 2 --warmup 1 --methods none --no-wgrad_stream
step tn_layout 180 python -u scripts/bench_sgd_epilogue.py --layouts
export PYTHONUNBUFFERED=1
R="--steps 3 --warmup 1 --method_steps 2 --layers 2 --llama_layers 2 --backend gloo_gpu"
step rehearse_n2 400 python3 bench.py --gpus 2 $R --json_out gpurun_out/rehearse_n2.json
step rehearse_n4 400 python3 bench.py --gpus 4 $R --json_out gpurun_out/rehearse_n4.json
