#!/bin/bash
# fp32 (reference dtype) flagship step: bf16x6 split GEMMs vs the fp32 MFMA kernel; kernel stats of the split path;
# TP engine/custom-AR tests after deferring the last layer's TP output exchange
source scripts/gpu_steps.sh
step tp_tests 400 python -u -m pytest tests/test_car_gpu.py tests/test_engine_gpu.py -q --timeout 120 --timeout-method thread
step f32_split 300 python bench.py --dtype fp32 --grad_dtype fp32 --methods none --steps 5 --warmup 2 --fp32_gemm bf16x6
step f32_mfma 300 python bench.py --dtype fp32 --grad_dtype fp32 --methods none --steps 5 --warmup 2 --fp32_gemm mfma_f32
step f32_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f32 -o f32 -- python bench.py --dtype fp32 --grad_dtype fp32 --methods none --steps 3 --warmup 1
step cli_fp32 600 python train_ffns.py -s 16 -bs 8 -n 1024 -l 1 -d 8192 -m 0 -r 1
