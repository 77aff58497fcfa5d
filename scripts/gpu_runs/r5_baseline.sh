#!/bin/bash
# Round 5: native-only tree (hipBLASLt routing removed).  Balanced 8-phase reads (DLLM_BPRE=1, production) vs the
# round-4 read order (variant build bpre0): bitwise equality + interleaved per-GEMM timing, the per-barrier stamp
# timeline (DLLM_STAMP build), the driver's command on both builds, a rocprofv3 kernel trace of the production
# headline, the new GPU tests, and the config-5 AdamW A/B (fused epilogue vs side-stream AdamW).
source scripts/gpu_steps.sh
B0=$PWD/distributed-llm-code-samples_amd/_dllm_native_bpre0.so
step gemm_ab 400 python3 scripts/bench_gemm.py --libs $B0 --rounds 3 --iters 10 --no_torch
if [ -f distributed-llm-code-samples_amd/_dllm_native_stamp.so ]; then
  step stamps 200 env DLLM_NATIVE_LIB=$PWD/distributed-llm-code-samples_amd/_dllm_native_stamp.so python3 scripts/stamp_gemm.py
fi
step driver_new 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --methods none --json_out gpurun_out/r5_driver_new.json
step driver_old 200 env DLLM_NATIVE_LIB=$B0 python3 bench.py --gpus 1 --steps 20 --warmup 5 --methods none --json_out gpurun_out/r5_driver_old.json
step driver_new2 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --methods none --json_out gpurun_out/r5_driver_new2.json
step prof 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5 -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --methods none
step newtests 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_streams_gpu.py tests/test_side_opt_gpu.py tests/test_comm_gpu.py tests/test_car_gpu.py -x -q --timeout 200 --timeout-method thread -k "vendor or loaded or role or queue or side or fsdp_copying or tp_engine"
step adam_fused 200 python3 bench.py --methods none --optimizer adam --gated --act silu --ffn_dim 14336 --layers 32 --steps 10 --warmup 3 --json_out gpurun_out/r5_adam_fused.json
step adam_side32 200 python3 bench.py --methods none --optimizer adam --gated --act silu --ffn_dim 14336 --layers 32 --steps 10 --warmup 3 --side_opt 32 --json_out gpurun_out/r5_adam_side32.json
