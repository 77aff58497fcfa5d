#!/bin/bash
# Round 5: nontemporal epilogue stores (build variant DLLM_EPI_NT=1) vs the production build: isolated GEMMs
# (bitwise-checked) and the flagship step, interleaved.
source scripts/gpu_steps.sh
export PYTHONUNBUFFERED=1
LIB=distributed-llm-code-samples_amd/_dllm_native_ntst.so
step gemm_ntst 300 python3 scripts/bench_gemm.py --variants 8phase_stagger --no_torch --libs $LIB --rounds 3
for i in 1 2 3; do
  step head_base_$i 240 python3 bench.py --steps 20 --warmup 5 --methods none --json_out gpurun_out/ntst_base_$i.json
  step head_ntst_$i 240 env DLLM_NATIVE_LIB=$LIB python3 bench.py --steps 20 --warmup 5 --methods none --json_out gpurun_out/ntst_nt_$i.json
done
