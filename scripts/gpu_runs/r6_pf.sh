#!/bin/bash
# Round 6: epilogue-operand prefetch (counted LDS-DMA of the fused-optimizer planes / ReLU mask / SwiGLU pre-activations
# during the tile's last K-tiles).  Per-GEMM bitwise + timing vs the DLLM_EPI_PF=0 build, numerics tests, and the
# flagship step interleaved with both builds.
source scripts/gpu_steps.sh
NOPF=distributed-llm-code-samples_amd/_dllm_native_nopf.so
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
step epi_pf 600 python -u scripts/bench_epilogue_cost.py --libs $NOPF --json gpurun_out/epi_pf.json
step t_gemm 900 $T tests/test_gemm_gpu.py tests/test_gemm_nnwgrad_gpu.py tests/test_split_master_gpu.py tests/test_engine_gpu.py
H="--steps 20 --warmup 5 --methods none --no_reference_init"
for i in 1 2 3; do
  step head_pf_$i 240 python -u bench.py $H --json_out gpurun_out/head_pf_$i.json
  step head_nopf_$i 240 env DLLM_NATIVE_LIB=$NOPF python -u bench.py $H --json_out gpurun_out/head_nopf_$i.json
done
