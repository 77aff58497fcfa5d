#!/bin/bash
# Round 6: the ReLU-mask dgrad loads its mask word at the start of the tile (DLLM_MASK_PRE=1, default) vs in the
# epilogue (build variant nomp): GEMM tests, per-GEMM bitwise + timing, the step interleaved (profiles/r6/mask_preload_r6.txt).
source scripts/gpu_steps.sh
NOMP=$PWD/distributed-llm-code-samples_amd/_dllm_native_nomp.so
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
step t_gemm 500 $T tests/test_gemm_gpu.py tests/test_gemm_nnwgrad_gpu.py
step epi_mp 300 python -u scripts/bench_epilogue_cost.py --libs $NOMP --rounds 5 --iters 6 --json gpurun_out/epi_mp.json
H="--steps 20 --warmup 5 --methods none --no_reference_init --phases"
for i in 1 2 3; do
  step head_mp_$i 300 python -u bench.py $H --json_out gpurun_out/head_mp_$i.json
  step head_nomp_$i 300 env DLLM_NATIVE_LIB=$NOMP python -u bench.py $H --json_out gpurun_out/head_nomp_$i.json
done
