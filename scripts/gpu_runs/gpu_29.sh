#!/bin/bash
# Persistence restricted to ReLU / store / SGD kernels: Llama, GELU and flagship, both settings, same box.
source scripts/gpu_steps.sh
step tests 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/tests.log && ! grep -q -E "[0-9]+ failed" gpurun_out/tests.log || exit 1
L="--steps 4 --warmup 2 --method hybrid --tp 1 --gated --act silu --ffn_dim 14336 --layers 32"
step llama_tpb2 600 python bench.py $L
step llama_tpb1 600 python bench.py $L --tpb 1
step flag_tpb2 300 python bench.py --steps 20 --warmup 5
step flag_tpb1 300 python bench.py --steps 20 --warmup 5 --tpb 1
step gelu_tpb2 300 python bench.py --steps 10 --warmup 3 --act gelu
step gelu_tpb1 300 python bench.py --steps 10 --warmup 3 --act gelu --tpb 1
step flag_tpb2b 300 python bench.py --steps 20 --warmup 5
