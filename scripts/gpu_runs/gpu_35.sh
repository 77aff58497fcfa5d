#!/bin/bash
# Paired-access DGLU epilogue: gated numerics tests, Llama-dims step, kernel stats.
source scripts/gpu_steps.sh
step tests 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_engine_gpu.py tests/test_api_gpu.py -x -q --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/tests.log && ! grep -q -E "[0-9]+ failed" gpurun_out/tests.log || exit 1
L="--steps 4 --warmup 2 --method hybrid --tp 1 --gated --act silu --ffn_dim 14336 --layers 32"
step llama1 600 python bench.py $L
step llama2 600 python bench.py $L
step prof_llama 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profl -o l -- python3 bench.py --steps 3 --warmup 1 --method hybrid --tp 1 --gated --act silu --ffn_dim 14336 --layers 32
