#!/bin/bash
source scripts/gpu_steps.sh
step cfg_c5_llama3_8b_ffn_L32_swiglu 900 python bench.py --json_out gpurun_out/cfg_c5_llama3_8b_ffn_L32_swiglu.json --steps 4 --warmup 2 --method hybrid --tp 1 --gated --act silu --ffn_dim 14336 --layers 32
step cfg_c5_llama3_8b_ffn_L32_swiglu_adam 900 python bench.py --json_out gpurun_out/cfg_c5_llama3_8b_ffn_L32_swiglu_adam.json --steps 4 --warmup 2 --method hybrid --tp 1 --gated --act silu --ffn_dim 14336 --layers 32 --optimizer adam
