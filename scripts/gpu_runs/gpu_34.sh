#!/bin/bash
# Kernel stats of the Llama-3-8B-dims gated stack (L32 D4096 F14336 SwiGLU, SGD) at the current defaults.
source scripts/gpu_steps.sh
step prof_llama 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profl -o l -- python3 bench.py --steps 3 --warmup 1 --method hybrid --tp 1 --gated --act silu --ffn_dim 14336 --layers 32
