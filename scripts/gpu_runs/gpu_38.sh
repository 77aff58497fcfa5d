#!/bin/bash
# Plain-PyTorch baseline of the reference algorithm (fp32 and bf16) vs the framework step, same box.
source scripts/gpu_steps.sh
step torch_bf16 600 python scripts/torch_baseline.py --dtype bf16 --steps 5
step torch_fp32 600 python scripts/torch_baseline.py --dtype fp32 --steps 2
step ours 300 python bench.py --steps 20 --warmup 5
