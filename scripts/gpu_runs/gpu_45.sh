#!/bin/bash
source scripts/gpu_steps.sh
step c6 600 python bench.py --steps 4 --warmup 2 --method ddp --model_size 8192 --layers 8 --json_out gpurun_out/cfg_c6.json
