#!/bin/bash
# Round 5: the driver's N=8 invocation rehearsed on one GPU -- 8 self-launched ranks sharing the card over gloo
# (RCCL refuses two ranks on one device; plumbing at world 8, not a measurement).
source scripts/gpu_steps.sh
export PYTHONUNBUFFERED=1
step rehearsal_n8_self 900 python bench.py --gpus 8 --steps 3 --warmup 1 --method_steps 2 --layers 2 --llama_layers 2 --backend gloo_gpu --json_out gpurun_out/rehearsal_n8_self.json
