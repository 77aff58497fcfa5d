#!/bin/bash
# Round 3 (session 2), end: the driver's N>1 invocation rehearsed at N=2 on one GPU (gloo on device tensors) with split
# masters, then every BASELINE.json configuration (scripts/bench_configs.sh) with the tiles-per-CU wgrad-stream rule.
source scripts/gpu_steps.sh
export PYTHONUNBUFFERED=1
step rehearsal_n2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29702 bench.py --gpus 2 --steps 3 --warmup 1 --method_steps 2 --layers 2 --llama_layers 2 --backend gloo_gpu --json_out gpurun_out/rehearsal_n2.json
bash scripts/bench_configs.sh
