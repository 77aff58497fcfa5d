#!/bin/bash
# Round 3 end (session 3): the driver's N=2 / N=4 invocations rehearsed on one GPU (ranks share the card over gloo).
source scripts/gpu_steps.sh
step rehearsal_n2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29702 bench.py --gpus 2 --steps 3 --warmup 1 --method_steps 2 --layers 2 --llama_layers 2 --backend gloo_gpu --json_out gpurun_out/rehearsal_n2.json
step rehearsal_n4 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29703 bench.py --gpus 4 --steps 3 --warmup 1 --method_steps 2 --layers 2 --llama_layers 2 --backend gloo_gpu --json_out gpurun_out/rehearsal_n4.json
