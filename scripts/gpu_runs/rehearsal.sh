#!/bin/bash
# The driver's N>1 bench invocations rehearsed on one GPU: ranks share the card over gloo (RCCL refuses two ranks on one
# device), both through torchrun and through bench.py's own launcher (no WORLD_SIZE: it starts the N ranks itself).
source scripts/gpu_steps.sh
export PYTHONUNBUFFERED=1
R="--steps 3 --warmup 1 --method_steps 2 --layers 2 --llama_layers 2 --backend gloo_gpu"
step rehearsal_n2_torchrun 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29702 bench.py --gpus 2 $R --json_out gpurun_out/rehearsal_n2.json
step rehearsal_n2_self 600 python bench.py --gpus 2 $R --json_out gpurun_out/rehearsal_n2_self.json
step rehearsal_n4_self 600 python bench.py --gpus 4 $R --json_out gpurun_out/rehearsal_n4_self.json
