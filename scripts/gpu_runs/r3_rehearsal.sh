#!/bin/bash
# Round 3: rehearse the driver's N>1 bench invocation on one GPU -- torchrun with 2 and 4 ranks sharing cuda:0,
# collectives over gloo on device tensors (--backend gloo_gpu): headline ZeRO-2 dp N plus every side method at N.
# Plumbing only (ranks share one GPU; gloo stages through the host), reduced depth to keep it short.
source scripts/gpu_steps.sh
export PYTHONUNBUFFERED=1
for n in 2 4; do
  step rehearsal_n$n 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29700 + n)) bench.py --gpus $n --steps 3 --warmup 1 --method_steps 2 --layers 2 --llama_layers 2 --backend gloo_gpu --json_out gpurun_out/rehearsal_n$n.json
done
