#!/bin/bash
# Round 5: the driver's N=2 / N=4 invocations rehearsed over gloo on one GPU with the NN weight-gradient default.
source scripts/gpu_steps.sh
export PYTHONUNBUFFERED=1
R="--steps 3 --warmup 1 --method_steps 2 --layers 2 --llama_layers 2 --backend gloo_gpu"
step rehearse_n2 400 python3 bench.py --gpus 2 $R --json_out gpurun_out/rehearse_nn_n2.json
step rehearse_n4 400 python3 bench.py --gpus 4 $R --json_out gpurun_out/rehearse_nn_n4.json
