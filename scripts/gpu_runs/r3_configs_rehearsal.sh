#!/bin/bash
# Round 3: the driver's N>1 invocation rehearsed at N=2 on one GPU (gloo on device tensors), the side-optimizer test, then
# every BASELINE.json configuration (scripts/bench_configs.sh).
# Regenerates profiles/r3/bench_rehearsal_gloo_gpu_n2_split_master_r3.json, bench_configs_split_master_r3.jsonl.
source scripts/gpu_steps.sh
export PYTHONUNBUFFERED=1
step rehearsal_n2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29702 bench.py --gpus 2 --steps 3 --warmup 1 --method_steps 2 --layers 2 --llama_layers 2 --backend gloo_gpu --json_out gpurun_out/rehearsal_n2.json
step pytest_sideopt 300 python -u -m pytest tests/test_side_opt_gpu.py -x -q --timeout 120 --timeout-method thread
bash scripts/bench_configs.sh
