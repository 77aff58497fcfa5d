#!/bin/bash
# Round 3: DLLM_SIDE_STREAMS=auto (only the weight-gradient stream at high priority) vs pool; headline without and
# with a live communicator, interleaved x3, and the methods once each (they never use the weight-gradient stream).
source scripts/gpu_steps.sh
H="python -u bench.py --gpus 1 --steps 20 --warmup 5"
M="python -u bench.py --gpus 1 --steps 10 --warmup 3 --method_steps 10 --methods ddp,zero,fsdp,hybrid"
step tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_split_master_gpu.py -k "side_streams or engine"
for r in 1 2 3; do
  step head_auto_$r 300 env DLLM_SIDE_STREAMS=auto $H --methods none
  step head_pool_$r 300 env DLLM_SIDE_STREAMS=pool $H --methods none
  step comm_auto_$r 300 env DLLM_SIDE_STREAMS=auto $H --methods ddp --dist_first
  step comm_pool_$r 300 env DLLM_SIDE_STREAMS=pool $H --methods ddp --dist_first
done
step m_auto 600 env DLLM_SIDE_STREAMS=auto $M --json_out gpurun_out/m_auto.json
step m_pool 600 env DLLM_SIDE_STREAMS=pool $M --json_out gpurun_out/m_pool.json
