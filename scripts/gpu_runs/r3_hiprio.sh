#!/bin/bash
# Round 3: engine side streams (wgrad / opt / fsdp) as native high-priority streams (DLLM_SIDE_STREAMS=high, own
# queue set per priority) vs torch pool streams; headline with and without a live communicator, methods; interleaved.
source scripts/gpu_steps.sh
H="python -u bench.py --gpus 1 --steps 20 --warmup 5"
M="python -u bench.py --gpus 1 --steps 10 --warmup 3 --method_steps 10 --methods ddp,zero,fsdp,hybrid"
step tests 300 env DLLM_SIDE_STREAMS=high python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py tests/test_split_master_gpu.py
for r in 1 2; do
  step head_high_$r 300 env DLLM_SIDE_STREAMS=high $H --methods none
  step head_pool_$r 300 env DLLM_SIDE_STREAMS=pool $H --methods none
  step comm_high_$r 300 env DLLM_SIDE_STREAMS=high $H --methods ddp --dist_first
  step comm_pool_$r 300 env DLLM_SIDE_STREAMS=pool $H --methods ddp --dist_first
  step m_high_$r 600 env DLLM_SIDE_STREAMS=high $M --json_out gpurun_out/m_high_$r.json
  step m_pool_$r 600 env DLLM_SIDE_STREAMS=pool $M --json_out gpurun_out/m_pool_$r.json
done
step tr_high 300 env DLLM_SIDE_STREAMS=high rocprofv3 --kernel-trace -d gpurun_out/tr_high -o t -- python3 bench.py --gpus 1 --steps 6 --warmup 2 --methods ddp --dist_first --method_steps 2
