#!/bin/bash
# Round 4: synchronous TP all-reduces on the compute stream (comm.all_reduce async_op=False, no communicator-stream
# hops) vs through the communicator stream (DLLM_SYNC_INLINE=0), for the methods with TP exchanges (tp, hybrid).
source scripts/gpu_steps.sh
step pytest_comm 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_comm_gpu.py
B="python3 bench.py --steps 5 --warmup 2 --methods tp,hybrid"
for r in 1 2; do
  step inl_$r 600 $B --json_out gpurun_out/inl_$r.json
  step hop_$r 600 env DLLM_SYNC_INLINE=0 $B --json_out gpurun_out/hop_$r.json
done
