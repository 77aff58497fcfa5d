#!/bin/bash
# Round 3: engine streams on dedicated hardware queues (CU-masked streams, utils/streams.py).  Probe the queue
# assignment under a 4-queue cap, run the engine / graph / split-master GPU tests, then A/B headline and the
# communicating methods with and without dedicated queues (interleaved).
source scripts/gpu_steps.sh
step probe 120 env GPU_MAX_HW_QUEUES=4 rocprofv3 --kernel-trace -d gpurun_out/tr_probe -o t -- python3 scripts/probe_dedicated_queues.py
step tests 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_engine_gpu.py tests/test_graph_gpu.py tests/test_split_master_gpu.py tests/test_side_opt_gpu.py
H="python -u bench.py --gpus 1 --steps 20 --warmup 5 --methods none"
M="python -u bench.py --gpus 1 --steps 10 --warmup 3 --method_steps 10 --methods ddp,zero,fsdp,hybrid"
for r in 1 2; do
  step head_ded_$r 300 env DLLM_DEDICATED_QUEUES=1 $H
  step head_pool_$r 300 env DLLM_DEDICATED_QUEUES=0 $H
  step m_ded_$r 600 env DLLM_DEDICATED_QUEUES=1 $M --json_out gpurun_out/m_ded_$r.json
  step m_pool_$r 600 env DLLM_DEDICATED_QUEUES=0 $M --json_out gpurun_out/m_pool_$r.json
done
step m_ded_q8 600 env DLLM_DEDICATED_QUEUES=1 GPU_MAX_HW_QUEUES=8 $M --json_out gpurun_out/m_ded_q8.json
step tr_ded 300 rocprofv3 --kernel-trace -d gpurun_out/tr_ded -o t -- python3 bench.py --gpus 1 --steps 6 --warmup 2 --methods ddp,zero --dist_first --method_steps 4
