#!/bin/bash
# Round 3: DLLM_SIDE_STREAMS=auto with the high-priority weight-gradient stream owned by its engine (destroyed, and its
# queue released, when the engine is collected): do the later collective methods still lose?  Interleaved.
source scripts/gpu_steps.sh
M="python -u bench.py --gpus 1 --steps 10 --warmup 3 --method_steps 10 --methods ddp,zero,fsdp,hybrid"
step tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_split_master_gpu.py tests/test_engine_gpu.py
for r in 1 2; do
  step m_auto_$r 600 env DLLM_SIDE_STREAMS=auto $M --json_out gpurun_out/m_auto_$r.json
  step m_pool_$r 600 env DLLM_SIDE_STREAMS=pool $M --json_out gpurun_out/m_pool_$r.json
done
step comm_auto 300 env DLLM_SIDE_STREAMS=auto python -u bench.py --gpus 1 --steps 20 --warmup 5 --methods ddp --dist_first
step comm_pool 300 env DLLM_SIDE_STREAMS=pool python -u bench.py --gpus 1 --steps 20 --warmup 5 --methods ddp --dist_first
