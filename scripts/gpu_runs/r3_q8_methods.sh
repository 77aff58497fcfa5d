#!/bin/bash
# Round 3: the communicating methods at N=1 (force_comm, RCCL communicators live) with 8 vs 16 HIP hardware queues,
# interleaved: does 8 keep the collective / GEMM overlap that 16 bought (profiles/r3/hwqueue_16_vs_4_r3.txt)?
source scripts/gpu_steps.sh
B="python -u bench.py --gpus 1 --steps 10 --warmup 3 --method_steps 10 --methods ddp,zero,fsdp,hybrid"
for r in 1 2; do
  step m_q16_$r 600 env GPU_MAX_HW_QUEUES=16 $B --json_out gpurun_out/m_q16_$r.json
  step m_q8_$r 600 env GPU_MAX_HW_QUEUES=8 $B --json_out gpurun_out/m_q8_$r.json
done
