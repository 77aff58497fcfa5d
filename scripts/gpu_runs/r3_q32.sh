#!/bin/bash
# Round 3: 32 HIP hardware queues (the pool cap this harness allows) so a live RCCL communicator's streams and
# torch's 32-stream pool no longer push the engine's side streams onto the compute stream's queue; interleaved.
source scripts/gpu_steps.sh
export TMPDIR=/tmp
B="python -u bench.py --gpus 1 --steps 20 --warmup 5"
for r in 1 2; do
  step comm_q16_$r 300 env GPU_MAX_HW_QUEUES=16 $B --methods ddp --dist_first
  step comm_q32_$r 300 env GPU_MAX_HW_QUEUES=32 $B --methods ddp --dist_first
  step none_q32_$r 300 env GPU_MAX_HW_QUEUES=32 $B --methods none
done
M="python -u bench.py --gpus 1 --steps 10 --warmup 3 --method_steps 10 --methods ddp,zero,fsdp,hybrid"
step m_q32 600 env GPU_MAX_HW_QUEUES=32 $M --json_out gpurun_out/m_q32.json
step m_q16 600 env GPU_MAX_HW_QUEUES=16 $M --json_out gpurun_out/m_q16.json
step tr_q32 300 env GPU_MAX_HW_QUEUES=32 rocprofv3 --kernel-trace -d gpurun_out/tr_q32 -o t -- python3 bench.py --gpus 1 --steps 6 --warmup 2 --methods ddp --dist_first --method_steps 2
