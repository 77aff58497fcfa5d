#!/bin/bash
# Round 3: hardware queues per process (GPU_MAX_HW_QUEUES, set to 16 by the package unless given).  Headline
# interleaved at 16 vs 4 queues; the ZeRO-2 forced-communicator step traced at 16 queues (do the reduce-scatter
# copies now run under the GEMMs?); the methods side by side with the comm observer.
source scripts/gpu_steps.sh
export PYTHONUNBUFFERED=1
for r in 1 2; do
  step head_q16_$r 300 python -u bench.py --methods none --steps 20 --warmup 5 --json_out gpurun_out/head_q16_$r.json
  step head_q4_$r 300 env GPU_MAX_HW_QUEUES=4 python -u bench.py --methods none --steps 20 --warmup 5 --json_out gpurun_out/head_q4_$r.json
done
step prof_zero16 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_zero16 -o run -- python3 bench.py --steps 10 --warmup 3 --methods none --method zero --force_comm
step methods 900 python -u bench.py --steps 10 --warmup 3 --json_out gpurun_out/methods16.json
