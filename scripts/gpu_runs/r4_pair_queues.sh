#!/bin/bash
# Round 4: grouped weight-gradient pair (TP8 shard) + compute-queue reservation: new GPU tests, the TP8-shard step
# with / without the pair (interleaved), the driver's N=1 command (queues, exposed_ms_diff), headline kernel trace
# with a live communicator (queue ids).
source scripts/gpu_steps.sh
{ echo "GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES-<unset>}"; env | grep -E '^(HIP|HSA|GPU|NCCL|RCCL|OMP)_' | sort; } > gpurun_out/env.txt 2>&1
step pytest_new 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_pair_gpu.py tests/test_streams_gpu.py "tests/test_engine_gpu.py::test_overlapped_data_mismatched_seed_bitwise"
for r in 1 2; do
  step tp8_pair_$r 300 python -u bench.py --methods none --method tp --ffn_dim 1792 --layers 1 --steps 20 --warmup 5 --json_out gpurun_out/tp8_pair_$r.json
  step tp8_nopair_$r 300 python -u bench.py --methods none --method tp --ffn_dim 1792 --layers 1 --steps 20 --warmup 5 --no_pair_wgrads --json_out gpurun_out/tp8_nopair_$r.json
done
step tp8_trace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tp8 -o run -- python3 bench.py --methods none --method tp --ffn_dim 1792 --layers 1 --steps 10 --warmup 3
step driver_1 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json_out gpurun_out/driver_1.json
step head_trace_comm 300 rocprofv3 --kernel-trace -d gpurun_out/prof_head_comm -o run -- python3 bench.py --gpus 1 --steps 6 --warmup 2 --methods zero --dist_first --method_steps 3 --diff_pairs 0
