#!/bin/bash
# Round 4: grouped weight-gradient pair + 224-row tiles / transposed-activation layout (TP8 shard), compute-queue
# reservation: new GPU tests, the TP8-shard step (transposed layout vs pair-only vs split-K, interleaved), device RNG,
# the driver's N=1 command (queues, exposed_ms_diff), kernel traces (TP8 shard; headline with a live communicator).
source scripts/gpu_steps.sh
{ echo "GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES-<unset>}"; env | grep -E '^(HIP|HSA|GPU|NCCL|RCCL|OMP)_' | sort; } > gpurun_out/env.txt 2>&1
step pytest_new 900 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_m224_gpu.py tests/test_gemm_pair_gpu.py tests/test_streams_gpu.py "tests/test_engine_gpu.py::test_overlapped_data_mismatched_seed_bitwise" "tests/test_split_master_gpu.py::test_fused_sgd_split_faulting_shape_of_parked_seam_patch" "tests/test_gemm_gpu.py::test_rng_matches_cpu_philox"
step rng 120 python -u scripts/bench_rng.py
TP="python -u bench.py --methods none --method tp --ffn_dim 1792 --layers 1 --steps 20 --warmup 5"
for r in 1 2; do
  step tp8_tmode_$r 300 $TP --json_out gpurun_out/tp8_tmode_$r.json
  step tp8_pair_$r 300 env DLLM_TP_TRANSPOSED=0 $TP --json_out gpurun_out/tp8_pair_$r.json
  step tp8_splitk_$r 300 env DLLM_TP_TRANSPOSED=0 $TP --no_pair_wgrads --json_out gpurun_out/tp8_splitk_$r.json
done
step tp8_trace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tp8 -o run -- python3 bench.py --methods none --method tp --ffn_dim 1792 --layers 1 --steps 10 --warmup 3
step driver_1 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json_out gpurun_out/driver_1.json
step head_trace_comm 300 rocprofv3 --kernel-trace -d gpurun_out/prof_head_comm -o run -- python3 bench.py --gpus 1 --steps 6 --warmup 2 --methods zero --dist_first --method_steps 3 --diff_pairs 0
