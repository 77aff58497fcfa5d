#!/bin/bash
# Round 4: 224-row tiles / transposed-activation layout tests and TP-shard A/B (F/tp = 1792, 3584, 7168: transposed vs
# regular layout), headline A/B at the box's 4 HW queues (queue reservation on/off, weight-gradient stream on/off).
source scripts/gpu_steps.sh
step pytest_m224 900 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_m224_gpu.py tests/test_gemm_pair_gpu.py tests/test_streams_gpu.py "tests/test_engine_gpu.py::test_overlapped_data_mismatched_seed_bitwise" "tests/test_split_master_gpu.py::test_fused_sgd_split_faulting_shape_of_parked_seam_patch" "tests/test_gemm_gpu.py::test_rng_matches_cpu_philox"
TP="python -u bench.py --methods none --method tp --layers 1 --steps 20 --warmup 5"
for r in 1 2; do
  for f in 1792 3584 7168; do
    step tp_f${f}_tmode_$r 300 $TP --ffn_dim $f --json_out gpurun_out/tp_f${f}_tmode_$r.json
    step tp_f${f}_reg_$r 300 env DLLM_TP_TRANSPOSED=0 $TP --ffn_dim $f --json_out gpurun_out/tp_f${f}_reg_$r.json
  done
done
H="python -u bench.py --methods none --steps 20 --warmup 5"
for r in 1 2; do
  step head_def_$r 300 $H --json_out gpurun_out/head_def_$r.json
  step head_noreserve_$r 300 $H --no_queue_reserve --json_out gpurun_out/head_noreserve_$r.json
  step head_nowgs_$r 300 $H --no-wgrad_stream --json_out gpurun_out/head_nowgs_$r.json
done
step tp8_trace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tp8 -o run -- python3 bench.py --methods none --method tp --ffn_dim 1792 --layers 1 --steps 10 --warmup 3
