#!/bin/bash
# Round 4: m224 / pair / streams tests, the engine + multi-rank suites after the dp=1 aliasing change, the driver's
# N=1 command (methods: fsdp / zero / hybrid with in-place size-1 collectives), TP8 shard with the data pipeline.
source scripts/gpu_steps.sh
step pytest_r4 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_m224_gpu.py tests/test_gemm_pair_gpu.py tests/test_streams_gpu.py tests/test_engine_gpu.py tests/test_multirank_gpu.py tests/test_split_master_gpu.py "tests/test_gemm_gpu.py::test_rng_matches_cpu_philox"
step driver_2 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json_out gpurun_out/driver_2.json
TP="python -u bench.py --methods none --method tp --ffn_dim 1792 --layers 1 --steps 20 --warmup 5"
for r in 1 2; do
  step tp8_sync_$r 300 $TP --json_out gpurun_out/tp8_sync_$r.json
  step tp8_ov_$r 300 $TP --data_overlap --json_out gpurun_out/tp8_ov_$r.json
done
