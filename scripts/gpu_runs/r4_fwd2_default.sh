#!/bin/bash
# Round 4: hipBLASLt for the forward's plain long-K NT store as the single-rank default -- tests, the driver's command,
# headline with it forced off (DLLM_NT_STORE_LIB=0) vs default, interleaved.
source scripts/gpu_steps.sh
step pytest_lib 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread "tests/test_gemm_gpu.py::test_lib_nt_store_routes_only_the_plain_long_k_store" tests/test_engine_gpu.py tests/test_comm_gpu.py tests/test_split_master_gpu.py
H="python -u bench.py --methods none --steps 20 --warmup 5"
for r in 1 2; do
  step def_$r 300 $H --json_out gpurun_out/def_$r.json
  step off_$r 300 env DLLM_NT_STORE_LIB=0 $H --json_out gpurun_out/off_$r.json
done
step driver_f 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json_out gpurun_out/driver_f.json
