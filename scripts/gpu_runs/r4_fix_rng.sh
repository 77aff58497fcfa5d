#!/bin/bash
# Round 4: the test-side fixes (wgrad-stream / pair / m224 tests), Philox rounds A/B for the device mock data (10 vs 7:
# build variant _dllm_native_philox7.so through DLLM_NATIVE_LIB), TP8 shard step with each.
source scripts/gpu_steps.sh
step pytest_fixed 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread "tests/test_engine_gpu.py::test_wgrad_stream_bitwise" tests/test_gemm_pair_gpu.py tests/test_m224_gpu.py "tests/test_split_master_gpu.py::test_engine_high_priority_side_streams_bitwise"
V=distributed-llm-code-samples_amd/_dllm_native_philox7.so
for r in 1 2; do
  step rng10_$r 120 python -u scripts/bench_rng.py
  step rng7_$r 120 env DLLM_NATIVE_LIB=$V python -u scripts/bench_rng.py
done
TP="python -u bench.py --methods none --method tp --ffn_dim 1792 --layers 1 --steps 20 --warmup 5"
for r in 1 2; do
  step tp8_r10_$r 300 $TP --json_out gpurun_out/tp8_r10_$r.json
  step tp8_r7_$r 300 env DLLM_NATIVE_LIB=$V $TP --json_out gpurun_out/tp8_r7_$r.json
done
