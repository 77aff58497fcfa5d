#!/bin/bash
# Round 4 experiment (knob since removed; result in profiles/r4/xcd_skew_sgd_epilogue_r4.txt): the fused split-master SGD weight-gradient epilogue with half the XCDs starting late
# (build knob DLLM_XCD_SKEW_US: _dllm_native_skew15.so / _skew30.so through DLLM_NATIVE_LIB), isolated GEMM and the
# headline step, interleaved with the default build.
source scripts/gpu_steps.sh
step pytest_hp 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread "tests/test_split_master_gpu.py::test_engine_high_priority_side_streams_bitwise"
D=distributed-llm-code-samples_amd
for r in 1 2; do
  step epi_base_$r 120 python -u scripts/bench_sgd_epilogue.py
  step epi_s15_$r 120 env DLLM_NATIVE_LIB=$D/_dllm_native_skew15.so python -u scripts/bench_sgd_epilogue.py
  step epi_s30_$r 120 env DLLM_NATIVE_LIB=$D/_dllm_native_skew30.so python -u scripts/bench_sgd_epilogue.py
done
H="python -u bench.py --methods none --steps 20 --warmup 5"
for r in 1 2; do
  step head_base_$r 300 $H --json_out gpurun_out/head_base_$r.json
  step head_s15_$r 300 env DLLM_NATIVE_LIB=$D/_dllm_native_skew15.so $H --json_out gpurun_out/head_s15_$r.json
done
