#!/bin/bash
# Round 3: the 256x128 two-blocks-per-CU GEMM family (csrc/gemm_pp.h): numerics/race/persistence tests for both
# families, then per-GEMM throughput on the flagship FFN shapes (interleaved in one process).
set -o pipefail
mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r3/pp_tests.log 2>&1 || { tail -30 gpurun_out/r3/pp_tests.log; exit 1; }
tail -3 gpurun_out/r3/pp_tests.log
timeout -k 10 400 python -u scripts/bench_gemm.py --variants tpb8,pp1,pp8 --rounds 3 --iters 10 \
  --json gpurun_out/r3/pp_gemm.json > gpurun_out/r3/pp_gemm.log 2>&1 || { tail -30 gpurun_out/r3/pp_gemm.log; exit 1; }
cat gpurun_out/r3/pp_gemm.log
