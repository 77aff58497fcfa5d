#!/bin/bash
# Static persistent 8-phase GEMM blocks (separate instantiations): bitwise tests, per-GEMM sweep, flagship step.
source scripts/gpu_steps.sh
step gemm_tests 300 python -u -m pytest tests/test_gemm_gpu.py -x -v --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/gemm_tests.log && ! grep -q -E "[0-9]+ failed" gpurun_out/gemm_tests.log || exit 1
step gemm_tpb 600 python scripts/bench_gemm.py --variants tpb1,tpb2,tpb8 --no_torch --rounds 3 --json gpurun_out/gemm_tpb.json
step bench_tpb1 300 python bench.py --steps 20 --warmup 5 --tpb 1
step bench_tpb2 300 python bench.py --steps 20 --warmup 5
step bench_tpb8 300 python bench.py --steps 20 --warmup 5 --tpb 8
step bench_tpb2b 300 python bench.py --steps 20 --warmup 5
step bench_tpb1b 300 python bench.py --steps 20 --warmup 5 --tpb 1
step engine_tests 600 python -u -m pytest tests/test_engine_gpu.py tests/test_graph_gpu.py tests/test_api_gpu.py -x -q --timeout 120 --timeout-method thread
