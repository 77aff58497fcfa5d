#!/bin/bash
# Round 3 (session 2): split-master GPU tests, the GEMM / engine GPU suites, smoke, and the headline with the split
# master (default) vs the fp32 master, interleaved on one box.
source scripts/gpu_steps.sh
step pytest_split 300 python -u -m pytest tests/test_split_master_gpu.py -x -v --timeout 120 --timeout-method thread
step pytest_core 900 python -u -m pytest tests/test_gemm_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
for r in 1 2; do
  step head_split_$r 300 python -u bench.py --methods none --steps 20 --warmup 5
  step head_fp32_$r 300 python -u bench.py --methods none --steps 20 --warmup 5 --master fp32
done
