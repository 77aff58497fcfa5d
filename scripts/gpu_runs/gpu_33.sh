#!/bin/bash
# Concurrent weight-gradient stream (N=1, fused SGD): bitwise test, flagship with / without, interleaved.
source scripts/gpu_steps.sh
step tests 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "wgrad_stream or mask"
grep -q " passed" gpurun_out/tests.log && ! grep -q -E "[0-9]+ failed" gpurun_out/tests.log || exit 1
step seq1 300 python bench.py --steps 20 --warmup 5
step ws1 300 python bench.py --steps 20 --warmup 5 --wgrad_stream
step seq2 300 python bench.py --steps 20 --warmup 5
step ws2 300 python bench.py --steps 20 --warmup 5 --wgrad_stream
step ws_tpb1 300 python bench.py --steps 20 --warmup 5 --wgrad_stream --tpb 1
