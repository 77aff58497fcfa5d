#!/bin/bash
# Side-by-side backward GEMMs on half-chip persistent grids (dW2_l | dx_l, dW1_l | da_{l-1}) vs the serial step
source scripts/gpu_steps.sh
step tests 600 python -u -m pytest tests/test_engine_gpu.py tests/test_gemm_gpu.py tests/test_graph_gpu.py -q -x --timeout 120 --timeout-method thread
for i in 1 2 3; do
  step serial_$i 120 python bench.py --steps 20 --warmup 5 --methods none
  step half_$i 120 python bench.py --steps 20 --warmup 5 --methods none --wgrad_stream --wgrad_stream_cus 128
  step full_$i 120 python bench.py --steps 20 --warmup 5 --methods none --wgrad_stream --wgrad_stream_cus 0
done
step prof_half 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_half -o half -- python bench.py --steps 6 --warmup 2 --methods none --wgrad_stream --wgrad_stream_cus 128
