#!/bin/bash
# TP8-shard weight gradients side by side (unsplit, two streams) vs sequential split-K + reduction
source scripts/gpu_steps.sh
step tests 400 python -u -m pytest tests/test_engine_gpu.py tests/test_car_gpu.py tests/test_graph_gpu.py -q -x --timeout 120 --timeout-method thread
for i in 1 2 3; do
  step pair_$i 120 python bench.py --method tp --ffn_dim 1792 --layers 1 --methods none --steps 100 --warmup 20
  step seq_$i 120 env DLLM_PAIR_WGRADS=0 python bench.py --method tp --ffn_dim 1792 --layers 1 --methods none --steps 100 --warmup 20
done
step prof_pair 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pair -o pair -- python bench.py --method tp --ffn_dim 1792 --layers 1 --methods none --steps 20 --warmup 5
