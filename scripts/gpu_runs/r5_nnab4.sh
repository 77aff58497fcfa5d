#!/bin/bash
# Round 5: nn_w2t (W2 stored transposed, both weight gradients NN-transposed) vs nn_w1 vs tn (serial), interleaved;
# engine tests first.
source scripts/gpu_steps.sh
step nn_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_nnwgrad_gpu.py
for i in 1 2 3; do
  step s_tn_$i 200 python -u bench.py --steps 20 --warmup 5 --methods none --wgrad_layout tn --no-wgrad_stream
  step s_w1_$i 200 python -u bench.py --steps 20 --warmup 5 --methods none --wgrad_layout nn_w1
  step s_w2t_$i 200 python -u bench.py --steps 20 --warmup 5 --methods none --wgrad_layout nn_w2t
done
step prof_w2t 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_w2t -o run -- python3 bench.py --steps 20 --warmup 5 --methods none --wgrad_layout nn_w2t
