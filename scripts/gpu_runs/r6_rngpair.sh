#!/bin/bash
# Round 6: x and dy drawn in one launch (rng_normal_bf16_pair_kernel) vs two (DLLM_RNG_PAIR=0): bitwise tests, the MP
# (TP8) shard interleaved, a kernel trace (profiles/r6/rng_pair_r6.txt).
source scripts/gpu_steps.sh
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
step t_rng 300 $T tests/test_gemm_gpu.py -k "rng or device_data"
T8="--method tp --ffn_dim 1792 --layers 1 --methods none --no_reference_init --steps 100 --warmup 20"
for i in 1 2 3; do
  step tp8_pair_$i 200 python -u bench.py $T8 --json_out gpurun_out/tp8_pair_$i.json
  step tp8_two_$i 200 env DLLM_RNG_PAIR=0 python -u bench.py $T8 --json_out gpurun_out/tp8_two_$i.json
done
step prof_tp8_pair 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tp8_pair -o run -- python3 bench.py $T8
