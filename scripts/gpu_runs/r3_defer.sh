#!/bin/bash
# Round 3 (session 2): deferred fused split-master SGD + in-kernel split-K combine -- tests first, then the headline
# with / without deferral (interleaved), the TP8 shard with / without the seam, and kernel traces.
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step pytest_defer 300 python -u -m pytest tests/test_defer_sgd_gpu.py -x -v --timeout 120 --timeout-method thread
step pytest_seam 600 python -u -m pytest tests/test_gemm_gpu.py -x -q -k "splitk or seam or persistent or race" --timeout 200 --timeout-method thread
step pytest_split 300 python -u -m pytest tests/test_split_master_gpu.py -x -v --timeout 120 --timeout-method thread
for r in 1 2; do
  step head_defer_$r 300 python -u bench.py --methods none --steps 20 --warmup 5
  step head_nodefer_$r 300 python -u bench.py --methods none --steps 20 --warmup 5 --no_defer_sgd
done
for r in 1 2; do
  step tp8_seam_$r 300 python -u bench.py --methods none --steps 20 --warmup 5 --method tp --ffn_dim 1792 --layers 1
  step tp8_reduce_$r 300 python -u bench.py --methods none --steps 20 --warmup 5 --method tp --ffn_dim 1792 --layers 1 --no_splitk_seam
done
step head_trace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_head -o head -- python bench.py --methods none --steps 10 --warmup 3
step tp8_trace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tp8 -o tp8 -- python bench.py --methods none --steps 10 --warmup 3 --method tp --ffn_dim 1792 --layers 1
