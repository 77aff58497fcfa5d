#!/bin/bash
# Round 3 (session 2): in-kernel split-K combine (seam) -- GEMM numerics / race tests, the TP8-shard step with the
# seam vs the splitk_reduce pass (interleaved), and a kernel trace of the seam step.
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step pytest_seam 600 python -u -m pytest tests/test_gemm_gpu.py -x -q -k "splitk or seam or persistent or race" --timeout 200 --timeout-method thread
step pytest_split 300 python -u -m pytest tests/test_split_master_gpu.py -x -q --timeout 120 --timeout-method thread
for r in 1 2; do
  step tp8_seam_$r 300 python -u bench.py --methods none --steps 20 --warmup 5 --method tp --ffn_dim 1792 --layers 1
  step tp8_reduce_$r 300 python -u bench.py --methods none --steps 20 --warmup 5 --method tp --ffn_dim 1792 --layers 1 --no_splitk_seam
done
step tp8_trace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tp8 -o tp8 -- python bench.py --methods none --steps 10 --warmup 3 --method tp --ffn_dim 1792 --layers 1
