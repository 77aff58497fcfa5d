#!/bin/bash
# Round 4: the persistent 8-phase family vs torch.matmul (hipBLASLt) on the flagship FFN shapes, final tree.
source scripts/gpu_steps.sh
step gemm_ffn_r4 400 python -u scripts/bench_gemm.py --variants tpb8 --rounds 3 --iters 10 --json gpurun_out/gemm_ffn_r4.json
