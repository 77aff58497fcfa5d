#!/bin/bash
# GEMM tables: native families (256x256 8-phase persistent, 256x128 two-per-CU) vs hipBLASLt on the FFN shapes,
# the MP / TP8-shard shapes, and the fp32 paths (bf16x6 split, fp32 MFMA, hipBLASLt fp32).
source scripts/gpu_steps.sh
step gemm_ffn 400 python -u scripts/bench_gemm.py --variants tpb8,pp1,pp8 --rounds 3 --iters 10 --json gpurun_out/gemm_ffn.json
step gemm_tp8 300 python -u scripts/bench_gemm.py --F 1792 --variants tpb8,pp8 --rounds 3 --iters 20 --json gpurun_out/gemm_tp8.json
step gemm_fp32 300 python -u scripts/bench_fp32.py
