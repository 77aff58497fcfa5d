#!/bin/bash
# Round 4: native vs hipBLASLt on the Llama-dims (F 14336) and the memory example's (D 8192, F 32768) FFN shapes --
# where the plain long-K NT store goes to hipBLASLt at N=1.
source scripts/gpu_steps.sh
step gemm_f14336 400 python -u scripts/bench_gemm.py --F 14336 --variants tpb8 --rounds 3 --iters 10
step gemm_d8192 600 python -u scripts/bench_gemm.py --D 8192 --F 32768 --variants tpb8 --rounds 3 --iters 5
