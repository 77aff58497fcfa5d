#!/bin/bash
# Native vs hipBLASLt for the plain forward GEMM (y = a·W2ᵀ), interleaved runs.
source scripts/gpu_steps.sh
step b_native1 600 python bench.py --steps 20 --warmup 3
step b_lib1 600 python bench.py --steps 20 --warmup 3 --lib_plain_nt
step b_native2 600 python bench.py --steps 20 --warmup 3
step b_lib2 600 python bench.py --steps 20 --warmup 3 --lib_plain_nt
