#!/bin/bash
source scripts/gpu_steps.sh
step splitk_tests 900 python -m pytest tests/test_gemm_gpu.py -q -m gpu -k splitk
step gpu_tests 900 python -m pytest tests -q -m gpu
step bench_tp8shard 600 python bench.py --steps 20 --warmup 5 --method tp --ffn_dim 1792 --layers 1
step bench_small 600 python bench.py --steps 50 --warmup 5 --model_size 1024 --layers 4 --batch_size 2 --seq_len 1024
step bench_default 600 python bench.py --steps 10 --warmup 3
