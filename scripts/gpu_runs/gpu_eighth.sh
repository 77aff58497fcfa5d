#!/bin/bash
source scripts/gpu_steps.sh
step graph_tests 600 python -m pytest tests/test_graph_gpu.py tests/test_ipc_gpu.py -q -m gpu
step race_tests 900 python -m pytest tests/test_comm_gpu.py -q -m gpu -k race
step bench_graph 600 python bench.py --steps 10 --warmup 3 --graph
step bench_tp8shard_graph 600 python bench.py --steps 20 --warmup 5 --method tp --ffn_dim 1792 --layers 1 --graph
step bench_small_graph 600 python bench.py --steps 50 --warmup 5 --model_size 1024 --layers 4 --batch_size 2 --seq_len 1024 --graph
step bench_small_eager 600 python bench.py --steps 50 --warmup 5 --model_size 1024 --layers 4 --batch_size 2 --seq_len 1024
