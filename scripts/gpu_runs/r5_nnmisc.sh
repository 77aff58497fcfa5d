#!/bin/bash
# Round 5: NN layout on 2 ranks (DDP / ZeRO-2, checkpoint crossing), HIP-graph capture of the NN step, TP8 shard trace.
source scripts/gpu_steps.sh
step mr_nn 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_multirank_gpu.py -k nn_weight
step graph_nn 200 python -u bench.py --steps 20 --warmup 5 --methods none --graph
step prof_tp8 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tp8 -o run -- python3 bench.py --method tp --ffn_dim 1792 --layers 1 --steps 100 --warmup 20 --methods none
