#!/bin/bash
# Round 3 diagnostic: kernel traces of the N=1 headline with and without a live RCCL communicator -- slower kernels
# (a GPU-side effect) or gaps between them (host side)?
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step tr_none 300 rocprofv3 --kernel-trace -d gpurun_out/tr_none -o t -- python3 bench.py --gpus 1 --steps 10 --warmup 3 --methods none
step tr_comm 300 rocprofv3 --kernel-trace -d gpurun_out/tr_comm -o t -- python3 bench.py --gpus 1 --steps 10 --warmup 3 --methods ddp --dist_first --method_steps 2
