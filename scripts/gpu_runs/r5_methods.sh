#!/bin/bash
# Round 5: the driver's full N=1 command (steady-state side-method windows,
# role-queue report, fsdp_copy, collectives_noop), the TP8 shard over 100 steps, and per-kernel traces of the config-5
# AdamW step fused vs side-stream.
source scripts/gpu_steps.sh
step driver_full 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json_out gpurun_out/r5_driver_full.json
step tp8 200 python3 bench.py --method tp --ffn_dim 1792 --layers 1 --steps 100 --warmup 20 --methods none --json_out gpurun_out/r5_tp8.json
step prof_adam_fused 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_adam_fused -o run -- python3 bench.py --methods none --optimizer adam --gated --act silu --ffn_dim 14336 --layers 32 --steps 4 --warmup 2
step prof_adam_side 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_adam_side -o run -- python3 bench.py --methods none --optimizer adam --gated --act silu --ffn_dim 14336 --layers 32 --steps 4 --warmup 2 --side_opt 32
