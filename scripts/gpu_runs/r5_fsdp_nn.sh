#!/bin/bash
# Round 5: NN layout with FSDP -- 2-rank GPU test (DDP / ZeRO-2 / FSDP, checkpoints), then the driver's full N=1
# command (every side method).
source scripts/gpu_steps.sh
step mr_nn 700 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_multirank_gpu.py -k nn_weight
step driver_full 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json_out gpurun_out/r5_driver_full_nn2.json
