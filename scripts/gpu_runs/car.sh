#!/bin/bash
# Custom all-reduce (csrc/car.hip): protocol tests (staged and zero-copy arena, 2-4 processes on one GPU, TP
# training, stalled peer) and the per-size timing of both modes.
source scripts/gpu_steps.sh
step car_tests 600 python -u -m pytest tests/test_car_gpu.py -q --timeout 240 --timeout-method thread
step car_bench 400 python -u scripts/bench_car.py --ranks 2,4
