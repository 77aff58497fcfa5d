#!/bin/bash
source scripts/gpu_steps.sh
step raster_t 300 python -u scripts/bench_nn_wgrad.py --raster_t
