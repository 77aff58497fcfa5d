#!/bin/bash
# Round 5: fused-SGD epilogue cost by master row pitch (NN natural [4096, 16384], K = 8192).
source scripts/gpu_steps.sh
step epi_pitch 300 python -u scripts/bench_nn_wgrad.py --epilogue_pitch
