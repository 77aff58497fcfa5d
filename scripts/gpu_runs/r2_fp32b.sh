#!/bin/bash
# fp32 256x256x32 (2-stage) kernel: numerics + throughput vs torch
source scripts/gpu_steps.sh
step test_fp32 600 python -u -m pytest tests/test_gemm_gpu.py -x -q -k "fp32" --timeout 120 --timeout-method thread
step bench_fp32 300 python scripts/bench_fp32.py
