#!/bin/bash
# Round 3: multi-rank engine paths on one GPU (2-4 processes sharing cuda:0 over gloo): oracle, cross-method and
# overlapped-vs-serialized checks of DDP / ZeRO-2 / FSDP / TP / hybrid with the HIP kernels and side streams.
source scripts/gpu_steps.sh
export PYTHONUNBUFFERED=1
step multirank 900 python -u -m pytest -v -s --timeout 400 --timeout-method thread tests/test_multirank_gpu.py
