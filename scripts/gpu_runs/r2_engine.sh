#!/bin/bash
# GPU engine tests (incl. the teacher-forced bf16 ReLU stack check)
source scripts/gpu_steps.sh
step test_engine 600 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread
