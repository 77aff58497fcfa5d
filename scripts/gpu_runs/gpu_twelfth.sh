#!/bin/bash
# Functional API on the GPU, RCCL single-process selftest binary, comm tests, bench JSON.
source scripts/gpu_steps.sh
step api_tests 600 python -m pytest tests/test_api_gpu.py -q -m gpu -x
step comm_tests 900 python -m pytest tests/test_comm_gpu.py -q -m gpu -x
step rccl_bin 120 distributed-llm-code-samples_amd/bin/dllm_rccl_selftest
step bench_default 600 python bench.py --steps 10 --warmup 3
