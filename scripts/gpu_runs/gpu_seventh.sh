#!/bin/bash
source scripts/gpu_steps.sh
step comm_tests 900 python -m pytest tests/test_comm_gpu.py -q -m gpu -x
step all_gpu_tests 900 python -m pytest tests -q -m gpu
step bench_zero_native 600 python bench.py --steps 10 --warmup 3 --force_comm --method zero --comm native
step bench_default 600 python bench.py --steps 10 --warmup 3
