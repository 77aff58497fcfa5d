#!/bin/bash
source scripts/gpu_steps.sh
step gemm_tests 600 python -m pytest tests/test_gemm_gpu.py -x -q -m gpu
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step engine_tests 600 python -m pytest tests/test_engine_gpu.py -x -q -m gpu
step bench1 600 python bench.py --steps 5 --warmup 2
