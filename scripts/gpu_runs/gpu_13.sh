#!/bin/bash
# Layer-0 wgrad reorder + side-stream ZeRO tail: engine/comm/graph tests, then ZeRO + default benches.
source scripts/gpu_steps.sh
step engine_tests 900 python -m pytest tests/test_engine_gpu.py tests/test_graph_gpu.py tests/test_api_gpu.py -q -m gpu -x
step comm_tests 900 python -m pytest tests/test_comm_gpu.py -q -m gpu -x
step bench_zero1 600 python bench.py --steps 10 --warmup 3 --force_comm --method zero
step bench_default 600 python bench.py --steps 10 --warmup 3
