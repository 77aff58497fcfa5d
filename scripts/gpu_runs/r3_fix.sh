#!/bin/bash
# Round 3: re-run the two GPU tests whose configurations were fixed, the custom all-reduce protocol tests and its
# staged-vs-arena timing, and the side-by-side methods on the native RCCL layer (vs the torch backend).
source scripts/gpu_steps.sh
export PYTHONUNBUFFERED=1
step fixed_tests 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_car_gpu.py "tests/test_engine_gpu.py::test_wgrad_stream_bitwise_full_size"
step car_bench 300 python -u scripts/bench_car.py --ranks 2,4
step methods_native 900 python -u bench.py --steps 10 --warmup 3 --comm native --json_out gpurun_out/methods_native.json
