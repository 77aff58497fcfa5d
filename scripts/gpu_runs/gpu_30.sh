#!/bin/bash
# Race screen + full GPU suite, flagship profile, ZeRO-path profile, BASELINE config sweep (current defaults).
source scripts/gpu_steps.sh
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/gputests.log && ! grep -q -E "[0-9]+ failed" gpurun_out/gputests.log || exit 1
step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o p -- python3 bench.py --steps 5 --warmup 2
step prof_zero 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profz -o z -- python3 bench.py --steps 5 --warmup 2 --force_comm --method zero
bash scripts/bench_configs.sh > gpurun_out/bench_configs.log 2>&1
