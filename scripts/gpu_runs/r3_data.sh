#!/bin/bash
# Round 3: one-deep device data pipeline (next batch drawn on a side stream under the backward): bitwise test,
# headline and TP8-shard config interleaved with / without it, a trace of the shard step, then every BASELINE config.
source scripts/gpu_steps.sh
export PYTHONUNBUFFERED=1
step data_test 300 python -u -m pytest -v --timeout 200 --timeout-method thread "tests/test_engine_gpu.py::test_overlapped_data_pipeline_bitwise"
for r in 1 2; do
  step head_ov_$r 300 python -u bench.py --methods none --steps 20 --warmup 5 --json_out gpurun_out/head_ov_$r.json
  step head_sync_$r 300 python -u bench.py --methods none --steps 20 --warmup 5 --no_data_overlap --json_out gpurun_out/head_sync_$r.json
  step tp8_ov_$r 300 python -u bench.py --methods none --steps 40 --warmup 5 --method tp --ffn_dim 1792 --layers 1 --json_out gpurun_out/tp8_ov_$r.json
  step tp8_sync_$r 300 python -u bench.py --methods none --steps 40 --warmup 5 --method tp --ffn_dim 1792 --layers 1 --no_data_overlap --json_out gpurun_out/tp8_sync_$r.json
done
step tp8_prof 300 rocprofv3 --kernel-trace -d gpurun_out/tp8_prof -o run -- python3 bench.py --methods none --steps 20 --warmup 5 --method tp --ffn_dim 1792 --layers 1
bash scripts/bench_configs.sh
