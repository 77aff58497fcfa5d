#!/bin/bash
# Round 4: bf16 mock data from 16-bit uniforms (8 normals per Philox call): RNG tests, draw time, TP8 shard step and
# the headline (before: profiles/r4/philox_rounds_ab_r4.txt, 28.4-28.5 us per bf16 [8192, 4096] draw).
source scripts/gpu_steps.sh
step pytest_rng 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread "tests/test_gemm_gpu.py::test_rng_matches_cpu_philox" tests/test_graph_gpu.py tests/test_engine_gpu.py
step rng_1 120 python -u scripts/bench_rng.py
step rng_2 120 python -u scripts/bench_rng.py
TP="python -u bench.py --methods none --method tp --ffn_dim 1792 --layers 1 --steps 20 --warmup 5"
for r in 1 2 3; do
  step tp8_$r 300 $TP --json_out gpurun_out/tp8_$r.json
done
step head_1 300 python -u bench.py --methods none --steps 20 --warmup 5 --json_out gpurun_out/head_1.json
