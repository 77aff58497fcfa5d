#!/bin/bash
# Round 4: the new default side-stream policy (DLLM_SIDE_STREAMS=role: the FSDP stream at high priority) vs all-pool,
# forced-comm methods interleaved; the comm / split-master tests; host enqueue time vs GPU time per FSDP step.
source scripts/gpu_steps.sh
step pytest_streams 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_comm_gpu.py tests/test_streams_gpu.py "tests/test_split_master_gpu.py::test_engine_high_priority_side_streams_bitwise"
B="python3 bench.py --steps 10 --warmup 3 --methods zero,fsdp,hybrid"
for r in 1 2; do
  step role_$r 600 $B --json_out gpurun_out/role_$r.json
  step pool_$r 600 env DLLM_SIDE_STREAMS=pool $B --json_out gpurun_out/pool_$r.json
done
step host_fsdp 300 python -u scripts/host_vs_gpu.py --method fsdp
step host_fsdp_elide 300 python -u scripts/host_vs_gpu.py --method fsdp --elide
