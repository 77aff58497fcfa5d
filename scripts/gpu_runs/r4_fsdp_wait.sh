#!/bin/bash
# Round 4 (A/B knob since removed; profiles/r4/fsdp_dp1_rs_wait_r4.txt): FSDP at dp = 1 without the compute-stream wait on the reduce-scatters (no ring slot to protect) vs with it
# (DLLM_FSDP_ALIAS_WAIT=1), interleaved; the comm tests (race screens, side-stream priority bitwise).
source scripts/gpu_steps.sh
step pytest_comm 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_comm_gpu.py
B="python3 bench.py --steps 10 --warmup 3 --methods fsdp,hybrid"
for r in 1 2; do
  step nowait_$r 600 $B --json_out gpurun_out/nowait_$r.json
  step wait_$r 600 env DLLM_FSDP_ALIAS_WAIT=1 $B --json_out gpurun_out/wait_$r.json
done
