#!/bin/bash
# Round 4: the elided reference steps now keep the collectives' issue-point dependencies (comm.Elided); kernel traces
# of zero / fsdp elided again, then the driver's N=1 command (exposed_ms_diff of every method).
source scripts/gpu_steps.sh
B="python3 bench.py --steps 10 --warmup 3 --methods none --force_comm --diff_pairs 0"
for m in zero fsdp; do
  step prof_${m}_elided2 300 rocprofv3 --kernel-trace -d gpurun_out/prof_${m}_elided2 -o run -- $B --method $m --elide_collectives
  echo "== ${m}_elided2" >> gpurun_out/comm_gaps2.txt
  python scripts/trace_gaps.py gpurun_out/prof_${m}_elided2/run_results.db --last_ms 250 >> gpurun_out/comm_gaps2.txt || exit 1
done
step pytest_elided 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread "tests/test_comm_gpu.py::test_elided_collective_keeps_dependency"
step driver_c 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json_out gpurun_out/driver_c.json
