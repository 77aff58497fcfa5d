#!/bin/bash
# Round 4: where the forced-communicator methods' exposed_ms_diff goes -- kernel traces of zero / fsdp at N=1 with
# their size-1 collectives and with them elided (bench.py --elide_collectives), summarised by scripts/trace_gaps.py.
source scripts/gpu_steps.sh
B="python3 bench.py --steps 10 --warmup 3 --methods none --force_comm --diff_pairs 0"
for m in zero fsdp; do
  step prof_${m} 300 rocprofv3 --kernel-trace -d gpurun_out/prof_${m} -o run -- $B --method $m
  step prof_${m}_elided 300 rocprofv3 --kernel-trace -d gpurun_out/prof_${m}_elided -o run -- $B --method $m --elide_collectives
done
for d in zero zero_elided fsdp fsdp_elided; do
  echo "== $d" >> gpurun_out/comm_gaps.txt
  python scripts/trace_gaps.py gpurun_out/prof_$d/run_results.db --last_ms 250 >> gpurun_out/comm_gaps.txt || exit 1
done
