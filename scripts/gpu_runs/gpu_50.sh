#!/bin/bash
# Fresh evidence for the final round-1 tree: flagship kernel profile, ZeRO-path profile, bench on each N>1 code path at world 1.
source scripts/gpu_steps.sh
step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o p -- python3 bench.py --steps 5 --warmup 2
step prof_zero 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profz -o z -- python3 bench.py --steps 5 --warmup 2 --force_comm --method zero
step b_default 300 python bench.py --steps 20 --warmup 5
step b_zero_fc 300 python bench.py --steps 20 --warmup 5 --force_comm --method zero
step b_ddp_fc 300 python bench.py --steps 20 --warmup 5 --force_comm --method ddp
step b_fsdp_fc 300 python bench.py --steps 20 --warmup 5 --force_comm --method fsdp
