#!/bin/bash
# Round 6 baseline: the finite-data bar (plain torch, recompute on/off) interleaved with the headline; the zero
# (ZeRO-2 at dp 1, forced communicators) vs headline gap by phase and per kernel, at min_bpc 1 and 2.
source scripts/gpu_steps.sh
H="--steps 20 --warmup 5 --methods none --no_reference_init"
for i in 1 2; do
  step head_$i 240 python -u bench.py $H --phases --json_out gpurun_out/head_$i.json
  step torch_rc_$i 240 python -u scripts/torch_baseline.py --recompute on
  step torch_norc_$i 240 python -u scripts/torch_baseline.py --recompute off
  step zero_$i 240 python -u bench.py $H --phases --force_comm --json_out gpurun_out/zero_$i.json
  step zero_bpc2_$i 240 python -u bench.py $H --phases --force_comm --min_bpc 2 --json_out gpurun_out/zero_bpc2_$i.json
done
step torch_ref_init 240 python -u scripts/torch_baseline.py --recompute on --init 0.02
step prof_head 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_head -o run -- python3 bench.py --steps 10 --warmup 3 --methods none --no_reference_init
step prof_zero 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_zero -o run -- python3 bench.py --steps 10 --warmup 3 --methods none --no_reference_init --force_comm
