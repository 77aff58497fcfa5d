#!/bin/bash
# rocprofv3 kernel traces of the flagship step (both GEMM families), the ZeRO-2 forced-communicator step and the
# TP8-shard MP step; summarised with scripts/kstats.py / scripts/rocpd_stats.py into profiles/.
source scripts/gpu_steps.sh
step prof_dp1 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dp1 -o run -- python3 bench.py --steps 10 --warmup 3 --methods none
step prof_dp1_pp 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dp1_pp -o run -- python3 bench.py --steps 10 --warmup 3 --methods none --gemm_variant pp
step prof_zero 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_zero -o run -- python3 bench.py --steps 10 --warmup 3 --methods none --method zero --force_comm
step prof_tp8 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tp8 -o run -- python3 bench.py --steps 20 --warmup 3 --methods none --method tp --ffn_dim 1792 --layers 1
