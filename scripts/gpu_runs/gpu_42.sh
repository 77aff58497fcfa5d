#!/bin/bash
# Persistent GEMM grids under CU contention (side-stream occupiers standing in for RCCL channels).
source scripts/gpu_steps.sh
step intf_tpb1 300 python scripts/interference.py --cus 0,8,32 --tpb 1
step intf_tpb2_bpc1 300 python scripts/interference.py --cus 0,8,32 --tpb 2 --min_bpc 1
step intf_tpb2_bpc2 300 python scripts/interference.py --cus 0,8,32 --tpb 2 --min_bpc 2
step bench 300 python bench.py --steps 20 --warmup 5
step bench_fc 300 python bench.py --steps 10 --warmup 3 --force_comm --method zero
