#!/bin/bash
# fp32 256x256 LDS-DMA kernel: numerics + throughput vs torch (hipBLASLt); native RCCL split/grouped comm tests
source scripts/gpu_steps.sh
step test_fp32 600 python -u -m pytest tests/test_gemm_gpu.py -x -q -k "fp32" --timeout 120 --timeout-method thread
step test_comm 600 python -u -m pytest tests/test_comm_gpu.py -x -q --timeout 120 --timeout-method thread
step bench_fp32 300 python scripts/bench_fp32.py
step prof_tp8shard 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tp8 -o run -- python3 bench.py --steps 10 --warmup 3 --methods none --method tp --ffn_dim 1792 --layers 8
step cli_fp32 600 python train_ffns.py -s 8 -bs 8 -n 1024 -l 2 -d 4096 -m 1 -r 1 --dtype fp32 --data device
