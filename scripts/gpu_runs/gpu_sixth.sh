#!/bin/bash
source scripts/gpu_steps.sh
step bench_zero_rccl 600 python bench.py --steps 10 --warmup 3 --force_comm --method zero --grad_dtype bf16
step bench_ddp_rccl_bf16 600 python bench.py --steps 10 --warmup 3 --force_comm --method ddp --grad_dtype bf16
step bench_fsdp_rccl_bf16 600 python bench.py --steps 10 --warmup 3 --force_comm --method fsdp --grad_dtype bf16
step bench_default 600 python bench.py --steps 10 --warmup 3
step prof_zero 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_zero -o z -- python bench.py --steps 5 --warmup 2 --force_comm --method zero --grad_dtype bf16
