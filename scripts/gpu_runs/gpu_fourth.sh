#!/bin/bash
source scripts/gpu_steps.sh
step gpu_tests 900 python -m pytest tests -q -m gpu
step bench_fused 600 python bench.py --steps 10 --warmup 3
step rccl_selftest 300 python -c "import dllm.parallel.selftest as s; s.run(1, \"nccl\", 29641); print(\"selftest ok\")" --backend nccl --world 1
step bench_ddp_rccl 600 python bench.py --steps 10 --warmup 3 --force_comm
step bench_ddp_rccl_bf16g 600 python bench.py --steps 10 --warmup 3 --force_comm --grad_dtype bf16
step bench_fsdp_rccl 600 python bench.py --steps 10 --warmup 3 --force_comm --method fsdp
step bench_tp1 600 python bench.py --steps 10 --warmup 3 --method tp
