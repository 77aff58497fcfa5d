#!/bin/bash
# Full GPU suite + smoke + kernel stats with persistent GEMM blocks on by default.
source scripts/gpu_steps.sh
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o p -- python3 bench.py --steps 5 --warmup 2
step bench_zero_fc 300 python bench.py --steps 10 --warmup 3 --force_comm --method zero
step bench_fsdp_fc 300 python bench.py --steps 10 --warmup 3 --force_comm --method fsdp
step bench_llama 600 python bench.py --steps 3 --warmup 1 --layers 32 --ffn_dim 14336 --gated --act silu --method hybrid --tp 1 --force_comm
