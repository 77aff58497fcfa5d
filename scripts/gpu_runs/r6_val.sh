#!/bin/bash
# Round 6 validation: the whole GPU suite + smoke on the current tree; config 5's FSDP x TP (hybrid) entry against the
# plain single-device step by phase; the driver's N=1 command (headline, reference_init, methods).
source scripts/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
C5="--ffn_dim 14336 --layers 32 --act silu --gated --methods none --no_reference_init --steps 10 --warmup 3 --phases"
for i in 1 2; do
  step c5_plain_$i 400 python -u bench.py $C5 --json_out gpurun_out/c5_plain_$i.json
  step c5_hybrid_$i 400 python -u bench.py $C5 --method hybrid --force_comm --json_out gpurun_out/c5_hybrid_$i.json
done
step prof_c5_hybrid 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5h -o run -- python3 bench.py --ffn_dim 14336 --layers 32 --act silu --gated --methods none --no_reference_init --steps 3 --warmup 2 --method hybrid --force_comm
step prof_c5_plain 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5p -o run -- python3 bench.py --ffn_dim 14336 --layers 32 --act silu --gated --methods none --no_reference_init --steps 3 --warmup 2
step driver 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 --json_out gpurun_out/driver.json
