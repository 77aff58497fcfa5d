#!/bin/bash
# Full validation (GPU suite, smoke, default bench) + interleaved tiles-per-persistent-block A/B (2 vs 4 vs 8)
source scripts/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py --steps 20 --warmup 5
for i in 1 2 3; do
  for t in 2 4 8; do
    step t${t}_$i 120 python bench.py --steps 20 --warmup 5 --methods none --tpb $t
  done
done
