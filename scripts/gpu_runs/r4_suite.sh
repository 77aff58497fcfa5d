#!/bin/bash
# Round 4: the whole GPU suite + smoke on the current tree, the N=2 / N=4 rehearsals (torchrun and bench.py's own
# launcher, ranks sharing the card over gloo), headline kernel stats.
source scripts/gpu_steps.sh
step pytest_gpu 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
bash scripts/gpu_runs/rehearsal.sh || exit $?   # a fatal step there ends this call too
step headline_stats 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_head -o run -- python3 bench.py --gpus 1 --steps 10 --warmup 3 --methods none
