#!/bin/bash
# Round 3 (session 2) validation of the split-master tree: GPU suite, smoke, the driver's default bench line (with the
# side-by-side methods), the headline A/B against the fp32 master, and rocprofv3 kernel traces of the headline step.
source scripts/gpu_steps.sh
export TMPDIR=/tmp
step pytest_gpu 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 600 python -u bench.py --gpus 1 --steps 20 --warmup 5
step head_split 300 python -u bench.py --methods none --steps 20 --warmup 5
step head_fp32 300 python -u bench.py --methods none --steps 20 --warmup 5 --master fp32
step head_trace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_head -o head -- python bench.py --methods none --steps 10 --warmup 3
