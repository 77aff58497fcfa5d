#!/bin/bash
# Round 3 diagnostics: comm observer raw intervals (ZeRO / FSDP at N=1) + its known-schedule test; a rocprofv3 trace
# of the ZeRO forced-comm step for the trace's own overlap fraction; the gated Llama-dims stack without the
# concurrent weight-gradient stream (tpb 8 / 1).
source scripts/gpu_steps.sh
export PYTHONUNBUFFERED=1
step observe_test 300 python -u -m pytest tests/test_observe_gpu.py -q -s --timeout 240 --timeout-method thread
step diag_zero 300 python -u scripts/observe_diag.py --method zero --steps 2
step diag_fsdp 300 python -u scripts/observe_diag.py --method fsdp --steps 2
step prof_zero 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_zero -o run -- python3 bench.py --steps 10 --warmup 3 --methods none --method zero --force_comm
step zero_overlap 120 python scripts/rocpd_stats.py gpurun_out/prof_zero/run_results.db --overlap copyBuffer,nccl,rccl --last_ms 160
step gated_tpb8_nows 300 python -u bench.py --methods none --steps 6 --warmup 2 --layers 32 --ffn_dim 14336 --gated --act silu --tpb 8 --no-wgrad_stream
step gated_tpb1_nows 300 python -u bench.py --methods none --steps 6 --warmup 2 --layers 32 --ffn_dim 14336 --gated --act silu --tpb 1 --no-wgrad_stream
