#!/bin/bash
# Round 6: W2ᵀ storage on row-major TP layers and the one-pass draw + transpose of the step's inputs: GPU tests,
# config 5's FSDP x TP entry with W2ᵀ vs row-major (per-kernel profiles), the headline with the fused draw vs the
# engine's transposes (DLLM_DRAW_T=0), interleaved (profiles/r6/config5_hybrid_phases_r6.txt, fused_draw_r6.txt).
source scripts/gpu_steps.sh
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
step t_new 300 $T tests/test_gemm_gpu.py tests/test_comm_gpu.py -k "rng or device_data or w2_transposed"
step t_multirank 600 $T tests/test_multirank_gpu.py
C5="--ffn_dim 14336 --layers 32 --act silu --gated --methods none --no_reference_init --method hybrid --force_comm"
for w in auto rowmajor; do
  step prof_c5h_$w 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5h_$w -o run -- python3 bench.py $C5 --steps 3 --warmup 2 --w2_storage $w
done
H="--steps 20 --warmup 5 --methods none --no_reference_init --phases"
for i in 1 2 3; do
  step head_drawt_$i 300 python -u bench.py $H --json_out gpurun_out/head_drawt_$i.json
  step head_engt_$i 300 env DLLM_DRAW_T=0 python -u bench.py $H --json_out gpurun_out/head_engt_$i.json
done
step prof_head_drawt 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_head_drawt -o run -- python3 bench.py --steps 5 --warmup 2 --methods none --no_reference_init
