#!/bin/bash
# Round 4 experiment (knob since removed; profiles/r4/adam_wgrad_pp_family_r4.txt): the Llama-dims AdamW stack with its fused-AdamW weight gradients on the 256x128 two-blocks-per-CU
# family (DLLM_PP_EPI=adam_split: one block's 24 B/param epilogue under the other's MFMAs) vs the 256x256 default.
source scripts/gpu_steps.sh
C="python bench.py --methods none --steps 4 --warmup 2 --method hybrid --tp 1 --gated --act silu --ffn_dim 14336 --layers 32 --optimizer adam"
for r in 1 2; do
  step adam_def_$r 600 $C --json_out gpurun_out/adam_def_$r.json
  step adam_pp_$r 600 env DLLM_PP_EPI=adam_split $C --json_out gpurun_out/adam_pp_$r.json
done
