#!/bin/bash
# All BASELINE.json configs on the GPUs of this box (1 GPU: multi-GPU configs run their per-rank shapes).
source scripts/gpu_steps.sh
OUT=gpurun_out/bench_configs.jsonl; : > $OUT
b() { local name=$1; shift; step "cfg_$name" 900 python bench.py --methods none --json_out gpurun_out/cfg_$name.json "$@" && \
      python -c "import json,sys; d=json.load(open('gpurun_out/cfg_$name.json')); d['bench_config']='$name'; print(json.dumps(d))" >> $OUT; }
b c2_ddp_L8_D4096 --steps 10 --warmup 3 --method ddp
b c2_zero_L8_D4096 --steps 10 --warmup 3 --method zero
b c2_fp32_reference_dtype_L8_D4096 --steps 5 --warmup 2 --dtype fp32 --grad_dtype fp32
b c3_fsdp_L8_D4096_forcecomm --steps 10 --warmup 3 --method fsdp --force_comm
b c4_tp_F14336_L1_full --steps 50 --warmup 10 --method tp --ffn_dim 14336 --layers 1
b c4_tp8_rank_shard_F1792 --steps 100 --warmup 20 --method tp --ffn_dim 1792 --layers 1
b c5_llama3_8b_ffn_L32_swiglu --steps 4 --warmup 2 --method hybrid --tp 1 --gated --act silu --ffn_dim 14336 --layers 32
b c5_llama3_8b_ffn_L32_swiglu_adam --steps 4 --warmup 2 --method hybrid --tp 1 --gated --act silu --ffn_dim 14336 --layers 32 --optimizer adam
# the reference's memory example (train_ffns.py:8-10): D=8192 L=8 "does not fit with DDP" on 4x24 GB -- one MI355X holds it
b c6_ref_memory_example_D8192_L8 --steps 4 --warmup 2 --method ddp --model_size 8192 --layers 8
cat $OUT
