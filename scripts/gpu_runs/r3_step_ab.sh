#!/bin/bash
# Round 3: end-to-end step A/Bs, interleaved on one box -- split vs fp32 master (flagship and the D8192 memory example),
# the concurrent weight-gradient stream on / off (4 vs 16 tiles per CU), the forward raster band 8 vs 4.
# Regenerates profiles/r3/headline_split_vs_fp32_master_r3.txt, wgrad_stream_tiles_per_cu_r3.txt, group_m_nt_step_r3.txt.
source scripts/gpu_steps.sh
B="python -u bench.py --methods none --steps 20 --warmup 5"
C="python -u bench.py --methods none --steps 4 --warmup 2 --method ddp --model_size 8192 --layers 8"
for r in 1 2; do
  step head_split_$r 300 $B
  step head_fp32_$r 300 $B --master fp32
  step head_serial_$r 300 $B --no-wgrad_stream
  step head_gm8_$r 300 $B --group_m_nt 8
  step c6_split_$r 300 $C
  step c6_fp32_$r 300 $C --master fp32
  step c6_wgs_$r 300 $C --wgrad_stream_max_tpc 64
done
