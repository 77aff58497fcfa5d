#!/bin/bash
# Round 3 (session 2): the reference's memory example (D8192 L8) with split vs fp32 masters, interleaved.
source scripts/gpu_steps.sh
for r in 1 2; do
  step c6_split_$r 300 python -u bench.py --methods none --steps 4 --warmup 2 --method ddp --model_size 8192 --layers 8
  step c6_fp32_$r 300 python -u bench.py --methods none --steps 4 --warmup 2 --method ddp --model_size 8192 --layers 8 --master fp32
done
