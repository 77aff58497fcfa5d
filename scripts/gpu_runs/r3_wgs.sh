#!/bin/bash
# Round 3 (session 2): concurrent weight-gradient stream on / off with split masters -- flagship (L8 D4096) and the
# reference's memory example (L8 D8192), interleaved.
source scripts/gpu_steps.sh
for r in 1 2; do
  step head_wgs_$r 300 python -u bench.py --methods none --steps 20 --warmup 5
  step head_serial_$r 300 python -u bench.py --methods none --steps 20 --warmup 5 --no-wgrad_stream
  step c6_wgs_$r 300 python -u bench.py --methods none --steps 4 --warmup 2 --method ddp --model_size 8192 --layers 8
  step c6_serial_$r 300 python -u bench.py --methods none --steps 4 --warmup 2 --method ddp --model_size 8192 --layers 8 --no-wgrad_stream
done
