#!/bin/bash
# Round 5: the reference CLI on the final tree (all methods, bf16, strict cross-checks) at flagship-like dims.
source scripts/gpu_steps.sh
step cli_all 500 python -u train_ffns.py -s 4 -bs 8 -n 1024 -l 2 -d 4096 -m 0 -r 1 --dtype bf16 --data device --strict
step cli_adam 300 python -u train_ffns.py -s 4 -bs 8 -n 1024 -l 2 -d 4096 -m 1 -r 1 --dtype bf16 --data device --optimizer adam --gated --act silu
