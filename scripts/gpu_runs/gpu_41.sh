#!/bin/bash
# Reference CLI on one MI355X: all methods (-m 0) at the README command's shape (1 layer), and bf16.
source scripts/gpu_steps.sh
step cli_m0 600 python train_ffns.py -s 4 -bs 8 -n 1024 -l 1 -d 4096 -m 0 -r 1
step cli_m1_bf16 600 python train_ffns.py -s 16 -bs 8 -n 1024 -l 1 -d 8192 -m 1 -r 1 --dtype bf16
