#!/bin/bash
# Round 4: where a short timed window loses time (TP8 shard and the flagship stack): per-step GPU events vs wall.
source scripts/gpu_steps.sh
step window_tp8 300 python -u scripts/window_probe.py
step window_flagship 300 python -u scripts/window_probe.py --ffn_dim 16384 --layers 8 --windows 5,10,20,40
