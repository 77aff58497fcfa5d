#!/bin/bash
# Weight-gradient GEMMs on the 4-phase schedule vs persistent 8-phase, in the flagship step (interleaved).
source scripts/gpu_steps.sh
step d1 300 python bench.py --steps 20 --warmup 5
step t1 300 python bench.py --steps 20 --warmup 5 --tn_4phase
step d2 300 python bench.py --steps 20 --warmup 5
step t2 300 python bench.py --steps 20 --warmup 5 --tn_4phase
