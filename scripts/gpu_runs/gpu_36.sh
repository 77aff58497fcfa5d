#!/bin/bash
source scripts/gpu_steps.sh
step w2probe 300 python scripts/w2_layout_probe.py
