#!/bin/bash
source scripts/gpu_steps.sh
step probe_div 300 python -u scripts/probe_divergence.py
