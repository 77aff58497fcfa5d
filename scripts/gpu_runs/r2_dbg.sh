#!/bin/bash
source scripts/gpu_steps.sh
step dbg_new 200 python scripts/debug_fp32_adam.py
step dbg_old 200 env DLLM_NATIVE_LIB=distributed-llm-code-samples_amd/_dllm_native_f32old.so python scripts/debug_fp32_adam.py
