#!/bin/bash
# Round 5: cost of non-MFMA instructions interleaved into a one-wave-per-SIMD MFMA stream (scripts/mfma_mix.hip).
source scripts/gpu_steps.sh
hipcc -O3 --offload-arch=gfx950 -std=c++17 -w scripts/mfma_mix.hip -o /tmp/mfma_mix || exit 1
step mix 120 /tmp/mfma_mix
