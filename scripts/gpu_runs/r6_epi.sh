#!/bin/bash
# Round 6: numerics of the changed kernels (runtime-activation epilogues, TN restriction, transposed W2 storage, zero
# copy); the epilogue-cost decomposition (K vs 2K, epilogue-skip build); the zero / zero_copy side entries.
source scripts/gpu_steps.sh
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
step t_gemm 900 $T tests/test_gemm_gpu.py tests/test_gemm_nnwgrad_gpu.py tests/test_split_master_gpu.py
step t_comm 600 $T tests/test_comm_gpu.py -k "zero or fsdp_copying"
step epi_cost 600 python -u scripts/bench_epilogue_cost.py --libs distributed-llm-code-samples_amd/_dllm_native_episkip.so --json gpurun_out/epi_cost.json
step zero_side 400 python -u bench.py --steps 20 --warmup 5 --methods zero --no_reference_init --json_out gpurun_out/zero_side.json
