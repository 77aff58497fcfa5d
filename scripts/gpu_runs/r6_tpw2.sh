#!/bin/bash
# Round 6: W2ᵀ storage on row-major TP layers (auto): numerics (bitwise vs row-major, 2-rank TP / hybrid on one GPU),
# config 5's FSDP x TP entry and the MP entry with W2ᵀ vs row-major, interleaved.
source scripts/gpu_steps.sh
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
step t_tpw2 600 $T tests/test_comm_gpu.py -k "w2_transposed" tests/test_multirank_gpu.py
C5="--ffn_dim 14336 --layers 32 --act silu --gated --methods none --no_reference_init --steps 10 --warmup 3 --phases --method hybrid --force_comm"
MP="--method tp --ffn_dim 14336 --layers 1 --methods none --no_reference_init --steps 100 --warmup 20 --force_comm"
for i in 1 2; do
  step c5h_auto_$i 400 python -u bench.py $C5 --json_out gpurun_out/c5h_auto_$i.json
  step c5h_row_$i 400 python -u bench.py $C5 --w2_storage rowmajor --json_out gpurun_out/c5h_row_$i.json
  step mp_auto_$i 200 python -u bench.py $MP --json_out gpurun_out/mp_auto_$i.json
  step mp_row_$i 200 python -u bench.py $MP --w2_storage rowmajor --json_out gpurun_out/mp_row_$i.json
done
