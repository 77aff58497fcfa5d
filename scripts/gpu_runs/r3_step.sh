#!/bin/bash
# Round 3: end-to-end steps: the gated Llama-dims stack with persistent vs one-tile GEMM blocks, and the
# communicating methods at N=1 (force_comm) with the comm observer; then the observer's own known-schedule test.
set -o pipefail
mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1
G="timeout -k 10 300 python -u bench.py --methods none --steps 6 --warmup 2 --layers 32 --ffn_dim 14336 --gated --act silu"
for t in 1 8; do
  $G --tpb $t > gpurun_out/r3/gated_tpb$t.json 2> gpurun_out/r3/gated_tpb$t.err || { tail -20 gpurun_out/r3/gated_tpb$t.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r3/gated_tpb$t.json'));print('gated tpb$t', d['value'], d['ms_per_step'], d['tflops_per_gpu'])"
done
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --methods ddp,zero,fsdp,tp,hybrid > gpurun_out/r3/methods.json 2> gpurun_out/r3/methods.err || { tail -20 gpurun_out/r3/methods.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r3/methods.json"))
for k, v in d.get("methods", {}).items():
    print(k, v.get("ms_per_step"), json.dumps(v.get("comm")))
PY
timeout -k 10 300 python -u -m pytest tests/test_observe_gpu.py -x -q -s --timeout 240 --timeout-method thread > gpurun_out/r3/observe_test.log 2>&1; tail -8 gpurun_out/r3/observe_test.log
