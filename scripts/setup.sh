#!/bin/bash
# Dev-box setup check and build (the reference's setup.sh configures git on its dev box, C24; here the
# box needs ROCm + PyTorch-ROCm and an in-tree build of the gfx950 library).
#   bash scripts/setup.sh            # check toolchain, build, import
#   bash scripts/setup.sh --test     # ... and run the CPU test suite
set -euo pipefail
cd "$(dirname "$0")/.."
ROCM=${ROCM_PATH:-/opt/rocm}
echo "== toolchain"
command -v hipcc >/dev/null || { echo "hipcc not on PATH (ROCm at $ROCM?)"; exit 1; }
hipcc --version | head -2
python3 -c "import torch; print('torch', torch.__version__, 'hip', torch.version.hip); assert torch.version.hip, 'need a ROCm build of PyTorch'"
python3 -c "import torch; n = torch.cuda.device_count(); print('visible GPUs:', n)"
echo "== build (hipcc --offload-arch=gfx950, in-tree)"
python3 -c "import __graft_entry__ as g; g.build()"
python3 -c "import dllm, dllm._native as n; print('native library:', n.lib()._name)"
if [[ "${1:-}" == "--test" ]]; then
  echo "== CPU tests"
  python3 -m pytest tests -q -m "not gpu"
fi
echo "setup ok"
