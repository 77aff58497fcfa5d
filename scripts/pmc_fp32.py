"""Target program for PMC passes over the fp32 GEMMs (native exact-fp32 kernel and torch.matmul on the same
shape); run under rocprofv3 --pmc, see scripts/gpu_runs/r2_pmc_fp32.sh."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dllm  # noqa: E402,F401
from dllm.ops.gemm import gemm  # noqa: E402

M, N, K = 8192, 16384, 4096
layout = sys.argv[1] if len(sys.argv) > 1 else "nt"
a = torch.randn((M, K) if layout != "tn" else (K, M), device="cuda")
b = torch.randn((N, K) if layout == "nt" else (K, N), device="cuda")
c = torch.empty(M, N, device="cuda")
ref = {"nt": lambda: a @ b.t(), "nn": lambda: a @ b, "tn": lambda: a.t() @ b}[layout]
for _ in range(3):
    gemm(a, b, layout, out=c)
    ref()
torch.cuda.synchronize()
print("done", flush=True)
