"""fp32 (reference-parity) GEMM throughput: native exact-fp32 MFMA kernel vs torch.matmul (rocBLAS/hipBLASLt)."""
import os, sys, statistics
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import dllm  # noqa
from dllm.ops.gemm import gemm

def t(fn, it=10):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize(); return s.elapsed_time(e) / it
for (M, N, K) in [(8192, 16384, 4096), (4096, 4096, 4096)]:
    for layout in ("nt", "nn", "tn"):
        a = torch.randn((M, K) if layout != "tn" else (K, M), device="cuda")
        b = torch.randn((N, K) if layout == "nt" else (K, N), device="cuda")
        c = torch.empty(M, N, device="cuda")
        ref = {"nt": lambda: a @ b.t(), "nn": lambda: a @ b, "tn": lambda: a.t() @ b}[layout]
        tm = statistics.median([t(lambda: gemm(a, b, layout, out=c)) for _ in range(3)])
        tr = statistics.median([t(ref) for _ in range(3)])
        f = 2 * M * N * K
        print(f"fp32 {layout} {M}x{N}x{K}: dllm {f / tm / 1e9:6.1f} TF  torch {f / tr / 1e9:6.1f} TF", flush=True)
