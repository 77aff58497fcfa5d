"""fp32 (reference-parity) GEMM throughput on the FFN shapes: the native bf16x6 split GEMM (default fp32 mode), the
native exact-fp32 MFMA kernel, and torch.matmul (rocBLAS/hipBLASLt) as the library point of comparison.
Also prints each method's max error relative to an fp64 reference on the same operands."""
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


for (M, N, K) in [(8192, 16384, 4096), (8192, 4096, 16384), (4096, 4096, 4096)]:
    for layout in ("nt", "nn", "tn"):
        if layout == "tn" and (M, N, K) == (8192, 4096, 16384):
            continue
        # FFN roles: nt = x·W1ᵀ, nn = dy·W2, tn = hᵀ·dy (weight gradient, K = tokens)
        a = torch.randn((M, K) if layout != "tn" else (K, M), device="cuda")
        b = torch.randn((N, K) if layout == "nt" else (K, N), device="cuda")
        c = torch.empty(M, N, device="cuda")
        ref = {"nt": lambda: a @ b.t(), "nn": lambda: a @ b, "tn": lambda: a.t() @ b}[layout]
        f = 2 * M * N * K
        row = []
        errs = []
        ad, bd = a[:512].double() if layout != "tn" else a[:, :512].double(), b.double()
        exact = {"nt": lambda: ad @ bd.t(), "nn": lambda: ad @ bd, "tn": lambda: ad.t() @ bd}[layout]()
        for name, fn in (("bf16x6", lambda: gemm(a, b, layout, out=c, force="bf16x6")),
                         ("mfma_f32", lambda: gemm(a, b, layout, out=c, force="mfma_f32")),
                         ("torch", ref)):
            tm = statistics.median([t(fn) for _ in range(3)])
            r = fn()
            r = (c if r is None or name != "torch" else r)[:512].double()
            errs.append(f"{name} {((r - exact).abs().max() / exact.abs().max()).item():.1e}")
            row.append(f"{name} {f / tm / 1e9:6.1f} TF")
        print(f"fp32 {layout} {M}x{N}x{K}: " + "  ".join(row) + "   | rel err " + ", ".join(errs), flush=True)
