"""Same GEMM shape in the three storage layouts (isolates the cost of MN-contiguous operands)."""
import os, sys, statistics
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import dllm  # noqa
from dllm.ops.gemm import gemm, set_bf16_variant


def timeit(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn(); torch.cuda.synchronize(); s.record()
    for _ in range(iters):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


set_bf16_variant("8phase_stagger")
for (M, N, K) in [(4096, 16384, 8192), (8192, 4096, 16384), (8192, 16384, 4096)]:
    bf = torch.bfloat16
    A_kc = torch.randn(M, K, device="cuda", dtype=bf); A_mc = torch.randn(K, M, device="cuda", dtype=bf)
    B_kc = torch.randn(N, K, device="cuda", dtype=bf); B_mc = torch.randn(K, N, device="cuda", dtype=bf)
    C16 = torch.empty(M, N, device="cuda", dtype=bf); C32 = torch.empty(M, N, device="cuda", dtype=torch.float32)
    fl = 2 * M * N * K
    cases = {"NT bf16out": lambda: gemm(A_kc, B_kc, "nt", out=C16),
             "NN bf16out": lambda: gemm(A_kc, B_mc, "nn", out=C16),
             "TN bf16out": lambda: gemm(A_mc, B_mc, "tn", out=C16),
             "NT f32out": lambda: gemm(A_kc, B_kc, "nt", out=C32),
             "TN f32out": lambda: gemm(A_mc, B_mc, "tn", out=C32)}
    res = {k: [] for k in cases}
    for _ in range(3):
        for k, f in cases.items():
            res[k].append(timeit(f))
    print(f"M={M} N={N} K={K}: " + "  ".join(f"{k} {fl / statistics.median(v) / 1e9:.0f}TF" for k, v in res.items()),
          flush=True)
