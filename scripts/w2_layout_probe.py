"""Probe: W2 stored [D, F] (reference layout) vs transposed [F, D] for the two GEMMs that read it.

fwd2 y = a·W2ᵀ : NT with W2 [D, F]  vs  NN with W2T [F, D]
da   = dy·W2  (ReLU mask epilogue): NN with W2 [D, F]  vs  NT with W2T [F, D]
ReLU-sparse activations (as in the real step), interleaved rounds in one process.
"""
import os, sys, statistics
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import dllm  # noqa
from dllm.ops.gemm import gemm


def timeit(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn(); torch.cuda.synchronize(); s.record()
    for _ in range(iters):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


T, D, F = 8192, 4096, 16384
bf = torch.bfloat16
a = torch.relu(torch.randn(T, F, device="cuda", dtype=bf))
w2 = (torch.randn(D, F, device="cuda") * 0.02).to(bf)
w2t = w2.t().contiguous()
dy = (torch.randn(T, D, device="cuda") * 0.1).to(bf)
y = torch.empty(T, D, device="cuda", dtype=bf)
da = torch.empty(T, F, device="cuda", dtype=bf)
cases = {
    "fwd2 NT W2[D,F]": lambda: gemm(a, w2, "nt", out=y),
    "fwd2 NN W2T[F,D]": lambda: gemm(a, w2t, "nn", out=y),
    "da NN W2[D,F] dact": lambda: gemm(dy, w2, "nn", out=da, epi="dact", act="relu", aux=a),
    "da NT W2T[F,D] dact": lambda: gemm(dy, w2t, "nt", out=da, epi="dact", act="relu", aux=a),
}
r = {k: [] for k in cases}
for _ in range(5):
    for k, f in cases.items():
        r[k].append(timeit(f))
flops = 2 * T * D * F
for k, v in r.items():
    m = statistics.median(v)
    print(f"{k:24s} {m * 1e3:8.1f} us  {flops / m / 1e9:7.1f} TF")
