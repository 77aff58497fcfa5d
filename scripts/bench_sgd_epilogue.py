"""Fused split-master SGD weight-gradient GEMM vs the same GEMM storing a bf16 gradient (the flagship's dW1 shape,
[16384, 4096] = 1024 tiles, K = T = 8192, persistent 4 tiles per CU): the epilogue's cost per GEMM.  Interleaved rounds,
median.  Run it against an alternate build with DLLM_NATIVE_LIB to A/B an epilogue change; ``--layouts`` also times
the same product with K-contiguous operands (NT) and with only A K-contiguous (NN): the TN layout's own cost.

    python scripts/bench_sgd_epilogue.py [--iters 10 --rounds 5]"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dllm  # noqa: E402,F401
from dllm.ops.gemm import gemm  # noqa: E402
from dllm.ops.master import split_master  # noqa: E402


def timeit(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--layouts", action="store_true", help="also time the same GEMM as NT and NN")
    a = ap.parse_args()
    T, D, F = 8192, 4096, 16384
    g = torch.Generator().manual_seed(0)
    da = torch.randn(T, F, generator=g).to(torch.bfloat16).cuda()
    x = torch.randn(T, D, generator=g).to(torch.bfloat16).cuda()
    hi, lo = split_master((torch.randn(F, D, generator=g) * 0.02).cuda())
    grad = torch.empty(F, D, dtype=torch.bfloat16, device="cuda")
    daT, xT = da.t().contiguous(), x.t().contiguous()   # the same GEMM with K-contiguous operands (NT) / A only (NN)
    res = {"sgd_split": [], "store_bf16": [], "nt_store_bf16": [], "nn_store_bf16": []}
    for _ in range(a.rounds):
        res["sgd_split"].append(timeit(lambda: gemm(da, x, "tn", out=lo, epi="sgd_split", lr=1e-9, aux_out=hi),
                                       a.iters))
        res["store_bf16"].append(timeit(lambda: gemm(da, x, "tn", out=grad), a.iters))
        if a.layouts:
            res["nt_store_bf16"].append(timeit(lambda: gemm(daT, xT, "nt", out=grad), a.iters))
            res["nn_store_bf16"].append(timeit(lambda: gemm(daT, x, "nn", out=grad), a.iters))
    med = {k: statistics.median(v) for k, v in res.items() if v}
    print(f"lib={os.environ.get('DLLM_NATIVE_LIB', 'default')} sgd_split {med['sgd_split']:.1f} us  "
          f"store_bf16 {med['store_bf16']:.1f} us  epilogue cost {med['sgd_split'] - med['store_bf16']:.1f} us",
          flush=True)
    if a.layouts:
        print(f"same GEMM storing bf16: TN {med['store_bf16']:.1f} us, NN (A K-contiguous) {med['nn_store_bf16']:.1f} "
              f"us, NT (both K-contiguous) {med['nt_store_bf16']:.1f} us", flush=True)


if __name__ == "__main__":
    main()
