"""Fused-SGD weight-gradient GEMM: fp32 master + bf16 copy ("sgd") vs split master ("sgd_split", ops/master.py).

    python scripts/bench_sgd_split.py [--T 8192 --D 4096 --F 16384] [--rounds 7] [--iters 10]

Checks first that one update through each form leaves the same fp32 master, bit for bit, and that the split form's
working copy is that master rounded half away from zero; then times both forms interleaved in one process
(guide §5.4 rule 24) on the dW2 [D, F] and dW1 [F, D] shapes (K = T) and prints the medians.
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dllm  # noqa: E402,F401
from dllm.ops.gemm import gemm  # noqa: E402
from dllm.ops.master import join_master, split_master  # noqa: E402


def timeit(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=8192)
    ap.add_argument("--D", type=int, default=4096)
    ap.add_argument("--F", type=int, default=16384)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    T, D, F = a.T, a.D, a.F
    bf = torch.bfloat16
    dy = torch.randn(T, D, device="cuda", dtype=bf)
    act = torch.randn(T, F, device="cuda", dtype=bf)
    flops = 2 * T * D * F
    lr = 1e-3
    for name, (A, B) in {"dW2 [D,F]": (dy, act), "dW1 [F,D]": (act, dy)}.items():
        M, N = A.shape[1], B.shape[1]
        w = torch.randn(M, N, device="cuda", dtype=torch.float32) * 0.02
        # numerics: one update through each form from the same master
        m32, c16 = w.clone(), w.to(bf)
        gemm(A, B, "tn", out=m32, epi="sgd", lr=lr, aux_out=c16)
        hi, lo = split_master(w)
        gemm(A, B, "tn", out=lo, epi="sgd_split", lr=lr, aux_out=hi)
        torch.cuda.synchronize()
        same = torch.equal(join_master(hi, lo).view(torch.int32), m32.view(torch.int32))
        h_ref, _ = split_master(m32)
        same_hi = torch.equal(hi.view(torch.int16), h_ref.view(torch.int16))
        rne_diff = (hi.view(torch.int16) != c16.view(torch.int16)).sum().item()
        print(f"{name}: master bitwise equal {same}, hi == rhaz(master) {same_hi}, hi != rne copy at {rne_diff} "
              f"of {hi.numel()} (exact ties)", flush=True)
        if not (same and same_hi):
            raise SystemExit(f"{name}: split-master update differs")
        lr_t = 1e-9  # timing: keep the weights bounded over many updates
        f32 = lambda: gemm(A, B, "tn", out=m32, epi="sgd", lr=lr_t, aux_out=c16)  # noqa: E731
        spl = lambda: gemm(A, B, "tn", out=lo, epi="sgd_split", lr=lr_t, aux_out=hi)  # noqa: E731
        t32, tsp = [], []
        for _ in range(a.rounds):
            t32.append(timeit(f32, a.iters))
            tsp.append(timeit(spl, a.iters))
        m1, m2 = statistics.median(t32), statistics.median(tsp)
        print(f"{name}: sgd fp32-master {m1 * 1e3:7.1f} us ({flops / m1 / 1e9:6.1f} TF) | sgd split-master "
              f"{m2 * 1e3:7.1f} us ({flops / m2 / 1e9:6.1f} TF) | {100 * (m1 - m2) / m1:+.1f} %", flush=True)


if __name__ == "__main__":
    main()
