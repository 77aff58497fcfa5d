"""The NN weight-gradient layout against the TN one on the flagship layer (T = 8192, D = 4096, F = 16384), per GEMM:

* dW2 [D, F]: TN ``dyᵀ·a`` fused split-master SGD  vs  NN ``(dyᵀ)·a`` with ``dyᵀ`` [D, T] stored (A K-contiguous)
* dW1 [F, D]: TN ``daᵀ·x``                          vs  NN ``(xᵀ)·da`` written transposed into W1 (``out_t``)
* the producers of the transposed copies: y = a·W2ᵀ (NT) and dx = da·W1 (NN) with and without ``aux_t``, and the
  standalone transpose of a [T, D] bf16 matrix (layer 0's x, the top layer's dy)

Every pair is checked bitwise (same fp32 master before, same master after) before it is timed.  Interleaved rounds,
median of rounds, microseconds.

    python scripts/bench_nn_wgrad.py [--iters 10 --rounds 5]"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dllm  # noqa: E402,F401
from dllm.ops.gemm import gemm, transpose_bf16  # noqa: E402
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
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    T, D, F = 8192, 4096, 16384
    g = torch.Generator().manual_seed(0)
    bf = torch.bfloat16

    def rnd(*shape, s=1.0):
        return (torch.randn(*shape, generator=g) * s).to(bf).cuda()

    da, x, dy, act = rnd(T, F), rnd(T, D), rnd(T, D), rnd(T, F)
    w1, w2 = rnd(F, D, s=0.02), rnd(D, F, s=0.02)
    xT, dyT = x.t().contiguous(), dy.t().contiguous()
    m1 = (torch.randn(F, D, generator=g) * 0.02).cuda()
    m2 = (torch.randn(D, F, generator=g) * 0.02).cuda()
    hi1, lo1 = split_master(m1)
    hi2, lo2 = split_master(m2)
    h1b, l1b, h2b, l2b = hi1.clone(), lo1.clone(), hi2.clone(), lo2.clone()
    lr = 1e-3

    checks = {}
    # bitwise: one update each way from the same master
    gemm(da, x, "tn", out=lo1, epi="sgd_split", lr=lr, aux_out=hi1)
    gemm(xT, da, "nn", out=l1b, epi="sgd_split", lr=lr, aux_out=h1b, out_t=True)
    checks["dW1 nn out_t == tn"] = bool(torch.equal(hi1, h1b) and torch.equal(lo1, l1b))
    gemm(dy, act, "tn", out=lo2, epi="sgd_split", lr=lr, aux_out=hi2)
    gemm(dyT, act, "nn", out=l2b, epi="sgd_split", lr=lr, aux_out=h2b)
    checks["dW2 nn == tn"] = bool(torch.equal(hi2, h2b) and torch.equal(lo2, l2b))
    y0, y1, yT = (torch.empty(T, D, dtype=bf, device="cuda") for _ in range(3))
    yT = torch.empty(D, T, dtype=bf, device="cuda")
    gemm(act, w2, "nt", out=y0)
    gemm(act, w2, "nt", out=y1, aux_t=yT)
    checks["y with aux_t == y"] = bool(torch.equal(y0, y1))
    checks["yT == y.t()"] = bool(torch.equal(yT, y0.t()))
    dx0, dx1, dxT = torch.empty(T, D, dtype=bf, device="cuda"), torch.empty(T, D, dtype=bf, device="cuda"), \
        torch.empty(D, T, dtype=bf, device="cuda")
    gemm(da, w1, "nn", out=dx0)
    gemm(da, w1, "nn", out=dx1, aux_t=dxT)
    checks["dx with aux_t == dx"] = bool(torch.equal(dx0, dx1))
    checks["dxT == dx.t()"] = bool(torch.equal(dxT, dx0.t()))
    tT = torch.empty(D, T, dtype=bf, device="cuda")
    transpose_bf16(x, tT)
    checks["transpose"] = bool(torch.equal(tT, xT))
    print("bitwise:", json.dumps(checks), flush=True)

    cases = {
        "dW1_tn_sgd": lambda: gemm(da, x, "tn", out=lo1, epi="sgd_split", lr=1e-9, aux_out=hi1),
        "dW1_nn_t_sgd": lambda: gemm(xT, da, "nn", out=lo1, epi="sgd_split", lr=1e-9, aux_out=hi1, out_t=True),
        "dW2_tn_sgd": lambda: gemm(dy, act, "tn", out=lo2, epi="sgd_split", lr=1e-9, aux_out=hi2),
        "dW2_nn_sgd": lambda: gemm(dyT, act, "nn", out=lo2, epi="sgd_split", lr=1e-9, aux_out=hi2),
        "y_nt": lambda: gemm(act, w2, "nt", out=y0),
        "y_nt_aux_t": lambda: gemm(act, w2, "nt", out=y1, aux_t=yT),
        "dx_nn": lambda: gemm(da, w1, "nn", out=dx0),
        "dx_nn_aux_t": lambda: gemm(da, w1, "nn", out=dx1, aux_t=dxT),
        "transpose_TxD": lambda: transpose_bf16(x, tT),
    }
    res = {k: [] for k in cases}
    for _ in range(a.rounds):
        for k, fn in cases.items():
            res[k].append(timeit(fn, a.iters))
    med = {k: round(statistics.median(v), 1) for k, v in res.items()}
    for k, v in med.items():
        print(f"{k:16s} {v:8.1f} us", flush=True)
    per_layer_old = med["dW1_tn_sgd"] + med["dW2_tn_sgd"] + med["y_nt"] + med["dx_nn"]
    per_layer_new = med["dW1_nn_t_sgd"] + med["dW2_nn_sgd"] + med["y_nt_aux_t"] + med["dx_nn_aux_t"]
    print(f"per middle layer (dW1 + dW2 + y + dx): TN {per_layer_old:.1f} us, NN layout {per_layer_new:.1f} us "
          f"({per_layer_new - per_layer_old:+.1f}); + 2 transposes per step {2 * med['transpose_TxD']:.1f} us",
          flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"checks": checks, "median_us": med}, f, indent=1)


def operand_order():
    """Same product, same operands, the two MFMA operand orders: the plain store (B fragment first, lanes hold 4
    consecutive columns) vs ``out_t`` (A fragment first, lanes hold 4 consecutive rows, output written transposed), for
    the three layouts on flagship shapes."""
    g = torch.Generator().manual_seed(1)
    bf = torch.bfloat16
    T, D, F = 8192, 4096, 16384

    def rnd(*shape):
        return torch.randn(*shape, generator=g).to(bf).cuda()

    a, w2, da, w1, dy = rnd(T, F), rnd(D, F), rnd(T, F), rnd(F, D), rnd(T, D)
    dyT = dy.t().contiguous()
    cases = {  # name: (A, B, layout, out shape)
        "nt y=a.W2t": (a, w2, "nt", (T, D)),
        "nn dx=da.W1": (da, w1, "nn", (T, D)),
        "nn dW2=dyT.a": (dyT, a, "nn", (D, F)),
        "tn dW2=dy^T.a": (dy, a, "tn", (D, F)),
    }
    for name, (A, B, lay, (M, N)) in cases.items():
        o, ot = torch.empty(M, N, dtype=bf, device="cuda"), torch.empty(N, M, dtype=bf, device="cuda")
        gemm(A, B, lay, out=o)
        gemm(A, B, lay, out=ot, out_t=True)
        same = bool(torch.equal(o, ot.t()))
        r0, r1 = [], []
        for _ in range(5):
            r0.append(timeit(lambda: gemm(A, B, lay, out=o), 10))
            r1.append(timeit(lambda: gemm(A, B, lay, out=ot, out_t=True), 10))
        print(f"{name:16s} B-first {statistics.median(r0):7.1f} us  A-first(out_t) {statistics.median(r1):7.1f} us  "
              f"bitwise {same}", flush=True)




def epilogue_shapes():
    """Fused split-master SGD epilogue cost by output shape and map: the same NN product (K = 8192) updating a
    [4096, 16384] or a [16384, 4096] master, natural (lanes along the row) or transposed (``out_t``); cost = fused minus
    the same GEMM's plain bf16 store."""
    g = torch.Generator().manual_seed(2)
    bf = torch.bfloat16
    K = 8192

    def rnd(*shape, s=1.0):
        return (torch.randn(*shape, generator=g) * s).to(bf).cuda()

    for (M, N) in ((4096, 16384), (16384, 4096)):
        A, B = rnd(M, K), rnd(K, N)
        for out_t in (False, True):
            shp = (N, M) if out_t else (M, N)
            hi, lo = split_master((torch.randn(*shp, generator=g) * 0.02).cuda())
            st = torch.empty(*shp, dtype=bf, device="cuda")
            r0, r1 = [], []
            for _ in range(5):
                r0.append(timeit(lambda: gemm(A, B, "nn", out=st, out_t=out_t), 10))
                r1.append(timeit(lambda: gemm(A, B, "nn", out=lo, epi="sgd_split", lr=1e-9, aux_out=hi, out_t=out_t),
                                 10))
            s0, s1 = statistics.median(r0), statistics.median(r1)
            print(f"NN M={M:5d} N={N:5d} {'out_t' if out_t else 'natural'}: master {shp}, store {s0:7.1f} us, "
                  f"fused SGD {s1:7.1f} us, epilogue {s1 - s0:6.1f} us", flush=True)




def epilogue_raster():
    """The natural [4096, 16384] fused-SGD weight gradient (dW2's master) by raster band height group_m."""
    g = torch.Generator().manual_seed(3)
    bf = torch.bfloat16
    M, N, K = 4096, 16384, 8192
    A = torch.randn(M, K, generator=g).to(bf).cuda()
    B = torch.randn(K, N, generator=g).to(bf).cuda()
    hi, lo = split_master((torch.randn(M, N, generator=g) * 0.02).cuda())
    st = torch.empty(M, N, dtype=bf, device="cuda")
    for gm in (1, 2, 4, 8, 16):
        r0, r1 = [], []
        for _ in range(5):
            r0.append(timeit(lambda: gemm(A, B, "nn", out=st, group_m=gm), 10))
            r1.append(timeit(lambda: gemm(A, B, "nn", out=lo, epi="sgd_split", lr=1e-9, aux_out=hi, group_m=gm), 10))
        s0, s1 = statistics.median(r0), statistics.median(r1)
        print(f"group_m {gm:2d}: store {s0:7.1f} us, fused SGD {s1:7.1f} us, epilogue {s1 - s0:6.1f} us", flush=True)




def epilogue_pitch():
    """The natural [4096, 16384] fused-SGD weight gradient with the master rows padded (row pitch 16384 + pad
    elements): does the 32-KiB power-of-two row pitch cost the epilogue's HBM writes?"""
    g = torch.Generator().manual_seed(4)
    bf = torch.bfloat16
    M, N, K = 4096, 16384, 8192
    A = torch.randn(M, K, generator=g).to(bf).cuda()
    B = torch.randn(K, N, generator=g).to(bf).cuda()
    for pad in (0, 64, 128, 256, 2048):
        hi_f, lo_f = split_master((torch.randn(M, N + pad, generator=g) * 0.02).cuda())
        hi, lo = hi_f[:, :N], lo_f[:, :N]
        st = torch.empty(M, N + pad, dtype=bf, device="cuda")[:, :N]
        r0, r1 = [], []
        for _ in range(5):
            r0.append(timeit(lambda: gemm(A, B, "nn", out=st), 10))
            r1.append(timeit(lambda: gemm(A, B, "nn", out=lo, epi="sgd_split", lr=1e-9, aux_out=hi), 10))
        s0, s1 = statistics.median(r0), statistics.median(r1)
        print(f"pitch {N + pad:6d}: store {s0:7.1f} us, fused SGD {s1:7.1f} us, epilogue {s1 - s0:6.1f} us", flush=True)




def raster_t():
    """The step's NN-layout GEMMs by raster band height group_m: the transposed-map fused SGD weight gradient
    (M = 4096, N = 16384, K = 8192) and the NN stores with a transposed copy (fwd-2 / dx shape [8192, 4096], K = 16384)."""
    g = torch.Generator().manual_seed(5)
    bf = torch.bfloat16
    T, D, F = 8192, 4096, 16384
    xT = torch.randn(D, T, generator=g).to(bf).cuda()
    da = torch.randn(T, F, generator=g).to(bf).cuda()
    hi, lo = split_master((torch.randn(F, D, generator=g) * 0.02).cuda())
    a = torch.randn(T, F, generator=g).to(bf).cuda()
    w2t = (torch.randn(F, D, generator=g) * 0.02).to(bf).cuda()
    y = torch.empty(T, D, dtype=bf, device="cuda")
    yT = torch.empty(D, T, dtype=bf, device="cuda")
    for gm in (1, 2, 4, 8):
        r0, r1 = [], []
        for _ in range(5):
            r0.append(timeit(lambda: gemm(xT, da, "nn", out=lo, epi="sgd_split", lr=1e-9, aux_out=hi, out_t=True,
                                          group_m=gm), 10))
            r1.append(timeit(lambda: gemm(a, w2t, "nn", out=y, aux_t=yT, group_m=gm), 10))
        print(f"group_m {gm}: dW1 NN-T fused SGD {statistics.median(r0):7.1f} us, y NN + copy {statistics.median(r1):7.1f} us",
              flush=True)


if __name__ == "__main__":
    if "--operand_order" in sys.argv:   # python scripts/bench_nn_wgrad.py --operand_order
        operand_order()
    elif "--raster_t" in sys.argv:
        raster_t()
    elif "--epilogue_pitch" in sys.argv:
        epilogue_pitch()
    elif "--epilogue_raster" in sys.argv:
        epilogue_raster()
    elif "--epilogue_shapes" in sys.argv:
        epilogue_shapes()
    else:
        main()
