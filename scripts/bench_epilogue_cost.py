"""Where a flagship GEMM's time goes: steady-state main loop vs per-tile fixed cost (epilogue, pipeline fill, tail).

For each GEMM family of the flagship step (T = 8192, D = 4096, F = 16384, finite N(0,1)-scaled bf16 data) the same
output tile grid is timed at K and 2K.  The 2K - K difference is K's worth of steady-state main loop (same tiles, same
tile transitions), so

    main(K) = t(2K) - t(K)        fixed = t(K) - main(K) = 2 t(K) - t(2K)

``fixed`` is everything a K-independent part of the kernel costs: the epilogue (stores, fused optimizer planes,
transposed copies, ReLU masks), the per-tile pipeline restart, the last-wave tail.  With ``--libs`` (diagnostic builds,
e.g. ``python -m dllm._build --variant episkip -DDLLM_EPI_SKIP=1``: every epilogue elided, wrong results) the same
cases run on each library, interleaved, so the epilogue's own share of ``fixed`` is measured directly.

    python scripts/bench_epilogue_cost.py [--libs path,...] [--rounds 5 --iters 6]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dllm  # noqa: E402,F401
from dllm import _native  # noqa: E402
from dllm.ops.gemm import gemm, relu_mask_bytes  # noqa: E402
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


def cases(T, D, F, g):
    bf = torch.bfloat16

    def rnd(*shape, s=1.0):
        return (torch.randn(*shape, generator=g) * s).to(bf).cuda()

    out = {}
    for mult in (1, 2):
        Dk, Fk, Tk = D * mult, F * mult, T * mult
        # fwd-1: h = x·W1ᵀ (NT), ReLU + 1-bit mask, K = D
        x, w1 = rnd(T, Dk), rnd(F, Dk, s=Dk ** -0.5)
        a = torch.empty(T, F, dtype=bf, device="cuda")
        mask = torch.empty(relu_mask_bytes(T, F), dtype=torch.uint8, device="cuda")
        out[("fwd1_nt_act", mult)] = (lambda x=x, w1=w1, a=a, mask=mask:
                                      gemm(x, w1, "nt", out=a, epi="act", act="relu", mask=mask), 2 * T * Dk * F,
                                      [a, mask])
        # fwd-2: y = a·W2ᵀ with W2ᵀ [F, D] stored (NN), store + transposed copy yᵀ, K = F
        av, w2t = rnd(T, Fk).relu_(), rnd(Fk, D, s=Fk ** -0.5)
        y, yT = torch.empty(T, D, dtype=bf, device="cuda"), torch.empty(D, T, dtype=bf, device="cuda")
        out[("fwd2_nn_store_dt", mult)] = (lambda av=av, w2t=w2t, y=y, yT=yT: gemm(av, w2t, "nn", out=y, aux_t=yT),
                                           2 * T * Fk * D, [y, yT])
        # dgrad: da = dy·W2 ⊙ mask (NT on W2ᵀ), K = D
        dy, w2tk = rnd(T, Dk), rnd(F, Dk, s=Dk ** -0.5)
        da = torch.empty(T, F, dtype=bf, device="cuda")
        out[("dgrad_nt_dact", mult)] = (lambda dy=dy, w2tk=w2tk, da=da, mask=mask:
                                        gemm(dy, w2tk, "nt", out=da, epi="dact", act="relu", aux=a, mask=mask),
                                        2 * T * Dk * F, [da])
        # weight gradient: dW1ᵀ = xᵀ·da (NN, K = T), written transposed into the split master of W1 [F, D] + SGD
        xT, dak = rnd(D, Tk), rnd(Tk, F, s=0.1)
        hi, lo = split_master((torch.randn(F, D, generator=g) * D ** -0.5).cuda())
        out[("wgrad_nn_t_sgd", mult)] = (lambda xT=xT, dak=dak, hi=hi, lo=lo:
                                         gemm(xT, dak, "nn", out=lo, epi="sgd_split", lr=1e-3, aux_out=hi, out_t=True),
                                         2 * D * Tk * F, [hi, lo])
        # weight gradient storing a bf16 gradient (the ZeRO / DDP path), same product
        gw = torch.empty(F, D, dtype=bf, device="cuda")
        out[("wgrad_nn_t_store", mult)] = (lambda xT=xT, dak=dak, gw=gw: gemm(xT, dak, "nn", out=gw, out_t=True),
                                           2 * D * Tk * F, [gw])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="", help="comma list of alternate builds (DLLM_NATIVE_LIB paths)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    T, D, F = 8192, 4096, 16384
    libs = {"base": _native.lib()}
    for i, path in enumerate(p for p in a.libs.split(",") if p):
        os.environ["DLLM_NATIVE_LIB"] = path
        libs[os.path.basename(path)] = _native._load()
    os.environ.pop("DLLM_NATIVE_LIB", None)
    cs = cases(T, D, F, torch.Generator().manual_seed(0))
    # bitwise: every case's outputs from the same starting state on each library (the first is the reference; an
    # epilogue-skip build is expected to differ).  The fused-SGD case updates its master planes in place: restore them.
    if len(libs) > 1:
        ref, same = {}, {}
        for ln, lib in libs.items():
            _native._LIB = lib
            for k, (fn, _, outs) in cs.items():
                if k[1] != 1:
                    continue
                saved = [t.clone() for t in outs]
                fn()
                torch.cuda.synchronize()
                got = [t.clone() for t in outs]
                for t, sv in zip(outs, saved):
                    t.copy_(sv)
                if ln == "base":
                    ref[k] = got
                else:
                    same[f"{ln}:{k[0]}"] = all(torch.equal(g_.view(torch.uint8), r_.view(torch.uint8))
                                               for g_, r_ in zip(got, ref[k]))
        _native._LIB = libs["base"]
        print("bitwise vs base:", json.dumps(same), flush=True)
    res = {(ln, k): [] for ln in libs for k in cs}
    for _ in range(a.rounds):
        for ln, lib in libs.items():
            _native._LIB = lib
            for k, (fn, _, _) in cs.items():
                res[(ln, k)].append(timeit(fn, a.iters))
    _native._LIB = libs["base"]
    table = {}
    for ln in libs:
        for fam in sorted({k[0] for k in cs}):
            t1 = statistics.median(res[(ln, (fam, 1))])
            t2 = statistics.median(res[(ln, (fam, 2))])
            main_k = t2 - t1
            fl = cs[(fam, 1)][1]
            row = {"t_K_us": round(t1, 1), "t_2K_us": round(t2, 1), "main_us": round(main_k, 1),
                   "fixed_us": round(t1 - main_k, 1), "fixed_frac": round((t1 - main_k) / t1, 3),
                   "tflops": round(fl / t1 / 1e6, 1), "main_tflops": round(fl / main_k / 1e6, 1)}
            table[f"{ln}:{fam}"] = row
            print(f"{ln:>10s} {fam:18s} " + " ".join(f"{k} {v}" for k, v in row.items()), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(table, f, indent=1)


if __name__ == "__main__":
    main()
