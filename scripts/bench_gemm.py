"""Per-GEMM throughput of the native gfx950 kernels vs torch.matmul (hipBLASLt) on the FFN shapes.

    python scripts/bench_gemm.py [--T 8192 --D 4096 --F 16384] [--iters 20]

Random N(0,1) bf16 operands (zero-filled operands read high on MI355X, guide §5.4 rule 25); variants are
interleaved in one process (rule 24) and the median of the rounds is reported.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dllm  # noqa: E402,F401
from dllm.ops.gemm import gemm, set_bf16_variant, set_tiles_per_block  # noqa: E402


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
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--group_m", type=int, default=4)
    ap.add_argument("--json", default="")
    ap.add_argument("--variants", default="2stage,8phase,8phase_stagger",
                    help="main-loop variants; 'tpbN' = 8-phase staggered with N tiles per persistent block, "
                         "'dyn' = dynamic persistent blocks")
    ap.add_argument("--cases", default="", help="comma-separated substrings selecting cases")
    ap.add_argument("--no_torch", action="store_true")
    ap.add_argument("--libs", default="",
                    help="comma-separated alternate native builds (python -m dllm._build --variant NAME -D...): each "
                         "becomes variant 'libI' (production kernels, tpb 8), timed interleaved with the others, and its "
                         "outputs are checked bitwise against the first variant's")
    a = ap.parse_args()
    T, D, F = a.T, a.D, a.F
    bf = torch.bfloat16
    dev = "cuda"
    x = torch.randn(T, D, device=dev, dtype=bf)
    w1 = torch.randn(F, D, device=dev, dtype=bf) * 0.02
    w2 = torch.randn(D, F, device=dev, dtype=bf) * 0.02
    h = torch.randn(T, F, device=dev, dtype=bf)
    act = torch.empty(T, F, device=dev, dtype=bf)
    y = torch.empty(T, D, device=dev, dtype=bf)
    dy = torch.randn(T, D, device=dev, dtype=bf)
    da = torch.empty(T, F, device=dev, dtype=bf)
    dx = torch.empty(T, D, device=dev, dtype=bf)
    gw1 = torch.empty(F, D, device=dev, dtype=torch.float32)
    gw2 = torch.empty(D, F, device=dev, dtype=torch.float32)
    mw2 = torch.randn(D, F, device=dev, dtype=torch.float32) * 0.02   # fp32 master + bf16 copy (fused SGD)
    cw2 = mw2.to(bf)
    rw2 = torch.zeros(D, F, device=dev, dtype=torch.int16)   # split master: bf16 copy + int16 residual plane
    gm = a.group_m
    cases = {
        "fwd1 h=x.W1t (NT,act)": (lambda: gemm(x, w1, "nt", out=act, epi="act", act="relu", group_m=gm),
                                  lambda: torch.relu(x @ w1.t())),
        "fwd2 y=a.W2t (NT)": (lambda: gemm(h, w2, "nt", out=y, group_m=gm), lambda: h @ w2.t()),
        "dW2=dyT.a (TN,f32)": (lambda: gemm(dy, h, "tn", out=gw2, group_m=gm),
                               lambda: (dy.t() @ h).float()),
        "dW2 sgd (TN,fused)": (lambda: gemm(dy, h, "tn", out=mw2, epi="sgd", lr=1e-9, aux_out=cw2, group_m=gm),
                               lambda: mw2.add_((dy.t() @ h).float(), alpha=-1e-9)),
        "dW2 sgd_split (TN,fused)": (lambda: gemm(dy, h, "tn", out=rw2, epi="sgd_split", lr=1e-9, aux_out=cw2,
                                                  group_m=gm), lambda: mw2.add_((dy.t() @ h).float(), alpha=-1e-9)),
        "da=dy.W2 (NN,dact)": (lambda: gemm(dy, w2, "nn", out=da, epi="dact", act="relu", aux=h, group_m=gm),
                               lambda: (dy @ w2) * (h > 0)),
        "dx=da.W1 (NN)": (lambda: gemm(h, w1, "nn", out=dx, group_m=gm), lambda: h @ w1),
        "dW1=daT.x (TN,f32)": (lambda: gemm(h, x, "tn", out=gw1, group_m=gm), lambda: (h.t() @ x).float()),
    }
    flops = 2 * T * D * F
    variants = a.variants.split(",")
    libs = {}
    if a.libs:
        from dllm import _native
        base = _native.lib()
        for i, path in enumerate(a.libs.split(",")):
            os.environ["DLLM_NATIVE_LIB"] = path
            libs[f"lib{i}"] = _native._load()
        os.environ.pop("DLLM_NATIVE_LIB")
        libs["lib_base"] = base
        variants = ["lib_base"] + sorted(k for k in libs if k != "lib_base")
        state = [mw2, cw2, rw2]
        outs = {"fwd1": act, "fwd2": y, "dW2=": gw2, "dW2 sgd ": mw2, "dW2 sgd_split": rw2, "da=": da, "dx=": dx,
                "dW1=": gw1}
    res = {}
    if a.cases:
        cases = {k: v for k, v in cases.items() if any(c in k for c in a.cases.split(","))}
    for name, (mine, ref) in cases.items():
        run_variants = variants
        times = {v: [] for v in run_variants}
        if libs:   # bitwise check of every build against the first, from the same initial state
            init = [t.clone() for t in state]
            got = {}
            for v in variants:
                for t, t0 in zip(state, init):
                    t.copy_(t0)
                _native._LIB = libs[v]
                set_bf16_variant("8phase_stagger")
                set_tiles_per_block(8)
                mine()
                torch.cuda.synchronize()
                o = next(t for k, t in outs.items() if name.startswith(k))
                got[v] = o.clone()
                if name.startswith("dW2 sgd_split"):
                    got[v] = torch.cat([o.view(torch.int16).flatten(), cw2.view(torch.int16).flatten()])
            for v in variants[1:]:
                same = torch.equal(got[v].view(torch.uint8), got[variants[0]].view(torch.uint8))
                print(f"  bitwise {v} == {variants[0]}: {same}", flush=True)
        tr = []
        for _ in range(a.rounds):  # interleaved rounds in one process (guide §5.4 rule 24)
            for v in run_variants:
                if v in libs:
                    _native._LIB = libs[v]
                    set_bf16_variant("8phase_stagger")
                    set_tiles_per_block(8)
                elif v.startswith("tpb"):
                    set_bf16_variant("8phase_stagger")
                    set_tiles_per_block(int(v[3:]))
                elif v.startswith("pp"):   # 256x128 two-blocks-per-CU family; ppN[sK]: N tiles per persistent
                    set_bf16_variant("pp")    # block, odd workgroup slot of each CU delayed K x 64 clocks
                    tpb, _, sk = v[2:].partition("s")
                    set_tiles_per_block(int(tpb or 1))
                    os.environ["DLLM_PP_SKEW"] = sk or "0"
                else:
                    set_bf16_variant(v)
                    set_tiles_per_block(1)
                times[v].append(timeit(mine, a.iters))
            if not a.no_torch:
                tr.append(timeit(ref, a.iters))
        row, msg = {}, f"{name:26s}"
        if tr:  # --no_torch: hipBLASLt not timed, no torch fields
            r = statistics.median(tr)
            row = {"torch_ms": r, "torch_tflops": flops / r / 1e9}
            msg += f" torch {flops / r / 1e9:7.1f} TF |"
        for v in run_variants:
            m = statistics.median(times[v])
            row[v + "_ms"], row[v + "_tflops"] = m, flops / m / 1e9
            msg += f" {v} {flops / m / 1e9:7.1f} TF"
        res[name] = row
        print(msg, flush=True)
    set_bf16_variant("auto")
    set_tiles_per_block(8)
    if libs:
        _native._LIB = libs["lib_base"]
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"T": T, "D": D, "F": F, "cases": res}, f, indent=1)


if __name__ == "__main__":
    main()
