"""GEMM grids under a concurrent collective's CU footprint.

    python scripts/bench_occupancy.py [--blocks 0,16,32,64] [--cases fwd1,dx]

At N > 1 the RCCL kernels of the overlapped collectives keep some CUs busy (one workgroup per channel) while the
FFN GEMMs run.  A persistent grid of exactly one 128 KiB-LDS block per CU then has blocks with no CU to start on
until a collective workgroup leaves, and the makespan stretches by up to a whole block's work; a grid of two
blocks per CU (the engine's ``min_bpc`` 2 when it communicates) or one block per tile lets the dispatcher fill
the CUs that are free.  This script launches ``ops.elementwise.occupy_cus`` (B workgroups resident for about the
GEMM's own duration, on a side stream, dispatched first) next to each GEMM and reports the GEMM stream's time per
iteration for each grid policy, next to the ideal 256/(256-B) stretch.
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dllm  # noqa: E402,F401
from dllm.ops.elementwise import occupy_cus  # noqa: E402
from dllm.ops.gemm import gemm, set_bf16_variant, set_min_blocks_per_cu, set_tiles_per_block  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=8192)
    ap.add_argument("--D", type=int, default=4096)
    ap.add_argument("--F", type=int, default=16384)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--blocks", default="0,16,32,64")
    ap.add_argument("--policies", default="tpb1,tpb8,tpb8b2")
    ap.add_argument("--cases", default="")
    a = ap.parse_args()
    T, D, F = a.T, a.D, a.F
    bf, dev = torch.bfloat16, "cuda"
    x = torch.randn(T, D, device=dev, dtype=bf)
    w1 = torch.randn(F, D, device=dev, dtype=bf) * 0.02
    w2 = torch.randn(D, F, device=dev, dtype=bf) * 0.02
    h = torch.randn(T, F, device=dev, dtype=bf)
    act = torch.empty(T, F, device=dev, dtype=bf)
    y = torch.empty(T, D, device=dev, dtype=bf)
    dy = torch.randn(T, D, device=dev, dtype=bf)
    dx = torch.empty(T, D, device=dev, dtype=bf)
    mw2 = torch.randn(D, F, device=dev, dtype=torch.float32) * 0.02
    cw2 = mw2.to(bf)
    cases = {
        "fwd1 h=x.W1t (NT,act)": lambda: gemm(x, w1, "nt", out=act, epi="act", act="relu"),
        "fwd2 y=a.W2t (NT)": lambda: gemm(h, w2, "nt", out=y),
        "dW2 sgd (TN,fused)": lambda: gemm(dy, h, "tn", out=mw2, epi="sgd", lr=1e-9, aux_out=cw2),
        "dx=da.W1 (NN)": lambda: gemm(h, w1, "nn", out=dx),
    }
    if a.cases:
        cases = {k: v for k, v in cases.items() if any(c in k for c in a.cases.split(","))}
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    side = torch.cuda.Stream()
    main_s = torch.cuda.current_stream()

    def policy(p):
        set_bf16_variant("8phase_stagger")
        set_tiles_per_block(1 if p == "tpb1" else int(p[3:].split("b")[0]))
        set_min_blocks_per_cu(2 if p.endswith("b2") else 1)

    def run(fn, blocks, us):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        go = torch.cuda.Event()
        fn()
        torch.cuda.synchronize()
        s.record()
        for _ in range(a.iters):
            if blocks:
                go.record(main_s)
                side.wait_event(go)        # the stand-in starts when the previous GEMM ends ...
                with torch.cuda.stream(side):
                    occupy_cus(blocks, us)  # ... and is dispatched before this iteration's GEMM
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / a.iters

    blocks = [int(b) for b in a.blocks.split(",")]
    pols = a.policies.split(",")
    print(f"{ncu} CUs; GEMM-stream ms per iteration (x ideal {ncu}/({ncu}-B) stretch over the B=0 time)", flush=True)
    for name, fn in cases.items():
        policy("tpb8")
        us = run(fn, 0, 0) * 1e3
        res = {(p, b): [] for p in pols for b in blocks}
        for _ in range(a.rounds):
            for p in pols:
                policy(p)
                for b in blocks:
                    res[(p, b)].append(run(fn, b, us))
        for p in pols:
            base = statistics.median(res[(p, 0)]) if 0 in blocks else None
            msg = f"{name:24s} {p:7s}"
            for b in blocks:
                m = statistics.median(res[(p, b)])
                rel = f" ({m / (base * ncu / (ncu - b)):.2f}x ideal)" if base and b else ""
                msg += f" B={b:<3d} {m:7.3f}{rel}"
            print(msg, flush=True)
    set_bf16_variant("auto")
    set_tiles_per_block(8)
    set_min_blocks_per_cu(1)


if __name__ == "__main__":
    main()
