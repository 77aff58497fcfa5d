"""Plain-PyTorch baseline of the reference algorithm on the same GPU and config (the bar for bench.py).

The reference (train_ffns.py) publishes no numbers, so this measures its algorithm as a
straightforward PyTorch program on one MI355X -- GEMMs on hipBLASLt through torch.matmul, elementwise ops as
ATen kernels:

  --recompute on  : the reference algorithm: the forward saves only each layer's input, the backward recomputes
                    h (train_ffns.py:61-70): 7 GEMMs per layer
  --recompute off : the framework's algorithm: the forward keeps h, the backward runs 4 GEMMs (6 per layer)
  --dtype fp32    : the reference's dtype (fp32 everywhere)
  --dtype bf16    : bf16 compute with fp32 master weights (the framework's numerics), plain torch ops
  --init fan_in   : std 1/sqrt(fan_in) per matrix, the bench's default (finite data throughout); 0.02 is the
                    reference's init (train_ffns.py:35-36), under which the 8-layer D=4096 stack overflows to
                    inf / NaN after its first update (docs/DESIGN.md §1, "the step on finite data")

Every step draws fresh x ~ N(0,1) and dL/dy ~ 0.1 N(0,1) on the device (as the bench's timed region does) and
runs in-place SGD (train_ffns.py:172).  Flagship config: L8 D4096 F16384 ReLU, T = 8x1024 tokens.
"""
import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import dllm  # noqa: F401
from dllm.models.reference import layer_bwd, layer_fwd


def step(masters, x, dy, lr, cdt, recompute):
    layers = [{k: v.to(cdt) for k, v in p.items()} for p in masters] if cdt != torch.float32 else masters
    if recompute:
        acts, y = [], x
        for p in layers:
            acts.append(y)
            y = layer_fwd(p, y)
        g = dy
        for i in reversed(range(len(layers))):
            g, gr = layer_bwd(g, layers[i], acts[i])
            for k in gr:
                masters[i][k].add_(gr[k].float(), alpha=-lr)
        return
    saved, y = [], x
    for p in layers:
        h = y @ p["w1"].t()
        a = torch.relu(h)
        saved.append((y, h, a))
        y = a @ p["w2"].t()
    g = dy
    for i in reversed(range(len(layers))):
        xin, h, a = saved[i]
        p = layers[i]
        gw2 = g.t() @ a
        da = (g @ p["w2"]).masked_fill_(h <= 0, 0)
        gw1 = da.t() @ xin
        if i > 0:
            g = da @ p["w1"]       # the layer-0 input gradient is unused (the framework skips it too)
        masters[i]["w2"].add_(gw2.float(), alpha=-lr)
        masters[i]["w1"].add_(gw1.float(), alpha=-lr)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", choices=["fp32", "bf16"], default="bf16")
    ap.add_argument("--recompute", choices=["on", "off"], default="on")
    ap.add_argument("--init", default="fan_in", help="fan_in or a fixed std (0.02 = the reference's)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--layers", type=int, default=8)
    a = ap.parse_args()
    D, F, T = 4096, 16384, 8192
    dev = "cuda"
    cdt = torch.float32 if a.dtype == "fp32" else torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    s1, s2 = ((1 / math.sqrt(D), 1 / math.sqrt(F)) if a.init == "fan_in" else (float(a.init), float(a.init)))
    masters = [{"w1": s1 * torch.randn(F, D, device=dev, generator=g),
                "w2": s2 * torch.randn(D, F, device=dev, generator=g)} for _ in range(a.layers)]
    recompute = a.recompute == "on"

    def one():
        x = torch.randn(T, D, device=dev, generator=g, dtype=cdt)
        dy = torch.randn(T, D, device=dev, generator=g, dtype=cdt).mul_(0.1)
        step(masters, x, dy, 1e-5, cdt, recompute)

    for _ in range(a.warmup):
        one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        one()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / a.steps
    gemms = 7 if recompute else 6
    flops = a.layers * 2 * gemms * T * D * F - (0 if recompute else 2 * T * D * F)   # no layer-0 dx without recompute
    finite = all(bool(torch.isfinite(p[k]).all()) for p in masters for k in p)
    print(json.dumps({"baseline": f"plain torch, {a.dtype}, recompute {a.recompute}, init {a.init}",
                      "tokens_per_s": round(T / el, 1), "ms_per_step": round(el * 1e3, 2),
                      "executed_tflops": round(flops / el / 1e12, 1), "finite": finite,
                      "peak_hbm_gib": round(torch.cuda.max_memory_allocated() / 2**30, 2)}), flush=True)


if __name__ == "__main__":
    main()
