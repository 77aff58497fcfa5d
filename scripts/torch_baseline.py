"""Plain-PyTorch baseline of the reference algorithm on the same GPU and config (context for bench.py).

The reference (train_ffns.py) publishes no numbers, so this measures its algorithm as a
straightforward PyTorch program on one MI355X: per-layer forward saving only the layer input, backward that
recomputes h (train_ffns.py:61-70), in-place SGD (:172) -- GEMMs on hipBLASLt through torch.matmul.

  fp32 : the reference's dtype (fp32 everywhere)
  bf16 : bf16 compute with fp32 master weights (the framework's numerics), still plain torch ops

Flagship config: L8 D4096 F16384 ReLU, T = 8x1024 tokens, synthetic device data, random-init weights.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import dllm  # noqa: F401
from dllm.models.reference import layer_bwd, layer_fwd


def step(masters, x, dy, lr, cdt):
    layers = [{k: v.to(cdt) for k, v in p.items()} for p in masters] if cdt != torch.float32 else masters
    acts, y = [], x
    for p in layers:
        acts.append(y)
        y = layer_fwd(p, y)
    g = dy
    for i in reversed(range(len(layers))):
        g, gr = layer_bwd(g, layers[i], acts[i])
        for k in gr:
            masters[i][k].add_(gr[k].float(), alpha=-lr)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", choices=["fp32", "bf16"], default="bf16")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--layers", type=int, default=8)
    a = ap.parse_args()
    D, F, T = 4096, 16384, 8192
    dev = "cuda"
    cdt = torch.float32 if a.dtype == "fp32" else torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    masters = [{"w1": 0.02 * torch.randn(F, D, device=dev, generator=g),
                "w2": 0.02 * torch.randn(D, F, device=dev, generator=g)} for _ in range(a.layers)]
    x = torch.randn(T, D, device=dev, generator=g).to(cdt)
    dy = (0.1 * torch.randn(T, D, device=dev, generator=g)).to(cdt)
    for _ in range(a.warmup):
        step(masters, x, dy, 1e-5, cdt)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(masters, x, dy, 1e-5, cdt)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / a.steps
    flops = a.layers * 14 * T * D * F  # 7 GEMMs per layer with the reference's recompute
    print(json.dumps({"baseline": f"plain torch, reference algorithm, {a.dtype}", "tokens_per_s": round(T / el, 1),
                      "ms_per_step": round(el * 1e3, 2), "executed_tflops": round(flops / el / 1e12, 1),
                      "peak_hbm_gib": round(torch.cuda.max_memory_allocated() / 2**30, 2)}))


if __name__ == "__main__":
    main()
