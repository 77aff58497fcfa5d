"""Pure-torch oracle of the reference's training semantics (single process, any float dtype).

Used by the tests as ground truth for the engine and the kernels.  Semantics reproduced:

* layer: ``y = act(x·W1ᵀ)·W2ᵀ``; backward recomputes ``h`` from the layer input (train_ffns.py:54-70);
* 1-GPU: ``num_steps`` sequential SGD steps ``p ← p − lr·g`` (:101-116);
* DDP / FSDP: rank ``r`` takes seeds ``r, r+n, …``; each of the ``num_steps/n`` optimizer steps applies the
  **sum** of the n ranks' gradients (:164-172, :253-259) — DDP and FSDP are the same algorithm;
* TP: every rank sees every batch; mathematically identical to 1-GPU (:290-312).
"""
from __future__ import annotations

import torch

from ..ops.activations import act_fwd, act_grad


def layer_fwd(p: dict, x: torch.Tensor, act: str = "relu") -> torch.Tensor:
    h = x @ p["w1"].t()
    a = act_fwd(act, h)
    if "w3" in p:
        a = a * (x @ p["w3"].t())
    return a @ p["w2"].t()


def layer_bwd(dy: torch.Tensor, p: dict, x: torch.Tensor, act: str = "relu"):
    h = x @ p["w1"].t()
    g = {}
    if "w3" in p:
        u = x @ p["w3"].t()
        a = act_fwd(act, h) * u
        g["w2"] = dy.t() @ a
        da = dy @ p["w2"]
        dh = da * u * act_grad(act, h)
        du = da * act_fwd(act, h)
        g["w1"] = dh.t() @ x
        g["w3"] = du.t() @ x
        dx = dh @ p["w1"] + du @ p["w3"]
    else:
        a = act_fwd(act, h)
        g["w2"] = dy.t() @ a
        dh = (dy @ p["w2"]) * act_grad(act, h)
        g["w1"] = dh.t() @ x
        dx = dh @ p["w1"]
    return dx, g


def stack_grads(layers: list[dict], x: torch.Tensor, dy: torch.Tensor, act: str = "relu"):
    acts = []
    y = x
    for p in layers:
        acts.append(y)
        y = layer_fwd(p, y, act)
    grads = [None] * len(layers)
    g = dy
    for i in reversed(range(len(layers))):
        g, grads[i] = layer_bwd(g, layers[i], acts[i], act)
    return y, grads


def _clone(layers):
    return [{k: v.clone() for k, v in p.items()} for p in layers]


def train_single(layers: list[dict], batches: list, lr: float, act: str = "relu") -> list[dict]:
    ps = _clone(layers)
    for x, dy in batches:
        _, grads = stack_grads(ps, x, dy, act)
        ps = [{k: p[k] - lr * g[k] for k in p} for p, g in zip(ps, grads)]
    return ps


def train_data_parallel(layers: list[dict], batches: list, n: int, lr: float, act: str = "relu") -> list[dict]:
    """Each optimizer step consumes n consecutive batches (rank r gets batch j*n + r) and applies the
    summed gradient."""
    if len(batches) % n:
        raise ValueError("num_steps must be divisible by n")
    ps = _clone(layers)
    for j in range(len(batches) // n):
        total = None
        for r in range(n):
            x, dy = batches[j * n + r]
            _, grads = stack_grads(ps, x, dy, act)
            if total is None:
                total = grads
            else:
                total = [{k: t[k] + g[k] for k in t} for t, g in zip(total, grads)]
        ps = [{k: p[k] - lr * g[k] for k in p} for p, g in zip(ps, total)]
    return ps


def _q(t: torch.Tensor, dt) -> torch.Tensor:
    return t if dt is None else t.to(dt).to(t.dtype)


def stack_grads_mixed(layers: list[dict], x: torch.Tensor, dy: torch.Tensor, act: str = "relu",
                      compute_dtype=torch.bfloat16):
    """Oracle of the engine's mixed-precision dataflow (non-gated): weights, activations and activation
    gradients rounded to ``compute_dtype`` exactly where the engine stores them; fp32 accumulation and
    fp32 weight gradients (recompute='none')."""
    q = lambda t: _q(t, compute_dtype)  # noqa: E731
    w = [{k: q(v) for k, v in p.items()} for p in layers]
    xs, hs, as_ = [q(x)], [], []
    for p in w:
        h = xs[-1] @ p["w1"].t()
        hs.append(q(h))
        as_.append(q(act_fwd(act, h)))
        xs.append(q(as_[-1] @ p["w2"].t()))
    grads = [None] * len(layers)
    g = q(dy)
    for i in reversed(range(len(layers))):
        p = w[i]
        gw2 = g.t() @ as_[i]
        aux = as_[i] if act == "relu" else hs[i]
        da = q((g @ p["w2"]) * act_grad(act, aux))
        gw1 = da.t() @ xs[i]
        grads[i] = {"w1": gw1, "w2": gw2}
        g = q(da @ p["w1"])
    return grads


def train_single_mixed(layers, batches, lr, act="relu", compute_dtype=torch.bfloat16):
    ps = _clone(layers)
    for x, dy in batches:
        grads = stack_grads_mixed(ps, x, dy, act, compute_dtype)
        ps = [{k: p[k] - lr * g[k] for k in p} for p, g in zip(ps, grads)]
    return ps


def train_adam_single(layers, batches, lr, b1=0.9, b2=0.95, eps=1e-8, wd=0.0, act="relu"):
    ps = _clone(layers)
    m = [{k: torch.zeros_like(v) for k, v in p.items()} for p in ps]
    v = [{k: torch.zeros_like(t) for k, t in p.items()} for p in ps]
    for step, (x, dy) in enumerate(batches, start=1):
        _, grads = stack_grads(ps, x, dy, act)
        for p, g, mm, vv in zip(ps, grads, m, v):
            for k in p:
                mm[k] = b1 * mm[k] + (1 - b1) * g[k]
                vv[k] = b2 * vv[k] + (1 - b2) * g[k] * g[k]
                mh, vh = mm[k] / (1 - b1 ** step), vv[k] / (1 - b2 ** step)
                p[k] = p[k] - lr * (mh / (torch.sqrt(vh) + eps) + wd * p[k])
    return ps
