"""Checkpoint / resume in the reference's logical parameter layout.

The reference writes nothing to disk: ``train_*`` return ``list[layer] of (W1 [F,D], W2 [D,F])`` fp32 on
``cuda:0`` (train_ffns.py:116,193,287,338).  This module persists exactly that layout —
per layer ``w1 [F,D]``, ``w2 [D,F]`` (+ ``w3 [F,D]`` for gated FFNs), ``[out, in]`` order, fp32 — plus
optimizer state (same layout), the step counter and the run config, in two formats:

* ``consolidated``: one ``model.safetensors`` (+ ``optim.safetensors``) written by rank 0 from the
  gathered full tensors;
* ``sharded``: every rank writes its owned flat buffers (``rank{r}.safetensors``) + a layout record;
  the loader reassembles logical tensors from any saved mesh (DDP replicas, FSDP dim-0 row shards,
  TP dim-0/dim-1 splits, 2-D hybrids) and reshards them for the current mesh.

Files are read only with safetensors / JSON (no pickle).
"""
from __future__ import annotations

import json
import os

import torch
import torch.distributed as dist
from safetensors.torch import load_file, save_file

from ..models.ffn import deinterleave_w13


def _rank() -> int:
    return dist.get_rank() if dist.is_initialized() else 0


def _barrier():
    if dist.is_initialized():
        dist.barrier()


def _flat_logical(layers: list[dict], prefix: str = "layers") -> dict:
    out = {}
    for l, p in enumerate(layers):
        for k, v in p.items():
            out[f"{prefix}.{l}.{k}"] = v.detach().to(torch.float32).contiguous().cpu()
    return out


def _unflat_logical(tensors: dict, prefix: str = "layers") -> list[dict]:
    layers: dict[int, dict] = {}
    for k, v in tensors.items():
        pre, l, name = k.split(".")
        if pre != prefix:
            continue
        layers.setdefault(int(l), {})[name] = v
    return [layers[i] for i in sorted(layers)]


def save_checkpoint(eng, path: str, step: int, fmt: str = "consolidated", meta: dict | None = None) -> None:
    os.makedirs(path, exist_ok=True)
    rank = _rank()
    info = {"step": int(step), "format": fmt, "layers": eng.L, "gated": eng.gated,
            "optimizer": eng.cfg.optimizer, "opt_step": eng.step_count, **(meta or {})}
    if fmt == "consolidated":
        bufs = eng.flat_buffers()
        gathered = {name: eng.gather_full_params(flat) for name, flat in bufs.items()}
        if rank == 0:
            save_file(_flat_logical(gathered["params"]), os.path.join(path, "model.safetensors"))
            opt = {}
            for name, layers in gathered.items():
                if name != "params":
                    opt.update(_flat_logical(layers, prefix=name))
            if opt:
                save_file(opt, os.path.join(path, "optim.safetensors"))
            with open(os.path.join(path, "meta.json"), "w") as f:
                json.dump(info, f, indent=1, default=str)
    elif fmt == "sharded":
        bufs = {k: v.detach().cpu().contiguous() for k, v in eng.flat_buffers().items()}
        save_file(bufs, os.path.join(path, f"rank{rank}.safetensors"))
        layout = {"dp": eng.mesh.dp, "tp": eng.mesh.tp, "fsdp": eng.fsdp, "rank": rank,
                  "dp_rank": eng.mesh.dp_rank, "tp_rank": eng.mesh.tp_rank,
                  "entries": [[e.layer, e.name, list(e.shape), list(e.full_shape), e.offset] for e in eng.entries]}
        with open(os.path.join(path, f"rank{rank}.json"), "w") as f:
            json.dump(layout, f)
        if rank == 0:
            with open(os.path.join(path, "meta.json"), "w") as f:
                json.dump({**info, "world": eng.mesh.world}, f, indent=1, default=str)
    else:
        raise ValueError(fmt)
    _barrier()


def load_logical(path: str) -> tuple[dict, dict]:
    """Read a checkpoint of either format into ``{buffer_name: list[layer dict]}`` + meta (CPU)."""
    with open(os.path.join(path, "meta.json")) as f:
        meta = json.load(f)
    if meta["format"] == "consolidated":
        out = {"params": _unflat_logical(load_file(os.path.join(path, "model.safetensors")))}
        op = os.path.join(path, "optim.safetensors")
        if os.path.exists(op):
            t = load_file(op)
            for name in ("adam_m", "adam_v"):
                ls = _unflat_logical(t, prefix=name)
                if ls:
                    out[name] = ls
        return out, meta
    # sharded: reassemble logical tensors
    world = meta["world"]
    L, gated = meta["layers"], meta["gated"]
    parts: dict[str, dict] = {}
    for r in range(world):
        with open(os.path.join(path, f"rank{r}.json")) as f:
            lay = json.load(f)
        bufs = load_file(os.path.join(path, f"rank{r}.safetensors"))
        for bname, flat in bufs.items():
            for l, name, shape, full_shape, off in lay["entries"]:
                n = shape[0] * shape[1]
                t = flat[off:off + n].view(shape)
                key = (bname, l, name, lay["tp_rank"])
                parts.setdefault(key, {})[lay["dp_rank"]] = (t, lay["fsdp"], lay["tp"])
    out: dict[str, list] = {}
    for (bname, l, name, tpr), by_dp in parts.items():
        ts = [by_dp[k][0] for k in sorted(by_dp)]
        fsdp, tp = by_dp[min(by_dp)][1], by_dp[min(by_dp)][2]
        local = torch.cat(ts, dim=0) if fsdp else ts[0]
        out.setdefault(bname, {}).setdefault(l, {}).setdefault(name, {})[tpr] = (local, tp)
    res: dict[str, list] = {}
    for bname, layers in out.items():
        lst = []
        for l in range(L):
            p = {}
            w1s = [layers[l]["w1"][k][0] for k in sorted(layers[l]["w1"])]
            w2s = [layers[l]["w2"][k][0] for k in sorted(layers[l]["w2"])]
            if gated:
                pairs = [deinterleave_w13(w) for w in w1s]
                p["w1"] = torch.cat([a for a, _ in pairs], 0)
                p["w3"] = torch.cat([b for _, b in pairs], 0)
            else:
                p["w1"] = torch.cat(w1s, 0)
            p["w2"] = torch.cat(w2s, 1)
            lst.append(p)
        res[bname] = lst
    return res, meta


def load_checkpoint(eng, path: str) -> int:
    """Load params (+ optimizer state) into ``eng`` for its current mesh; returns the saved step."""
    state, meta = load_logical(path)
    eng.load_full_params(state["params"])
    bufs = eng.flat_buffers()
    for name in ("adam_m", "adam_v"):
        if name in bufs and name in state:
            eng.load_full_params(state[name], flat=bufs[name])
    eng.step_count = int(meta.get("opt_step", 0))
    return int(meta["step"])
