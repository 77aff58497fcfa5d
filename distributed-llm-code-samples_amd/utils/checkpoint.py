"""Checkpoint / resume in the reference's logical parameter layout, with scalable sharded files.

The reference writes nothing to disk: ``train_*`` return ``list[layer] of (W1 [F,D], W2 [D,F])`` fp32 on
``cuda:0`` (train_ffns.py:116,193,287,338).  This module persists exactly that layout —
per layer ``w1 [F,D]``, ``w2 [D,F]`` (+ ``w3 [F,D]`` for gated FFNs), ``[out, in]`` order, fp32 — plus
optimizer state (same layout), the step counter and the run config, in two formats:

* ``consolidated``: one ``model.safetensors`` (+ ``optim.safetensors``) written by rank 0 from the
  gathered full tensors (small / medium models, interchange);
* ``sharded``: every rank writes ONLY the state it owns — FSDP dim-0 row shards, ZeRO-2 flat shards of the
  fp32 master / Adam moments, TP slices; a replicated buffer (DDP, pure TP over dp) is written by its
  dp-rank-0 copy only — as ``rank{r}.safetensors`` + a piece index ``rank{r}.json``.  The loader reads,
  for the CURRENT mesh (any dp / tp / FSDP / ZeRO layout, any world size), only the byte ranges that
  overlap this rank's partition, through ``safetensors.safe_open`` slices (memory-mapped, no full-file
  loads): a reshard from world 4 to world 2 reads ~1/2 of the checkpoint per rank, not all of it.

Coordinates.  Every weight lives in one *global storage matrix*: the W1 family is ``G1 [R1, D]`` — ``w1``
rows, or for gated FFNs ``w1``/``w3`` interleaved in 16-row blocks over the whole F axis (a TP rank's local
interleaved ``W13`` is exactly rows ``[2·r·F/t, 2·(r+1)·F/t)`` of it) — and ``W2`` is ``G2 [D, F]`` (TP rank r:
columns ``[r·F/t, (r+1)·F/t)``).  A saved piece covers rows of a rank's local tensor (FSDP / replicas) or a
flat element range of it (ZeRO), i.e. at most three boxes of its global matrix; a loading rank needs boxes
of the same matrices, and every needed box is filled from the intersecting saved boxes.

Files are read only with safetensors / JSON (no pickle).
"""
from __future__ import annotations

import json
import os

import torch
import torch.distributed as dist
from safetensors import safe_open
from safetensors.torch import load_file, save_file

from ..models.ffn import GLU_BLOCK, deinterleave_w13, interleave_w13

FORMAT_VERSION = 2


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


# ------------------------------------------------------------------------------------------------------
# geometry: local tensors <-> global storage matrices
# ------------------------------------------------------------------------------------------------------
def _local_geom(eng, name: str) -> tuple[int, int, int, int]:
    """(rows, cols, global row offset, global col offset) of this rank's TP-local tensor of ``name``."""
    r = eng.mesh.tp_rank
    if name == "w1":
        return eng.R1, eng.D, r * eng.R1, 0
    return eng.D, eng.F_loc, 0, r * eng.F_loc


def _stored_t(eng, name: str) -> bool:
    """Whether ``name`` is stored transposed (W2ᵀ [F_loc, D]: the transposed-activation TP layout or the row-major
    layer's ``w2_storage``): its flat ranges are row-major in the STORED geometry, the checkpoint stays logical."""
    return bool(getattr(eng, "w2t", False)) and name == "w2"


def _flat_boxes(e0: int, e1: int, cols: int) -> list[tuple[int, int, int, int, int]]:
    """Split flat range [e0, e1) of a row-major ``[*, cols]`` tensor into boxes
    ``(r0, r1, c0, c1, flat_start)``: a partial first row, the full rows, a partial last row."""
    out = []
    while e0 < e1:
        r, c = divmod(e0, cols)
        if c == 0 and e1 - e0 >= cols:
            nr = (e1 - e0) // cols
            out.append((r, r + nr, 0, cols, e0))
            e0 += nr * cols
        else:
            c1 = min(cols, c + (e1 - e0))
            out.append((r, r + 1, c, c1, e0))
            e0 += c1 - c
    return out


def _owned_pieces(eng) -> list[dict]:
    """This rank's owned pieces of every (layer, weight): local-row ranges or local flat ranges."""
    pieces = []
    d, dr = eng.mesh.dp, eng.mesh.dp_rank
    for e in eng.entries:
        rows, cols, roff, coff = _local_geom(eng, e.name)
        base = {"layer": e.layer, "name": e.name, "rows": rows, "cols": cols, "row_off": roff, "col_off": coff}
        if eng.zero and _stored_t(eng, e.name):
            # flat ranges of the stored W2ᵀ: stored geometry [cols, rows] (``t``); boxes map back transposed
            base.update(rows=cols, cols=rows, t=True)
        if eng.zero:
            for a, b, go in eng._owned_segments(e.offset, e.offset + e.numel):
                pieces.append({**base, "kind": "flat", "e0": a - e.offset, "e1": b - e.offset,
                               "src": go})  # src: offset in the stored shard buffer
        elif eng.fsdp and _stored_t(eng, e.name):
            # FSDP row shards of the stored W2ᵀ are logical COLUMN ranges of W2 [D, F]
            own = cols // d
            pieces.append({**base, "kind": "cols", "c0": dr * own, "c1": (dr + 1) * own, "src": e.offset})
        elif eng.fsdp:
            own = rows // d
            pieces.append({**base, "kind": "rows", "r0": dr * own, "r1": (dr + 1) * own, "src": e.offset})
        elif dr == 0:  # replicated over dp: one copy is enough
            pieces.append({**base, "kind": "rows", "r0": 0, "r1": rows, "src": e.offset})
    return pieces


def _piece_boxes(p: dict) -> list[tuple]:
    """Global boxes of a piece: (R0, R1, C0, C1, local_r0, local_c0, flat_start | None)."""
    ro, co = p["row_off"], p["col_off"]
    if p["kind"] == "rows":
        return [(ro + p["r0"], ro + p["r1"], co, co + p["cols"], p["r0"], 0, None)]
    if p["kind"] == "cols":
        return [(ro, ro + p["rows"], co + p["c0"], co + p["c1"], 0, p["c0"], None)]
    if p.get("t"):   # stored transposed: stored rows are logical columns
        return [(ro + c0, ro + c1, co + r0, co + r1, r0, c0, fs) for r0, r1, c0, c1, fs in
                _flat_boxes(p["e0"], p["e1"], p["cols"])]
    return [(ro + r0, ro + r1, co + c0, co + c1, r0, c0, fs) for r0, r1, c0, c1, fs in
            _flat_boxes(p["e0"], p["e1"], p["cols"])]


# ------------------------------------------------------------------------------------------------------
# save
# ------------------------------------------------------------------------------------------------------
def save_checkpoint(eng, path: str, step: int, fmt: str = "consolidated", meta: dict | None = None) -> None:
    os.makedirs(path, exist_ok=True)
    rank = _rank()
    info = {"step": int(step), "format": fmt, "version": FORMAT_VERSION, "layers": eng.L, "gated": eng.gated,
            "D": eng.D, "F": eng.F, "optimizer": eng.cfg.optimizer, "opt_step": eng.step_count, **(meta or {})}
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
        bufs = eng.flat_buffers()
        pieces = _owned_pieces(eng)
        tensors, index = {}, []
        for bname, flat in bufs.items():
            for i, p in enumerate(pieces):
                key = f"{bname}/{p['layer']}/{p['name']}/{i}"
                if p["kind"] == "flat":
                    t = flat[p["src"]:p["src"] + (p["e1"] - p["e0"])]
                elif p["kind"] == "cols":   # FSDP shard of a stored W2ᵀ: the logical column block, whole
                    t = eng.logical_view(flat, eng.entry[(p["layer"], p["name"])])
                else:
                    e = eng.entry[(p["layer"], p["name"])]
                    own = eng.logical_view(flat, e)  # the stored 2-D tensor, [out, in] (FSDP: its row shard)
                    lo = p["r0"] - (p["r0"] if eng.fsdp else 0)
                    t = own[lo:lo + (p["r1"] - p["r0"])]
                tensors[key] = t.detach().to(torch.float32).contiguous().cpu()
                index.append({**{k: v for k, v in p.items() if k != "src"}, "key": key, "buf": bname})
        if tensors:
            save_file(tensors, os.path.join(path, f"rank{rank}.safetensors"))
        with open(os.path.join(path, f"rank{rank}.json"), "w") as f:
            json.dump({"rank": rank, "dp": eng.mesh.dp, "tp": eng.mesh.tp, "pieces": index}, f)
        if rank == 0:
            with open(os.path.join(path, "meta.json"), "w") as f:
                json.dump({**info, "world": eng.mesh.world}, f, indent=1, default=str)
    else:
        raise ValueError(fmt)
    _barrier()


# ------------------------------------------------------------------------------------------------------
# load
# ------------------------------------------------------------------------------------------------------
class _Reader:
    """Lazily opened safetensors files; counts the bytes actually sliced out of them."""

    def __init__(self, path: str):
        self.path, self.files, self.bytes_read = path, {}, 0

    def slice(self, fname: str, key: str, sl):
        f = self.files.get(fname)
        if f is None:
            f = self.files[fname] = safe_open(os.path.join(self.path, fname), framework="pt")
        t = f.get_slice(key)[sl]
        self.bytes_read += t.numel() * t.element_size()
        return t


def _needed_boxes(eng, e) -> list[tuple]:
    """Boxes of the global matrix this rank stores for entry ``e``, with their destination:
    (R0, R1, C0, C1, dest) where dest = ("rows", local_r0_of_stored_view) or ("flat", shard offset of the box's
    first element, local_r0, local_c0, cols); a flat box is one (partial) row or full-width rows."""
    rows, cols, ro, co = _local_geom(eng, e.name)
    if eng.zero:
        out = []
        t = _stored_t(eng, e.name)
        sc = rows if t else cols   # columns of the stored geometry
        for a, b, go in eng._owned_segments(e.offset, e.offset + e.numel):
            for r0, r1, c0, c1, fs in _flat_boxes(a - e.offset, b - e.offset, sc):
                dest = ("flatT" if t else "flat", go + (fs - (a - e.offset)), r0, c0, sc)
                if t:
                    out.append((ro + c0, ro + c1, co + r0, co + r1, dest))
                else:
                    out.append((ro + r0, ro + r1, co + c0, co + c1, dest))
        return out
    if eng.fsdp and _stored_t(eng, e.name):   # stored W2ᵀ row shard = logical column block
        own = cols // eng.mesh.dp
        c0 = eng.mesh.dp_rank * own
        return [(ro, ro + rows, co + c0, co + c0 + own, ("cols", c0))]
    if eng.fsdp:
        own = rows // eng.mesh.dp
        r0 = eng.mesh.dp_rank * own
        return [(ro + r0, ro + r0 + own, co, co + cols, ("rows", r0))]
    return [(ro, ro + rows, co, co + cols, ("rows", 0))]


def _fill(eng, target: torch.Tensor, e, sources, reader: _Reader) -> int:
    """Fill entry ``e`` of ``target`` from ``sources`` (list of (global box, read_fn)); returns elements written."""
    written = 0
    for R0, R1, C0, C1, dest in _needed_boxes(eng, e):
        for (S0, S1, T0, T1), read in sources:
            a, b, c, d = max(R0, S0), min(R1, S1), max(C0, T0), min(C1, T1)
            if a >= b or c >= d:
                continue
            blk = read(a, b, c, d).to(device=target.device, dtype=target.dtype)  # [b-a, d-c]
            if dest[0] in ("rows", "cols"):  # the stored 2-D view (FSDP: its shard) starts at global (R0, C0)
                eng.logical_view(target, e)[(a - R0):(b - R0), (c - C0):(d - C0)].copy_(blk)
            elif dest[0] == "flatT":
                # stored transposed: logical rows [a, b) are stored columns, logical columns [c, d) stored rows
                _, start, lr0, lc0, cols = dest
                base = start + (c - C0) * cols + (a - R0)
                bt = blk.t()
                if d - c == 1:
                    target[base:base + (b - a)].copy_(bt.reshape(-1))
                else:
                    target[base:base + (d - c - 1) * cols + (b - a)].as_strided((d - c, b - a), (cols, 1)).copy_(bt)
            else:
                _, start, lr0, lc0, cols = dest
                # box rows are local rows lr0.. of the flat segment; flat index of (row, col) relative to
                # the box start = (row - lr0) * cols + (col - lc0)
                base = start + (a - R0) * cols + (c - C0)
                if b - a == 1:
                    target[base:base + (d - c)].copy_(blk.reshape(-1))
                else:  # full-width box rows: a strided 2-D view
                    target[base:base + (b - a - 1) * cols + (d - c)].as_strided((b - a, d - c), (cols, 1)).copy_(blk)
            written += (b - a) * (d - c)
    return written


def _sharded_sources(path: str, meta: dict, reader: _Reader) -> dict:
    """{(buf, layer, name): [(global box, read_fn)]} over every rank file of a sharded checkpoint."""
    src: dict = {}
    for r in range(meta["world"]):
        with open(os.path.join(path, f"rank{r}.json")) as f:
            idx = json.load(f)
        fname = f"rank{r}.safetensors"
        for p in idx["pieces"]:
            for R0, R1, C0, C1, lr0, lc0, fs in _piece_boxes(p):
                if p["kind"] in ("rows", "cols"):
                    def read(a, b, c, d, p=p, R0=R0, C0=C0, fname=fname):
                        return reader.slice(fname, p["key"], (slice(a - R0, b - R0), slice(c - C0, d - C0)))
                elif p.get("t"):
                    def read(a, b, c, d, p=p, R0=R0, C0=C0, fs=fs, fname=fname):
                        # stored transposed: logical rows [a, b) = stored columns, logical columns [c, d) = stored
                        # rows; read the stored block, return it transposed
                        cols = p["cols"]
                        first = fs - p["e0"] + (c - C0) * cols + (a - R0)
                        if d - c == 1:
                            return reader.slice(fname, p["key"], slice(first, first + (b - a))).view(1, b - a).t()
                        span = reader.slice(fname, p["key"], slice(first, first + (d - c - 1) * cols + (b - a)))
                        return span.as_strided((d - c, b - a), (cols, 1)).t()
                else:
                    def read(a, b, c, d, p=p, R0=R0, C0=C0, lr0=lr0, lc0=lc0, fs=fs, fname=fname):
                        cols = p["cols"]
                        rel = fs - p["e0"]  # box start inside the saved 1-D tensor
                        first = rel + (a - R0) * cols + (c - C0)
                        if b - a == 1:
                            return reader.slice(fname, p["key"], slice(first, first + (d - c))).view(1, d - c)
                        span = reader.slice(fname, p["key"], slice(first, first + (b - a - 1) * cols + (d - c)))
                        return span.as_strided((b - a, d - c), (cols, 1))
                src.setdefault((p["buf"], p["layer"], p["name"]), []).append(((R0, R1, C0, C1), read))
    return src


def _consolidated_sources(path: str, meta: dict, reader: _Reader) -> dict:
    """Sources over a consolidated checkpoint: W2 and plain W1 are sliced straight out of the file; a gated
    W1 family (w1/w3 interleaved in the storage matrix) is rebuilt from the two logical tensors."""
    src: dict = {}
    L, gated, D, F = meta["layers"], meta["gated"], meta.get("D"), meta.get("F")
    files = {"params": ("model.safetensors", "layers")}
    if os.path.exists(os.path.join(path, "optim.safetensors")):
        with safe_open(os.path.join(path, "optim.safetensors"), framework="pt") as f:
            pres = {k.split(".")[0] for k in f.keys()}
        for pre in pres:
            files[pre] = ("optim.safetensors", pre)
    for bname, (fname, pre) in files.items():
        for l in range(L):
            if D is None:
                with safe_open(os.path.join(path, fname), framework="pt") as f:
                    Fx, Dx = f.get_slice(f"{pre}.{l}.w1").get_shape()
            else:
                Fx, Dx = F, D
            key2 = f"{pre}.{l}.w2"
            src.setdefault((bname, l, "w2"), []).append(
                ((0, Dx, 0, Fx), lambda a, b, c, d, k=key2, fn=fname: reader.slice(fn, k, (slice(a, b), slice(c, d)))))
            if not gated:
                key1 = f"{pre}.{l}.w1"
                src.setdefault((bname, l, "w1"), []).append(
                    ((0, Fx, 0, Dx),
                     lambda a, b, c, d, k=key1, fn=fname: reader.slice(fn, k, (slice(a, b), slice(c, d)))))
            else:
                def read13(a, b, c, d, l=l, pre=pre, fn=fname):
                    # interleaved rows [a, b) lie in 2*GLU_BLOCK-row periods p0 .. p1-1, i.e. logical rows
                    # [p0*GLU_BLOCK, p1*GLU_BLOCK) of w1 and of w3: slice only those (and columns [c, d)), re-interleave,
                    # crop.  Reads (b - a) rows + < 2 periods, never the whole tensors.
                    per = 2 * GLU_BLOCK
                    p0, p1 = a // per, -(-b // per)
                    rows = slice(p0 * GLU_BLOCK, p1 * GLU_BLOCK)
                    w1 = reader.slice(fn, f"{pre}.{l}.w1", (rows, slice(c, d)))
                    w3 = reader.slice(fn, f"{pre}.{l}.w3", (rows, slice(c, d)))
                    return interleave_w13(w1, w3)[a - p0 * per:b - p0 * per]

                src.setdefault((bname, l, "w1"), []).append(((0, 2 * Fx, 0, Dx), read13))
    return src


def load_into(eng, path: str) -> tuple[dict, int]:
    """Load a checkpoint of either format into ``eng``'s state buffers for its current mesh, reading only
    the ranges this rank stores.  Returns (meta, bytes read by this rank)."""
    with open(os.path.join(path, "meta.json")) as f:
        meta = json.load(f)
    reader = _Reader(path)
    if meta["format"] == "sharded":
        if meta.get("version", 1) < 2:
            raise ValueError("sharded checkpoint written by an older format version; re-save it")
        src = _sharded_sources(path, meta, reader)
    else:
        src = _consolidated_sources(path, meta, reader)
    if meta["layers"] != eng.L or bool(meta["gated"]) != bool(eng.gated):
        raise ValueError(f"checkpoint is L={meta['layers']} gated={meta['gated']}, engine L={eng.L} gated={eng.gated}")
    # a larger checkpoint would contain every needed box and silently load a sub-block of the wrong-sized matrices
    for dim in ("D", "F"):
        if meta.get(dim) is not None and int(meta[dim]) != int(getattr(eng, dim)):
            raise ValueError(f"checkpoint has {dim}={meta[dim]}, engine {dim}={getattr(eng, dim)}")
    bufs = eng.flat_buffers()
    for bname, target in bufs.items():
        for e in eng.entries:
            sources = src.get((bname, e.layer, e.name))
            if not sources:
                if bname == "params":
                    raise ValueError(f"checkpoint has no {bname} for layer {e.layer} {e.name}")
                continue
            need = sum((R1 - R0) * (C1 - C0) for R0, R1, C0, C1, _ in _needed_boxes(eng, e))
            got = _fill(eng, target, e, sources, reader)
            if got != need:
                raise ValueError(f"checkpoint covers {got} of {need} elements of {bname} layer {e.layer} {e.name}")
    eng.refresh_copy()
    eng.step_count = int(meta.get("opt_step", 0))
    return meta, reader.bytes_read


def load_logical(path: str) -> tuple[dict, dict]:
    """Read a checkpoint of either format into ``{buffer_name: list[layer dict]}`` + meta (CPU, full logical
    tensors: for inspection and interchange; training resumes through ``load_into``)."""
    with open(os.path.join(path, "meta.json")) as f:
        meta = json.load(f)
    if meta["format"] == "consolidated":
        out = {"params": _unflat_logical(load_file(os.path.join(path, "model.safetensors")))}
        op = os.path.join(path, "optim.safetensors")
        if os.path.exists(op):
            t = load_file(op)
            for name in sorted({k.split(".")[0] for k in t}):
                out[name] = _unflat_logical(t, prefix=name)
        return out, meta
    reader = _Reader(path)
    src = _sharded_sources(path, meta, reader)
    L, gated, D, F = meta["layers"], meta["gated"], meta["D"], meta["F"]
    R1 = 2 * F if gated else F
    out: dict = {}
    for (bname, l, name), sources in src.items():
        shape = (R1, D) if name == "w1" else (D, F)
        full = torch.zeros(shape, dtype=torch.float32)
        for (S0, S1, T0, T1), read in sources:
            full[S0:S1, T0:T1] = read(S0, S1, T0, T1)
        out.setdefault(bname, [dict() for _ in range(L)])[l][name] = full
    for bname, layers in out.items():
        for p in layers:
            if gated and "w1" in p:
                p["w1"], p["w3"] = deinterleave_w13(p["w1"])
    return out, meta


def load_checkpoint(eng, path: str) -> int:
    """Load params (+ optimizer state) into ``eng`` for its current mesh; returns the saved step."""
    meta, _ = load_into(eng, path)
    return int(meta["step"])


__all__ = ["save_checkpoint", "load_checkpoint", "load_into", "load_logical", "GLU_BLOCK"]
