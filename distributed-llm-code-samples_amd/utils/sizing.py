"""Per-rank HBM accounting for a model and mesh (size everything for 288 GB per MI355X).

The reference's one quantitative claim is a memory argument: at D=8192, L=8 ("over 4B model, 16GB of space,
as fp32 is used") training "will work if FSDP is used ... but not with DDP" on 4 x 24 GB GPUs
(train_ffns.py:8-10).  ``plan()`` computes, for any configuration this framework runs, the persistent state
and the activation working set one rank allocates -- mirroring the engine's own buffers
(``parallel/engine.py``: flat fp32 master, compute copy, gradient buffer, Adam moments, ZeRO shard, FSDP rings,
saved activations, ReLU masks, dgrad buffers) -- and the headroom left in a device's HBM.  A test checks the
prediction against a constructed engine's buffers, so the table in README.md stays true.

    python -m dllm.utils.sizing --model_size 4096 --ffn_dim 14336 --layers 32 --gated --optimizer adam --gpus 8
"""
from __future__ import annotations

import argparse
import json

HBM_GIB = 288e9 / 2**30  # MI355X: 288 GB HBM3E


def _round_up(n: int, a: int) -> int:
    return (n + a - 1) // a * a


def resolve_wgrad_layout(layout: str, D: int, F_loc: int, R1: int, T: int, mode: str = "none", tp: int = 1,
                         dtype: str = "bf16", recompute: str = "none", sp: bool = False, master: str = "split",
                         on_gpu: bool = True) -> str:
    """The weight-gradient layout the engine runs for ``layout`` (mirrors ``FFNTrainer._wgrad_nn_supported``): "auto"
    -> "nn_w2t" on a GPU in bf16 for row-major data-parallel / single-device layers (no TP / SP, kept activations, a
    fused optimizer only on split masters) whose GEMMs all sit unsplit on the 256x256 tiles; otherwise "tn"."""
    if layout != "auto":
        return layout
    fused = mode == "none"
    if not on_gpu or dtype != "bf16" or tp > 1 or sp or recompute != "none" or (fused and master != "split"):
        return "tn"
    from ..parallel.engine import wgrad_nn_shape_problem

    return "tn" if wgrad_nn_shape_problem(T, D, F_loc, R1) else "nn_w2t"


def plan(D: int, F: int, L: int, tokens: int, dp: int = 1, tp: int = 1, mode: str = "none", gated: bool = False,
         act: str = "relu", dtype: str = "bf16", grad_dtype: str = "bf16", optimizer: str = "sgd",
         recompute: str = "none", relu_mask: bool = True, sequence_parallel: bool = False,
         align: int = 64, wgrad_stream: bool = False, master: str = "split", wgrad_layout: str = "auto",
         on_gpu: bool = True) -> dict:
    """Per-rank bytes by buffer (and GiB totals).  ``mode``: none | ddp | zero | fsdp (over ``dp`` ranks).
    ``wgrad_stream``: the concurrent weight-gradient stream (single device, fused optimizer, kept activations, no
    TP) rotates two dgrad and three dx buffers instead of one and two (``FFNTrainer.da_ring`` / ``dxb``).
    ``master``: "split" keeps a bf16 run's fp32 master as the working copy plus an int16 residual plane
    (``master_residual``, 2 B/param) instead of a separate fp32 buffer (``master_fp32``, 4 B/param).
    ``wgrad_layout`` (the engine's resolved mode, ``FFNTrainer.wgrad_nn`` / ``wgrad_nn_w2``): nn_w1 keeps a transposed
    copy xᵀ [D, T] of every layer input, nn / nn_w2t also dyᵀ copies rotating with the dx buffers plus the top layer's;
    the NN modes run the backward serially (no weight-gradient stream).  "auto" resolves as the engine does
    (``resolve_wgrad_layout``): nn_w2t on a GPU wherever the layout runs, else tn."""
    cd = 2 if dtype == "bf16" else 4
    gd = 2 if grad_dtype == "bf16" else 4
    multi = dp > 1
    fsdp, zero, ddp = mode == "fsdp" and multi, mode == "zero" and multi, mode == "ddp" and multi
    F_loc = F // tp
    R1 = (2 if gated else 1) * F_loc
    al = align * dp if zero else align
    own = (lambda n: n // dp) if fsdp else (lambda n: n)
    total = L * (_round_up(own(R1 * D), al) + _round_up(own(D * F_loc), al))
    master_n = total // dp if zero else total
    b = {}
    if master == "split" and dtype == "bf16":
        b["master_residual"] = master_n * 2
    else:
        b["master_fp32"] = master_n * 4
    shared_copy = cd == 4 and not zero
    b["compute_copy"] = 0 if shared_copy else total * cd
    fused = not (ddp or zero or fsdp)
    b["grads"] = 0 if fused else total * gd
    if optimizer == "adam":
        b["adam_moments"] = 2 * master_n * 4
    if zero:
        b["zero_grad_shard"] = (total // dp) * gd
    if fsdp:
        layer = (R1 * D + D * F_loc)
        b["fsdp_weight_ring"] = 2 * layer * cd
        b["fsdp_grad_ring"] = 2 * layer * gd
    T = tokens
    sp = sequence_parallel and tp > 1
    Tl = T // tp if sp else T
    keep = recompute == "none"
    nA = L if keep else 1
    need_h = gated or act != "relu"
    b["layer_inputs"] = (L + 1) * Tl * D * cd
    b["activations"] = nA * T * F_loc * cd
    if need_h:
        b["preactivations"] = nA * T * R1 * cd
    if relu_mask and act == "relu" and not gated and dtype == "bf16":
        b["relu_masks"] = nA * (T // 256) * (F_loc // 256) * 8192
    wgrad_layout = resolve_wgrad_layout(wgrad_layout, D, F_loc, R1, T, mode=mode if multi else "none", tp=tp,
                                        dtype=dtype, recompute=recompute, sp=sp, master=master, on_gpu=on_gpu)
    # the engine runs the stream only while a weight gradient has <= 4 tiles per CU (TrainConfig.wgrad_stream_max_tpc)
    nn = wgrad_layout in ("nn_w1", "nn", "nn_w2t")
    ws = (wgrad_stream and fused and tp == 1 and keep and not sp and not nn
          and -(-R1 // 256) * -(-D // 256) <= 4 * 256)
    b["dgrad_buffer"] = (2 if ws else 1) * T * R1 * cd
    b["dx_buffers"] = (3 if ws else 2) * T * D * cd
    if nn:
        b["nn_transposed_copies"] = (L + (3 if wgrad_layout != "nn_w1" else 0)) * D * T * cd
    if sp:
        b["sp_buffers"] = (3 + (L if keep else 0)) * T * D * cd + 2 * Tl * D * cd
    state = sum(v for k, v in b.items() if k in ("master_fp32", "master_residual", "compute_copy", "grads", "adam_moments",
                                                   "zero_grad_shard", "fsdp_weight_ring", "fsdp_grad_ring"))
    tot = sum(b.values())
    g = 2**30
    return {"bytes": b, "state_gib": round(state / g, 2), "activations_gib": round((tot - state) / g, 2),
            "total_gib": round(tot / g, 2), "headroom_gib": round(HBM_GIB - tot / g, 1),
            "params_per_rank": total, "params_total": L * ((2 if gated else 1) * F * D + D * F),
            "wgrad_layout": wgrad_layout}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model_size", type=int, default=4096)
    ap.add_argument("--ffn_dim", type=int, default=0)
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--tokens", type=int, default=8192)
    ap.add_argument("--gated", action="store_true")
    ap.add_argument("--act", default="relu")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--grad_dtype", default="bf16")
    ap.add_argument("--optimizer", default="sgd")
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--wgrad_layout", default="auto", choices=["auto", "tn", "nn", "nn_w1", "nn_w2t"],
                    help="weight-gradient layout (auto: as the engine resolves it)")
    a = ap.parse_args()
    F = a.ffn_dim or 4 * a.model_size
    n = a.gpus
    meshes = {"1gpu": (1, 1, "none"), f"ddp{n}": (n, 1, "ddp"), f"zero{n}": (n, 1, "zero"),
              f"fsdp{n}": (n, 1, "fsdp"), f"tp{n}": (1, n, "none")}
    if n >= 4:
        meshes[f"fsdp{n // 2}xtp2"] = (n // 2, 2, "fsdp")
    for name, (dp, tp, mode) in meshes.items():
        r = plan(a.model_size, F, a.layers, a.tokens, dp, tp, mode, a.gated, a.act, a.dtype, a.grad_dtype,
                 a.optimizer, wgrad_layout=a.wgrad_layout)
        print(json.dumps({"mesh": name, "wgrad_layout": r["wgrad_layout"],
                          **{k: v for k, v in r.items() if k not in ("bytes", "wgrad_layout")}}))


if __name__ == "__main__":
    main()
