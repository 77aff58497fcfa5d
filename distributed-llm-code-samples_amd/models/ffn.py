"""Transformer FFN sub-block stack with explicit ("first principles") forward and backward.

Reference semantics (train_ffns.py:35-94):

* parameters ``W1 [F, D]``, ``W2 [D, F]`` in ``[out, in]`` layout, ``scale·randn`` with scale 2e-2,
  drawn W1 then W2, layer by layer, after the step seeds (``:35-39``, ``:360-361``);
* ``y = act(x·W1ᵀ)·W2ᵀ`` — no bias, no residual, no norm (``:54-58``);
* backward by hand: ``dW2 = dyᵀ·a``, ``da = (dy·W2)⊙act'(h)``, ``dW1 = daᵀ·x``, ``dx = da·W1``
  (``:61-70``); the reference recomputes ``h`` from the saved layer input (``recompute="full"`` here).

MI355X design: each layer is 6 GEMMs in forward+backward order ``fwd1, fwd2 | da, dW2, dx, dW1``, every
elementwise op fused into a GEMM epilogue (activation into fwd1, activation-derivative mask into the
``da`` dgrad), so the only HBM traffic is GEMM operands.  With ``recompute="none"`` (default) the forward
keeps ``a`` (and ``h`` for non-ReLU activations) so the backward runs 4 GEMMs instead of the reference's
5 — 6·P·T model FLOPs instead of 7·P·T.  ReLU needs no ``h``: ``act'(h) = [a > 0]``.  Without a gradient
collective (one GPU, pure TP) the SGD/AdamW update is fused into the two weight-gradient GEMMs.

Gated (SwiGLU, Llama-3 FFN): ``a = act(x·W1ᵀ) ⊙ (x·W3ᵀ)``.  W1 and W3 are stored row-interleaved in
16-row blocks as one ``W13 [2F, D]`` so a single GEMM produces both pre-activations and its epilogue
combines each gate/up pair inside one lane (``epi="glu"``); the backward ``epi="dglu"`` writes the
interleaved ``[dg|du]`` that feeds one dgrad and one wgrad GEMM against W13.
"""
from __future__ import annotations

from typing import NamedTuple

import torch

from ..ops.gemm import gemm, gemm_pair
from ..utils.config import INIT_SCALE

GLU_BLOCK = 16


# --------------------------------------------------------------------------------------------------
# parameter init
# --------------------------------------------------------------------------------------------------
def init_linear_layer(m: int, n: int, gen: torch.Generator | None, scale: float = INIT_SCALE) -> torch.Tensor:
    """``[n, m]`` weight (``[out, in]``), reference init (train_ffns.py:35-36)."""
    return scale * torch.randn((n, m), generator=gen)


def init_ffn_layer(D: int, F: int, gen: torch.Generator | None, gated: bool = False) -> dict:
    """One layer's logical parameters in the reference RNG order (W1 then W2; W3 last if gated)."""
    p = {"w1": init_linear_layer(D, F, gen), "w2": init_linear_layer(F, D, gen)}
    if gated:
        p["w3"] = init_linear_layer(D, F, gen)
    return p


def init_ffn_params_device(D: int, F: int, L: int, seed: int, device, gated: bool = False,
                           scale: float | str = INIT_SCALE) -> list[dict]:
    """Device-side init (Philox, one stream per (layer, matrix)); identical on every rank and on CPU.
    ``scale="fan_in"``: std 1/sqrt(fan_in) per matrix (variance-preserving).  The reference's fixed 2e-2
    grows activations ~2x per layer at D=4096 and, through the gate's product of two projections,
    doubly exponentially in a deep gated stack without norms/residuals (a 32-layer SwiGLU stack
    overflows bf16 within a few layers); fan-in scaling keeps such stacks finite."""
    from ..ops.elementwise import rng_normal_

    out = []
    for l in range(L):
        p = {}
        for j, (name, shape) in enumerate((("w1", (F, D)), ("w2", (D, F)), ("w3", (F, D)))):
            if name == "w3" and not gated:
                continue
            t = torch.empty(shape, dtype=torch.float32, device=device)
            sc = shape[1] ** -0.5 if scale == "fan_in" else float(scale)
            rng_normal_(t, seed=seed, stream_id=1000 + 4 * l + j, scale=sc)
            p[name] = t
        out.append(p)
    return out


def interleave_w13(w1: torch.Tensor, w3: torch.Tensor) -> torch.Tensor:
    """[F,D],[F,D] -> [2F,D] with 16-row blocks alternating W1, W3."""
    F, D = w1.shape
    if F % GLU_BLOCK:
        raise ValueError(f"gated FFN needs F % {GLU_BLOCK} == 0 (F={F})")
    return torch.stack([w1.reshape(F // GLU_BLOCK, GLU_BLOCK, D), w3.reshape(F // GLU_BLOCK, GLU_BLOCK, D)],
                       dim=1).reshape(2 * F, D)


def deinterleave_w13(w13: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    R, D = w13.shape
    v = w13.reshape(R // (2 * GLU_BLOCK), 2, GLU_BLOCK, D)
    return v[:, 0].reshape(R // 2, D), v[:, 1].reshape(R // 2, D)


# --------------------------------------------------------------------------------------------------
# one layer
# --------------------------------------------------------------------------------------------------
def needs_preact(act: str, gated: bool) -> bool:
    """Whether the backward needs the pre-activation h (ReLU recovers act' from a itself)."""
    return gated or act != "relu"


def layer_fwd(x: torch.Tensor, w1: torch.Tensor, w2: torch.Tensor, act: str, gated: bool,
              a_out: torch.Tensor, h_out: torch.Tensor | None, y_out: torch.Tensor,
              before_fwd2=None, mask: torch.Tensor | None = None, y_t: torch.Tensor | None = None,
              w2t: bool = False) -> torch.Tensor:
    """y = act(x·W1ᵀ)·W2ᵀ  (gated: (act(x·W1ᵀ)⊙x·W3ᵀ)·W2ᵀ with ``w1`` = interleaved W13).
    ``before_fwd2()`` runs between the two GEMMs (e.g. waiting for W2's all-gather).  ``mask`` (ReLU):
    the first GEMM also writes the activation-gradient bitmask the backward's dgrad reads.  ``y_t`` (NN weight-gradient
    layout): the second GEMM's epilogue also writes yᵀ [D, T], the next layer's dW1 operand.  ``w2t``: ``w2`` is the
    stored W2ᵀ [F, D] (y = a·W2ᵀ then runs NN)."""
    if gated:
        gemm(x, w1, "nt", out=a_out, epi="glu", act=act, aux_out=h_out)
    else:
        gemm(x, w1, "nt", out=a_out, epi="act", act=act, aux_out=h_out, mask=mask)
    if before_fwd2 is not None:
        before_fwd2()
    gemm(a_out, w2, "nn" if w2t else "nt", out=y_out, aux_t=y_t)
    return y_out


class NNWgrad(NamedTuple):
    """Operands of the NN weight-gradient layout (round 5) for one layer's backward.

    The TN weight gradients ``dW2 = dyᵀ·a`` and ``dW1 = daᵀ·x`` read both operands through transposed LDS fragment
    reads (twice the read instructions of a K-contiguous operand).  With transposed copies of the two D-sized
    operands -- ``x_t`` = xᵀ [D, T] (the previous layer's fwd-2 epilogue writes it, ``layer_fwd(y_t=)``) and ``dy_t``
    = dyᵀ [D, T] (the layer above's dx epilogue writes it, ``dx_t``) -- both run as NN GEMMs with a K-contiguous A:
    ``dW2 = (dyᵀ)·a`` [D, F] and ``dW1ᵀ = (xᵀ)·da`` [D, F] written transposed into W1 [F, D] (``gemm(out_t=True)``).
    Same products, same accumulation order: bitwise the TN results (tests/test_gemm_nnwgrad_gpu.py).  ``dy_t`` None:
    dW2 stays TN (and dx needs no transposed copy) -- the ``nn_w1`` mode."""
    x_t: torch.Tensor
    dy_t: torch.Tensor | None
    dx_t: torch.Tensor | None


def wgrad_w2(dy: torch.Tensor, a: torch.Tensor, kw2: dict, nn: NNWgrad | None, w2t: bool = False) -> None:
    """dW2 [D, F]; ``w2t``: W2 is stored as W2ᵀ [F, D] and the gradient / fused update goes through the transposed
    output map (``gemm(out_t=True)``)."""
    if nn is None or nn.dy_t is None:
        gemm(dy, a, "tn", out_t=w2t, **kw2)                           # dW2 = dyᵀ·a        [D, F] (or -> W2ᵀ)
    else:
        gemm(nn.dy_t, a, "nn", out_t=w2t, **kw2)                      # dW2 = (dyᵀ)·a      [D, F] (or -> W2ᵀ)


def wgrad_w1(da: torch.Tensor, x: torch.Tensor, kw1: dict, nn: NNWgrad | None) -> None:
    if nn is None:
        gemm(da, x, "tn", **kw1)                                      # dW1 = daᵀ·x        [F, D]
    else:
        gemm(nn.x_t, da, "nn", out_t=True, **kw1)                     # dW1ᵀ = (xᵀ)·da     -> W1 [F, D]


def layer_bwd(dy: torch.Tensor, x: torch.Tensor, w1: torch.Tensor, w2: torch.Tensor, act: str, gated: bool,
              a: torch.Tensor, h: torch.Tensor | None, gw1, gw2, da_buf: torch.Tensor,
              dx_out: torch.Tensor | None, hooks=None, mask: torch.Tensor | None = None,
              dx_first: bool = False, pair_wgrads: bool = False,
              nn: NNWgrad | None = None, w2t: bool = False) -> torch.Tensor | None:
    """Backward of one layer; returns dx.

    ``gw1``/``gw2`` are either gradient tensors (overwritten) or dicts of ``gemm`` keyword arguments for the
    weight-gradient GEMMs — e.g. ``{"out": master, "epi": "sgd", "lr": …, "aux_out": bf16_copy}`` to fuse
    the optimizer update into the GEMM epilogue when no gradient collective is needed.

    Order ``da, dW2, dx, dW1``: every dgrad that reads a weight runs before that weight's (possibly fused)
    update, a TP all-reduce of ``dx`` overlaps the dW1 GEMM, and ``hooks`` (``after_w2``, ``after_dx``,
    ``after_w1``) mark the points where gradient collectives can be issued.  ``dx_first`` (tensor parallel):
    ``da, dx, dW2, dW1`` -- the input-gradient all-reduce, on which the next layer's whole backward waits,
    then overlaps BOTH weight-gradient GEMMs.  Without ``dx`` (layer 0) the order is ``da, dW1, dW2`` (the
    engine's flat layout follows the completion order).

    ``pair_wgrads`` (small tile grids, e.g. the MP / TP8 shard): ``da, dx, (dW2 | dW1)`` -- both weight gradients
    in ONE grouped launch (``ops.gemm.gemm_pair``) that fills the chip with whole tiles instead of two split-K GEMMs
    and their reduction passes; dx still runs before W1's fused update, and a TP all-reduce of dx overlaps the pair.

    ``nn`` (``NNWgrad``): the weight gradients in the NN layout; dx's epilogue also writes dxᵀ into ``nn.dx_t``.
    ``w2t``: ``w2`` is the stored W2ᵀ [F, D]: the dgrad runs NT and dW2 goes through the transposed output map.
    """
    w2_layout = "nt" if w2t else "nn"                                  # w2t: w2 is the stored W2ᵀ [F, D]
    if gated:
        gemm(dy, w2, w2_layout, out=da_buf, epi="dglu", act=act, aux=h)   # [dg|du] interleaved [T, 2F]
    else:
        gemm(dy, w2, w2_layout, out=da_buf, epi="dact", act=act, aux=h if h is not None else a, mask=mask)
    kw1 = gw1 if isinstance(gw1, dict) else {"out": gw1}
    kw2 = gw2 if isinstance(gw2, dict) else {"out": gw2}
    if pair_wgrads:
        assert not w2t, "grouped weight-gradient pairs keep W2 row-major"
        dx = None
        if dx_out is not None:
            dx = gemm(da_buf, w1, "nn", out=dx_out)                   # dx = da·W1 (before W1's update)
            if hooks is not None:
                hooks.after_dx(dx)
        gemm_pair(dy, a, kw2, da_buf, x, kw1)                          # dW2 = dyᵀ·a  |  dW1 = daᵀ·x
        if hooks is not None:
            if dx_out is None:   # layer 0's completion order (flat layout): W1 first
                hooks.after_w1()
                hooks.after_w2()
            else:
                hooks.after_w2()
                hooks.after_w1()
        return dx
    dx_t = nn.dx_t if nn is not None else None
    if dx_out is None:
        # no input gradient (layer 0): dW1 first, so W1's gradient collective / update starts while dW2
        # runs and the next forward's first GEMM (which needs W1) is not behind the step's last collective
        wgrad_w1(da_buf, x, kw1, nn)                                  # dW1 = daᵀ·x        [F, D]
        if hooks is not None:
            hooks.after_w1()
        wgrad_w2(dy, a, kw2, nn, w2t)                                 # dW2 = dyᵀ·a        [D, F]
        if hooks is not None:
            hooks.after_w2()
        return None
    if dx_first:
        dx = gemm(da_buf, w1, "nn", out=dx_out, aux_t=dx_t)           # dx = da·W1         [T, D]
        if hooks is not None:
            hooks.after_dx(dx)
    wgrad_w2(dy, a, kw2, nn, w2t)                                     # dW2 = dyᵀ·a        [D, F]
    if hooks is not None:
        hooks.after_w2()
    if not dx_first:
        dx = gemm(da_buf, w1, "nn", out=dx_out, aux_t=dx_t)           # dx = da·W1         [T, D]
        if hooks is not None:
            hooks.after_dx(dx)
    wgrad_w1(da_buf, x, kw1, nn)                                      # dW1 = daᵀ·x        [F, D]
    if hooks is not None:
        hooks.after_w1()
    return dx


# ------------------------------------------------------------------------------------------------------------------
# Transposed-activation layer (tensor-parallel shards whose F/tp is a multiple of 224 that 224-row tiles cover better
# than 256-row ones, e.g. the MP config's F = 14336 over 8 GPUs: 1792 = 8 x 224 = 7 x 256 rows).  The activations are kept as aᵀ / hᵀ / daᵀ [F, T] and W2 as W2ᵀ [F, D],
# so in every GEMM whose output has an F dimension that dimension is M, which the 224-row tiles cover exactly
# (F/tp = 8 x 224): h, da -> 8 x 32 = 256 tiles, dW2ᵀ | dW1 -> 128 + 128 tiles in one grouped launch, i.e. the
# whole chip with no split-K and no idle CU.  The math is the reference layer's (train_ffns.py:54-70, K1-K8) with
# every [T, F] operand transposed; only NT / NN / TN layouts occur:
#   hᵀ  = W1·xᵀ           NT  [F, T]   + act epilogue (ReLU bitmask)
#   y   = (aᵀ)ᵀ·W2ᵀ        TN  [T, D]
#   daᵀ = W2ᵀ·dyᵀ ⊙ act'   NT  [F, T]   + act' epilogue (bitmask)
#   dx  = (daᵀ)ᵀ·W1        TN  [T, D]
#   dW2ᵀ = aᵀ·dy | dW1 = daᵀ·x   NN [F, D] (+ fused optimizer), one grouped launch
# ------------------------------------------------------------------------------------------------------------------
def layer_fwd_t(x: torch.Tensor, w1: torch.Tensor, w2t: torch.Tensor, act: str, aT: torch.Tensor,
                hT: torch.Tensor | None, y_out: torch.Tensor, before_fwd2=None,
                mask: torch.Tensor | None = None) -> torch.Tensor:
    """Transposed-activation forward: ``aT = act(W1·xᵀ)`` [F, T], ``y = aTᵀ·W2ᵀ`` [T, D] (``w2t`` = W2ᵀ [F, D])."""
    gemm(w1, x, "nt", out=aT, epi="act", act=act, aux_out=hT, mask=mask)
    if before_fwd2 is not None:
        before_fwd2()
    gemm(aT, w2t, "tn", out=y_out)
    return y_out


def layer_bwd_t(dy: torch.Tensor, x: torch.Tensor, w1: torch.Tensor, w2t: torch.Tensor, act: str, aT: torch.Tensor,
                hT: torch.Tensor | None, gw1, gw2, daT: torch.Tensor, dx_out: torch.Tensor | None, hooks=None,
                mask: torch.Tensor | None = None) -> torch.Tensor | None:
    """Transposed-activation backward (order ``da, dx, dW2 | dW1``: dx reads W1 before its fused update, a TP
    all-reduce of dx overlaps the grouped weight-gradient launch).  ``gw2`` targets W2ᵀ [F, D]."""
    gemm(w2t, dy, "nt", out=daT, epi="dact", act=act, aux=hT if hT is not None else aT, mask=mask)
    dx = None
    if dx_out is not None:
        dx = gemm(daT, w1, "tn", out=dx_out)                           # dx = da·W1        [T, D]
        if hooks is not None:
            hooks.after_dx(dx)
    kw1 = gw1 if isinstance(gw1, dict) else {"out": gw1}
    kw2 = gw2 if isinstance(gw2, dict) else {"out": gw2}
    gemm_pair(aT, dy, kw2, daT, x, kw1, layout="nn")                   # dW2ᵀ = aᵀ·dy | dW1 = daᵀ·x   [F, D]
    if hooks is not None:
        if dx_out is None:   # layer 0's completion order (flat layout): W1 first
            hooks.after_w1()
            hooks.after_w2()
        else:
            hooks.after_w2()
            hooks.after_w1()
    return dx


def recompute_fwd1(x: torch.Tensor, w1: torch.Tensor, act: str, gated: bool, a_out: torch.Tensor,
                   h_out: torch.Tensor | None, mask: torch.Tensor | None = None) -> None:
    """Reference-style activation recompute (train_ffns.py:63,66) for ``recompute='full'``."""
    if gated:
        gemm(x, w1, "nt", out=a_out, epi="glu", act=act, aux_out=h_out)
    else:
        gemm(x, w1, "nt", out=a_out, epi="act", act=act, aux_out=h_out, mask=mask)
