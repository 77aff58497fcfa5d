"""GEMM op with fused FFN epilogues.

``gemm(a, b, layout, ...)`` computes, with fp32 accumulation,

* ``"nt"``: ``C[M,N] = A[M,K] · B[N,K]ᵀ``   (linear forward, reference ``linear_fwd`` train_ffns.py:41-42)
* ``"nn"``: ``C[M,N] = A[M,K] · B[K,N]``    (input gradient, ``einsum('bc,cd->bd')`` train_ffns.py:45)
* ``"tn"``: ``C[M,N] = A[K,M]ᵀ · B[K,N]``   (weight gradient, ``einsum('bc,bd->cd')`` train_ffns.py:45)

followed by an epilogue:

* ``"store"``: ``C = alpha·acc + beta·C``
* ``"act"``:   ``C = act(acc)``; ``aux_out = acc`` if given (pre-activation kept for the backward)
* ``"dact"``:  ``C = acc · act'(aux)``  (``aux`` = pre-activation; for ReLU the activation itself works)
* ``"glu"``:   gated forward on a 16-row-interleaved [W1|W3] weight; ``C = act(g)·u`` (N/2 columns),
  ``aux_out`` = interleaved pre-activations
* ``"dglu"``:  gated backward; ``acc`` = ``da`` (N columns), ``aux`` = interleaved [g|u], ``C`` = interleaved
  [dg|du] (2N columns)
* ``"sgd"``:   weight-gradient GEMM fused with the optimizer: ``C`` is the fp32 master weight, updated in place
  ``C += -lr·alpha·acc`` (reference ``param.add_(-LR*grad)``), ``aux_out`` = its bf16 working copy
* ``"adam"``:  same with fused AdamW; ``opt_m``/``opt_v`` share ``C``'s layout
* ``"sgd_split"``: ``"sgd"`` on a split master (``ops/master.py``): ``C`` is the int16 residual plane, ``aux_out``
  (required) the bf16 working copy; together they hold the fp32 master, updated exactly as ``"sgd"`` updates it
* ``"adam_split"``: ``"adam"`` on a split master (fp32 moments ``opt_m``/``opt_v`` in ``C``'s layout)

Transposed outputs (the NN weight-gradient layout, ``ffn.layer_bwd(..., wgrad_nn=...)``; 256x256 8-phase tiles):

* ``out_t=True`` (``"store"`` in any layout, ``"sgd_split"`` / ``"adam_split"`` in ``"nn"`` / ``"tn"``; any epilogue on
  the CPU reference): ``out`` (and ``aux_out``,
  the moments) hold ``Cᵀ``
  [N, M] -- e.g.
  ``dW1ᵀ = xᵀ·da`` written into (or updating) ``W1`` [F, D] while ``xᵀ`` is the K-contiguous A operand
* ``aux_t=`` (``"store"``, beta 0, bf16, layouts ``"nt"`` / ``"nn"``): also writes ``Cᵀ`` [N, M] into ``aux_t`` --
  e.g. a layer's output ``y`` and its ``yᵀ``, the next layer's K-contiguous weight-gradient operand

CUDA (HIP) tensors run the hand-written gfx950 kernels of ``csrc/gemm_kernels.h``; CPU tensors run the torch
reference below (used by the CPU/gloo tests and as the numerics oracle).  There is no silent fallback:
a GPU tensor with the native library missing raises.
"""
from __future__ import annotations

import torch

from .. import _native
from ..utils import observe as _observe
from .activations import act_code, act_fwd, act_grad
from .master import join_master, set_master_

LAYOUTS = {"nt": 0, "nn": 1, "tn": 2}
EPIS = {"store": 0, "act": 1, "dact": 2, "glu": 3, "dglu": 4, "sgd": 5, "adam": 6, "sgd_split": 7, "adam_split": 8}
FORCE = {None: -1, "mfma_bf16": 0, "mfma_f32": 1, "generic": 2, "bf16x6": -1, "mfma_bf16_m224": 3}


def gemm_shape(a: torch.Tensor, b: torch.Tensor, layout: str) -> tuple[int, int, int]:
    if layout == "nt":
        (M, K), (N, K2) = a.shape, b.shape
    elif layout == "nn":
        (M, K), (K2, N) = a.shape, b.shape
    elif layout == "tn":
        (K, M), (K2, N) = a.shape, b.shape
    else:
        raise ValueError(layout)
    if K != K2:
        raise ValueError(f"gemm {layout}: inner dims differ {tuple(a.shape)} vs {tuple(b.shape)}")
    return M, N, K


def out_cols(N: int, epi: str) -> int:
    if epi == "glu":
        return N // 2
    if epi == "dglu":
        return N * 2
    return N


def _check_rowmajor(t: torch.Tensor, name: str) -> None:
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError(f"{name} must be a row-major 2-D view (stride(1)==1), got strides {t.stride()}")


def _glu_split(h: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """Split 16-column-interleaved [g|u] blocks into (g, u)."""
    M, N = h.shape
    v = h.reshape(M, N // 32, 2, 16)
    return v[:, :, 0, :].reshape(M, N // 2), v[:, :, 1, :].reshape(M, N // 2)


def _glu_merge(g: torch.Tensor, u: torch.Tensor) -> torch.Tensor:
    M, F = g.shape
    return torch.stack([g.reshape(M, F // 16, 16), u.reshape(M, F // 16, 16)], dim=2).reshape(M, 2 * F)


def _torch_gemm(a, b, layout, out, epi, act, aux, aux_out, alpha, beta, opt=None, out_t=False, aux_t=None):
    acc_dt = torch.promote_types(a.dtype, torch.float32)  # fp32 accumulation (fp64 stays fp64 for oracles)
    af, bf = a.to(acc_dt), b.to(acc_dt)
    if layout == "nt":
        acc = af @ bf.t()
    elif layout == "nn":
        acc = af @ bf
    else:
        acc = af.t() @ bf
    if out_t:
        acc = acc.t()
    if epi == "store":
        r = alpha * acc
        if beta != 0.0:
            r = r + beta * out.to(acc_dt)
        out.copy_(r)
        if aux_t is not None:
            aux_t.copy_(out.t())
    elif epi == "act":
        if aux_out is not None:
            aux_out.copy_(acc)
        out.copy_(act_fwd(act, acc))
    elif epi == "dact":
        out.copy_(acc * act_grad(act, aux.to(acc_dt)))
    elif epi == "glu":
        if aux_out is not None:
            aux_out.copy_(acc)
        g, u = _glu_split(acc)
        out.copy_(act_fwd(act, g) * u)
    elif epi == "dglu":
        g, u = _glu_split(aux.to(acc_dt))
        du = acc * act_fwd(act, g)
        dg = acc * u * act_grad(act, g)
        out.copy_(_glu_merge(dg, du))
    elif epi == "sgd":
        out.add_(-opt["lr"] * (alpha * acc).to(out.dtype))
        if aux_out is not None:
            aux_out.copy_(out)
    elif epi == "sgd_split":
        w = join_master(aux_out, out)
        w.add_(-opt["lr"] * (alpha * acc).to(torch.float32))
        set_master_(aux_out, out, w)
    elif epi == "adam_split":
        w = join_master(aux_out, out)
        _torch_gemm(a, b, layout, w, "adam", act, aux, None, alpha, beta, opt)
        set_master_(aux_out, out, w)
        return out
    elif epi == "adam":
        g = (alpha * acc).to(out.dtype)
        b1, b2, step = opt["b1"], opt["b2"], opt["step"]
        m, v = opt["m"], opt["v"]
        m.mul_(b1).add_((1 - b1) * g)
        v.mul_(b2).add_((1 - b2) * g * g)
        upd = (m / (1 - b1 ** step)) / (torch.sqrt(v / (1 - b2 ** step)) + opt["eps"]) + opt["wd"] * out
        out.sub_(opt["lr"] * upd)
        if aux_out is not None:
            aux_out.copy_(out)
    return out


# fp32 GEMMs on the GPU: "bf16x6" (default) runs the exact three-way bf16 split on the bf16 MFMA kernels
# (fp32 accuracy, ~1.7x the fp32 MFMA rate); "mfma_f32" runs the fp32 MFMA kernel (v_mfma_f32_16x16x4_f32)
_FP32 = {"mode": "bf16x6"}
FP32_MODES = ("bf16x6", "mfma_f32")
# split operands, cached per (device, stream, operand): a GEMM only reuses its own stream's buffers
_SPLIT_WS: dict = {}


def set_fp32_mode(mode: str) -> str:
    """Select how fp32 GEMMs run on the GPU (``FP32_MODES``); returns the previous mode."""
    if mode not in FP32_MODES:
        raise ValueError(f"unknown fp32 GEMM mode {mode!r}")
    old = _FP32["mode"]
    _FP32["mode"] = mode
    return old


def bf16x6_supported(M: int, N: int, K: int) -> bool:
    """Shapes the split fp32 GEMM takes: 256x256 output tiles and K' = 6K a multiple of the 128-deep K step."""
    return M % 256 == 0 and N % 256 == 0 and K % 64 == 0


def _use_bf16x6(M: int, N: int, K: int, force) -> bool:
    if force == "bf16x6":
        if not bf16x6_supported(M, N, K):
            raise ValueError(f"bf16x6 fp32 GEMM needs M, N % 256 == 0 and K % 64 == 0, got {(M, N, K)}")
        return True
    return force is None and _FP32["mode"] == "bf16x6" and bf16x6_supported(M, N, K)


def split3(x: torch.Tensor, role: int, rows_form: bool) -> torch.Tensor:
    """Three-way bf16 split of an fp32 operand, six planes along its K dimension (``role`` 0 = A, 1 = B).

    ``rows_form`` False: ``x`` is ``[R, K]`` -> ``[R, 6K]``; True: ``x`` is ``[K, C]`` -> ``[6K, C]``.  The planes
    carry (a0, a1, a2, a0, a1, a0) for A and (b2, b1, b0, b1, b0, b0) for B, so a bf16 GEMM over the 6K axis sums
    the six partial products a_i b_j with i + j <= 2."""
    R, C = x.shape
    n = 6 * R * C
    key = (x.device.index, torch.cuda.current_stream(x.device).cuda_stream, role)
    ws = _SPLIT_WS.get(key)
    if ws is None or ws.numel() < n:
        ws = torch.empty(n, dtype=torch.bfloat16, device=x.device)
        _SPLIT_WS[key] = ws
    out = ws[:n].view(6 * R, C) if rows_form else ws[:n].view(R, 6 * C)
    _native.check(_native.lib().dllm_split3(x.data_ptr(), x.stride(0), R, C, out.data_ptr(), role, int(rows_form),
                                            _native.stream_ptr(x.device)), "dllm_split3")
    return out


NUM_CUS = 256   # MI355X; the device's own count is used when a GPU is present (num_cus)
_NCU: list = []


def num_cus() -> int:
    """Compute units of the current GPU (the native side's tile-grid decisions use the same count, csrc/gemm.hip
    use_m224 -> num_cu()); 256 (MI355X) without a GPU, e.g. in CPU tests."""
    if not _NCU:
        n = NUM_CUS
        if torch.cuda.is_available():
            n = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
        _NCU.append(int(n))
    return _NCU[0]


_SPLITK = {"enabled": True}


def choose_ksplit(M: int, N: int, K: int) -> int:
    """Split-K factor for the 256x256 bf16 kernel: raise CU occupancy when the tile grid is small.

    One block per CU (128 KiB LDS), 256 CUs: pick the factor s (K-tiles per slice even, >= 8) that
    maximises tiles*s / (waves*256), and only when it beats s = 1 by >= 25 % (the partials cost one
    fp32 round trip through HBM)."""
    if not _SPLITK["enabled"] or M % 256 or N % 256 or K % 128:
        return 1
    pp = _VARIANT["name"] == "pp"   # 256x128 tiles, two resident blocks per CU
    tiles = (M // 256) * (N // (128 if pp else 256))
    slots = num_cus() * (2 if pp else 1)
    if tiles >= slots * 0.75:
        return 1

    def util(s):
        blocks = tiles * s
        return blocks / (-(-blocks // slots) * slots)

    best, best_u = 1, util(1)
    for s in (2, 3, 4, 6, 8):
        nkt = K // 64
        if nkt % (2 * s) or nkt // s < 8:
            continue
        u = util(s)
        if u > best_u * 1.25:
            best, best_u = s, u
    return best


def set_splitk(enabled: bool) -> bool:
    old = _SPLITK["enabled"]
    _SPLITK["enabled"] = enabled
    return old


_VARIANT = {"name": "auto"}
# Launch policy of the 256x256 bf16 kernels (tiles per persistent block, minimum blocks per CU): Python-level
# defaults that every call passes to the library explicitly -- the native side keeps no mutable state, so
# GEMMs issued concurrently on different streams never race on a setting.
# group_m_nt: tiles per raster band of the NT (forward) GEMMs.  8 is 1-1.3 % faster on the standalone forward shapes
# (profiles/r3/group_m_sweep_r3.txt) but not in the step (30.15-30.37 vs 30.17-30.26 ms, interleaved,
# profiles/r3/group_m_nt_step_r3.txt), so every layout keeps 4
# group_m_nn: 8 -- the NN-layout GEMMs of the finite-data step (NN stores with transposed copies, transposed-map weight
# gradients) ran 34.13-34.18 ms against 34.26-34.35 at 4 and 34.97-35.01 at 16 (5 interleaved pairs,
# profiles/r5/group_m_nn_finite_r5.txt)
_POLICY = {"tpb": 8, "min_bpc": 1, "group_m_nt": 4, "group_m_nn": 8, "group_m_tn": 4}  # tpb: the cap; the library picks the makespan-optimal tiles per block
# split-K fp32 partial workspaces, cached per (device, stream): a GEMM only ever reuses its own stream's
# buffer, so stream order serialises the reuse
_WS: dict = {}


def _splitk_workspace(numel: int, device: torch.device) -> torch.Tensor:
    key = (device.index, torch.cuda.current_stream(device).cuda_stream)
    ws = _WS.get(key)
    if ws is None or ws.numel() < numel:
        ws = torch.empty(numel, dtype=torch.float32, device=device)
        _WS[key] = ws
    return ws


def gemm(a: torch.Tensor, b: torch.Tensor, layout: str, out: torch.Tensor | None = None, *, epi: str = "store",
         act: str = "none", aux: torch.Tensor | None = None, aux_out: torch.Tensor | None = None,
         alpha: float = 1.0, beta: float = 0.0, out_dtype: torch.dtype | None = None, group_m: int | None = None,
         force: str | None = None, lr: float = 0.0, betas: tuple = (0.9, 0.95), eps: float = 1e-8,
         wd: float = 0.0, step: int = 0, opt_m: torch.Tensor | None = None,
         opt_v: torch.Tensor | None = None, mask: torch.Tensor | None = None, out_t: bool = False,
         aux_t: torch.Tensor | None = None) -> torch.Tensor:
    """``mask`` (ReLU only, GPU, see ``relu_mask_supported``): ``epi="act"`` also writes the activation-gradient
    bitmask, ``epi="dact"`` reads it instead of ``aux`` (1 bit instead of a bf16 per element).  CPU tensors
    ignore it (``aux`` stays the source of truth there).  ``out_t`` / ``aux_t``: transposed outputs (module doc)."""
    M, N, K = gemm_shape(a, b, layout)
    if out_t or aux_t is not None:
        _check_transposed(a, layout, epi, M, N, K, out_t, aux_t, beta)
    if group_m is None:   # raster band height: the layout's policy (profiles/r3/group_m_sweep_r3.txt)
        group_m = _POLICY["group_m_nt"] if layout == "nt" else _POLICY["group_m_nn"] if layout == "nn" else \
            _POLICY["group_m_tn"]
    if a.dtype != b.dtype:
        raise TypeError(f"gemm operands differ in dtype: {a.dtype} vs {b.dtype}")
    nout = out_cols(N, epi)
    oshape = (nout, M) if out_t else (M, nout)
    if out is None:
        out = torch.empty(oshape, dtype=out_dtype or a.dtype, device=a.device)
    if out.shape != oshape:
        raise ValueError(f"out has shape {tuple(out.shape)}, expected {oshape}")
    if epi in ("dact", "dglu") and aux is None:
        raise ValueError(f"epilogue {epi} needs aux (pre-activation)")
    if epi == "glu" and N % 32:
        raise ValueError("gated GEMM needs N % 32 == 0 (16-row interleave)")
    if epi in ("act", "dact", "glu", "dglu") and a.device.type == "cuda" and (layout == "tn" or act == "none"):
        # the native library has activation kernels per activation, in the NT / NN layouts only
        raise ValueError(f"epilogue {epi} on the GPU: relu / silu / gelu in the NT / NN layouts (got {act}, {layout})")
    # fused optimizers: the weight-gradient layouts -- TN, NN on 224-row tiles (transposed-activation TP layout), or
    # the NN weight-gradient layout's 256x256 tiles (split masters)
    opt_layout_ok = layout == "tn" or (layout == "nn" and a.device.type == "cuda" and (
        use_m224(M, N) or (epi in ("sgd_split", "adam_split") and nn_wgrad_supported(M, N, K))))
    if epi in ("sgd", "adam"):
        if not (opt_layout_ok or (layout == "nn" and a.device.type != "cuda")) or out.dtype != torch.float32:
            raise ValueError("fused-optimizer epilogues need the TN (weight-gradient) layout and an fp32 master")
        if epi == "adam" and (opt_m is None or opt_v is None or step < 1):
            raise ValueError("adam epilogue needs opt_m, opt_v and step >= 1")
        for t in (opt_m, opt_v):
            if t is not None and (t.shape != out.shape or t.stride() != out.stride()):
                raise ValueError("optimizer moments must share the master weight's layout")
    if epi in ("sgd_split", "adam_split"):
        if epi == "adam_split" and (opt_m is None or opt_v is None or step < 1):
            raise ValueError("adam_split epilogue needs opt_m, opt_v and step >= 1")
        if not (opt_layout_ok or (layout == "nn" and a.device.type != "cuda")) or out.dtype != torch.int16 \
                or aux_out is None or aux_out.dtype != torch.bfloat16 \
                or aux_out.shape != out.shape or a.dtype != torch.bfloat16:
            raise ValueError(f"{epi} needs the TN layout, bf16 operands, an int16 residual plane as out and its "
                             "bf16 working copy as aux_out")
    if a.device.type != "cuda":
        opt = {"lr": lr, "b1": betas[0], "b2": betas[1], "eps": eps, "wd": wd, "step": step, "m": opt_m, "v": opt_v}
        return _torch_gemm(a, b, layout, out, epi, act, aux, aux_out, alpha, beta, opt, out_t, aux_t)

    for t, nm in ((a, "a"), (b, "b"), (out, "out")):
        _check_rowmajor(t, nm)
    if (a.dtype == torch.float32 and mask is None and _use_bf16x6(M, N, K, force)
            and all(t.data_ptr() % 16 == 0 and t.stride(0) % 4 == 0 for t in (a, b))):
        # fp32-accurate GEMM on the bf16 matrix cores: split both operands into three bf16 parts and run one
        # bf16 GEMM over K' = 6K with the same fused epilogue (see split3 / csrc/elementwise.hip split3_kernel)
        a6 = split3(a, 0, layout == "tn")
        b6 = split3(b, 1, layout != "nt")
        return gemm(a6, b6, layout, out, epi=epi, act=act, aux=aux, aux_out=aux_out, alpha=alpha, beta=beta,
                    group_m=group_m, lr=lr, betas=betas, eps=eps, wd=wd, step=step, opt_m=opt_m, opt_v=opt_v)
    code = EPIS[epi]
    if out_t:
        code = EPI_T[epi]
    elif aux_t is not None:
        code, aux_out = EPI_STORE_DT, aux_t
    auxt = aux if aux is not None else aux_out
    if aux_t is not None:
        _check_rowmajor(aux_t, "aux_t")
        if aux_t.dtype != out.dtype or aux_t.shape != (N, M):
            raise ValueError(f"aux_t must be the [N, M] = {(N, M)} transposed output in the output dtype")
    elif auxt is not None:
        _check_rowmajor(auxt, "aux")
        if epi in ("sgd", "adam", "sgd_split", "adam_split"):
            if auxt.dtype != torch.bfloat16 or auxt.shape != out.shape:
                raise TypeError("fused-optimizer aux_out must be the bf16 copy of the master weight")
        elif auxt.dtype != out.dtype:
            raise TypeError("aux / aux_out must have the output dtype")
    L = _native.lib()
    in_dt = _native.dtype_code(a.dtype)
    out_dt = _native.dtype_code(torch.bfloat16 if out.dtype == torch.int16 else out.dtype)  # 16-bit planes
    ksplit, ws = 1, None
    if a.dtype == torch.bfloat16 and force in (None, "mfma_bf16") and code == EPIS[epi]:
        ksplit = choose_ksplit(M, N, K)
        if ksplit > 1 and L.dllm_gemm_path(in_dt, out_dt, M, N, K, a.stride(0), b.stride(0), out.stride(0)) == 0:
            ws = _splitk_workspace(ksplit * M * N, a.device)
        else:
            ksplit = 1
    obs = _observe.active()
    if obs is not None:
        obs.gemm_begin()
    rc = L.dllm_gemm(in_dt, out_dt, LAYOUTS[layout], code, act_code(act),
                     a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), out.data_ptr(), out.stride(0),
                     aux.data_ptr() if aux is not None else None,
                     aux_out.data_ptr() if aux_out is not None else None,
                     auxt.stride(0) if auxt is not None else 0,
                     M, N, K, float(alpha), float(beta), int(group_m), FORCE[force],
                     _native.stream_ptr(a.device), float(lr), float(betas[0]), float(betas[1]), float(eps),
                     float(wd), int(step), opt_m.data_ptr() if opt_m is not None else None,
                     opt_v.data_ptr() if opt_v is not None else None, ksplit,
                     ws.data_ptr() if ws is not None else None,
                     _mask_ptr(mask, M, N) if mask is not None else None,
                     BF16_VARIANTS[_VARIANT["name"]], _POLICY["tpb"], _POLICY["min_bpc"])
    _native.check(rc, f"dllm_gemm({layout},{epi},M={M},N={N},K={K})")
    if obs is not None:
        obs.gemm_end()
    return out


EPI_T = {"store": 10, "sgd_split": 9, "adam_split": 12}     # csrc/common.h EPI_STORE_T / EPI_SGDS_T / EPI_ADAMS_T
EPI_STORE_DT = 11


def nn_wgrad_supported(M: int, N: int, K: int) -> bool:
    """Shapes of the NN weight-gradient layout's kernels (transposed outputs / copies, NN fused SGD): 256x256 output
    tiles on the 8-phase kernel (K a multiple of its 128-deep step) and not the 224-row family."""
    return M % 256 == 0 and N % 256 == 0 and K % 128 == 0 and not use_m224(M, N)


def _check_transposed(a, layout, epi, M, N, K, out_t, aux_t, beta) -> None:
    if out_t and aux_t is not None:
        raise ValueError("out_t and aux_t are exclusive")
    if out_t and a.device.type == "cuda" and (epi not in EPI_T or (epi != "store" and layout == "nt")):
        raise ValueError(f"out_t: 'store' (any layout) or the split-master optimizers (NN / TN) only (got {epi}, {layout})")
    if aux_t is not None and (epi != "store" or layout not in ("nt", "nn")):
        raise ValueError(f"aux_t: the store epilogue in the NT / NN layouts only (got {epi}, {layout})")
    if beta != 0.0:
        raise ValueError("transposed outputs: beta must be 0")
    if a.device.type == "cuda" and (a.dtype != torch.bfloat16 or not nn_wgrad_supported(M, N, K)):
        raise ValueError(f"transposed outputs need bf16 operands on 256x256 tiles with K % 128 == 0, got {(M, N, K)}")


def transpose_bf16(src: torch.Tensor, dst: torch.Tensor) -> torch.Tensor:
    """``dst = srcᵀ`` for bf16 row-major views (rows and columns multiples of 64 on the GPU kernel)."""
    R, C = src.shape
    if dst.shape != (C, R) or src.dtype != dst.dtype:
        raise ValueError(f"transpose: dst {tuple(dst.shape)} / {dst.dtype} for src {tuple(src.shape)} / {src.dtype}")
    if src.device.type != "cuda":
        dst.copy_(src.t())
        return dst
    _check_rowmajor(src, "src")
    _check_rowmajor(dst, "dst")
    _native.check(_native.lib().dllm_transpose_bf16(src.data_ptr(), src.stride(0), dst.data_ptr(), dst.stride(0), R, C,
                                                    _native.stream_ptr(src.device)), "dllm_transpose_bf16")
    return dst


_PAIR = {"enabled": True}


def set_pair_wgrads(enabled: bool) -> bool:
    """Allow grouped weight-gradient pairs (``gemm_pair``); returns the previous setting."""
    old = _PAIR["enabled"]
    _PAIR["enabled"] = bool(enabled)
    return old


def use_m224(M: int, N: int) -> bool:
    """Whether an ``[M, N]`` bf16 GEMM output (K-contiguous A: NT / NN) runs on 224-row tiles: M = 224k and the 224-row
    grid fills the CUs strictly better than the 256-row one -- e.g. the MP / TP8 shard's F/8 = 1792 rows against
    T = 8192: 8 x 32 = 256 tiles instead of 7 x 32 = 224 (mirrors csrc/gemm.hip use_m224)."""
    if M % 224 or N % 256:
        return False
    if M % 256:
        return True

    def fill(bm):
        t = (M // bm) * (N // 256)
        ncu = num_cus()
        return t / (-(-t // ncu) * ncu)

    return fill(224) > fill(256)


def tile_rows(M: int, N: int) -> int:
    """Output-tile rows the bf16 MFMA kernels use for an ``[M, N]`` output with a K-contiguous A (224 or 256)."""
    return 224 if use_m224(M, N) else 256


def pair_supported(shapes, dtype: torch.dtype = torch.bfloat16, layout: str = "tn") -> bool:
    """Whether two weight-gradient GEMMs ``shapes = ((M0, N0, K), (M1, N1, K))`` run as one grouped launch: bf16, the
    8-phase K step, both tile grids together <= the CUs, and each alone too small to fill the chip.  ``"tn"``: 256-row
    tiles, each GEMM would otherwise run split-K (a part-empty chip plus a reduction pass) -- e.g. the MP (TP8) shard's
    dW2 [4096, 1792] and dW1 [1792, 4096].  ``"nn"``: 224-row tiles (the transposed-activation TP layout's dW2ᵀ and dW1,
    both [1792, 4096]: 128 + 128 tiles, exactly the 256 CUs)."""
    (M0, N0, K0), (M1, N1, K1) = shapes
    if not _PAIR["enabled"] or dtype != torch.bfloat16 or K0 != K1 or K0 % 128:
        return False
    if _VARIANT["name"] not in ("auto", "8phase_stagger"):
        return False
    if layout == "nn":
        if not (use_m224(M0, N0) and use_m224(M1, N1)):
            return False
        return (M0 // 224) * (N0 // 256) + (M1 // 224) * (N1 // 256) <= num_cus()
    if any(m % 256 or n % 256 for m, n in ((M0, N0), (M1, N1))):
        return False
    tiles = (M0 // 256) * (N0 // 256) + (M1 // 256) * (N1 // 256)
    return tiles <= num_cus() and (choose_ksplit(M0, N0, K0) > 1 or choose_ksplit(M1, N1, K1) > 1)


def gemm_pair(a0: torch.Tensor, b0: torch.Tensor, kw0: dict, a1: torch.Tensor, b1: torch.Tensor, kw1: dict,
              layout: str = "tn") -> None:
    """Two weight-gradient GEMMs ``gemm(a0, b0, layout, **kw0)`` and ``gemm(a1, b1, layout, **kw1)`` -- same epilogue
    and K -- as ONE grouped launch with one tile per block (``csrc/gemm_kernels.h`` ``gemm_bf16_8ph_pair``; ``"tn"``
    on 256x256 tiles, ``"nn"`` on 224x256 tiles).  Each result is bitwise the single unsplit GEMM's.  Falls back to two
    ``gemm`` calls where the grouped kernel does not apply (CPU tensors, shapes, alignment)."""
    M0, N0, K0 = gemm_shape(a0, b0, layout)
    M1, N1, K1 = gemm_shape(a1, b1, layout)
    epi = kw0.get("epi", "store")
    if a0.device.type != "cuda" or kw1.get("epi", "store") != epi or not pair_supported(((M0, N0, K0), (M1, N1, K1)),
                                                                                         a0.dtype, layout):
        gemm(a0, b0, layout, **kw0)
        gemm(a1, b1, layout, **kw1)
        return
    for kw in (kw0, kw1):
        bad = set(kw) - {"out", "epi", "lr", "aux_out", "betas", "eps", "wd", "step", "opt_m", "opt_v", "alpha"}
        if bad or kw.get("out") is None:
            raise ValueError(f"gemm_pair: unsupported arguments {sorted(bad) or ['out missing']}")
        for k in ("lr", "betas", "eps", "wd", "step", "alpha"):
            if kw.get(k) != kw0.get(k):
                raise ValueError(f"gemm_pair: both GEMMs must share {k}")
    outs = [kw0["out"], kw1["out"]]
    for (M, N), o in zip(((M0, N0), (M1, N1)), outs):
        if o.shape != (M, N):
            raise ValueError(f"gemm_pair: out {tuple(o.shape)} != {(M, N)}")
    for t, nm in ((a0, "a0"), (b0, "b0"), (a1, "a1"), (b1, "b1"), *((o, "out") for o in outs)):
        _check_rowmajor(t, nm)
    if epi in ("sgd", "adam") and any(o.dtype != torch.float32 for o in outs):
        raise ValueError("fused-optimizer epilogues need an fp32 master")
    if epi in ("sgd_split", "adam_split") and any(o.dtype != torch.int16 or kw.get("aux_out") is None
                                                  for o, kw in zip(outs, (kw0, kw1))):
        raise ValueError(f"{epi} needs int16 residual planes and bf16 working copies")
    from ctypes import c_float, c_int, c_long, c_void_p

    def arr(ctype, vals):
        return (ctype * 2)(*vals)

    kws = (kw0, kw1)
    aux = [kw.get("aux_out") for kw in kws]
    om = [kw.get("opt_m") for kw in kws]
    ov = [kw.get("opt_v") for kw in kws]
    ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    betas = kw0.get("betas", (0.9, 0.95))
    out_dt = _native.dtype_code(torch.bfloat16 if outs[0].dtype == torch.int16 else outs[0].dtype)
    L = _native.lib()
    obs = _observe.active()
    if obs is not None:
        obs.gemm_begin()
    rc = L.dllm_gemm_pair(LAYOUTS[layout], out_dt, EPIS[epi], arr(c_void_p, [a0.data_ptr(), a1.data_ptr()]),
                          arr(c_long, [a0.stride(0), a1.stride(0)]), arr(c_void_p, [b0.data_ptr(), b1.data_ptr()]),
                          arr(c_long, [b0.stride(0), b1.stride(0)]), arr(c_void_p, [o.data_ptr() for o in outs]),
                          arr(c_long, [o.stride(0) for o in outs]), arr(c_void_p, [ptr(t) for t in aux]),
                          arr(c_long, [t.stride(0) if t is not None else 0 for t in aux]),
                          arr(c_void_p, [ptr(t) for t in om]), arr(c_void_p, [ptr(t) for t in ov]),
                          arr(c_int, [M0, M1]), arr(c_int, [N0, N1]), K0, c_float(float(kw0.get("alpha", 1.0))),
                          c_float(float(kw0.get("lr", 0.0))), c_float(float(betas[0])), c_float(float(betas[1])),
                          c_float(float(kw0.get("eps", 1e-8))), c_float(float(kw0.get("wd", 0.0))),
                          int(kw0.get("step", 0)), _native.stream_ptr(a0.device))
    if obs is not None:
        obs.gemm_end()
    if rc == -1:   # not expressible as one grouped launch (alignment, CU count): two GEMMs
        gemm(a0, b0, layout, **kw0)
        gemm(a1, b1, layout, **kw1)
        return
    _native.check(rc, f"dllm_gemm_pair({epi},{(M0, N0)},{(M1, N1)},K={K0})")


def relu_mask_bytes(M: int, N: int) -> int:
    """Size of the ReLU bitmask of an ``[M, N]`` activation (8 KiB per 256x256 or 224x256 tile)."""
    return (M // tile_rows(M, N)) * (N // 256) * 8192


def relu_mask_supported(M: int, N: int, K: int, dtype: torch.dtype = torch.bfloat16) -> bool:
    """Whether the forward (``x·W1ᵀ``, K = D) / dgrad (``dy·W2``, K = D) pair of an ``[M, N]`` ReLU activation runs
    on the 8-phase kernels that share the bitmask's tile-native layout."""
    kstep = 64 if _VARIANT["name"] == "pp" else 128
    if dtype == torch.bfloat16 and use_m224(M, N) and K % 128 == 0:
        return _VARIANT["name"] in ("auto", "8phase_stagger")   # 224-row tiles (transposed-activation TP layout)
    return (dtype == torch.bfloat16 and M % 256 == 0 and N % 256 == 0 and K % kstep == 0
            and choose_ksplit(M, N, K) == 1 and _VARIANT["name"] != "2stage")


def _mask_ptr(mask: torch.Tensor, M: int, N: int) -> int:
    if mask.dtype != torch.uint8 or not mask.is_contiguous() or mask.numel() < relu_mask_bytes(M, N):
        raise ValueError(f"ReLU mask must be a contiguous uint8 buffer of >= {relu_mask_bytes(M, N)} bytes")
    return mask.data_ptr()


# "pp": 256x128 tiles, 4 waves, 80 KiB LDS -> two blocks per CU (csrc/gemm_pp.h); the others are 256x256 main loops
BF16_VARIANTS = {"auto": 0, "2stage": 1, "8phase": 2, "8phase_stagger": 3, "4phase_stagger": 4, "pp": 5}


def set_bf16_variant(name: str) -> str:
    """Select the bf16 256x256 main loop for subsequent calls; returns the previous setting's name."""
    if name not in BF16_VARIANTS:
        raise ValueError(f"unknown bf16 GEMM variant {name!r}")
    old = _VARIANT["name"]
    _VARIANT["name"] = name
    return old


def set_tiles_per_block(n: int) -> int:
    """Persistent GEMM blocks for the FFN's own GEMMs: each block runs up to ``n`` output tiles back to back, the next
    tile's first K-tiles prefetched while the current tile's epilogue runs (no pipeline drain or block relaunch per
    tile).  ``n`` is a cap: the launcher picks the makespan-optimal tiles per block under it (never fewer blocks than
    CUs x ``min_bpc`` up to rounding); ``n <= 1``: one block per tile.  Default 8 (the engine's default for every
    stack).  Returns the previous setting."""
    old = _POLICY["tpb"]
    _POLICY["tpb"] = max(1, int(n))
    return old


def set_group_m_nt(n: int) -> int:
    """Tiles per raster band (L2 panel sharing) of the NT-layout GEMMs; returns the previous setting."""
    old = _POLICY["group_m_nt"]
    _POLICY["group_m_nt"] = max(1, int(n))
    return old


def set_group_m_nn(n: int) -> int:
    """Tiles per raster band of the NN-layout GEMMs (dgrad / NN weight gradients / NN stores); returns the previous."""
    old = _POLICY["group_m_nn"]
    _POLICY["group_m_nn"] = max(1, int(n))
    return old


def set_group_m_tn(n: int) -> int:
    """Tiles per raster band of the TN-layout GEMMs (weight gradients, the TP shard's forward); returns the previous."""
    old = _POLICY["group_m_tn"]
    _POLICY["group_m_tn"] = max(1, int(n))
    return old


def set_min_blocks_per_cu(n: int) -> int:
    """Minimum blocks per CU of a persistent GEMM grid (default 1).  The engine sets 2 when collectives run
    concurrently with the GEMMs, so a CU held by an RCCL kernel delays one of several blocks per CU rather than
    the only one.  Returns the previous setting."""
    old = _POLICY["min_bpc"]
    _POLICY["min_bpc"] = max(1, int(n))
    return old


def gemm_path(a_dtype: torch.dtype, out_dtype: torch.dtype, M: int, N: int, K: int,
              lda: int, ldb: int, ldc: int) -> str:
    """Which native kernel family a call would use: 'mfma_bf16', 'mfma_f32' or 'generic'."""
    p = _native.lib().dllm_gemm_path(_native.dtype_code(a_dtype), _native.dtype_code(out_dtype), M, N, K,
                                     lda, ldb, ldc)
    return {0: "mfma_bf16", 1: "mfma_f32", 2: "generic", 3: "mfma_bf16_m224"}[p]
