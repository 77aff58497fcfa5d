"""Device RNG, fused optimizer steps and casts (native on HIP tensors, torch reference on CPU)."""
from __future__ import annotations

import math

import torch

from .. import _native

# Philox stream separation for the mock data of one step (x and dloss_dx, train_ffns.py:149-150)
STREAM_X, STREAM_DY = 0, 1


def rng_normal_t_supported(out: torch.Tensor) -> bool:
    """Whether ``rng_normal_(out, ..., out_t=...)`` runs the one-pass draw + transpose kernel on ``out``."""
    return (out.device.type == "cuda" and out.dtype == torch.bfloat16 and out.dim() == 2 and out.is_contiguous()
            and out.shape[0] % 64 == 0 and out.shape[1] % 64 == 0 and out.shape[0] // 64 <= 65535)


def rng_normal_(out: torch.Tensor, seed: int, stream_id: int = 0, scale: float = 1.0,
                out_t: torch.Tensor | None = None) -> torch.Tensor:
    """Fill ``out`` with ``scale·N(0,1)``, deterministic in (seed, stream_id, numel) on any device.

    GPU: Philox4x32-10 kernel.  CPU: the same Philox stream computed in torch (bitwise-identical
    uniform draws; normals equal up to libm differences), so CPU tests and GPU runs see the same data.
    fp32 outputs take 32-bit uniforms (4 normals per Philox call); bf16 outputs, which keep 8 mantissa bits, take
    16-bit uniforms (8 normals per call, csrc/elementwise.hip ``rng_normal_bf16_kernel``).
    ``out_t`` ([C, R] for a 2-D ``out`` [R, C]): also write the transpose -- on the GPU in the same pass
    (``rng_normal_bf16_t_kernel``, bitwise the draw + ``transpose_bf16``) where ``rng_normal_t_supported(out)``.
    """
    if not out.is_contiguous():
        raise ValueError("rng_normal_ needs a contiguous tensor")
    n = out.numel()
    if out_t is not None:
        if out.dim() != 2 or tuple(out_t.shape) != (out.shape[1], out.shape[0]) or out_t.dtype != out.dtype:
            raise ValueError(f"out_t must be [{out.shape[-1]}, {out.shape[0]}] {out.dtype}")
        if rng_normal_t_supported(out) and out_t.is_contiguous():
            rc = _native.lib().dllm_rng_normal_bf16_t(out.data_ptr(), out_t.data_ptr(), out.shape[0], out.shape[1],
                                                      seed & (2**64 - 1), None, stream_id & (2**64 - 1),
                                                      float(scale), _native.stream_ptr(out.device))
            _native.check(rc, "dllm_rng_normal_bf16_t")
            return out
        rng_normal_(out, seed, stream_id, scale)
        out_t.copy_(out.t())
        return out
    if out.device.type == "cuda":
        rc = _native.lib().dllm_rng_normal(out.data_ptr(), _native.dtype_code(out.dtype), n, seed & (2**64 - 1),
                                           stream_id & (2**64 - 1), float(scale), _native.stream_ptr(out.device))
        _native.check(rc, "dllm_rng_normal")
        return out
    out.copy_(_philox_normal_cpu(n, seed, stream_id, scale, u16=out.dtype == torch.bfloat16).view(out.shape))
    return out


def _pair_ok(a: torch.Tensor, b: torch.Tensor) -> bool:
    return (a.device.type == "cuda" and a.dtype == b.dtype == torch.bfloat16 and a.numel() == b.numel() and
            a.is_contiguous() and b.is_contiguous() and a.device == b.device and a.numel() // 8 < 2**31)


def rng_normal_pair_(a: torch.Tensor, b: torch.Tensor, seed: int, stream_a: int, scale_a: float, stream_b: int,
                     scale_b: float, seed_dev: torch.Tensor | None = None) -> None:
    """``rng_normal_(a, seed, stream_a, scale_a)`` and ``rng_normal_(b, seed, stream_b, scale_b)`` -- on the GPU for two
    contiguous bf16 tensors of one size in a single launch (``rng_normal_bf16_pair_kernel``, bitwise the two draws).
    ``seed_dev``: read the seed from this 1-element int64 device tensor at execution time (HIP-graph replays)."""
    if _pair_ok(a, b):
        if seed_dev is not None and (seed_dev.dtype != torch.int64 or seed_dev.device != a.device):
            raise TypeError("seed_dev must be an int64 tensor on the outputs' device")
        rc = _native.lib().dllm_rng_normal_bf16_pair(a.data_ptr(), b.data_ptr(), a.numel(), seed & (2**64 - 1),
                                                     seed_dev.data_ptr() if seed_dev is not None else None,
                                                     stream_a & (2**64 - 1), stream_b & (2**64 - 1), float(scale_a),
                                                     float(scale_b), _native.stream_ptr(a.device))
        _native.check(rc, "dllm_rng_normal_bf16_pair")
        return
    if seed_dev is not None:
        rng_normal_devseed_(a, seed_dev, stream_a, scale_a)
        rng_normal_devseed_(b, seed_dev, stream_b, scale_b)
        return
    rng_normal_(a, seed, stream_a, scale_a)
    rng_normal_(b, seed, stream_b, scale_b)


def rng_normal_devseed_(out: torch.Tensor, seed_dev: torch.Tensor, stream_id: int = 0,
                        scale: float = 1.0) -> torch.Tensor:
    """``rng_normal_`` with the seed read from a 1-element int64 device tensor at execution time, so the
    launch can live inside a captured HIP graph and still draw new data on every replay."""
    if out.device.type != "cuda":
        return rng_normal_(out, int(seed_dev.item()), stream_id, scale)
    if seed_dev.dtype != torch.int64 or seed_dev.device != out.device:
        raise TypeError("seed_dev must be an int64 tensor on the output's device")
    rc = _native.lib().dllm_rng_normal_devseed(out.data_ptr(), _native.dtype_code(out.dtype), out.numel(),
                                               seed_dev.data_ptr(), stream_id & (2**64 - 1), float(scale),
                                               _native.stream_ptr(out.device))
    _native.check(rc, "dllm_rng_normal_devseed")
    return out


def _mulhilo(a: int, b: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    p = b.to(torch.int64) * a  # < 2^64, fits as unsigned; use int64 with masking
    lo = p & 0xFFFFFFFF
    hi = (p >> 32) & 0xFFFFFFFF
    return hi, lo


def philox4x32_10(c0, c1, c2, c3, k0: int, k1: int):
    """Vectorised Philox4x32-10 on int64 tensors holding uint32 lanes (same rounds as csrc/elementwise.hip)."""
    M0, M1, W0, W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85
    for _ in range(10):
        hi0, lo0 = _mulhilo(M0, c0)
        hi1, lo1 = _mulhilo(M1, c2)
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        k0 = (k0 + W0) & 0xFFFFFFFF
        k1 = (k1 + W1) & 0xFFFFFFFF
    return c0, c1, c2, c3


def _philox_normal_cpu(n: int, seed: int, stream_id: int, scale: float, u16: bool = False) -> torch.Tensor:
    """``u16``: the bf16 stream -- counter i yields outputs 8i..8i+7 from Box-Muller pairs (lo16, hi16) of its four
    words, u1 = 1 - a/2^16 in (0, 1], u2 = b/2^16 in [0, 1)."""
    per = 8 if u16 else 4
    n4 = (n + per - 1) // per
    idx = torch.arange(n4, dtype=torch.int64)
    c0, c1, c2, c3 = philox4x32_10(idx & 0xFFFFFFFF, (idx >> 32) & 0xFFFFFFFF,
                                   torch.full_like(idx, stream_id & 0xFFFFFFFF),
                                   torch.full_like(idx, (stream_id >> 32) & 0xFFFFFFFF),
                                   seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    inv = 2.3283064365386963e-10

    def bm(a, b):
        u1 = (a.to(torch.float32) + 1.0) * inv
        u2 = b.to(torch.float32) * inv
        r = torch.sqrt(-2.0 * torch.log(u1))
        th = 2 * math.pi * u2
        return r * torch.cos(th), r * torch.sin(th)

    if u16:
        zs = []
        for c in (c0, c1, c2, c3):
            u1 = 1.0 - (c & 0xFFFF).to(torch.float32) * 2.0 ** -16
            th = 2 * math.pi * ((c >> 16) & 0xFFFF).to(torch.float32) * 2.0 ** -16
            r = torch.sqrt(-2.0 * torch.log(u1)) * scale
            zs += [r * torch.cos(th), r * torch.sin(th)]
        return torch.stack(zs, dim=1).reshape(-1)[:n]
    z0, z1 = bm(c0, c1)
    z2, z3 = bm(c2, c3)
    z = torch.stack([z0, z1, z2, z3], dim=1).reshape(-1)[:n]
    return z * scale


def _grad_code(g: torch.Tensor) -> int:
    return _native.dtype_code(g.dtype)


def sgd_step_(master: torch.Tensor, grad: torch.Tensor, lr: float, copy: torch.Tensor | None = None,
              grad_scale: float = 1.0, max_blocks: int = 0) -> None:
    """``master += (-lr)·grad`` in place (reference ``param.add_(-LR*grad)``), then ``copy = bf16(master)``.
    ``max_blocks > 0``: the streaming variant on at most that many workgroups (a side-stream optimizer
    that leaves the rest of the GPU to concurrent GEMMs); bitwise the same update."""
    if master.dtype != torch.float32:
        raise TypeError("master weights must be fp32")
    if master.device.type == "cuda":
        n = master.numel()
        if n % 4 == 0 and master.is_contiguous() and grad.is_contiguous():
            cp = copy.data_ptr() if copy is not None else None
            if max_blocks > 0:
                rc = _native.lib().dllm_sgd_step_stream(master.data_ptr(), grad.data_ptr(), _grad_code(grad), cp, n,
                                                        float(lr), float(grad_scale), int(max_blocks),
                                                        _native.stream_ptr(master.device))
                _native.check(rc, "dllm_sgd_step_stream")
                return
            rc = _native.lib().dllm_sgd_step(master.data_ptr(), grad.data_ptr(), _grad_code(grad), cp, n, float(lr),
                                             float(grad_scale), _native.stream_ptr(master.device))
            _native.check(rc, "dllm_sgd_step")
            return
        raise ValueError("sgd_step_ on GPU needs contiguous buffers with numel % 4 == 0")
    g = grad.float()
    if grad_scale != 1.0:
        g = g * grad_scale
    master.add_(-lr * g)
    if copy is not None:
        copy.copy_(master)


def sgd_split_step_(lo: torch.Tensor, hi: torch.Tensor, grad: torch.Tensor, lr: float,
                    grad_scale: float = 1.0) -> None:
    """``sgd_step_`` on a split master (``ops/master.py``): ``lo`` the int16 residual plane, ``hi`` the bf16
    working copy; the fp32 master they encode is updated exactly as ``sgd_step_`` updates an fp32 master."""
    if lo.dtype != torch.int16 or hi.dtype != torch.bfloat16 or lo.numel() != hi.numel():
        raise TypeError("sgd_split_step_ takes an int16 residual plane and its bf16 working copy")
    if lo.device.type == "cuda":
        n = lo.numel()
        if n % 4 or not (lo.is_contiguous() and hi.is_contiguous() and grad.is_contiguous()):
            raise ValueError("sgd_split_step_ on GPU needs contiguous buffers with numel % 4 == 0")
        rc = _native.lib().dllm_sgd_split_step(lo.data_ptr(), hi.data_ptr(), grad.data_ptr(), _grad_code(grad), n,
                                               float(lr), float(grad_scale), _native.stream_ptr(lo.device))
        _native.check(rc, "dllm_sgd_split_step")
        return
    from .master import join_master, set_master_

    w = join_master(hi, lo)
    g = grad.float()
    if grad_scale != 1.0:
        g = g * grad_scale
    w.add_(-lr * g)
    set_master_(hi, lo, w)


def adam_split_step_(lo: torch.Tensor, hi: torch.Tensor, grad: torch.Tensor, m: torch.Tensor, v: torch.Tensor,
                     step: int, lr: float, b1: float = 0.9, b2: float = 0.95, eps: float = 1e-8, wd: float = 0.0,
                     grad_scale: float = 1.0) -> None:
    """``adam_step_`` on a split master (``ops/master.py``); the moments ``m`` / ``v`` stay fp32."""
    if lo.dtype != torch.int16 or hi.dtype != torch.bfloat16 or lo.numel() != hi.numel():
        raise TypeError("adam_split_step_ takes an int16 residual plane and its bf16 working copy")
    if lo.device.type == "cuda":
        n = lo.numel()
        if n % 4:
            raise ValueError("adam_split_step_ on GPU needs numel % 4 == 0")
        rc = _native.lib().dllm_adam_split_step(lo.data_ptr(), hi.data_ptr(), grad.data_ptr(), _grad_code(grad),
                                                m.data_ptr(), v.data_ptr(), n, float(lr), float(b1), float(b2),
                                                float(eps), float(wd), int(step), float(grad_scale),
                                                _native.stream_ptr(lo.device))
        _native.check(rc, "dllm_adam_split_step")
        return
    from .master import join_master, set_master_

    w = join_master(hi, lo)
    adam_step_(w, grad, m, v, step, lr, b1, b2, eps, wd, grad_scale=grad_scale)
    set_master_(hi, lo, w)


def adam_step_(master: torch.Tensor, grad: torch.Tensor, m: torch.Tensor, v: torch.Tensor, step: int, lr: float,
               b1: float = 0.9, b2: float = 0.95, eps: float = 1e-8, wd: float = 0.0,
               copy: torch.Tensor | None = None, grad_scale: float = 1.0) -> None:
    """Fused AdamW on flat fp32 buffers (decoupled weight decay)."""
    if master.device.type == "cuda":
        n = master.numel()
        if n % 4:
            raise ValueError("adam_step_ on GPU needs numel % 4 == 0")
        rc = _native.lib().dllm_adam_step(master.data_ptr(), grad.data_ptr(), _grad_code(grad), m.data_ptr(),
                                          v.data_ptr(), copy.data_ptr() if copy is not None else None, n,
                                          float(lr), float(b1), float(b2), float(eps), float(wd), int(step),
                                          float(grad_scale), _native.stream_ptr(master.device))
        _native.check(rc, "dllm_adam_step")
        return
    g = grad.float() * grad_scale
    m.mul_(b1).add_((1 - b1) * g)
    v.mul_(b2).add_((1 - b2) * g * g)
    bc1, bc2 = 1 - b1 ** step, 1 - b2 ** step
    upd = (m / bc1) / (torch.sqrt(v / bc2) + eps) + wd * master
    master.sub_(lr * upd)
    if copy is not None:
        copy.copy_(master)


def cast_(src: torch.Tensor, dst: torch.Tensor) -> torch.Tensor:
    if src.numel() != dst.numel():
        raise ValueError("cast_: size mismatch")
    if src.device.type == "cuda" and src.dtype != dst.dtype and src.is_contiguous() and dst.is_contiguous():
        rc = _native.lib().dllm_cast(src.data_ptr(), _native.dtype_code(src.dtype), dst.data_ptr(),
                                     _native.dtype_code(dst.dtype), src.numel(), _native.stream_ptr(src.device))
        _native.check(rc, "dllm_cast")
        return dst
    dst.copy_(src.view(dst.shape) if src.shape != dst.shape else src)
    return dst


def occupy_cus(blocks: int, us: float, threads: int = 256, device: torch.device | None = None) -> None:
    """Keep ``blocks`` workgroups of ``threads`` lanes resident for ``us`` microseconds on the current stream: a
    stand-in for a collective kernel's CU footprint (RCCL channels), to measure how a GEMM grid behaves when part
    of the chip is taken (scripts/bench_occupancy.py).  Native only."""
    dev = device or torch.device("cuda", torch.cuda.current_device())
    rc = _native.lib().dllm_occupy(int(blocks), int(threads), float(us), None, _native.stream_ptr(dev))
    _native.check(rc, "dllm_occupy")
