"""Split fp32 master weights: the fp32 master stored as its bf16 working copy plus a 16-bit residual plane.

``bits(w) = (bits(hi) << 16) + sext(lo)`` (mod 2^32), with ``t = bits(w) + 0x8000``, ``hi = t >> 16`` and
``lo = (t & 0xffff) ^ 0x8000``.  The map is a bijection on 32-bit patterns, so the master stays exactly the fp32
value an unsplit update computes; ``hi`` is that value rounded to bf16 half away from zero (RNE differs only on exact
ties).  A bf16 run then keeps 4 B per parameter of weight state instead of 6 B (fp32 master + bf16 copy), and the
fused optimizer epilogue reads 4 B and writes 4 B per parameter instead of reading 4 B and writing 6 B
(``csrc/common.h`` ``split_join2`` / ``split_part2``, ``csrc/gemm_kernels.h`` ``EPI_SGDS``).

These are the torch forms (any device): the engine's hot path never calls them; checkpoints, tests and parameter
export do.  The reference keeps plain fp32 parameters (``train_ffns.py:114``, ``:172``).
"""
from __future__ import annotations

import torch


def split_master(w: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """fp32 ``w`` -> (hi bf16, lo int16) of the same shape."""
    if w.dtype != torch.float32:
        raise TypeError("split_master takes fp32")
    u = w.contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    t = (u + 0x8000) & 0xFFFFFFFF
    hi = _u16_to_i16(t >> 16)
    lo = _u16_to_i16((t & 0xFFFF) ^ 0x8000)
    return hi.view(torch.bfloat16).view(w.shape), lo.view(w.shape)


def join_master(hi: torch.Tensor, lo: torch.Tensor) -> torch.Tensor:
    """(hi bf16, lo int16) -> the fp32 master they encode."""
    if hi.dtype != torch.bfloat16 or lo.dtype != torch.int16 or hi.shape != lo.shape:
        raise TypeError("join_master takes (bf16 hi, int16 lo) of one shape")
    h = hi.contiguous().view(torch.int16).to(torch.int64) & 0xFFFF
    u = ((h << 16) + lo.contiguous().to(torch.int64)) & 0xFFFFFFFF
    u = torch.where(u >= 2 ** 31, u - 2 ** 32, u)
    return u.to(torch.int32).view(torch.float32).view(hi.shape)


def set_master_(hi: torch.Tensor, lo: torch.Tensor, w: torch.Tensor) -> None:
    """Store the fp32 ``w`` into the split planes ``hi`` / ``lo`` in place."""
    h, l = split_master(w.to(torch.float32))
    hi.copy_(h)
    lo.copy_(l)


def join_flat(hi: torch.Tensor, lo: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """Flat (1-D) join: the native kernel on GPU buffers, ``join_master`` on CPU."""
    if out is None:
        out = torch.empty(lo.numel(), dtype=torch.float32, device=lo.device)
    if lo.device.type == "cuda":
        from .. import _native

        _native.check(_native.lib().dllm_split_master(hi.data_ptr(), lo.data_ptr(), out.data_ptr(), lo.numel(), 0,
                                                      _native.stream_ptr(lo.device)), "dllm_split_master(join)")
        return out
    out.copy_(join_master(hi, lo))
    return out


def part_flat(w: torch.Tensor, hi: torch.Tensor, lo: torch.Tensor) -> None:
    """Flat (1-D) split of fp32 ``w`` into ``hi`` / ``lo`` in place (native on GPU)."""
    if lo.device.type == "cuda":
        from .. import _native

        w = w.contiguous()
        _native.check(_native.lib().dllm_split_master(hi.data_ptr(), lo.data_ptr(), w.data_ptr(), lo.numel(), 1,
                                                      _native.stream_ptr(lo.device)), "dllm_split_master(split)")
        return
    set_master_(hi, lo, w)


def _u16_to_i16(x: torch.Tensor) -> torch.Tensor:
    return torch.where(x >= 2 ** 15, x - 2 ** 16, x).to(torch.int16)
