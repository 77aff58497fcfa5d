"""Activation functions and their derivatives (torch reference path + codes shared with the HIP epilogues).

Reference: ReLU forward ``torch.where(x<=0, 0, x)`` and the in-place backward mask
``dloss_dx.masked_fill_(x<=0, 0)`` (train_ffns.py:47-52).  SiLU and GELU(tanh) are the north-star
activations (BASELINE.json); the same formulas are implemented in ``csrc/common.h``.
"""
from __future__ import annotations

import math

import torch

ACT_CODES = {"none": 0, "relu": 1, "silu": 2, "gelu": 3}


def act_code(name: str) -> int:
    if name not in ACT_CODES:
        raise ValueError(f"unknown activation {name!r}; choose from {sorted(ACT_CODES)}")
    return ACT_CODES[name]


def act_fwd(name: str, x: torch.Tensor) -> torch.Tensor:
    if name == "relu":
        return torch.where(x <= 0, torch.zeros((), dtype=x.dtype, device=x.device), x)
    if name == "silu":
        return x * torch.sigmoid(x)
    if name == "gelu":
        return torch.nn.functional.gelu(x, approximate="tanh")
    if name == "none":
        return x
    raise ValueError(name)


def act_grad(name: str, x: torch.Tensor) -> torch.Tensor:
    """d act(x) / dx evaluated at the pre-activation ``x``."""
    if name == "relu":
        return (x > 0).to(x.dtype)
    if name == "silu":
        s = torch.sigmoid(x)
        return s * (1 + x * (1 - s))
    if name == "gelu":
        k0, k1 = math.sqrt(2.0 / math.pi), 0.044715
        u = k0 * (x + k1 * x ** 3)
        t = torch.tanh(u)
        return 0.5 * (1 + t) + 0.5 * x * (1 - t * t) * k0 * (1 + 3 * k1 * x * x)
    if name == "none":
        return torch.ones_like(x)
    raise ValueError(name)


def relu_bkwd_(dloss_dx: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """In-place ReLU backward with the reference's exact semantics (train_ffns.py:50-52)."""
    dloss_dx.masked_fill_(x <= 0, 0)
    return dloss_dx
