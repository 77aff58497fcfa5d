"""Mock data: random inputs ``x`` and a random ``dloss/dx`` standing in for the loss (train_ffns.py:12).

* ``reference_mock_data`` — the reference's exact stream: for each seed, reseed a CPU ``Generator`` and draw
  ``x = randn(T, D)`` then ``dloss_dx = 0.1·randn(T, D)`` (train_ffns.py:144-151).  Used for parity
  (``--data cpu_compat``); costs ~0.4 s/step on the host at T=8192, D=4096.
* ``DeviceMockData`` — throughput mode: the same two tensors drawn on the GPU by the Philox kernel
  (``ops.elementwise.rng_normal_``), keyed by the step seed, directly in the compute dtype, into
  preallocated buffers (no H2D copy, no allocator traffic).
"""
from __future__ import annotations

import torch

from ..ops.elementwise import STREAM_DY, STREAM_X, rng_normal_
from .config import DLOSS_DX_COEF


def reference_mock_data(seeds, batch_size: int, model_size: int):
    gen = torch.Generator()
    for seed in (seeds.tolist() if hasattr(seeds, "tolist") else list(seeds)):
        gen.manual_seed(int(seed))
        x = torch.randn((batch_size, model_size), generator=gen)
        dloss_dx = DLOSS_DX_COEF * torch.randn((batch_size, model_size), generator=gen)
        yield x, dloss_dx


class DeviceMockData:
    def __init__(self, tokens: int, model_size: int, dtype: torch.dtype, device: torch.device):
        self.x = torch.empty((tokens, model_size), dtype=dtype, device=device)
        self.dy = torch.empty((tokens, model_size), dtype=dtype, device=device)

    def fill(self, seed: int) -> tuple[torch.Tensor, torch.Tensor]:
        rng_normal_(self.x, seed=int(seed), stream_id=STREAM_X, scale=1.0)
        rng_normal_(self.dy, seed=int(seed), stream_id=STREAM_DY, scale=DLOSS_DX_COEF)
        return self.x, self.dy


class CpuCompatData:
    """Reference stream, copied into preallocated device buffers (pinned staging for async H2D)."""

    def __init__(self, tokens: int, model_size: int, dtype: torch.dtype, device: torch.device):
        self.x = torch.empty((tokens, model_size), dtype=dtype, device=device)
        self.dy = torch.empty((tokens, model_size), dtype=dtype, device=device)
        self.tokens, self.model_size = tokens, model_size

    def fill(self, seed: int) -> tuple[torch.Tensor, torch.Tensor]:
        (x, dy), = list(reference_mock_data([int(seed)], self.tokens, self.model_size))
        self.x.copy_(x)
        self.dy.copy_(dy)
        return self.x, self.dy


def make_data(kind: str, tokens: int, model_size: int, dtype: torch.dtype, device: torch.device):
    if kind == "device":
        return DeviceMockData(tokens, model_size, dtype, device)
    if kind == "cpu_compat":
        return CpuCompatData(tokens, model_size, dtype, device)
    raise ValueError(kind)


def stripe_seeds(seeds: torch.Tensor, n: int, r: int) -> torch.Tensor:
    """Rank r's share of the step seeds for data parallelism: ``seeds[r::n]``
    (= the reference's ``seeds.reshape((-1, n)).chunk(n, dim=1)[r]``, train_ffns.py:182, :273)."""
    if len(seeds) % n:
        raise ValueError(f"num_steps ({len(seeds)}) must be divisible by the data-parallel size ({n}) "
                         "(train_ffns.py:175)")
    return seeds.reshape(-1, n)[:, r].reshape(-1)
