"""Mock data: random inputs ``x`` and a random ``dloss/dx`` standing in for the loss (train_ffns.py:12).

* ``reference_mock_data`` — the reference's exact stream: for each seed, reseed a CPU ``Generator`` and draw
  ``x = randn(T, D)`` then ``dloss_dx = 0.1·randn(T, D)`` (train_ffns.py:144-151).  Used for parity
  (``--data cpu_compat``); costs ~0.4 s/step on the host at T=8192, D=4096.
* ``DeviceMockData`` — throughput mode: the same two tensors drawn on the GPU by the Philox kernel
  (``ops.elementwise.rng_normal_``), keyed by the step seed, directly in the compute dtype, into
  preallocated buffers (no H2D copy, no allocator traffic).
"""
from __future__ import annotations

import os

import torch

from ..ops.elementwise import STREAM_DY, STREAM_X, rng_normal_, rng_normal_pair_
from .config import DLOSS_DX_COEF


def reference_mock_data(seeds, batch_size: int, model_size: int):
    gen = torch.Generator()
    for seed in (seeds.tolist() if hasattr(seeds, "tolist") else list(seeds)):
        gen.manual_seed(int(seed))
        x = torch.randn((batch_size, model_size), generator=gen)
        dloss_dx = DLOSS_DX_COEF * torch.randn((batch_size, model_size), generator=gen)
        yield x, dloss_dx


class DeviceMockData:
    """Device-generated batches.  ``overlap=True`` (GPU) turns it into a one-deep data pipeline: two batch slots,
    and the next step's batch is drawn on a side stream while the current step's backward runs -- the engine
    calls ``release()`` at the start of its backward (``FFNTrainer.before_backward``); the next ``fill`` makes
    the compute stream wait for that draw only.  The slot being drawn into was last read by the previous step,
    which the compute stream has finished by then (stream order, and the weight-gradient stream is joined at
    the end of every step).  Values are identical to the synchronous mode (same seeds, same kernel)."""

    def __init__(self, tokens: int, model_size: int, dtype: torch.dtype, device: torch.device,
                 overlap: bool = False):
        self.x = torch.empty((tokens, model_size), dtype=dtype, device=device)
        self.dy = torch.empty((tokens, model_size), dtype=dtype, device=device)
        self.overlap = bool(overlap) and torch.device(device).type == "cuda"
        self.depth = 1 if self.overlap else 0  # how far ahead callers name next_seed (0: no prefetch)
        if self.overlap:
            self._slots = [(self.x, self.dy), (torch.empty_like(self.x), torch.empty_like(self.dy))]
            self._stream = torch.cuda.Stream(device=device)
            self._n = 0
            self._pending = None  # (seed, slot) to draw at the next release()
            self._ready = None    # (seed, slot, event) drawn ahead

    def prefetch(self, seed: int) -> None:
        return None

    def bind_transposed(self, x_t: torch.Tensor | None, dy_t: torch.Tensor | None) -> None:
        """Draw the transposes xᵀ / dyᵀ too, into the engine's buffers (``FFNEngine.input_transposes()``: the NN
        weight-gradient layout's layer-0 xᵀ and top-layer dyᵀ), in the same pass as the batch
        (``rng_normal_bf16_t_kernel``).  Each filled tensor is tagged ``_dllm_t`` = its transpose buffer, which the
        engine's next ``train_step`` takes instead of transposing (and clears).  Synchronous mode only: with the
        one-deep pipeline the next draw would overwrite a transpose the current step's backward still reads."""
        off = self.overlap or os.environ.get("DLLM_DRAW_T", "1") == "0"   # DLLM_DRAW_T=0: engine transposes (A/B)
        self._t = (None, None) if off else (x_t, dy_t)

    def _draw(self, x: torch.Tensor, dy: torch.Tensor, seed: int) -> None:
        x_t, dy_t = getattr(self, "_t", (None, None))
        if x_t is None and dy_t is None and os.environ.get("DLLM_RNG_PAIR", "1") != "0":
            # both in one launch on the GPU (rng_normal_bf16_pair_kernel; the same values)
            rng_normal_pair_(x, dy, int(seed), STREAM_X, 1.0, STREAM_DY, DLOSS_DX_COEF)
        else:
            rng_normal_(x, seed=int(seed), stream_id=STREAM_X, scale=1.0, out_t=x_t)
            rng_normal_(dy, seed=int(seed), stream_id=STREAM_DY, scale=DLOSS_DX_COEF, out_t=dy_t)
        x._dllm_t, dy._dllm_t = x_t, dy_t

    def fill(self, seed: int, next_seed: int | None = None) -> tuple[torch.Tensor, torch.Tensor]:
        if not self.overlap:
            self._draw(self.x, self.dy, seed)
            return self.x, self.dy
        k = self._n % 2
        self._n += 1
        if self._ready is not None:
            # order after the side-stream draw whether or not it is the batch asked for: on a mismatch (resume,
            # skipped step, an eval fill) the redraw below may target the very slot that draw is still writing
            torch.cuda.current_stream(self.x.device).wait_event(self._ready[2])
        if self._ready is None or self._ready[:2] != (int(seed), k):
            self._draw(*self._slots[k], seed)
        self._ready = None
        self._pending = (int(next_seed), k ^ 1) if next_seed is not None else None
        return self._slots[k]

    def release(self) -> None:
        """Start drawing the announced next batch on the side stream (after everything issued so far)."""
        if not self.overlap or self._pending is None:
            return
        seed, k = self._pending
        self._pending = None
        go = torch.cuda.Event()
        go.record(torch.cuda.current_stream(self.x.device))
        self._stream.wait_event(go)
        with torch.cuda.stream(self._stream):
            self._draw(*self._slots[k], seed)
            done = torch.cuda.Event()
            done.record(self._stream)
        self._ready = (seed, k, done)


class CpuCompatData:
    """Reference stream (CPU ``Generator``), copied into preallocated device buffers.

    The reference draws each batch on the host inside the timed step (~0.4 s at T=8192, D=4096, one core).
    Every step reseeds its own generator (train_ffns.py:148), so steps are independent streams: a pool of
    ``depth`` host threads draws the next ``depth`` seeds' batches concurrently into pinned memory while the
    GPU trains on the current one (torch's CPU RNG releases the GIL), and the copy to the device is an async
    H2D on the current stream.  Values are identical to the reference's ``mock_data`` (same generator, same
    draw order per seed).  ``depth`` defaults to the host cores available to this rank (at most 8)."""

    def __init__(self, tokens: int, model_size: int, dtype: torch.dtype, device: torch.device,
                 prefetch: bool = True, depth: int = 0):
        self.x = torch.empty((tokens, model_size), dtype=dtype, device=device)
        self.dy = torch.empty((tokens, model_size), dtype=dtype, device=device)
        self.tokens, self.model_size = tokens, model_size
        self.dtype, self.device = dtype, torch.device(device)
        self.pin = self.device.type == "cuda"
        self._pool = None
        self._pending = {}
        if not depth:
            import os

            ranks = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1")))
            depth = max(1, min(8, (os.cpu_count() or 2) // ranks - 1))
        self.depth = depth if prefetch else 0
        if prefetch:
            import concurrent.futures as cf

            self._pool = cf.ThreadPoolExecutor(max_workers=self.depth)
        self._host = None

    def _draw(self, seed: int):
        (x, dy), = list(reference_mock_data([int(seed)], self.tokens, self.model_size))
        x, dy = x.to(self.dtype), dy.to(self.dtype)
        if self.pin:
            x, dy = x.pin_memory(), dy.pin_memory()
        return x, dy

    def prefetch(self, seed: int) -> None:
        if self._pool is not None and seed not in self._pending:
            self._pending[seed] = self._pool.submit(self._draw, seed)

    def fill(self, seed: int, next_seed: int | None = None) -> tuple[torch.Tensor, torch.Tensor]:
        fut = self._pending.pop(int(seed), None)
        x, dy = fut.result() if fut is not None else self._draw(seed)
        # no host synchronisation: the device buffers are reused in stream order, and a pinned host batch
        # released here goes back to torch's caching host allocator, which records an event on the stream
        # of every non_blocking copy out of it and reuses the block only after that event -- so the host
        # keeps enqueueing ahead of the GPU instead of waiting for the previous step
        self.x.copy_(x, non_blocking=self.pin)
        self.dy.copy_(dy, non_blocking=self.pin)
        self._host = (x, dy)
        if next_seed is not None:
            self.prefetch(int(next_seed))
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
