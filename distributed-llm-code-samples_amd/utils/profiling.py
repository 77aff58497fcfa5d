"""Tracing: torch.profiler on ROCm (Kineto/roctracer) for rank 0, roctx ranges, phase timers.

Reference: the ``torch_profile_rank_0`` decorator (train_ffns.py:129-141) wraps a worker in
``torch.profiler.profile(CPU+CUDA, record_shapes, with_stack)`` and exports ``trace_profiler_trace.json``
on rank 0; it rebinds a module-level ``global`` so ``spawn`` can pickle it, which breaks when applied to
a second function.  Here profiling is a context manager (nothing to pickle) and
kernel-level evidence comes from ``rocprofv3 --kernel-trace --stats`` (``profiles/README.md`` lists the
commands; ``scripts/rocpd_stats.py`` summarises a run's database).
"""
from __future__ import annotations

import contextlib
import functools
import os

import torch


@contextlib.contextmanager
def maybe_profile(path: str, rank: int, all_ranks: bool = False):
    """Profile the enclosed region with torch.profiler and write a chrome trace (rank 0 unless all_ranks)."""
    if not path or (rank != 0 and not all_ranks):
        yield None
        return
    from torch.profiler import ProfilerActivity, profile

    acts = [ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(ProfilerActivity.CUDA)
    with profile(activities=acts, record_shapes=True, with_stack=True) as prof:
        yield prof
    out = path if rank == 0 else f"{os.path.splitext(path)[0]}.rank{rank}.json"
    prof.export_chrome_trace(out)
    print(f"Profiler exported {out}", flush=True)


def profile_rank0(path: str = "trace_profiler_trace.json"):
    """Decorator form of ``maybe_profile`` (first positional arg = rank, as in the reference)."""

    def deco(fn):
        @functools.wraps(fn)
        def wrapper(*args, **kwargs):
            with maybe_profile(path, int(args[0]) if args else 0):
                return fn(*args, **kwargs)

        return wrapper

    return deco


_ROCTX = None


def _roctx():
    """The roctx library rocprofv3 intercepts (ROCm's rocprofiler-sdk roctx), else torch's legacy one."""
    global _ROCTX
    if _ROCTX is None:
        import ctypes

        _ROCTX = False
        rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
        for d in (os.path.join(rocm, "lib", "librocprofiler-sdk-roctx.so.1"),
                  os.path.join(os.path.dirname(torch.__file__), "lib", "libroctx64.so")):
            if os.path.exists(d):
                try:
                    _ROCTX = ctypes.CDLL(d)
                    _ROCTX.roctxRangePushA.argtypes = [ctypes.c_char_p]
                    break
                except (OSError, AttributeError):
                    _ROCTX = False
    return _ROCTX


def roctx_push(name: str) -> None:
    """Open a roctx range when DLLM_ROCTX=1 (no-op otherwise)."""
    if os.environ.get("DLLM_ROCTX") == "1":
        lib = _roctx()
        if lib:
            lib.roctxRangePushA(name.encode())


def roctx_pop() -> None:
    if os.environ.get("DLLM_ROCTX") == "1":
        lib = _roctx()
        if lib:
            lib.roctxRangePop()


@contextlib.contextmanager
def range_(name: str):
    """roctx range (visible to rocprofv3 --marker-trace) + torch.profiler record_function."""
    lib = _roctx() if os.environ.get("DLLM_ROCTX") == "1" else None
    if lib:
        lib.roctxRangePushA(name.encode())
    try:
        with torch.profiler.record_function(name):
            yield
    finally:
        if lib:
            lib.roctxRangePop()


class PhaseTimer:
    """HIP-event timing of named phases on the current stream (no host sync until ``summary``)."""

    def __init__(self, enabled: bool = True):
        self.enabled = enabled and torch.cuda.is_available()
        self.events: list[tuple[str, torch.cuda.Event, torch.cuda.Event]] = []

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled:
            yield
            return
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        yield
        e.record()
        self.events.append((name, s, e))

    def summary(self) -> dict:
        if not self.enabled:
            return {}
        torch.cuda.synchronize()
        out: dict[str, float] = {}
        for n, s, e in self.events:
            out[n] = out.get(n, 0.0) + s.elapsed_time(e)
        self.events.clear()
        return out
