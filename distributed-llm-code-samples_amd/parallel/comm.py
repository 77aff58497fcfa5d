"""Collective wrappers: flat, zero-copy, async, one stream per role.

Every call site of the reference maps to one function here:

* X1 ``dist.all_reduce(grad, async_op=True)`` per tensor (train_ffns.py:165)  -> ``all_reduce`` on bucket views
* X2 ``dist.all_gather(list, shard, async_op=True)`` + ``torch.cat`` (:203,:209) -> ``all_gather_into``
  writing straight into the full-weight buffer (row shards concatenate contiguously, no cat, no zeros_like)
* X3 sync ``dist.reduce_scatter(shard, list(chunk(g)))`` (:255-256)            -> async ``reduce_scatter_into``
  from the flat full-grad buffer on its own communicator/stream (fixes the TODO at :14/:252)
* X4/X5 sync ``dist.all_reduce(y / dx)`` (:303,:309)                           -> ``all_reduce`` on the tp role,
  async where a consumer can wait later.

With the ``nccl`` backend (RCCL over xGMI) the returned handle's ``wait()`` only makes the *current HIP
stream* wait on the collective's stream (no host block), so compute keeps flowing.  ``world == 1`` is a
no-op returning an already-completed handle.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from ..utils import observe


class Done:
    """Completed-work placeholder (single-rank groups, or nothing to do)."""

    def wait(self):
        return True

    def is_completed(self):
        return True


class Elided:
    """An infinitely fast collective (``set_elide``): issued on the current stream, ``wait()`` orders the waiting
    stream after that issue point.  The step keeps every data dependency a real collective carries (e.g. the next
    forward still waits for the shard update whose result the all-gather would ship); only the transfer and the
    collective stream's hops are gone."""

    def __init__(self, t: torch.Tensor):
        self.ev = None
        if t.is_cuda:
            self.ev = torch.cuda.Event()
            self.ev.record(torch.cuda.current_stream(t.device))
        self.device = t.device

    def wait(self):
        if self.ev is not None:
            torch.cuda.current_stream(self.device).wait_event(self.ev)
        return True

    def is_completed(self):
        return self.ev is None or self.ev.query()


_SERIALIZE = False
_ELIDE = False
# synchronous collectives on the caller's stream (all_reduce); DLLM_SYNC_INLINE=0 routes them through the
# communicator stream as before (A/B)
_SYNC_INLINE = os.environ.get("DLLM_SYNC_INLINE", "1") != "0"


def set_elide(flag: bool) -> bool:
    """Timing mode for the differential exposed-communication measurement (bench.py ``exposed_ms_diff``): every
    collective on a communicator returns an ``Elided`` handle at once without running, so a step costs its compute
    and its dependency edges alone.  The results of such steps are meaningless (gradients are not reduced, shards
    not gathered); only their time is used.  Returns the previous setting."""
    global _ELIDE
    old, _ELIDE = _ELIDE, bool(flag)
    return old


def eliding() -> bool:
    return _ELIDE


def set_serialize(flag: bool) -> None:
    """Race-detection mode: every collective is waited for at issue and the device is
    synchronised, so communication never overlaps compute.  Results must be bitwise identical to the
    overlapped schedule; any difference exposes a missing stream/event edge."""
    global _SERIALIZE
    _SERIALIZE = flag


def _finish(w, async_op: bool):
    if _SERIALIZE and not isinstance(w, Done):
        w.wait()
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()
        return Done()
    return w if async_op else Done()


def _native(group) -> bool:
    from .rccl import NativeGroup

    return isinstance(group, NativeGroup)


def _active(group) -> bool:
    """A collective on ``None`` (a mesh axis of size 1 without a communicator) is a local no-op; a real
    group — even of size 1 (``Mesh.build(force=True)``) — always goes through the backend."""
    return group is not None and dist.is_initialized()


_COUNTS: dict | None = None


class count_collectives:
    """Context manager counting the collectives issued through this module, per group object (any backend,
    CPU or GPU): ``with count_collectives() as c: ...; c.by_role(mesh.groups)``."""

    def __enter__(self):
        global _COUNTS
        self.counts = _COUNTS = {}
        return self

    def __exit__(self, *exc):
        global _COUNTS
        _COUNTS = None
        return False

    def by_role(self, groups: dict) -> dict:
        """{role: count} for a mesh's role groups (roles sharing one group object share its count)."""
        return {r: self.counts.get(id(g), 0) for r, g in groups.items() if g is not None}


def _group_size(group) -> int:
    return group.size() if _native(group) else dist.get_world_size(group)


def _moves(group, out: torch.Tensor, inp: torch.Tensor) -> bool:
    """Whether a collective moves data: on a size-1 communicator (``force_comm`` at N=1) an in-place
    all-reduce / all-gather / reduce-scatter launches no kernel, so the observer keeps it out of the
    comm intervals (it still counts it)."""
    return not (_group_size(group) == 1 and out.data_ptr() == inp.data_ptr())


def _issue(group, fn, moves: bool = True):
    """Run ``fn()`` (which issues one collective and returns its work); with a ``CommObserver`` active the
    collective's issue and completion are recorded (utils/observe.py)."""
    if _COUNTS is not None:
        _COUNTS[id(group)] = _COUNTS.get(id(group), 0) + 1
    obs = observe.active()
    if obs is None:
        return fn()
    ev = obs.issue()
    w = fn()
    obs.issued(group, ev, w, moves=moves)
    return w


def all_reduce(t: torch.Tensor, group, async_op: bool = True):
    """``async_op=False`` (a consumer right behind it, e.g. the TP forward's output exchange): issued as a synchronous
    collective -- native: ``NativeGroup.all_reduce_inline``, on the caller's current stream, so it costs no event
    hops to a communicator stream and back, each a cross-queue wait (``profiles/r4/forced_comm_gaps_r4.txt``);
    torch: ``dist.all_reduce(async_op=False)``, which recent ProcessGroupNCCL versions also launch on the current
    stream (older ones wait on their own stream, as the async form + wait does).  Under a ``CommObserver`` it stays
    on the communicator stream, where the observer times it."""
    if _ELIDE and group is not None:
        return Elided(t)
    inline = not async_op and not _SERIALIZE and observe.active() is None and _SYNC_INLINE
    if group is not None and _native(group):
        if inline:
            _issue(group, lambda: group.all_reduce_inline(t))
            return Done()
        w = _issue(group, lambda: group.all_reduce(t), _moves(group, t, t))
        return _finish(w, async_op) if (async_op or _SERIALIZE) else (w.wait(), Done())[1]
    if not _active(group):
        return Done()
    if inline:
        _issue(group, lambda: dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group, async_op=False))
        return Done()
    w = _issue(group, lambda: dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group, async_op=True),
               _moves(group, t, t))
    return _finish(w, async_op) if (async_op or _SERIALIZE) else (w.wait(), Done())[1]


def all_gather_into(out: torch.Tensor, shard: torch.Tensor, group, async_op: bool = True):
    if _ELIDE and group is not None:
        return Elided(out)
    if group is not None and _native(group):
        w = _issue(group, lambda: group.all_gather_into(out.view(-1), shard.reshape(-1)), _moves(group, out, shard))
        return _finish(w, async_op) if (async_op or _SERIALIZE) else (w.wait(), Done())[1]
    if not _active(group):
        if out.data_ptr() != shard.data_ptr():
            out.copy_(shard.view_as(out))
        return Done()
    n = dist.get_world_size(group)
    if out.numel() != shard.numel() * n:
        raise ValueError(f"all_gather_into: out {out.numel()} != {n} x shard {shard.numel()}")
    w = _issue(group, lambda: dist.all_gather_into_tensor(out.view(-1), shard.reshape(-1), group=group,
                                                         async_op=True), _moves(group, out, shard))
    return _finish(w, async_op) if (async_op or _SERIALIZE) else (w.wait(), Done())[1]


def reduce_scatter_into(out: torch.Tensor, full: torch.Tensor, group, async_op: bool = True):
    if _ELIDE and group is not None:
        return Elided(out)
    if group is not None and _native(group):
        w = _issue(group, lambda: group.reduce_scatter_into(out.view(-1), full.reshape(-1)), _moves(group, out, full))
        return _finish(w, async_op) if (async_op or _SERIALIZE) else (w.wait(), Done())[1]
    if not _active(group):
        if out.data_ptr() != full.data_ptr():
            out.copy_(full.view_as(out))
        return Done()
    n = dist.get_world_size(group)
    if full.numel() != out.numel() * n:
        raise ValueError(f"reduce_scatter_into: full {full.numel()} != {n} x out {out.numel()}")
    w = _issue(group, lambda: dist.reduce_scatter_tensor(out.view(-1), full.reshape(-1), op=dist.ReduceOp.SUM,
                                                        group=group, async_op=True), _moves(group, out, full))
    return _finish(w, async_op) if (async_op or _SERIALIZE) else (w.wait(), Done())[1]


class _Many:
    """Completion of several collectives issued together."""

    def __init__(self, works):
        self.works = works

    def wait(self):
        for w in self.works:
            w.wait()
        return True

    def is_completed(self):
        return all(w.is_completed() for w in self.works)


def all_gather_into_many(pairs, group, async_op: bool = True):
    """All-gathers ``(out, shard)`` issued as ONE group: the native layer fuses them with
    ncclGroupStart/End (one launch, one completion event); torch / gloo issue them back to back."""
    if _ELIDE and group is not None:
        return Elided(pairs[0][0])
    if group is not None and _native(group) and not _SERIALIZE:
        w = _issue(group, lambda: group.all_gather_into_many([(o.view(-1), sh.reshape(-1)) for o, sh in pairs]),
                   any(_moves(group, o, sh) for o, sh in pairs))
        return w if async_op else (w.wait(), Done())[1]
    w = _Many([all_gather_into(o, sh, group, async_op=True) for o, sh in pairs])
    return w if async_op else (w.wait(), Done())[1]


def reduce_scatter_into_many(pairs, group, async_op: bool = True):
    """Reduce-scatters ``(out, full)`` issued as ONE group (see ``all_gather_into_many``)."""
    if _ELIDE and group is not None:
        return Elided(pairs[0][0])
    if group is not None and _native(group) and not _SERIALIZE:
        w = _issue(group, lambda: group.reduce_scatter_into_many([(o.view(-1), f.reshape(-1)) for o, f in pairs]),
                   any(_moves(group, o, f) for o, f in pairs))
        return w if async_op else (w.wait(), Done())[1]
    w = _Many([reduce_scatter_into(o, f, group, async_op=True) for o, f in pairs])
    return w if async_op else (w.wait(), Done())[1]


def gather_to_rank0(t: torch.Tensor, group=None) -> list[torch.Tensor] | None:
    """Gather equally-shaped tensors from every rank of ``group`` onto rank 0 of that group (CPU copies)."""
    if group is not None and _native(group):
        n = group.size()
        out = torch.empty((n,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        group.all_gather_into(out.view(-1), t.contiguous().view(-1)).wait()
        return [o.cpu() for o in out]
    if group is None or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return [t.detach().cpu()]
    n = dist.get_world_size(group)
    outs = [torch.empty_like(t) for _ in range(n)]
    dist.all_gather(outs, t.contiguous(), group=group)
    return [o.cpu() for o in outs]


def barrier(group=None, device: torch.device | None = None) -> None:
    if not dist.is_initialized():
        return
    if device is not None and device.type == "cuda":
        dist.barrier(group=group, device_ids=[device.index])
    else:
        dist.barrier(group=group)
