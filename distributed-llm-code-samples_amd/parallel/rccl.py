"""Python side of the native RCCL communicator layer (``csrc/comm.cpp``).

``NativeGroup`` = one RCCL communicator + one dedicated HIP stream for one communication role (DDP
gradient all-reduce, ZeRO/FSDP reduce-scatter, parameter all-gather, TP activations).  Collectives are
enqueued on the role stream behind a HIP event recorded on the caller's current (compute) stream; the
returned ``NativeWork.wait()`` makes the current stream wait on the completion event — the same
contract as ``torch.distributed``'s async ``Work`` with ProcessGroupNCCL, but with explicit streams and
events under our control.  The communicator's uniqueId travels through the job's
``torch.distributed`` store, so no extra rendezvous is needed.

Buffers passed to a collective must stay alive until the work is waited for: the engine only passes
views of its persistent flat buffers.
"""
from __future__ import annotations

import ctypes
import itertools

import torch
import torch.distributed as dist

from .. import _native
from ..utils import observe

c_int, c_long, c_void_p, c_char_p = ctypes.c_int, ctypes.c_long, ctypes.c_void_p, ctypes.c_char_p
_PP = ctypes.POINTER(ctypes.c_void_p)
for _name, _res, _args in (
    ("dllm_nccl_version", c_int, []),
    ("dllm_nccl_unique_id", c_int, [c_char_p, c_int]),
    ("dllm_nccl_unique_id_bytes", c_int, []),
    ("dllm_nccl_comm_init", c_int, [c_int, c_int, c_char_p, c_int, _PP]),
    ("dllm_nccl_comm_split", c_int, [c_void_p, c_int, c_int, _PP]),
    ("dllm_nccl_comm_destroy", c_int, [c_void_p]),
    ("dllm_nccl_comm_abort", c_int, [c_void_p]),
    ("dllm_nccl_comm_async_error", c_int, [c_void_p]),
    ("dllm_nccl_all_reduce", c_int, [c_void_p, c_void_p, c_void_p, c_long, c_int, c_void_p]),
    ("dllm_nccl_all_gather", c_int, [c_void_p, c_void_p, c_void_p, c_long, c_int, c_void_p]),
    ("dllm_nccl_reduce_scatter", c_int, [c_void_p, c_void_p, c_void_p, c_long, c_int, c_void_p]),
    ("dllm_nccl_group_start", c_int, []),
    ("dllm_nccl_group_end", c_int, []),
    ("dllm_nccl_error_string", ctypes.c_char_p, [c_int]),
    ("dllm_stream_create", c_int, [c_int, _PP]),
    ("dllm_stream_destroy", c_int, [c_void_p]),
    ("dllm_event_create", c_int, [_PP]),
    ("dllm_event_destroy", c_int, [c_void_p]),
    ("dllm_event_record", c_int, [c_void_p, c_void_p]),
    ("dllm_stream_wait_event", c_int, [c_void_p, c_void_p]),
    ("dllm_event_query", c_int, [c_void_p]),
    ("dllm_event_synchronize", c_int, [c_void_p]),
):
    _native.register_optional(_name, _res, _args)

_DT = {torch.bfloat16: 0, torch.float32: 1, torch.float16: 2, torch.int32: 3, torch.int64: 4}
_COUNTER = itertools.count()


def _lib():
    return _native.lib()


def _check(rc: int, what: str) -> None:
    if rc != 0:
        msg = _lib().dllm_nccl_error_string(rc) if rc >= 1000 else b"hip error"
        raise RuntimeError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


class _Event:
    __slots__ = ("h",)

    def __init__(self):
        h = ctypes.c_void_p()
        _check(_lib().dllm_event_create(ctypes.byref(h)), "hipEventCreate")
        self.h = h.value

    def __del__(self):
        try:
            if self.h:
                _lib().dllm_event_destroy(self.h)
        except Exception:
            pass


class NativeWork:
    """Completion handle: ``wait()`` = current HIP stream waits on the collective's completion event."""

    def __init__(self, ev: _Event, keep=(), span=None):
        self.ev, self.keep = ev, keep
        self.span = span  # (start, end) timing events on the communicator stream while a CommObserver is active

    def wait(self):
        _check(_lib().dllm_stream_wait_event(torch.cuda.current_stream().cuda_stream, self.ev.h),
               "hipStreamWaitEvent")
        return True

    def is_completed(self) -> bool:
        return _lib().dllm_event_query(self.ev.h) == 1

    def synchronize(self) -> None:
        _check(_lib().dllm_event_synchronize(self.ev.h), "hipEventSynchronize")


NCCL_SPLIT_NOCOLOR = -1


class NativeGroup:
    """One RCCL communicator over ``ranks`` (global ranks) with its own stream.  Collective over the
    members only (non-members do not participate), bootstrapped through the default store -- or carved out
    of a parent communicator with ``ncclCommSplit`` (``NativeGroup.split``, how 2-D meshes are built)."""

    def __init__(self, ranks: list[int], tag: str, device: torch.device, store=None, priority: int = 0,
                 _comm: int | None = None, avoid: list | None = None):
        self.ranks = list(ranks)
        me = dist.get_rank()
        if me not in self.ranks:
            raise ValueError("NativeGroup built on a non-member rank")
        self.rank, self._size = self.ranks.index(me), len(self.ranks)
        self.device = device
        if _comm is None:
            store = store or dist.distributed_c10d._get_default_store()
            key = f"dllm/rccl/{tag}/{'-'.join(map(str, self.ranks))}"
            nbytes = _lib().dllm_nccl_unique_id_bytes()
            if self.rank == 0:
                buf = ctypes.create_string_buffer(nbytes)
                _check(_lib().dllm_nccl_unique_id(buf, nbytes), "ncclGetUniqueId")
                uid = buf.raw
                store.set(key, uid)
            else:
                uid = store.get(key)
            comm = ctypes.c_void_p()
            _check(_lib().dllm_nccl_comm_init(self._size, self.rank, uid, device.index, ctypes.byref(comm)),
                   "ncclCommInitRank")
            _comm = comm.value
        self.comm = _comm
        if avoid is not None:
            # a stream on a hardware queue none of ``avoid`` (stream handles; 0 = compute) uses (utils/streams.py)
            from ..utils.streams import create_stream_off

            self.stream = create_stream_off(device, avoid, priority)
        else:
            st = ctypes.c_void_p()
            _check(_lib().dllm_stream_create(priority, ctypes.byref(st)), "hipStreamCreate")
            self.stream = st.value

    @classmethod
    def split(cls, parent: "NativeGroup", groups: list[list[int]], device: torch.device,
              avoid: list | None = None) -> "NativeGroup | None":
        """``ncclCommSplit`` of ``parent`` into ``groups`` (lists of global ranks, disjoint): collective over
        ALL of the parent's ranks; returns this rank's new group (its own communicator and stream), or None
        if this rank is in none of them (it passes NCCL_SPLIT_NOCOLOR)."""
        me = dist.get_rank()
        color, mine = NCCL_SPLIT_NOCOLOR, None
        for i, g in enumerate(groups):
            if me in g:
                color, mine = i, g
        comm = ctypes.c_void_p()
        _check(_lib().dllm_nccl_comm_split(parent.comm, color, mine.index(me) if mine else 0, ctypes.byref(comm)),
               "ncclCommSplit")
        if mine is None:
            return None
        return cls(mine, "split", device, _comm=comm.value, avoid=avoid)

    def size(self) -> int:
        return self._size

    # -- plumbing --------------------------------------------------------------------------------------
    def _span_event(self):
        """Under a CommObserver: a timing event recorded on this communicator's own stream, so the observer gets
        the collective's execution interval (after its input wait, around its kernel) instead of issue ->
        completion as seen from other streams."""
        if observe.active() is None:
            return None
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.ExternalStream(self.stream, device=self.device))
        return ev

    def _enqueue(self, fn, keep):
        cur = torch.cuda.current_stream(self.device).cuda_stream
        ev_in = _Event()
        _check(_lib().dllm_event_record(ev_in.h, cur), "hipEventRecord")
        _check(_lib().dllm_stream_wait_event(self.stream, ev_in.h), "hipStreamWaitEvent")
        t_s = self._span_event()
        fn(self.stream)
        t_e = self._span_event()
        ev_out = _Event()
        _check(_lib().dllm_event_record(ev_out.h, self.stream), "hipEventRecord")
        return NativeWork(ev_out, keep=(ev_in,) + tuple(keep), span=(t_s, t_e) if t_s is not None else None)

    # -- collectives (SUM) -----------------------------------------------------------------------------
    def all_reduce(self, t: torch.Tensor) -> NativeWork:
        dt = _DT[t.dtype]

        def run(s):
            _check(_lib().dllm_nccl_all_reduce(self.comm, t.data_ptr(), t.data_ptr(), t.numel(), dt, s),
                   "ncclAllReduce")

        return self._enqueue(run, (t,))

    def all_reduce_inline(self, t: torch.Tensor) -> None:
        """Synchronous form: the all-reduce on the caller's current stream itself (no event hop to this group's
        stream and back); the result is ready for whatever the current stream runs next."""
        cur = torch.cuda.current_stream(self.device).cuda_stream
        _check(_lib().dllm_nccl_all_reduce(self.comm, t.data_ptr(), t.data_ptr(), t.numel(), _DT[t.dtype], cur),
               "ncclAllReduce")

    def all_gather_into(self, out: torch.Tensor, shard: torch.Tensor) -> NativeWork:
        if out.numel() != shard.numel() * self._size:
            raise ValueError("all_gather_into: size mismatch")
        dt = _DT[shard.dtype]

        def run(s):
            _check(_lib().dllm_nccl_all_gather(self.comm, shard.data_ptr(), out.data_ptr(), shard.numel(), dt, s),
                   "ncclAllGather")

        return self._enqueue(run, (out, shard))

    def reduce_scatter_into(self, out: torch.Tensor, full: torch.Tensor) -> NativeWork:
        if full.numel() != out.numel() * self._size:
            raise ValueError("reduce_scatter_into: size mismatch")
        dt = _DT[full.dtype]

        def run(s):
            _check(_lib().dllm_nccl_reduce_scatter(self.comm, full.data_ptr(), out.data_ptr(), out.numel(), dt, s),
                   "ncclReduceScatter")

        return self._enqueue(run, (out, full))

    # -- grouped collectives (ncclGroupStart/End: one fused launch, one completion event) ---------------
    def _enqueue_group(self, calls, keep):
        cur = torch.cuda.current_stream(self.device).cuda_stream
        ev_in = _Event()
        _check(_lib().dllm_event_record(ev_in.h, cur), "hipEventRecord")
        _check(_lib().dllm_stream_wait_event(self.stream, ev_in.h), "hipStreamWaitEvent")
        t_s = self._span_event()
        _check(_lib().dllm_nccl_group_start(), "ncclGroupStart")
        try:
            for fn in calls:
                fn(self.stream)
        finally:
            # the collectives are launched at GroupEnd, so the completion event is recorded after it
            _check(_lib().dllm_nccl_group_end(), "ncclGroupEnd")
        t_e = self._span_event()
        ev_out = _Event()
        _check(_lib().dllm_event_record(ev_out.h, self.stream), "hipEventRecord")
        return NativeWork(ev_out, keep=(ev_in,) + tuple(keep), span=(t_s, t_e) if t_s is not None else None)

    def all_gather_into_many(self, pairs) -> NativeWork:
        """Several all-gathers ``(out, shard)`` as one group (e.g. a layer's W1 and W2 shards)."""
        calls, keep = [], []
        for out, shard in pairs:
            if out.numel() != shard.numel() * self._size:
                raise ValueError("all_gather_into_many: size mismatch")

            def run(s, out=out, shard=shard):
                _check(_lib().dllm_nccl_all_gather(self.comm, shard.data_ptr(), out.data_ptr(), shard.numel(),
                                                   _DT[shard.dtype], s), "ncclAllGather")

            calls.append(run)
            keep += [out, shard]
        return self._enqueue_group(calls, keep)

    def reduce_scatter_into_many(self, pairs) -> NativeWork:
        """Several reduce-scatters ``(out, full)`` as one group (a layer's W1 and W2 gradients)."""
        calls, keep = [], []
        for out, full in pairs:
            if full.numel() != out.numel() * self._size:
                raise ValueError("reduce_scatter_into_many: size mismatch")

            def run(s, out=out, full=full):
                _check(_lib().dllm_nccl_reduce_scatter(self.comm, full.data_ptr(), out.data_ptr(), out.numel(),
                                                       _DT[full.dtype], s), "ncclReduceScatter")

            calls.append(run)
            keep += [out, full]
        return self._enqueue_group(calls, keep)

    def check_async_error(self) -> None:
        _check(_lib().dllm_nccl_comm_async_error(self.comm), "ncclCommGetAsyncError")

    def abort(self) -> None:
        """Error path: abort the communicator without waiting for outstanding work."""
        if self.comm:
            _lib().dllm_nccl_comm_abort(self.comm)
            self.comm = None

    def destroy(self, abort: bool = False) -> None:
        if self.comm:
            torch.cuda.synchronize(self.device)
            (_lib().dllm_nccl_comm_abort if abort else _lib().dllm_nccl_comm_destroy)(self.comm)
            self.comm = None
        if self.stream:
            _lib().dllm_stream_destroy(self.stream)
            self.stream = None


def new_role_group(ranks: list[int], role: str, device: torch.device) -> NativeGroup | None:
    """Create the native communicator for ``role`` if this rank belongs to ``ranks`` (else None)."""
    if dist.get_rank() not in ranks:
        return None
    return NativeGroup(ranks, f"{role}/{next(_COUNTER)}", device)


def new_world_group(device: torch.device) -> NativeGroup:
    """The job-wide communicator every mesh communicator is split from (collective over all ranks)."""
    return NativeGroup(list(range(dist.get_world_size())), f"world/{next(_COUNTER)}", device)
