"""Python side of the custom two-shot xGMI all-reduce (``csrc/car.hip``) for TP activations.

``CustomAllReduce`` registers one buffer per rank (IN and OUT regions + signal slots), exchanges the
hipIpc handles through the job's ``torch.distributed`` store, maps every peer's buffer, and then
all-reduces a tensor in place on the current HIP stream: copy-in, flag barrier, reduce-scatter + push
over all peers at once, flag barrier, copy-out.  Every rank sums peers in the same order, so all ranks
hold bitwise identical results.  It is an opt-in backend for the ``tp`` activation all-reduces
(``TrainConfig.tp_allreduce = "custom"``); gradient collectives stay on RCCL.

Buffers up to ``cap_bytes`` (default: the largest TP message the engine sends, ``[T, D]`` in the compute
dtype).  The barrier spins are bounded: ``check()`` raises if one timed out.

Zero-copy (``arena_bytes``): the engine carves the TP-exchanged activations (layer outputs, input gradients) out of
an arena every peer maps; the producing GEMM writes its partial there and the all-reduce runs in place (the sum is
written back into every peer's range), so the copy-in / copy-out passes disappear.
"""
from __future__ import annotations

import ctypes
import itertools

import torch
import torch.distributed as dist

from .. import _native

c_int, c_long, c_void_p, c_char_p, c_double = ctypes.c_int, ctypes.c_long, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_double
_PP = ctypes.POINTER(ctypes.c_void_p)
for _name, _res, _args in (
    ("dllm_car_create", c_int, [c_int, c_int, c_long, c_int, _PP]),
    ("dllm_car_handle_bytes", c_int, []),
    ("dllm_car_get_handle", c_int, [c_void_p, c_char_p, c_int]),
    ("dllm_car_open", c_int, [c_void_p, c_char_p]),
    ("dllm_car_set_peer", c_int, [c_void_p, c_int, c_void_p]),
    ("dllm_car_all_reduce", c_int, [c_void_p, c_void_p, c_long, c_int, c_double, c_void_p]),
    ("dllm_car_error", c_int, [c_void_p]),
    ("dllm_car_destroy", c_int, [c_void_p]),
    ("dllm_car_arena_handle", c_int, [c_void_p, c_char_p, c_int, ctypes.POINTER(c_long)]),
    ("dllm_car_attach_arena", c_int, [c_void_p, c_void_p, c_long, c_char_p, ctypes.POINTER(c_long)]),
    ("dllm_car_set_peer_arena", c_int, [c_void_p, c_int, c_void_p]),
    ("dllm_car_all_reduce_arena", c_int, [c_void_p, c_long, c_long, c_int, c_double, c_void_p]),
):
    _native.register_optional(_name, _res, _args)

_DT = {torch.bfloat16: 0, torch.float32: 1}
_COUNTER = itertools.count()


class _Done:
    def wait(self):
        return True

    def is_completed(self):
        return True


class CustomAllReduce:
    """Custom all-reduce over ``ranks`` (global ranks; this rank must be one of them)."""

    def __init__(self, ranks: list[int], device: torch.device, cap_bytes: int, store=None, tag: str = "",
                 timeout_s: float = 30.0, _local_peers: list | None = None, _local_rank: int | None = None,
                 arena_bytes: int = 0):
        """``arena_bytes`` > 0: also allocate a zero-copy arena of that size (``arena_view``), mapped by every peer;
        tensors carved from it are all-reduced in place (no staging copies).  ``cap_bytes`` bounds the staged
        (copy-in / copy-out) path for tensors outside the arena."""
        self.ranks = list(ranks)
        self.arena = None
        self._arena_next = 0
        self.n = len(self.ranks)
        if not 1 <= self.n <= 8:
            raise ValueError("custom all-reduce supports 1..8 ranks")
        self.device, self.timeout_s = device, float(timeout_s)
        self.cap = (int(cap_bytes) + 15) // 16 * 16
        lib = _native.lib()
        me = _local_rank if _local_rank is not None else self.ranks.index(dist.get_rank())
        self.rank = me
        st = ctypes.c_void_p()
        _native.check(lib.dllm_car_create(me, self.n, self.cap, device.index, ctypes.byref(st)), "dllm_car_create")
        self.st = st.value
        if arena_bytes > 0:
            # identical size and carving order on every rank -> identical offsets (the in-place protocol needs it)
            self.arena = torch.empty((int(arena_bytes) + 255) // 256 * 256, dtype=torch.uint8, device=device)
        if _local_peers is not None:  # single-process testing: peers are other CustomAllReduce objects
            if self.arena is not None:
                _native.check(lib.dllm_car_attach_arena(self.st, self.arena.data_ptr(), self.arena.numel(), None, None),
                              "dllm_car_attach_arena")
            return
        if self.n > 1:
            nb = lib.dllm_car_handle_bytes()
            buf = ctypes.create_string_buffer(nb)
            _native.check(lib.dllm_car_get_handle(self.st, buf, nb), "hipIpcGetMemHandle")
            store = store or dist.distributed_c10d._get_default_store()
            key = f"dllm/car/{tag or next(_COUNTER)}/{'-'.join(map(str, self.ranks))}"
            store.set(f"{key}/{me}", buf.raw)
            allh = b"".join(store.get(f"{key}/{p}") for p in range(self.n))
            _native.check(lib.dllm_car_open(self.st, allh), "hipIpcOpenMemHandle")
            if self.arena is not None:
                off = c_long()
                abuf = ctypes.create_string_buffer(nb)
                _native.check(lib.dllm_car_arena_handle(self.arena.data_ptr(), abuf, nb, ctypes.byref(off)),
                              "hipIpcGetMemHandle(arena)")
                store.set(f"{key}/arena/{me}", abuf.raw + int(off.value).to_bytes(8, "little", signed=True))
                recs = [store.get(f"{key}/arena/{p}") for p in range(self.n)]
                handles = b"".join(r[:nb] for r in recs)
                offs = (c_long * self.n)(*[int.from_bytes(r[nb:nb + 8], "little", signed=True) for r in recs])
                _native.check(lib.dllm_car_attach_arena(self.st, self.arena.data_ptr(), self.arena.numel(), handles,
                                                        offs), "hipIpcOpenMemHandle(arena)")
        elif self.arena is not None:
            _native.check(lib.dllm_car_attach_arena(self.st, self.arena.data_ptr(), self.arena.numel(), None, None),
                          "dllm_car_attach_arena")

    @classmethod
    def local_group(cls, n: int, device: torch.device, cap_bytes: int, timeout_s: float = 10.0):
        """n ranks inside ONE process sharing buffers directly.  Each rank must run on its own HIP stream
        AND those streams on distinct hardware queues (a process has GPU_MAX_HW_QUEUES of them, shared
        with other streams): two ranks serialised on one queue time out in the barrier."""
        objs = [cls(list(range(n)), device, cap_bytes, timeout_s=timeout_s, _local_peers=[], _local_rank=r)
                for r in range(n)]
        lib = _native.lib()
        for a in objs:
            for p, b in enumerate(objs):
                _native.check(lib.dllm_car_set_peer(a.st, p, b.st), "dllm_car_set_peer")
        return objs

    def size(self) -> int:
        return self.n

    def arena_view(self, shape, dtype: torch.dtype) -> torch.Tensor:
        """Carve the next 256-B aligned tensor out of the zero-copy arena (same order on every rank)."""
        if self.arena is None:
            raise RuntimeError("custom all-reduce created without an arena")
        n = 1
        for d in shape:
            n *= int(d)
        nbytes = n * torch.empty(0, dtype=dtype).element_size()
        start = self._arena_next
        if start + nbytes > self.arena.numel():
            raise ValueError(f"arena exhausted: {start} + {nbytes} > {self.arena.numel()}")
        self._arena_next = (start + nbytes + 255) // 256 * 256
        return self.arena[start:start + nbytes].view(dtype).view(*shape)

    def _arena_offset(self, t: torch.Tensor) -> int | None:
        """Byte offset of ``t`` inside the arena, or None when it lies outside."""
        if self.arena is None:
            return None
        a0, a1 = self.arena.data_ptr(), self.arena.data_ptr() + self.arena.numel()
        p = t.data_ptr()
        return p - a0 if a0 <= p and p + t.numel() * t.element_size() <= a1 else None

    def all_reduce(self, t: torch.Tensor, stream: torch.cuda.Stream | None = None):
        if t.dtype not in _DT:
            raise TypeError(f"custom all-reduce supports bf16/fp32, got {t.dtype}")
        if not t.is_contiguous():
            raise ValueError("custom all-reduce needs a contiguous tensor")
        nbytes = t.numel() * t.element_size()
        if nbytes % 16:
            raise ValueError(f"custom all-reduce: {nbytes} B (needs a multiple of 16)")
        if t.data_ptr() % 16:
            raise ValueError("custom all-reduce: the tensor must be 16-byte aligned (uint4 copies)")
        s = stream.cuda_stream if stream is not None else torch.cuda.current_stream(self.device).cuda_stream
        off = self._arena_offset(t)
        if off is not None:  # zero-copy: in place on the arena range (same offset on every rank)
            _native.check(_native.lib().dllm_car_all_reduce_arena(self.st, off, nbytes, _DT[t.dtype], self.timeout_s,
                                                                  s), "dllm_car_all_reduce_arena")
            return _Done()
        if nbytes > self.cap:
            raise ValueError(f"custom all-reduce: {nbytes} B outside the arena exceeds the staging cap {self.cap}")
        _native.check(_native.lib().dllm_car_all_reduce(self.st, t.data_ptr(), nbytes, _DT[t.dtype], self.timeout_s, s),
                      "dllm_car_all_reduce")
        return _Done()

    def all_reduce_async(self, t: torch.Tensor):
        """Enqueue on this object's own stream behind the current stream; ``wait()`` makes the current
        stream wait for the result (the TP dx all-reduce overlapping the dW1 GEMM)."""
        from . import comm

        if comm.eliding():
            return comm.Elided(t)
        cur = torch.cuda.current_stream(self.device)
        if getattr(self, "_stream", None) is None:
            self._stream = torch.cuda.Stream(device=self.device)
        self._stream.wait_stream(cur)
        self.all_reduce(t, stream=self._stream)
        ev = torch.cuda.Event()
        ev.record(self._stream)
        t.record_stream(self._stream)

        class _Work:
            def wait(_self):
                torch.cuda.current_stream(self.device).wait_event(ev)
                return True

            def is_completed(_self):
                return ev.query()

        return _Work()

    def check(self) -> None:
        """Raise if a barrier timed out (synchronises the device first)."""
        torch.cuda.synchronize(self.device)
        e = _native.lib().dllm_car_error(self.st)
        if e != 0:
            raise RuntimeError(f"custom all-reduce barrier timed out (code {e})")

    def destroy(self) -> None:
        if self.st:
            _native.lib().dllm_car_destroy(self.st)
            self.st = None
        self.arena = None
