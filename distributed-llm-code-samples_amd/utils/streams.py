"""Where the engine's side streams (weight-gradient, shard-optimizer, FSDP tail) get their hardware queues.

HIP gives a process at most ``GPU_MAX_HW_QUEUES`` hardware queues per priority level; once they are taken it puts
each new stream on the least-used existing queue, picked in pointer order.  torch's stream pool (32 streams, created
together at its first use) and RCCL's internal streams take them early in a job with a process group, so a side
stream can land on the compute stream's queue and the two streams' kernels serialise
(``profiles/r3/hw_queue_collision_trace_r3.txt``: the weight-gradient stream lost all of its overlap that way).

``DLLM_SIDE_STREAMS`` picks the remedy:
  * ``role`` (default since round 4): the FSDP side stream (shard updates and the step-boundary update -> gather
    chains) is a native high-priority stream, every other role a torch pool stream.  On the pool, the FSDP stream
    shared a hardware queue with ProcessGroupNCCL's collective streams, so a collective's completion marker waited
    behind a shard update and the compute stream behind the marker: forced-comm hybrid (FSDP x TP) 172.7 / 172.9 vs
    173.5 / 174.2 ms with its exposed_ms_diff 0.8-1.0 vs 3.8-3.9 ms, FSDP 32.39 / 32.45 vs 32.44 / 32.72 ms, one box
    (``profiles/r4/side_streams_high_fsdp_r4.txt``).  ZeRO's optimizer stream loses at high priority (32.54-32.60 vs
    32.25 ms) and stays on the pool;
  * ``pool``: torch pool streams for every role;
  * ``high``: native non-blocking streams at high priority (``csrc/comm.cpp: dllm_stream_create``).  HIP keeps a
    separate queue set per priority, and nothing else in the process asks for high-priority queues, so these
    never share the compute stream's (normal-priority) queue;
  * ``auto``: ``high`` for the weight-gradient stream only (it runs only in steps without collectives).  It recovers
    a step next to a live communicator (29.86-29.96 vs 30.32-30.43 ms) and is neutral without one, but collective
    methods run later in the same process lose 5-14 % (``profiles/r3/side_streams_auto_r3.txt``); ``high`` costs
    them about as much (DDP +6 %, hybrid +10 %, ``side_streams_high_priority_r3.txt``).  A high-priority queue that
    exists is enough for that loss; why is not pinned down.  Hence not the default.

More hardware queues are not the remedy: at 32 the hardware scheduler time-slices them and the communicating
methods collapse (``profiles/r3/hw_queues_32_vs_16_r3.txt``); queues that own a CU mask cost 2 % on the headline
(``profiles/r3/dedicated_cu_mask_queues_r3.txt``).  Native handles live for the process.

**Reserving the compute stream's queue** (round 4, ``reserve_compute_queue``).  The compute stream is torch's default
(HIP null) stream.  At process start, before torch's stream pool, any process group or RCCL communicator exists,
``csrc/elementwise.hip: dllm_queue_reserve`` creates non-blocking candidate streams one by one and measures for each
whether it landed on the compute stream's hardware queue (a spinning wave on the compute stream, a timestamp kernel on
the candidate: a shared queue runs them in order).  Candidates on the compute queue are kept for the process, the
others destroyed, so the compute queue carries the highest use count and HIP's least-used placement puts every later
stream -- torch's pool (engine side streams, ProcessGroupNCCL's collective streams) and RCCL's own -- on the other
queues.  ``queue_report`` re-measures any set of streams against the compute stream (bench.py reports it per method).
Works at HIP's default of 4 queues per process; the package no longer changes ``GPU_MAX_HW_QUEUES`` (bench.py
``--hw_queues`` sets it explicitly for a run).
"""
from __future__ import annotations

import ctypes
import os
import weakref

import torch

from .. import _native

_native.register_optional("dllm_stream_create", ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)])
_RESERVED: dict[int, int] = {}
PROBE_SPIN_US = 100
_native.register_optional("dllm_stream_destroy", ctypes.c_int, [ctypes.c_void_p])
_HANDLES: dict[tuple[int, str], torch.cuda.ExternalStream] = {}


HIGH_ROLES_AUTO = ("wgrad",)
HIGH_ROLES = ("fsdp",)


def mode() -> str:
    m = os.environ.get("DLLM_SIDE_STREAMS", "role")
    if m not in ("role", "pool", "high", "auto"):
        raise ValueError(f"DLLM_SIDE_STREAMS={m!r}: expected role | pool | high | auto")
    return m


def high_priority(role: str) -> bool:
    m = mode()
    return (m == "high" or (m == "auto" and role in HIGH_ROLES_AUTO)
            or (m == "role" and role in HIGH_ROLES))


def _destroy(handle: int, idx: int) -> None:
    try:
        torch.cuda.synchronize(idx)
        _native.lib().dllm_stream_destroy(handle)
    except Exception:
        pass


def side_stream(device: torch.device, role: str, owner=None) -> torch.cuda.Stream:
    """The stream for side-work ``role`` on ``device``.  A high-priority one is native; with ``owner`` it is destroyed
    (its hardware queue released) when the owner is collected, else it is cached for the process."""
    if not high_priority(role):
        return torch.cuda.Stream(device=device)
    idx = device.index if device.index is not None else torch.cuda.current_device()
    key = (idx, role)
    if owner is None and key in _HANDLES:
        return _HANDLES[key]
    lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
    h = ctypes.c_void_p()
    with torch.cuda.device(idx):
        rc = _native.lib().dllm_stream_create(int(hi), ctypes.byref(h))
    if rc != 0 or not h.value:
        raise RuntimeError(f"hipStreamCreateWithPriority failed ({rc})")
    st = torch.cuda.ExternalStream(h.value, device=torch.device("cuda", idx))
    if owner is None:
        _HANDLES[key] = st
    else:
        weakref.finalize(owner, _destroy, h.value, idx)
    return st


def reserve_compute_queue(device: torch.device | int | None = None, candidates: int = 128) -> int:
    """Keep later streams off the compute (null) stream's hardware queue (see the module docstring); once per device
    and process, before anything else creates streams.  Returns the number of blocker streams kept (0 when disabled
    with ``DLLM_QUEUE_RESERVE=0``)."""
    if os.environ.get("DLLM_QUEUE_RESERVE", "1") == "0":
        return 0
    idx = _index(device)
    if idx not in _RESERVED:
        with torch.cuda.device(idx):
            n = _native.lib().dllm_queue_reserve(None, int(candidates), PROBE_SPIN_US)
        if n < 0:
            raise RuntimeError(f"dllm_queue_reserve failed ({n})")
        _RESERVED[idx] = n
    return _RESERVED[idx]


def _index(device) -> int:
    if device is None:
        return torch.cuda.current_device()
    if isinstance(device, int):
        return device
    return device.index if device.index is not None else torch.cuda.current_device()


def shares_compute_queue(stream: torch.cuda.Stream, device=None, tries: int = 3) -> bool:
    """Whether ``stream`` runs on the compute (null) stream's hardware queue (measured; synchronises both).  The
    majority of ``tries`` probes decides: a single probe can read "shared" when the candidate's dispatch is merely
    late (seen once in a round-4 methods run, against a consistent "own queue" for the same stream)."""
    votes = 0
    with torch.cuda.device(_index(device)):
        for _ in range(tries):
            r = _native.lib().dllm_queue_shared(None, ctypes.c_void_p(stream.cuda_stream), PROBE_SPIN_US)
            if r < 0:
                raise RuntimeError(f"dllm_queue_shared failed ({r})")
            votes += r
    return 2 * votes > tries


def shares_queue(a: int | None, b: int | None, device=None, tries: int = 3) -> bool:
    """Whether raw HIP streams ``a`` and ``b`` (handles; None / 0 = the null, i.e. compute, stream) run on one hardware
    queue (measured; majority of ``tries`` probes; synchronises both).  ``a`` spins, then ``b`` stamps: a shared queue
    runs them in order."""
    if (a or 0) == (b or 0):
        return True
    votes = 0
    with torch.cuda.device(_index(device)):
        for _ in range(tries):
            r = _native.lib().dllm_queue_shared(ctypes.c_void_p(a or None), ctypes.c_void_p(b or None), PROBE_SPIN_US)
            if r < 0:
                raise RuntimeError(f"dllm_queue_shared failed ({r})")
            votes += r
    return 2 * votes > tries


_QUEUE_BLOCKERS: dict[int, list[int]] = {}


def create_stream_off(device, avoid: list, priority: int = 0, max_tries: int = 16) -> int:
    """A new native stream (handle) on a hardware queue that none of the ``avoid`` streams (handles; 0 = compute) uses.
    Candidates that land on an avoided queue are kept for the process as blockers -- they raise that queue's use
    count, so HIP's least-used placement puts the next candidate elsewhere (the compute-queue reservation's
    mechanism).  After ``max_tries`` the last candidate is returned as is (``role_queue_report`` then shows the
    conflict)."""
    idx = _index(device)
    blockers = _QUEUE_BLOCKERS.setdefault(idx, [])
    h = None
    for _ in range(max_tries):
        st = ctypes.c_void_p()
        with torch.cuda.device(idx):
            rc = _native.lib().dllm_stream_create(int(priority), ctypes.byref(st))
            if rc != 0 or not st.value:
                raise RuntimeError(f"hipStreamCreateWithPriority failed ({rc})")
            h = st.value
            # first use acquires the queue: not part of the timed probes
            _native.lib().dllm_queue_shared(ctypes.c_void_p(h), ctypes.c_void_p(h), 0)
        if not any(shares_queue(a, h, idx) for a in avoid):
            return h
        blockers.append(h)
    return h


class PoolCursor:
    """torch's per-device pool of normal-priority streams, as an ordered ring with a known position.

    ``torch.cuda.Stream()`` and ProcessGroupNCCL's collective streams (``at::cuda::getStreamFromPool``) are handed out
    round-robin from one per-device counter over 32 streams.  Walking the ring once gives its order and the counter's
    position, so the stream the NEXT process group will take is known (``peek``), can be skipped when it sits on an
    unwanted hardware queue (``skip``), and what a group creation actually took is checked afterwards (``taken``)."""

    def __init__(self, device):
        self.idx = _index(device)
        first = torch.cuda.Stream(device=self.idx)
        ring = [first]
        while True:
            st = torch.cuda.Stream(device=self.idx)
            if st.cuda_stream == first.cuda_stream:
                break
            ring.append(st)
            if len(ring) > 256:
                raise RuntimeError("torch stream pool is not a ring")
        self.ring = ring
        self.pos = 1 % len(ring)   # ``first`` was handed out twice: the counter now points past it

    def peek(self) -> torch.cuda.Stream:
        return self.ring[self.pos]

    def skip(self) -> None:
        torch.cuda.Stream(device=self.idx)
        self.pos = (self.pos + 1) % len(self.ring)

    def taken(self) -> torch.cuda.Stream | None:
        """After something drew from the pool: if it drew exactly one stream (the one ``peek`` showed), return it
        (the cursor moves past it and past this check's own draw), else None (cursor resynchronised)."""
        expect = self.ring[self.pos]
        st = torch.cuda.Stream(device=self.idx)
        n = len(self.ring)
        at = next(i for i in range(n) if self.ring[i].cuda_stream == st.cuda_stream)
        took = (at - self.pos) % n
        self.pos = (at + 1) % n
        return expect if took == 1 else None

    def steer(self, avoid: list, max_skips: int = 32) -> torch.cuda.Stream:
        """Skip pool streams until the next one shares no hardware queue with ``avoid`` (handles; 0 = compute)."""
        for _ in range(max_skips):
            if not any(shares_queue(a, self.peek().cuda_stream, self.idx) for a in avoid):
                break
            self.skip()
        return self.peek()


# role pairs that must not share a hardware queue: any communicator role with the compute stream, and the FSDP
# gather with the FSDP reduce-scatter (the reference's serialisation, train_ffns.py:14, :252-256)
MUST_DIFFER = (("compute", "dp_ag"), ("compute", "dp_rs"), ("compute", "dp_ar"), ("compute", "tp"),
               ("dp_ag", "dp_rs"))


def role_queue_report(device, named: dict) -> dict:
    """Pairwise hardware-queue sharing among ``named`` streams ({name: handle or stream}; "compute" = the null stream
    is added; None entries are reported as unknown).  ``role_queue_conflicts``: the ``MUST_DIFFER`` pairs (plus every
    stream against compute) that share a queue."""
    idx = _index(device)
    h = {"compute": 0}
    unknown = []
    for n, st in named.items():
        if st is None:
            unknown.append(n)
            continue
        h[n] = st if isinstance(st, int) else st.cuda_stream
    names = list(h)
    sharing = []
    for i in range(len(names)):
        for j in range(i + 1, len(names)):
            a, b = names[i], names[j]
            if shares_queue(h[a], h[b], idx):
                sharing.append([a, b])
    must = {tuple(p) for p in MUST_DIFFER} | {("compute", n) for n in names if n != "compute"}
    conflicts = [p for p in sharing if tuple(p) in must or tuple(p[::-1]) in must]
    return {"role_queue_conflicts": conflicts, "queue_sharing_pairs": sharing, "unknown_streams": unknown}


def queue_report(device, streams: dict, pool: bool = True) -> dict:
    """Which of ``streams`` ({name: stream}, None entries skipped) -- plus, with ``pool``, torch's 32 normal-priority
    pool streams, which ProcessGroupNCCL's collective streams come from -- share the compute stream's hardware queue.
    Idle GPU expected (each probe synchronises)."""
    idx = _index(device)
    shared = [n for n, st in streams.items() if st is not None and st.cuda_stream != 0 and shares_compute_queue(st, idx)]
    npool = 0
    if pool:
        seen = set()
        for _ in range(32):
            st = torch.cuda.Stream(device=idx)
            if st.cuda_stream in seen:
                continue
            seen.add(st.cuda_stream)
            npool += shares_compute_queue(st, idx)
    return {"reserved_blockers": _RESERVED.get(idx, 0), "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES",
                                                                                            "hip default"),
            "side_streams_on_compute_queue": shared, "pool_streams_on_compute_queue": npool,
            "compute_queue_exclusive": not shared and npool == 0}
