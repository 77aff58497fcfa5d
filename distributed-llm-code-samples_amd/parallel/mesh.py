"""Process bootstrap and the 2-D (data × tensor) device mesh.

Reference: ``init_process`` sets ``MASTER_ADDR=127.0.0.1``/``MASTER_PORT=29500`` and calls
``dist.init_process_group("nccl", rank, world_size=nGPUs)`` (train_ffns.py:121-127); every method uses
all GPUs on one axis and one process group, so FSDP's reduce-scatter serialises behind its prefetch
all-gather on the single NCCL stream (the author's TODO, train_ffns.py:14,252).

Here: one process per GPU (torchrun env or our own spawner), backend ``nccl`` (= RCCL over xGMI on ROCm)
or ``gloo`` (CPU plumbing), and a ``Mesh`` of ``dp × tp`` ranks (tp fastest-varying, so a TP group is a
block of neighbouring GPUs).  Each communication *role* gets its own process group — and therefore its
own RCCL communicator and HIP stream — so DDP gradient all-reduce, FSDP parameter all-gather, FSDP
gradient reduce-scatter and TP activation all-reduce can run concurrently with each other and with
compute.  Two interchangeable communicator implementations: torch ProcessGroupNCCL (``comm_backend=
"torch"``, default) or the native C++ RCCL layer (``"native"``: ``csrc/comm.cpp`` + ``parallel/rccl.py``,
one ncclComm_t + one hipStream_t per role, store-bootstrapped, event-synchronised):

    role      ranks        used by
    dp_ar     dp group     DDP bucketed gradient all-reduce
    dp_ag     dp group     FSDP parameter all-gather (prefetch)
    dp_rs     dp group     FSDP gradient reduce-scatter
    tp        tp group     Megatron activation / input-grad all-reduce (or SP reduce-scatter/all-gather)
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass, field

import torch
import torch.distributed as dist

ROLES = ("dp_ar", "dp_ag", "dp_rs", "tp")


def init_distributed(backend: str, rank: int | None = None, world_size: int | None = None,
                     master_addr: str | None = None, master_port: int | None = None,
                     timeout_s: float = 600.0) -> tuple[int, int]:
    """Initialise the default process group from explicit args or the torchrun environment."""
    if dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    rank = int(os.environ.get("RANK", 0)) if rank is None else rank
    world_size = int(os.environ.get("WORLD_SIZE", 1)) if world_size is None else world_size
    os.environ["MASTER_ADDR"] = master_addr or os.environ.get("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(master_port or os.environ.get("MASTER_PORT", "29500"))
    kw = {}
    if backend == "nccl":
        local = int(os.environ.get("LOCAL_RANK", rank))
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
        # keep RCCL's / the process groups' streams off the compute stream's hardware queue (utils/streams.py);
        # must precede the communicators (idempotent: bench.py may have reserved already)
        from ..utils.streams import reserve_compute_queue

        reserve_compute_queue(torch.cuda.current_device())
        # eager communicator creation (device_id) unless DLLM_NCCL_EAGER=0: then RCCL builds it at the first collective
        if os.environ.get("DLLM_NCCL_EAGER", "1") != "0":
            kw["device_id"] = torch.device("cuda", torch.cuda.current_device())
    dist.init_process_group(backend, rank=rank, world_size=world_size,
                            timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return rank, world_size


@dataclass
class Mesh:
    """``world = dp × tp`` ranks; ``rank = dp_rank * tp + tp_rank``."""

    dp: int = 1
    tp: int = 1
    rank: int = 0
    groups: dict = field(default_factory=dict)
    dp_ranks: list = field(default_factory=list)
    tp_ranks: list = field(default_factory=list)
    native_world: object = None  # native backend: the communicator the role communicators are split from
    # the HIP stream each role communicator runs on ({role: raw handle}, None = not identified); see _queue_plan
    role_streams: dict = field(default_factory=dict)

    @property
    def world(self) -> int:
        return self.dp * self.tp

    @property
    def dp_rank(self) -> int:
        return self.rank // self.tp

    @property
    def tp_rank(self) -> int:
        return self.rank % self.tp

    def group(self, role: str):
        return self.groups.get(role)

    def destroy(self, abort: bool = False) -> None:
        """Tear down native communicators (torch process groups are destroyed with the default PG).
        ``abort``: error path -- ``ncclCommAbort`` instead of a synchronising destroy, so a rank whose
        peer died does not block in teardown."""
        from .car import CustomAllReduce
        from .rccl import NativeGroup

        seen = set()
        for g in self.groups.values():
            if isinstance(g, CustomAllReduce) and id(g) not in seen:
                seen.add(id(g))
                g.destroy()
                continue
            if isinstance(g, NativeGroup) and id(g) not in seen:
                seen.add(id(g))
                if abort:
                    g.abort()
                else:
                    g.destroy()
        self.groups.clear()
        if self.native_world is not None:
            if abort:
                self.native_world.abort()
            else:
                self.native_world.destroy()
            self.native_world = None

    @classmethod
    def build(cls, dp: int, tp: int, separate_streams: bool = True, force: bool = False,
              comm_backend: str = "torch", device: torch.device | None = None) -> "Mesh":
        """Create the role process groups (collective: every rank must call it with the same args).

        ``force`` also creates groups for axes of size 1 (used to exercise the RCCL code paths with a
        single GPU: a size-1 communicator still runs real collectives and stream waits)."""
        world = dist.get_world_size() if dist.is_initialized() else 1
        rank = dist.get_rank() if dist.is_initialized() else 0
        if dp * tp != world:
            raise ValueError(f"mesh dp={dp} x tp={tp} != world size {world}")
        m = cls(dp=dp, tp=tp, rank=rank)
        m.dp_ranks = [d * tp + m.tp_rank for d in range(dp)]
        m.tp_ranks = [m.dp_rank * tp + t for t in range(tp)]
        if not dist.is_initialized() or (world == 1 and not force):
            return m
        # Distinct hardware queues per role: the FSDP gather and reduce-scatter must not share
        # one, or the reference's serialisation (train_ffns.py:14, :252) just moves down to the queue; no role may
        # share the compute stream's.  ``avoid[role]`` = the roles whose streams its stream must not queue with.
        on_gpu = device is not None and device.type == "cuda" and os.environ.get("DLLM_ROLE_QUEUES", "1") != "0"
        avoid = {"dp_ar": ["compute"], "dp_ag": ["compute"], "dp_rs": ["compute", "dp_ag"], "tp": ["compute"]}

        def handles(role):
            return [0 if r == "compute" else m.role_streams.get(r) for r in avoid[role]
                    if r == "compute" or m.role_streams.get(r)]

        if comm_backend == "native":
            # one job-wide RCCL communicator (store-bootstrapped uniqueId), then every role communicator is
            # ncclCommSplit from it: color = this rank's dp group (dp roles) or tp group (tp role), key = its
            # position in that group -- the 2-D mesh is carved out of one bootstrap
            from .rccl import NativeGroup, new_world_group

            dev = device or torch.device("cuda", torch.cuda.current_device())
            world_comm = new_world_group(dev)
            m.native_world = world_comm
            dp_groups = [[d * tp + t for d in range(dp)] for t in range(tp)]
            tp_groups = [[d * tp + t for t in range(tp)] for d in range(dp)]
            for role in ROLES:
                axis = dp if role.startswith("dp") else tp
                if axis == 1 and not force:
                    continue
                if not separate_streams and role in ("dp_ag", "dp_rs") and "dp_ar" in m.groups:
                    m.groups[role] = m.groups["dp_ar"]
                    continue
                m.groups[role] = NativeGroup.split(world_comm, tp_groups if role == "tp" else dp_groups, dev,
                                                   avoid=handles(role) if on_gpu else None)
                if m.groups[role] is not None:
                    m.role_streams[role] = m.groups[role].stream
            return m
        cursor = None
        if on_gpu and dist.get_backend() == "nccl":
            from ..utils.streams import PoolCursor

            cursor = PoolCursor(device)

        def new_group(ranks, role):
            """dist.new_group + (nccl, GPU) steer torch's stream pool so the communicator's stream lands on an allowed
            queue, then identify the stream it took (a 1-element all-reduce makes sure the communicator exists)."""
            member = rank in ranks
            if cursor is not None and member:
                cursor.steer(handles(role))
            g = dist.new_group(ranks)
            if cursor is not None and member:
                t = torch.zeros(1, device=device)
                dist.all_reduce(t, group=g)
                torch.cuda.synchronize(device)
                st = cursor.taken()
                m.role_streams[role] = st.cuda_stream if st is not None else None
            return g

        # every rank creates every group in the same order (new_group is collective)
        for role in ROLES:
            if role.startswith("dp"):
                if dp == 1 and not force:
                    continue
                if not separate_streams and role != "dp_ar" and "dp_ar" in m.groups:
                    m.groups[role] = m.groups["dp_ar"]
                    continue
                if dp == world:
                    grp = new_group(list(range(world)), role)
                    m.groups[role] = grp
                else:
                    mine = None
                    for t in range(tp):
                        ranks = [d * tp + t for d in range(dp)]
                        g = new_group(ranks, role)
                        if rank in ranks:
                            mine = g
                    m.groups[role] = mine
            else:
                if tp == 1 and not force:
                    continue
                if tp == world:
                    m.groups[role] = new_group(list(range(world)), role)
                else:
                    mine = None
                    for d in range(dp):
                        ranks = [d * tp + t for t in range(tp)]
                        g = new_group(ranks, role)
                        if rank in ranks:
                            mine = g
                    m.groups[role] = mine
        return m
