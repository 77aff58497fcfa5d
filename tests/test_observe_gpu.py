"""The communication observer (utils/observe.py) against schedules whose overlap is known by construction.

A collective issued on its role stream right before a long GEMM on the compute stream runs under that GEMM
(overlap_frac ~ 1); the same collective waited for before the GEMM starts is fully exposed (overlap_frac ~ 0).
Both communicator backends (torch ProcessGroupNCCL, native RCCL layer), size-1 communicators on one GPU.
"""
import os

import pytest
import torch
import torch.distributed as dist

from dllm.ops.gemm import gemm
from dllm.parallel import comm
from dllm.parallel.mesh import Mesh, init_distributed
from dllm.utils.observe import CommObserver

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pg():
    os.environ["LOCAL_RANK"] = "0"
    init_distributed("nccl", 0, 1, "127.0.0.1", 29100 + os.getpid() % 1000)
    yield
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("backend", ["torch", "native"])
def test_observer_overlap_known_schedule(pg, backend):
    dev = torch.device("cuda", 0)
    mesh = Mesh.build(1, 1, force=True, comm_backend=backend, device=dev)
    grp = mesh.group("dp_rs")
    g = torch.Generator(device=dev).manual_seed(1)
    a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16, generator=g)
    b = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16, generator=g)
    c = torch.empty(8192, 8192, device=dev, dtype=torch.bfloat16)
    full = torch.randn(16 << 20, device=dev, generator=g)    # 64 MiB: a size-1 reduce-scatter is one copy
    out = torch.empty_like(full)

    side = torch.cuda.Stream(device=dev)

    def step(serial: bool):
        if serial:
            w = comm.reduce_scatter_into(out, full, grp, async_op=True)
            w.wait()          # the GEMM starts only after the collective completed
            gemm(a, b, "nt", out=c)
        else:
            gemm(a, b, "nt", out=c)   # the compute stream is busy ~1 ms ...
            with torch.cuda.stream(side):  # ... while the collective is issued and runs from another stream
                w = comm.reduce_scatter_into(out, full, grp, async_op=True)
            w.wait()

    for serial in (False, True):
        step(serial)
    torch.cuda.synchronize()
    res = {}
    for serial in (False, True):
        with CommObserver(dev, dict(mesh.groups)) as obs:
            for _ in range(4):
                step(serial)
        res[serial] = obs.summary(4)
        print(backend, "serial" if serial else "overlapped", res[serial], obs.intervals())
    assert torch.equal(out, full)
    assert res[False]["collectives_per_step"] == 1.0 and res[True]["collectives_per_step"] == 1.0
    assert res[False]["comm_ms"] > 0.005 and res[True]["comm_ms"] > 0.005
    assert res[False]["overlap_frac"] >= 0.8, res
    assert res[True]["overlap_frac"] <= 0.2, res
    mesh.destroy()


@pytest.mark.parametrize("backend", ["torch", "native"])
def test_observer_skips_collectives_that_move_nothing(pg, backend):
    """On a size-1 communicator an in-place all-reduce / all-gather launches no kernel: counted, no interval;
    an out-of-place one is a copy and gets an interval."""
    dev = torch.device("cuda", 0)
    mesh = Mesh.build(1, 1, force=True, comm_backend=backend, device=dev)
    grp = mesh.group("dp_ag")
    t = torch.randn(4 << 20, device=dev)
    o = torch.empty_like(t)
    with CommObserver(dev, dict(mesh.groups)) as obs:
        comm.all_reduce(t, grp).wait()
        comm.all_gather_into(t, t, grp).wait()
        comm.all_gather_into(o, t, grp).wait()
    s = obs.summary(1)
    assert s["collectives_per_step"] == 3.0 and s["noop_collectives_per_step"] == 2.0, s
    assert len(obs.colls) == 1 and s["comm_ms"] > 0.0, s
    assert torch.equal(o, t)
    mesh.destroy()
