"""Collective / stream-ordering self-tests runnable on gloo (CPU) or RCCL (GPU).

Replaces the reference's smoke scripts with asserting checks:

* ``test_nccl.py`` (single-process ``torch.cuda.nccl`` AG/AR/RS vs CPU expectations, :9-38) ->
  ``check_collectives``: all-gather-into, all-reduce, reduce-scatter through ``parallel.comm`` on every
  role group, compared with the expectation computed from every rank's deterministic input.
* ``test_torch_distributed.py`` (``new_group`` + async all-reduce + a side stream that must wait, :9-21,
  which printed instead of asserting and read the side-stream result without a ``wait_stream``) ->
  ``check_async_side_stream``: the side-stream update is ordered by explicit stream/event edges and
  the result is asserted (104 after ``ones -> AR(4) -> +100`` generalises to ``world + 100``).
* ``test_mp_barrier_gpus.py`` (children mutate parent-owned tensors) -> the engine returns results
  through rank 0's report instead of IPC; ``launch.spawn`` is covered by the tests.

``python -m dllm.parallel.selftest --backend gloo --world 4`` runs them standalone.
"""
from __future__ import annotations

import argparse
import os

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from . import comm
from .mesh import Mesh, init_distributed


def _input(rank: int, n: int, device) -> torch.Tensor:
    g = torch.Generator().manual_seed(1000 + rank)
    return torch.rand(n, generator=g).to(device)


def check_collectives(mesh: Mesh, device, n: int = 128) -> None:
    world = mesh.world
    rank = mesh.rank
    mine = _input(rank, n, device)
    allin = [_input(r, n, device) for r in range(world)]
    grp = dist.new_group(list(range(world))) if world > 1 else None
    # all-gather (X2 / X6)
    out = torch.zeros(n * world, device=device)
    comm.all_gather_into(out, mine, grp, async_op=True).wait()
    assert torch.equal(out.cpu(), torch.cat(allin).cpu()), "all_gather mismatch"
    # all-reduce (X1 / X7)
    t = mine.clone()
    comm.all_reduce(t, grp, async_op=True).wait()
    assert torch.allclose(t.cpu(), torch.stack(allin).sum(0).cpu()), "all_reduce mismatch"
    # reduce-scatter (X3 / X8)
    big = [_input(r, n * world, device) for r in range(world)]
    o = torch.zeros(n, device=device)
    comm.reduce_scatter_into(o, big[rank], grp, async_op=True).wait()
    want = torch.stack(big).sum(0)[rank * n:(rank + 1) * n]
    assert torch.allclose(o.cpu(), want.cpu()), "reduce_scatter mismatch"
    # grouped collectives (a layer's W2 + W1 pair, two different sizes, issued as one group): each output
    # must match its own collective, in order
    outs = [torch.zeros(n * world, device=device), torch.zeros(2 * n * world, device=device)]
    ins = [mine, _input(rank + 77, 2 * n, device)]
    comm.all_gather_into_many(list(zip(outs, ins)), grp, async_op=True).wait()
    assert torch.equal(outs[0].cpu(), torch.cat(allin).cpu()), "all_gather_into_many[0] mismatch"
    assert torch.equal(outs[1].cpu(), torch.cat([_input(r + 77, 2 * n, device) for r in range(world)]).cpu()), \
        "all_gather_into_many[1] mismatch"
    fulls = [big[rank], _input(rank + 99, 2 * n * world, device)]
    os_ = [torch.zeros(n, device=device), torch.zeros(2 * n, device=device)]
    comm.reduce_scatter_into_many(list(zip(os_, fulls)), grp, async_op=True).wait()
    assert torch.allclose(os_[0].cpu(), want.cpu()), "reduce_scatter_into_many[0] mismatch"
    want1 = torch.stack([_input(r + 99, 2 * n * world, device) for r in range(world)]).sum(0)
    assert torch.allclose(os_[1].cpu(), want1[rank * 2 * n:(rank + 1) * 2 * n].cpu()), \
        "reduce_scatter_into_many[1] mismatch"
    # role groups of a dp x tp mesh
    for role in ("dp_ar", "dp_ag", "dp_rs", "tp"):
        g = mesh.group(role)
        if g is None:
            continue
        ranks = mesh.tp_ranks if role == "tp" else mesh.dp_ranks
        t = mine.clone()
        comm.all_reduce(t, g).wait()
        assert torch.allclose(t.cpu(), sum(allin[r] for r in ranks).cpu()), f"{role} all_reduce mismatch"
        # grouped pair on the role communicator (native: ncclGroupStart/End around both)
        k, me = len(ranks), ranks.index(rank)
        ag = [torch.zeros(n * k, device=device), torch.zeros(2 * n * k, device=device)]
        comm.all_gather_into_many([(ag[0], mine), (ag[1], ins[1])], g).wait()
        assert torch.equal(ag[0].cpu(), torch.cat([allin[r] for r in ranks]).cpu()), f"{role} grouped AG"
        rs = [torch.zeros(n // k if n % k == 0 else n, device=device) for _ in range(2)]
        if n % k == 0:
            comm.reduce_scatter_into_many([(rs[0], mine), (rs[1], mine * 2)], g).wait()
            tot = sum(allin[r] for r in ranks)
            seg = slice(me * (n // k), (me + 1) * (n // k))
            assert torch.allclose(rs[0].cpu(), tot[seg].cpu()) and torch.allclose(rs[1].cpu(), 2 * tot[seg].cpu()), \
                f"{role} grouped RS"


def check_async_side_stream(world: int, device, iters: int = 10) -> None:
    grp = dist.new_group(list(range(world))) if world > 1 else None
    for _ in range(iters):
        t = torch.ones(1, device=device)
        w = comm.all_reduce(t, grp, async_op=True)
        w.wait()  # current stream waits on the collective
        if device.type == "cuda":
            s = torch.cuda.Stream(device)
            s.wait_stream(torch.cuda.current_stream(device))
            with torch.cuda.stream(s):
                t.add_(100)
            torch.cuda.current_stream(device).wait_stream(s)
        else:
            t.add_(100)
        assert t.item() == world + 100, t.item()


def worker(rank: int, world: int, backend: str, port: int, dp: int, tp: int) -> None:
    os.environ["LOCAL_RANK"] = str(rank)
    init_distributed(backend, rank, world, "127.0.0.1", port)
    device = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    mesh = Mesh.build(dp, tp)
    check_collectives(mesh, device)
    check_async_side_stream(world, device)
    dist.barrier()
    dist.destroy_process_group()


def run(world: int, backend: str = "gloo", port: int = 29650, dp: int | None = None, tp: int = 1) -> None:
    dp = dp or world // tp
    mp.spawn(worker, args=(world, backend, port, dp, tp), nprocs=world, join=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="gloo")
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--port", type=int, default=29650)
    a = ap.parse_args()
    run(a.world, a.backend, a.port, tp=a.tp)
    print("selftest ok")
