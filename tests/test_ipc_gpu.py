"""test_mp_barrier_gpus.py with assertions: a process pool mutates parent-owned tensors through IPC.

The reference's children update CUDA tensors the parent created (shared via CUDA IPC handles by torch's
multiprocessing reducers) behind an ``mp.Barrier`` and the parent reads the result (C17/C23).  The GPU
variant shares device memory between processes on one MI355X (dmabuf IPC); the CPU variant uses shared
memory.  The engine itself returns results through rank 0 instead (no IPC needed).
"""
import multiprocessing as mp

import pytest
import torch

_BARRIER = None
_TENSORS = None


def _init(barrier, tensors):
    global _BARRIER, _TENSORS
    _BARRIER, _TENSORS = barrier, tensors


def _add_rank(rank):
    a, b = _TENSORS[rank]
    a.add_(rank + 1)
    b.add_(10 * (rank + 1))
    if a.is_cuda:
        torch.cuda.synchronize()
    _BARRIER.wait()
    return float(a.sum())


def _run(device, n=2):
    ctx = mp.get_context("spawn")
    tensors = [(torch.zeros(2, 2, device=device), torch.zeros(2, 2, device=device)) for _ in range(n)]
    if device == "cpu":
        for a, b in tensors:
            a.share_memory_()
            b.share_memory_()
    barrier = ctx.Barrier(n)
    with ctx.Pool(n, initializer=_init, initargs=(barrier, tensors)) as pool:
        sums = pool.map(_add_rank, range(n))
    if device != "cpu":
        torch.cuda.synchronize()
    for r, (a, b) in enumerate(tensors):
        assert torch.all(a.cpu() == r + 1) and torch.all(b.cpu() == 10 * (r + 1))
        assert sums[r] == 4 * (r + 1)


def test_ipc_pool_cpu_shared_memory():
    _run("cpu")


@pytest.mark.gpu
def test_ipc_pool_gpu_device_memory():
    _run("cuda")
