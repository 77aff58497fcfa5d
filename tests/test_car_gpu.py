"""Custom two-shot xGMI all-reduce (csrc/car.hip) on one MI355X.

Several ranks share the GPU: in one process (buffers shared directly, one HIP stream per rank) and in
two processes (hipIpc handles exchanged through a gloo store).  The flag protocol, chunking and
reduction are the same as across GPUs; only the links differ.  Every rank must end with bitwise the
same result: the fp32 sum of the inputs in rank order, rounded once to the tensor dtype."""
import os

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _expected(xs):
    acc = torch.zeros_like(xs[0], dtype=torch.float32)
    for x in xs:
        acc += x.float()
    return acc.to(xs[0].dtype)


# Ranks run as separate processes on the one GPU: each process has its own hardware queues, so every
# rank's spinning barrier kernel can run next to its peers' kernels.  (Ranks as streams of ONE process
# are not used: with GPU_MAX_HW_QUEUES = 4 shared with torch's stream pool, two ranks can land on one
# queue and serialise behind a barrier -- measured as bounded-spin timeouts.)


def _proc(rank, n, port, numel, dtype, q):
    import torch.distributed as dist

    from dllm.parallel.car import CustomAllReduce

    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=n)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    car = CustomAllReduce(list(range(n)), dev, cap_bytes=numel * 4, tag="test")
    ok = True
    for it in range(3):
        xs = [torch.randn(numel, generator=torch.Generator().manual_seed(1000 * it + r)).to(dtype) for r in range(n)]
        want = _expected(xs)
        t = xs[rank].to(dev)
        dist.barrier()
        car.all_reduce(t)
        car.check()
        ok &= bool(torch.equal(t.cpu(), want))
    car.destroy()
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, ok))


@pytest.mark.parametrize("n,dtype", [(2, torch.bfloat16), (4, torch.float32), (3, torch.bfloat16)])
def test_processes_ipc(n, dtype, free_port):
    numel = (1 << 18) + 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_proc, args=(r, n, free_port, numel, dtype, q)) for r in range(n)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(180)
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    res = dict(q.get(timeout=10) for _ in range(n))
    assert all(res.values()), res
