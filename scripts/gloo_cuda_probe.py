"""Which torch.distributed collectives the gloo backend runs on GPU tensors (two processes sharing cuda:0).

    python scripts/gloo_cuda_probe.py

RCCL refuses two ranks on one device, so multi-rank GPU tests of the data-parallel engine paths would use gloo
with device tensors; this prints which of the collectives the engine needs (async, then a stream wait) work.
"""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _proc(rank, n, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=n)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    res = {}
    side = torch.cuda.Stream()

    def check(name, fn):
        try:
            ok = fn()
            torch.cuda.synchronize()
            res[name] = bool(ok)
        except Exception as e:  # noqa: BLE001
            res[name] = f"{type(e).__name__}: {str(e)[:120]}"

    def ar():
        t = torch.full((1 << 16,), float(rank + 1), device=dev)
        with torch.cuda.stream(side):
            w = dist.all_reduce(t, async_op=True)
        w.wait()
        return torch.all(t == n * (n + 1) / 2).item()

    def ag():
        s = torch.full((1 << 16,), float(rank), device=dev)
        o = torch.empty(n << 16, device=dev)
        dist.all_gather_into_tensor(o, s, async_op=True).wait()
        return all(torch.all(o[r << 16:(r + 1) << 16] == r).item() for r in range(n))

    def rs():
        f = torch.arange(n << 16, device=dev, dtype=torch.float32)
        o = torch.empty(1 << 16, device=dev)
        dist.reduce_scatter_tensor(o, f, async_op=True).wait()
        return torch.equal(o, n * f[rank << 16:(rank + 1) << 16])

    def rs_bf16():
        f = torch.ones(n << 16, device=dev, dtype=torch.bfloat16)
        o = torch.empty(1 << 16, device=dev, dtype=torch.bfloat16)
        dist.reduce_scatter_tensor(o, f, async_op=True).wait()
        return torch.all(o == n).item()

    for name, fn in (("all_reduce", ar), ("all_gather_into_tensor", ag), ("reduce_scatter_tensor", rs),
                     ("reduce_scatter_tensor_bf16", rs_bf16)):
        check(name, fn)
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def main():
    n, port = 2, 29000 + os.getpid() % 1000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_proc, args=(r, n, port, q)) for r in range(n)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
    out = dict(q.get(timeout=10) for _ in range(n))
    print(out[0])
    sys.exit(0 if all(p.exitcode == 0 for p in ps) else 1)


if __name__ == "__main__":
    main()
