"""Custom all-reduce (csrc/car.hip) timing with n ranks as processes sharing ONE MI355X (hipIpc buffers).

Not an xGMI measurement: the peers' buffers sit in the same HBM and the ranks' kernels share the CUs, so this
prices the protocol (flag barriers, the two-shot reduce-scatter / all-gather passes, the copy-in and copy-out)
and the small-message latency, not the links.  Prints one JSON line per (n, size, mode): median us per call (max over
ranks) and the algorithmic bandwidth 2(n-1)/n * bytes / time.  Modes: "staged" (copy-in / exchange / copy-out around
an ordinary tensor) and "arena" (zero-copy: the tensor lives in the peer-mapped arena and is all-reduced in place).

    python scripts/bench_car.py [--ranks 2,4] [--sizes_kib 64,1024,8192,65536]
"""
import argparse
import json
import os
import socket
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _proc(rank, n, port, sizes, iters, q):
    import torch.distributed as dist

    import dllm  # noqa: F401
    from dllm.parallel.car import CustomAllReduce

    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=n)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    car = CustomAllReduce(list(range(n)), dev, cap_bytes=max(sizes), tag="bench", arena_bytes=max(sizes))
    out = []
    for nbytes, mode in [(b, m) for b in sizes for m in ("staged", "arena")]:
        if mode == "arena":  # zero-copy: the tensor lives in the mapped arena, all-reduced in place
            car._arena_next = 0
            t = car.arena_view((nbytes // 2,), torch.bfloat16)
            t.copy_(torch.randn(nbytes // 2, device=dev))
        else:                # staged: copy-in -> exchange -> copy-out around an ordinary tensor
            t = torch.randn(nbytes // 2, device=dev).bfloat16()
        for _ in range(3):
            car.all_reduce(t)
        torch.cuda.synchronize()
        times = []
        for _ in range(iters):
            dist.barrier()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            car.all_reduce(t)
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) * 1e3)
        us = torch.tensor([statistics.median(times)], dtype=torch.float64)
        dist.all_reduce(us, op=dist.ReduceOp.MAX)
        out.append((nbytes, mode, float(us.item())))
    car.check()
    car.destroy()
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", default="2,4")
    ap.add_argument("--sizes_kib", default="64,1024,8192,65536")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    sizes = [int(s) * 1024 for s in a.sizes_kib.split(",")]
    ctx = mp.get_context("spawn")
    for n in (int(x) for x in a.ranks.split(",")):
        q = ctx.Queue()
        port = _port()
        ps = [ctx.Process(target=_proc, args=(r, n, port, sizes, a.iters, q)) for r in range(n)]
        for p in ps:
            p.start()
        res = dict(q.get(timeout=300) for _ in range(n))
        for p in ps:
            p.join(timeout=60)
        for nbytes, mode, us in res[0]:
            print(json.dumps({"ranks": n, "bytes": nbytes, "mode": mode, "us_per_call": round(us, 1),
                              "algbw_GBps": round(2 * (n - 1) / n * nbytes / us / 1e3, 1),
                              "note": "ranks share one GPU (HBM, CUs): protocol cost, not xGMI"}), flush=True)


if __name__ == "__main__":
    main()
