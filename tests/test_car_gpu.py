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


def _proc(rank, n, port, numel, dtype, q, arena=False):
    import torch.distributed as dist

    from dllm.parallel.car import CustomAllReduce

    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=n)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    car = CustomAllReduce(list(range(n)), dev, cap_bytes=numel * 4, tag="test",
                          arena_bytes=2 * (numel * 4 + 256) if arena else 0)  # views are 256-B aligned
    # arena: two tensors carved from the zero-copy arena (the second at a non-zero offset), all-reduced in place
    views = [car.arena_view((numel,), dtype) for _ in range(2)] if arena else None
    ok = True
    for it in range(3):
        xs = [torch.randn(numel, generator=torch.Generator().manual_seed(1000 * it + r)).to(dtype) for r in range(n)]
        want = _expected(xs)
        if arena:
            t = views[it % 2]
            t.copy_(xs[rank].to(dev))
        else:
            t = xs[rank].to(dev)
        dist.barrier()
        car.all_reduce(t)
        car.check()
        ok &= bool(torch.equal(t.cpu(), want))
    car.destroy()
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, ok))


@pytest.mark.parametrize("arena", [False, True])
@pytest.mark.parametrize("n,dtype", [(2, torch.bfloat16), (4, torch.float32), (3, torch.bfloat16)])
def test_processes_ipc(n, dtype, arena, free_port):
    """Staged (copy-in / copy-out) and zero-copy arena (in place on the peer-mapped range) all-reduces."""
    numel = (1 << 18) + 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_proc, args=(r, n, free_port, numel, dtype, q, arena)) for r in range(n)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(180)
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    res = dict(q.get(timeout=10) for _ in range(n))
    assert all(res.values()), res


def _tp_proc(rank, n, port, q, mode="custom"):
    import torch.distributed as dist

    from dllm.models.ffn import init_ffn_layer
    from dllm.parallel.engine import FFNTrainer
    from dllm.parallel.mesh import Mesh
    from dllm.utils.config import ModelConfig, TrainConfig
    from dllm.utils.data import reference_mock_data

    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=n)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    D, F, L, T = 256, 1024, 2, 512
    gen = torch.Generator().manual_seed(7)
    layers = [init_ffn_layer(D, F, gen) for _ in range(L)]
    batches = list(reference_mock_data(torch.randint(100_000, (3,), generator=gen), T, D))
    cfg = TrainConfig(model=ModelConfig(D, F, L), batch_size=1, seq_len=T, dtype="fp32", grad_dtype="fp32",
                      lr=1e-2, dp=1, tp=n, tp_allreduce=mode, skip_input_grad=False)
    mesh = Mesh.build(1, n, device=dev)
    eng = FFNTrainer(cfg, mesh, dev)
    if mode == "auto":   # both timed on the [T, D] message; every rank made the same choice
        ch = eng.tp_ar_choice
        assert ch["choice"] in ("rccl", "custom") and ch["rccl"]["ms"] > 0 and ch["custom"]["ms"] > 0, ch
        assert ch["bytes"] == T * D * 4 and ch["ranks"] == n
        assert (eng.tp_car is not None) == (ch["choice"] == "custom")
    if eng.tp_car is not None:
        assert eng.tp_car.arena is not None
        assert eng.tp_car._arena_offset(eng.xs[1]) is not None and eng.tp_car._arena_offset(eng.dxb[0]) is not None
    eng.load_full_params(layers)
    for x, dy in batches:
        eng.train_step(x.to(dev), dy.to(dev))
    if eng.tp_car is not None:
        eng.tp_car.check()
    loc = [{k: v.cpu() for k, v in p.items()} for p in eng.local_params()]
    q.put((rank, (loc, eng.tp_ar_choice)))
    dist.barrier()
    mesh.destroy()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["custom", "auto"])
def test_tp_engine_with_custom_allreduce(mode, free_port):
    """TP=2 training (two processes on the GPU, gloo only as the store) with the custom all-reduce for
    the activation exchange equals single-device training up to reduction order (train_ffns.py:290-312).
    ``auto``: the engine times the gloo tp group against the custom all-reduce on the [T, D] message and keeps the
    faster (the gloo_gpu rehearsal of the 8-GPU selection; both ranks must agree)."""
    from dllm.models import reference as R
    from dllm.models.ffn import init_ffn_layer
    from dllm.utils.data import reference_mock_data

    n = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_tp_proc, args=(r, n, free_port, q, mode)) for r in range(n)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(n))
    for p in ps:
        p.join(60)
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    res = {r: v[0] for r, v in got.items()}
    if mode == "auto":
        assert got[0][1]["choice"] == got[1][1]["choice"], got[0][1]
    D, F, L, T = 256, 1024, 2, 512
    gen = torch.Generator().manual_seed(7)
    layers = [init_ffn_layer(D, F, gen) for _ in range(L)]
    batches = list(reference_mock_data(torch.randint(100_000, (3,), generator=gen), T, D))
    want = R.train_single(layers, batches, 1e-2)
    for l in range(L):
        w1 = torch.cat([res[r][l]["w1"] for r in range(n)], 0)
        w2 = torch.cat([res[r][l]["w2"] for r in range(n)], 1)
        for got, k in ((w1, "w1"), (w2, "w2")):
            d_got = got.double() - layers[l][k].double()
            d_want = want[l][k].double() - layers[l][k].double()
            assert (d_got - d_want).norm() / d_want.norm() < 2e-3, (l, k)


def _stall_proc(rank, n, port, q, arena=False):
    import torch.distributed as dist

    from dllm.parallel.car import CustomAllReduce

    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=n)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    car = CustomAllReduce(list(range(n)), dev, cap_bytes=4096 * 4, tag="stall", timeout_s=0.5,
                          arena_bytes=4096 * 4 if arena else 0)
    res = None
    if rank == 0:  # rank 1 stalls: it never enters the all-reduce
        t = car.arena_view((4096,), torch.float32).fill_(1.0) if arena else torch.ones(4096, device=dev)
        car.all_reduce(t)
        try:
            car.check()
            res = "no error"
        except RuntimeError as e:
            res = ("raised", "timed out" in str(e), bool(torch.isnan(t).all().item()))
        car.all_reduce(t)  # a later call fails fast (no second spin) and stays poisoned
        torch.cuda.synchronize()
        res = res + (bool(torch.isnan(t).all().item()),)
    dist.barrier()
    car.destroy()
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, res))


@pytest.mark.parametrize("arena", [False, True])
def test_stalled_peer_fails_loudly(arena, free_port):
    """A peer that never arrives: the bounded barrier times out, the result is NaN-poisoned (never a
    silently partial sum) and ``check()`` -- which the engine runs at its sync points -- raises."""
    n = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_stall_proc, args=(r, n, free_port, q, arena)) for r in range(n)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(n))
    for p in ps:
        p.join(60)
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    assert res[0] == ("raised", True, True, True), res[0]
