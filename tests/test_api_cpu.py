"""The reference-compatible functional API (dllm.api) on CPU: primitives against the
reference's own formulas (train_ffns.py:41-94), trainers against the pure-torch oracle, and the
process-level worker entry points (init_process + train_process_*) under gloo."""
import torch
import torch.multiprocessing as mp

from dllm import api
from dllm.models import reference as R

D, F, T, L = 16, 64, 8, 2


def _params(seed=5):
    gen = torch.Generator()
    gen.manual_seed(seed)
    return [api.init_tlayer_ffn(D, F, gen) for _ in range(L)]


def _ref_bkwd(dy, lp, x):  # the reference's formulas, written out with torch
    h = x @ lp[0].t()
    a = torch.where(h <= 0, 0, h)
    dw2, da = torch.einsum("bc,bd->cd", dy, a), torch.einsum("bc,cd->bd", dy, lp[1])
    da = da.masked_fill(h <= 0, 0)
    dw1, dx = torch.einsum("bc,bd->cd", da, x), torch.einsum("bc,cd->bd", da, lp[0])
    return dx, (dw1, dw2)


def test_init_matches_reference_rng_order():
    gen = torch.Generator()
    gen.manual_seed(3)
    w1, w2 = api.init_tlayer_ffn(D, F, gen)
    gen.manual_seed(3)
    assert torch.equal(w1, 2e-2 * torch.randn((F, D), generator=gen))
    assert torch.equal(w2, 2e-2 * torch.randn((D, F), generator=gen))


def test_primitives():
    lp = _params()[0]
    x = torch.randn(T, D)
    torch.testing.assert_close(api.linear_fwd(lp[0], x), x @ lp[0].t())
    dy = torch.randn(T, F)
    dw, dx = api.t_linear_bkwd(dy, lp[0], x)
    torch.testing.assert_close(dw, torch.einsum("bc,bd->cd", dy, x))
    torch.testing.assert_close(dx, torch.einsum("bc,cd->bd", dy, lp[0]))
    h = torch.randn(T, F)
    assert torch.equal(api.t_relu_fwd(h), torch.where(h <= 0, 0, h))
    g = torch.randn(T, F)
    exp = g.clone().masked_fill_(h <= 0, 0)
    out = api.t_relu_bkwd_(g, h)
    assert out is g and torch.equal(g, exp)


def test_layer_and_stack():
    layers = _params()
    x, dy = torch.randn(T, D), torch.randn(T, D)
    y, acts = api.tlayers_ffn_fwd(layers, x)
    ref = x
    for lp in layers:
        torch.testing.assert_close(api.tlayer_ffn_fwd(lp, ref), torch.where(ref @ lp[0].t() <= 0, 0, ref @ lp[0].t()) @ lp[1].t())
        ref = torch.where(ref @ lp[0].t() <= 0, 0, ref @ lp[0].t()) @ lp[1].t()
    torch.testing.assert_close(y, ref)
    assert len(acts) == L and acts[0] is x
    seen = []
    grads, handles = api.tlayers_ffn_bkwd(dy, layers, acts, after_comms_hook=lambda dp: seen.append(dp) or len(seen))
    assert handles == [2, 1]  # forward order; the hook ran last layer first
    g = dy
    for i in reversed(range(L)):
        g, (dw1, dw2) = _ref_bkwd(g, layers[i], acts[i])
        torch.testing.assert_close(grads[i][0], dw1)
        torch.testing.assert_close(grads[i][1], dw2)
    calls = []
    api.tlayers_ffn_fwd(layers, x, before_comms_hook=lambda h: calls.append(h) or len(calls))
    assert calls == [None, 1]


def _oracle(layers, seeds, n, lr=api.LR * 1000):
    ls = [{"w1": lp[0].clone(), "w2": lp[1].clone()} for lp in layers]
    batches = list(api.mock_data(seeds, T, D))
    if n == 1:
        return R.train_single(ls, batches, lr)
    return R.train_data_parallel(ls, batches, n, lr)


def test_trainers_match_oracle(free_port):
    layers = _params()
    seeds = torch.tensor([11, 22, 33, 44])
    lr = api.LR * 1000
    one = api.train_1gpu(layers, seeds, T, D, port=free_port, lr=lr)
    ddp = api.train_ddp(layers, seeds, T, D, nprocs=2, port=free_port + 1, lr=lr)
    fsdp = api.train_fsdp(layers, seeds, T, D, nprocs=2, port=free_port + 2, lr=lr)
    tp = api.train_tp(layers, seeds, T, D, nprocs=2, port=free_port + 3, lr=lr)
    o1, o2 = _oracle(layers, seeds, 1), _oracle(layers, seeds, 2)
    for l in range(L):
        for k, name in ((0, "w1"), (1, "w2")):
            torch.testing.assert_close(one[l][k], o1[l][name], rtol=1e-5, atol=1e-7)
            torch.testing.assert_close(tp[l][k], o1[l][name], rtol=1e-5, atol=1e-7)
            torch.testing.assert_close(ddp[l][k], o2[l][name], rtol=1e-5, atol=1e-7)
            assert torch.allclose(ddp[l][k], fsdp[l][k])  # the reference's own check (:386-391)
    assert layers[0][0].shape == (F, D)  # the inputs are not modified


def _proc(rank, world, port, kind, shards, seeds):
    import os

    os.environ["MASTER_PORT"] = str(port)
    fn = {"ddp": api.train_process_ddp, "fsdp": api.train_process_fsdp, "tp": api.train_process_tp}[kind]
    # like the reference's drivers: DDP/FSDP workers get their own stripe (cpus_seeds[rank], train_ffns.py:182,
    # :273), TP workers every seed (:324)
    mine = seeds if kind == "tp" else seeds.reshape(-1, world)[:, rank]
    api.init_process(rank, shards[rank], mine, T, D, fn, world_size=world, backend="gloo")
    import torch.distributed as dist

    dist.destroy_process_group()


def test_process_entry_points_write_back_in_place(free_port):
    layers = _params(9)
    seeds = torch.tensor([5, 6, 7, 8])
    n = 2
    ctx = mp.get_context("spawn")
    ref = _oracle(layers, seeds, n, api.LR)  # the workers train at the reference LR (:29)
    ref1 = _oracle(layers, seeds, 1, api.LR)
    for j, kind in enumerate(("ddp", "fsdp", "tp")):
        if kind == "ddp":
            shards = [[[p.clone().share_memory_() for p in lp] for lp in layers] for _ in range(n)]
        elif kind == "fsdp":
            shards = [[[p.chunk(n, 0)[r].clone().share_memory_() for p in lp] for lp in layers] for r in range(n)]
        else:
            shards = [[[lp[0].chunk(n, 0)[r].clone().share_memory_(), lp[1].chunk(n, 1)[r].clone().share_memory_()]
                       for lp in layers] for r in range(n)]
        procs = [ctx.Process(target=_proc, args=(r, n, free_port + j, kind, shards, seeds)) for r in range(n)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(120)
            assert p.exitcode == 0, kind
        for l in range(L):
            if kind == "ddp":
                w1, w2 = shards[0][l]
                exp = ref
            elif kind == "fsdp":
                w1 = torch.cat([shards[r][l][0] for r in range(n)], 0)
                w2 = torch.cat([shards[r][l][1] for r in range(n)], 0)
                exp = ref
            else:
                w1 = torch.cat([shards[r][l][0] for r in range(n)], 0)
                w2 = torch.cat([shards[r][l][1] for r in range(n)], 1)
                exp = ref1
            assert not torch.equal(w1, layers[l][0]), kind  # trained in place
            torch.testing.assert_close(w1, exp[l]["w1"], rtol=1e-5, atol=1e-8)
            torch.testing.assert_close(w2, exp[l]["w2"], rtol=1e-5, atol=1e-8)
