"""Split fp32 master (bf16 working copy + int16 residual, ops/master.py): the encoding, the CPU update paths, the
engine's state accounting and checkpoints -- single process and ZeRO-2 / DDP / FSDP over gloo."""
import pytest
import torch

from dllm.ops.gemm import gemm
from dllm.ops.master import join_master, split_master
from dllm.parallel.engine import FFNTrainer
from dllm.parallel.mesh import Mesh
from dllm.utils.config import ModelConfig, TrainConfig


def test_split_is_lossless_and_rounds_half_away():
    g = torch.Generator().manual_seed(0)
    u = torch.randint(-2**31, 2**31 - 1, (200_000,), generator=g, dtype=torch.int32)
    h, l = split_master(u.view(torch.float32))
    assert torch.equal(join_master(h, l).view(torch.int32), u)
    w = torch.randn(100_000, generator=g)
    w = torch.cat([w, torch.tensor([0.0, -0.0, float("inf"), -float("inf"), 1e-42, -3e38])])
    h, _ = split_master(w)
    ref = w.to(torch.bfloat16)  # RNE: differs from half-away-from-zero only on exact ties
    tie = (w.view(torch.int32) & 0xFFFF) == 0x8000
    assert torch.equal(h.view(torch.int16)[~tie], ref.view(torch.int16)[~tie])
    # a tie rounds away from zero in magnitude
    t = torch.tensor([1.0 + 2.0 ** -8, -(1.0 + 2.0 ** -8)])   # exactly half-way between two bf16 values
    h, l = split_master(t)
    assert h.float().abs().tolist() == [1.0 + 2.0 ** -7] * 2 and torch.equal(join_master(h, l), t)


def test_cpu_fused_sgd_split_equals_sgd():
    g = torch.Generator().manual_seed(1)
    a, b = torch.randn(64, 32, generator=g).bfloat16(), torch.randn(64, 48, generator=g).bfloat16()
    w = torch.randn(32, 48, generator=g) * 0.02
    hi, lo = split_master(w)
    gemm(a, b, "tn", out=lo, epi="sgd_split", lr=0.1, aux_out=hi)
    m = w.clone()
    gemm(a, b, "tn", out=m, epi="sgd", lr=0.1)
    assert torch.equal(join_master(hi, lo), m)
    with pytest.raises(ValueError):
        gemm(a, b, "tn", out=lo.float(), epi="sgd_split", lr=0.1, aux_out=hi)


def _layers(D, F, L, seed=2):
    g = torch.Generator().manual_seed(seed)
    return [{"w1": (torch.randn(F, D, generator=g) * 0.05).bfloat16().float(),
             "w2": (torch.randn(D, F, generator=g) * 0.05).bfloat16().float()} for _ in range(L)]


def _engine(master, D=32, F=128, L=2, opt="sgd"):
    cfg = TrainConfig(model=ModelConfig(D, F, L), batch_size=1, seq_len=64, dtype="bf16", grad_dtype="bf16",
                      lr=1e-2, optimizer=opt, master=master)
    return FFNTrainer(cfg, Mesh(), torch.device("cpu"))


def test_engine_split_state_and_step():
    D, F, L = 32, 128, 2
    es, ef = _engine("split"), _engine("fp32")
    assert es.split and not ef.split and es.master_lo.dtype == torch.int16
    assert es.master_bytes * 2 == ef.master_bytes   # 2 B/param residual vs 4 B/param fp32
    layers = _layers(D, F, L)
    g = torch.Generator().manual_seed(3)
    x, dy = torch.randn(64, D, generator=g).bfloat16(), (torch.randn(64, D, generator=g) * 0.1).bfloat16()
    ea, eb = _engine("split", opt="adam"), _engine("fp32", opt="adam")   # AdamW: split master, fp32 moments
    assert ea.split and not eb.split
    for e in (es, ef, ea, eb):
        e.load_full_params(layers)
        e.train_step(x, dy)
    assert torch.equal(es.master.view(torch.int32), ef.master.view(torch.int32))
    assert torch.equal(ea.master.view(torch.int32), eb.master.view(torch.int32))
    assert torch.equal(ea.adam_v, eb.adam_v)
    assert torch.equal(es.master_slice(3, 70), es.master[3:70])
    assert torch.equal(es.copy.view(torch.int16), split_master(es.master)[0].view(torch.int16))


@pytest.mark.parametrize("fmt", ["consolidated", "sharded"])
def test_split_master_checkpoint_roundtrip(fmt, tmp_path):
    from dllm.utils.checkpoint import load_into, save_checkpoint

    D, F, L = 32, 128, 2
    a = _engine("split")
    a.load_full_params(_layers(D, F, L))
    g = torch.Generator().manual_seed(4)
    a.train_step(torch.randn(64, D, generator=g).bfloat16(), (torch.randn(64, D, generator=g) * 0.1).bfloat16())
    save_checkpoint(a, str(tmp_path), step=1, fmt=fmt)
    for fmt_b in ("split", "fp32"):   # resumes into either format: the file holds the fp32 master
        b = _engine(fmt_b)
        load_into(b, str(tmp_path))
        assert torch.equal(b.master.view(torch.int32), a.master.view(torch.int32))
        if fmt_b == "split":
            assert torch.equal(b.copy.view(torch.int16), a.copy.view(torch.int16))


@pytest.mark.parametrize("method,opt", [(6, "sgd"), (2, "sgd"), (3, "sgd"), (6, "adam"), (3, "adam")])
def test_split_master_data_parallel_equals_fp32(method, opt, free_port):
    """One step per rank over 2 gloo ranks from bf16-representable weights: the split-master engine's fp32 master equals the
    fp32-master engine's bit for bit (ZeRO-2 / DDP / FSDP shard updates run the flat split kernel)."""
    from dllm.parallel.launch import spawn

    D, F, L = 32, 128, 2
    layers = [{k: v.numpy() for k, v in p.items()} for p in _layers(D, F, L)]
    res = {}
    for i, fmt in enumerate(("split", "fp32")):
        cfg = TrainConfig(model=ModelConfig(D, F, L), batch_size=1, seq_len=64, num_steps=2, lr=1e-2, dtype="bf16",
                          grad_dtype="bf16", data="cpu_compat", master=fmt, optimizer=opt)
        res[fmt] = spawn(2, cfg, method, "gloo", free_port + i,
                         {"seed": 11, "params": layers, "return_full": True, "tp": 2})["params"]
    for ps, pf in zip(res["split"], res["fp32"]):
        for k in ps:
            assert torch.equal(torch.as_tensor(ps[k]).view(torch.int32), torch.as_tensor(pf[k]).view(torch.int32)), k
