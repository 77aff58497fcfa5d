"""Single-process engine on CPU vs the reference oracle (same fp32 precision -> tight agreement)."""
import pytest
import torch

from dllm.models import reference as R
from dllm.models.ffn import init_ffn_layer
from dllm.parallel.engine import FFNTrainer
from dllm.parallel.mesh import Mesh
from dllm.utils.config import ModelConfig, TrainConfig
from dllm.utils.data import reference_mock_data


def _run(act, gated, recompute, opt="sgd", lr=1e-2, steps=3, D=16, F=64, L=3, T=32, fused=True):
    gen = torch.Generator().manual_seed(3)
    layers = [init_ffn_layer(D, F, gen, gated) for _ in range(L)]
    batches = list(reference_mock_data(torch.randint(100_000, (steps,), generator=gen), T, D))
    cfg = TrainConfig(model=ModelConfig(D, F, L, act, gated), batch_size=1, seq_len=T, lr=lr, optimizer=opt,
                      recompute=recompute, fused_optimizer=fused)
    eng = FFNTrainer(cfg, Mesh(), torch.device("cpu"))
    eng.load_full_params(layers)
    for x, dy in batches:
        eng.train_step(x, dy)
    return eng.gather_full_params(), layers, batches


@pytest.mark.parametrize("act,gated", [("relu", False), ("silu", False), ("gelu", False), ("silu", True)])
@pytest.mark.parametrize("recompute", ["none", "full"])
def test_single_matches_oracle(act, gated, recompute):
    got, layers, batches = _run(act, gated, recompute)
    want = R.train_single(layers, batches, 1e-2, act)
    for g, w in zip(got, want):
        for k in w:
            torch.testing.assert_close(g[k], w[k], rtol=1e-5, atol=1e-7)


def test_adam_matches_oracle():
    got, layers, batches = _run("relu", False, "none", opt="adam", lr=1e-3)
    want = R.train_adam_single(layers, batches, 1e-3)
    for g, w in zip(got, want):
        for k in w:
            torch.testing.assert_close(g[k], w[k], rtol=1e-5, atol=1e-6)


def test_bf16_compute_on_cpu_tracks_fp32():
    gen = torch.Generator().manual_seed(3)
    D, F, L, T = 32, 128, 2, 64
    layers = [init_ffn_layer(D, F, gen) for _ in range(L)]
    (x, dy), = list(reference_mock_data([7], T, D))
    cfg = TrainConfig(model=ModelConfig(D, F, L), batch_size=1, seq_len=T, lr=1e-2, dtype="bf16")
    eng = FFNTrainer(cfg, Mesh(), torch.device("cpu"))
    eng.load_full_params(layers)
    eng.train_step(x.bfloat16(), dy.bfloat16())
    got = eng.gather_full_params()
    want = R.train_single(layers, [(x.bfloat16().float(), dy.bfloat16().float())], 1e-2)
    for g, w, p in zip(got, want, layers):
        for k in w:
            rel = ((g[k] - p[k]) - (w[k] - p[k])).norm() / (w[k] - p[k]).norm()
            assert rel < 1e-1, (k, rel.item())  # bf16 activations + ReLU-mask flips at tiny T


@pytest.mark.parametrize("opt", ["sgd", "adam"])
def test_fused_optimizer_equals_unfused(opt):
    a, _, _ = _run("silu", True, "none", opt=opt, lr=1e-3, fused=True)
    b, _, _ = _run("silu", True, "none", opt=opt, lr=1e-3, fused=False)
    for g, w in zip(a, b):
        for k in w:
            torch.testing.assert_close(g[k], w[k], rtol=1e-6, atol=1e-8)


@pytest.mark.parametrize("gated,act,opt,rec", [(False, "relu", "sgd", "none"), (True, "silu", "adam", "none"),
                                               (False, "gelu", "adam", "full")])
def test_sizing_plan_matches_engine_buffers(gated, act, opt, rec):
    """utils/sizing.plan (the README's per-rank HBM table) predicts the engine's own allocations."""
    from dllm.parallel.engine import FFNTrainer
    from dllm.parallel.mesh import Mesh
    from dllm.utils.config import ModelConfig, TrainConfig
    from dllm.utils.sizing import plan

    m = ModelConfig(64, 192, 3, act, gated)
    cfg = TrainConfig(model=m, batch_size=2, seq_len=64, dtype="bf16", grad_dtype="bf16", optimizer=opt,
                      recompute=rec)
    eng = FFNTrainer(cfg, Mesh(), "cpu")
    p = plan(64, 192, 3, 128, gated=gated, act=act, dtype="bf16", grad_dtype="bf16", optimizer=opt, recompute=rec,
             relu_mask=False)["bytes"]
    nb = lambda t: t.numel() * t.element_size()  # noqa: E731
    assert p.get("master_fp32", 0) + p.get("master_residual", 0) == eng.master_bytes
    assert p["compute_copy"] == nb(eng.copy) and p["grads"] == nb(eng.grads)
    if opt == "adam":
        assert p["adam_moments"] == nb(eng.adam_m) + nb(eng.adam_v)
    assert p["layer_inputs"] == sum(nb(t) for t in eng.xs[1:]) + 128 * 64 * 2
    assert p["activations"] == sum(nb(t) for t in eng.acts_a)
    assert p.get("preactivations", 0) == (sum(nb(t) for t in eng.acts_h) if eng.acts_h else 0)
    assert p["dgrad_buffer"] == nb(eng.da) and p["dx_buffers"] == sum(nb(t) for t in eng.dxb)


def test_tp_chunk_policy_avoids_split_k_chunks():
    """TP/SP forward chunks on the GPU: halve the chunk count until each chunk's GEMMs fill the chip without
    split-K (MP config T=8192, D=4096, F=14336: TP8 shard unchunked, TP2 / TP4 in 2 chunks)."""
    from dllm.parallel.engine import gpu_chunk_count

    T, D = 8192, 4096
    assert gpu_chunk_count(T, D, 14336 // 8, 14336 // 8, 4) == 1
    assert gpu_chunk_count(T, D, 14336 // 4, 14336 // 4, 4) == 2
    assert gpu_chunk_count(T, D, 14336 // 2, 14336 // 2, 4) == 2
    assert gpu_chunk_count(T, D, 14336 // 2, 14336, 4) == 2       # gated: R1 = 2 F_loc
    assert gpu_chunk_count(4 * T, D, 16384 // 2, 16384 // 2, 4) == 4
    assert gpu_chunk_count(T, D, 8192, 8192, 1) == 1


def _engine(D=16, F=64, L=2, gated=False, act="relu"):
    cfg = TrainConfig(model=ModelConfig(D, F, L, act, gated), batch_size=1, seq_len=32, lr=1e-2)
    eng = FFNTrainer(cfg, Mesh(), torch.device("cpu"))
    gen = torch.Generator().manual_seed(5)
    eng.load_full_params([init_ffn_layer(D, F, gen, gated) for _ in range(L)])
    return eng


@pytest.mark.parametrize("fmt", ["consolidated", "sharded"])
@pytest.mark.parametrize("dim", ["D", "F"])
def test_checkpoint_rejects_other_model_dims(fmt, dim, tmp_path):
    """A checkpoint of a LARGER model contains every box a smaller engine needs; resuming from it must raise, not
    silently load a sub-block of the wrong-sized matrices."""
    from dllm.utils.checkpoint import load_checkpoint, save_checkpoint

    save_checkpoint(_engine(D=32, F=128) if dim == "D" else _engine(F=128), str(tmp_path), step=1, fmt=fmt)
    with pytest.raises(ValueError, match=f"{dim}="):
        load_checkpoint(_engine(D=16, F=64), str(tmp_path))
    load_checkpoint(_engine(D=32, F=128) if dim == "D" else _engine(F=128), str(tmp_path))  # same dims: fine


def test_gated_consolidated_reads_only_needed_rows(tmp_path):
    """A gated consolidated checkpoint stores w1 / w3 separately; the loader rebuilds the interleaved storage rows
    [a, b) from just the w1 / w3 rows (and columns) that cover them, not from the whole tensors."""
    from dllm.models.ffn import interleave_w13
    from dllm.utils.checkpoint import _consolidated_sources, _Reader, save_checkpoint

    eng = _engine(D=16, F=128, L=1, gated=True, act="silu")
    save_checkpoint(eng, str(tmp_path), step=0)
    full = eng.gather_full_params()[0]
    meta = {"layers": 1, "gated": True, "D": 16, "F": 128}
    reader = _Reader(str(tmp_path))
    (_, read), = _consolidated_sources(str(tmp_path), meta, reader)[("params", 0, "w1")]
    got = read(40, 70, 4, 12)
    torch.testing.assert_close(got, interleave_w13(full["w1"], full["w3"])[40:70, 4:12], rtol=0, atol=0)
    # rows 40..69 lie in 32-row periods 1..2 -> w1 / w3 rows 16..47 (x 8 columns): 2 * 32 * 8 fp32 values
    assert reader.bytes_read == 2 * 32 * 8 * 4, reader.bytes_read


def test_sizing_counts_wgrad_stream_buffers():
    """The concurrent weight-gradient stream rotates 2 dgrad and 3 dx buffers (engine da_ring / dxb); the planner
    counts them only where the engine enables the stream (single device, fused optimizer, kept activations)."""
    from dllm.utils.sizing import plan

    kw = dict(dtype="bf16", grad_dtype="bf16")
    base = plan(64, 256, 2, 128, **kw)["bytes"]
    ws = plan(64, 256, 2, 128, wgrad_stream=True, **kw)["bytes"]
    assert ws["dgrad_buffer"] == 2 * base["dgrad_buffer"] and ws["dx_buffers"] == 3 * 128 * 64 * 2
    for off in (dict(dp=2, mode="ddp"), dict(tp=2), dict(recompute="full")):
        a = plan(64, 256, 2, 128, wgrad_stream=True, **kw, **off)["bytes"]
        b = plan(64, 256, 2, 128, **kw, **off)["bytes"]
        assert a["dgrad_buffer"] == b["dgrad_buffer"] and a["dx_buffers"] == b["dx_buffers"]


def test_wgrad_nn_shapes_cover_the_transposed_copies():
    """the NN weight-gradient layout also needs the fwd-2 / dx GEMMs that write the transposed copies on
    256x256 tiles.  T = 4224 (33 x 128 tokens) passes the weight-gradient shape checks but not the copies' (T % 256), so
    'auto' must fall back to TN (engine and sizing alike) instead of raising at the first forward."""
    from dllm.ops.gemm import nn_wgrad_supported
    from dllm.parallel.engine import wgrad_nn_shape_problem
    from dllm.utils.sizing import plan, resolve_wgrad_layout

    assert nn_wgrad_supported(4096, 16384, 4224)            # the weight gradients alone would pass
    assert wgrad_nn_shape_problem(4224, 4096, 16384, 16384)
    assert not wgrad_nn_shape_problem(8192, 4096, 16384, 16384)
    assert resolve_wgrad_layout("auto", 4096, 16384, 16384, 4224) == "tn"
    assert resolve_wgrad_layout("auto", 4096, 16384, 16384, 8192) == "nn_w2t"
    assert resolve_wgrad_layout("auto", 4096, 16384, 16384, 8192, tp=2) == "tn"
    assert resolve_wgrad_layout("auto", 4096, 16384, 16384, 8192, master="fp32") == "tn"           # fused: split only
    assert resolve_wgrad_layout("auto", 4096, 16384, 16384, 8192, mode="zero", master="fp32") == "nn_w2t"
    assert "nn_transposed_copies" not in plan(4096, 16384, 8, 4224)["bytes"]
    assert plan(4096, 16384, 8, 8192)["bytes"]["nn_transposed_copies"] == (8 + 3) * 4096 * 8192 * 2


def test_engine_t4224_keeps_tn_layout():
    """The engine built at T = 4224 (CPU-constructible) resolves 'auto' to the TN layout."""
    cfg = TrainConfig(model=ModelConfig(256, 1024, 2, "relu", False), batch_size=33, seq_len=128, dtype="bf16")
    eng = FFNTrainer(cfg, Mesh(), torch.device("cpu"))
    assert eng.T == 4224 and eng.wgrad_nn is False and eng.w2t is False
