"""The NN weight-gradient layout's kernels (round 5; csrc/gemm_kernels.h EPI_SGDS_T / EPI_STORE_T / EPI_STORE_DT,
dispatch_x): transposed outputs with the MFMA operands swapped, transposed copies out of the store epilogue, the NN
fused split-master SGD on 256x256 tiles, and the LDS transpose.  Each is checked against the fp32 torch reference of
the same op and bitwise against the TN-layout kernel it replaces (same accumulation order)."""
import pytest
import torch

from dllm.ops.gemm import gemm, nn_wgrad_supported, set_splitk, transpose_bf16
from dllm.ops.master import join_master, split_master

pytestmark = pytest.mark.gpu

BF = torch.bfloat16
# (T, D, F): a one-tile-per-block grid, and a persistent one (1024 tiles > 256 CUs) with a short K
SHAPES = [(1024, 512, 1024), (256, 4096, 16384)]


@pytest.fixture(autouse=True)
def _no_splitk():
    """The TN reference must run unsplit (small grids otherwise take split-K: another summation order)."""
    old = set_splitk(False)
    yield
    set_splitk(old)


def _rnd(g, *shape, s=1.0):
    return (torch.randn(*shape, generator=g) * s).to(BF).cuda()


@pytest.mark.parametrize("T,D,F", SHAPES)
def test_transposed_output_store_matches_tn(T, D, F):
    g = torch.Generator().manual_seed(1)
    da, x = _rnd(g, T, F), _rnd(g, T, D)
    assert nn_wgrad_supported(D, F, T)
    for dt in (torch.float32, BF):
        ref = gemm(da, x, "tn", out=torch.empty(F, D, dtype=dt, device="cuda"))            # dW1 = daᵀ·x
        got = gemm(x.t().contiguous(), da, "nn", out=torch.empty(F, D, dtype=dt, device="cuda"), out_t=True)
        assert torch.equal(got, ref), (dt, (got.float() - ref.float()).abs().max().item())
    exact = da.float().t() @ x.float()
    torch.testing.assert_close(got.float(), exact, rtol=2e-2, atol=2e-2 * exact.abs().max().item())


@pytest.mark.parametrize("T,D,F", SHAPES)
def test_nn_fused_sgd_matches_tn(T, D, F):
    """dW2 (NN, A = dyᵀ K-contiguous) and dW1 (NN, transposed output) fused split-master SGD updates are bitwise the
    TN kernels' and match the fp32 update."""
    g = torch.Generator().manual_seed(2)
    dy, a, da, x = _rnd(g, T, D), _rnd(g, T, F), _rnd(g, T, F), _rnd(g, T, D)
    lr = 1e-2
    for shape, tn, nn in (((D, F), lambda lo, hi: gemm(dy, a, "tn", out=lo, epi="sgd_split", lr=lr, aux_out=hi),
                           lambda lo, hi: gemm(dy.t().contiguous(), a, "nn", out=lo, epi="sgd_split", lr=lr,
                                               aux_out=hi)),
                          ((F, D), lambda lo, hi: gemm(da, x, "tn", out=lo, epi="sgd_split", lr=lr, aux_out=hi),
                           lambda lo, hi: gemm(x.t().contiguous(), da, "nn", out=lo, epi="sgd_split", lr=lr,
                                               aux_out=hi, out_t=True))):
        m = (torch.randn(*shape, generator=g) * 0.02).cuda()
        h0, l0 = split_master(m)
        h1, l1 = h0.clone(), l0.clone()
        tn(l0, h0)
        nn(l1, h1)
        assert torch.equal(h0, h1) and torch.equal(l0, l1), shape
        if shape == (D, F):
            grad = dy.float().t() @ a.float()
        else:
            grad = da.float().t() @ x.float()
        exact = m - lr * grad
        got = join_master(h1, l1)
        torch.testing.assert_close(got, exact, rtol=0, atol=2e-2 * lr * grad.abs().max().item() + 1e-6)


@pytest.mark.parametrize("T,D,F", SHAPES)
def test_nn_fused_adamw_matches_tn(T, D, F):
    """The split-master AdamW epilogue through the transposed map (EPI_ADAMS_T, dW1 into W1 [F, D]) and on NN 256x256
    tiles (dW2): masters and moments bitwise the TN kernel's."""
    g = torch.Generator().manual_seed(6)
    dy, a, da, x = _rnd(g, T, D), _rnd(g, T, F), _rnd(g, T, F), _rnd(g, T, D)
    kw = dict(epi="adam_split", lr=1e-3, betas=(0.9, 0.95), eps=1e-8, wd=0.1, step=3)
    for shape, tn, nn in (((D, F), lambda **k: gemm(dy, a, "tn", **k),
                           lambda **k: gemm(dy.t().contiguous(), a, "nn", **k)),
                          ((F, D), lambda **k: gemm(da, x, "tn", **k),
                           lambda **k: gemm(x.t().contiguous(), da, "nn", out_t=True, **k))):
        m = (torch.randn(*shape, generator=g) * 0.02).cuda()
        mom = (torch.randn(*shape, generator=g) * 1e-3).cuda(), (torch.rand(*shape, generator=g) * 1e-5).cuda()
        h0, l0 = split_master(m)
        st = [(h0, l0, mom[0].clone(), mom[1].clone()), (h0.clone(), l0.clone(), mom[0].clone(), mom[1].clone())]
        for (h, lo, mm, vv), fn in zip(st, (tn, nn)):
            fn(out=lo, aux_out=h, opt_m=mm, opt_v=vv, **kw)
        for u, v in zip(st[0], st[1]):
            assert torch.equal(u, v), shape


@pytest.mark.parametrize("T,D,F", SHAPES)
@pytest.mark.parametrize("layout", ["nt", "nn"])
def test_store_with_transposed_copy(T, D, F, layout):
    """y = a·W2ᵀ (NT) and dx = da·W1 (NN) with ``aux_t``: the output is bitwise the plain store's and the copy is
    exactly its transpose."""
    g = torch.Generator().manual_seed(3)
    a = _rnd(g, T, F)
    w = _rnd(g, D, F, s=0.02) if layout == "nt" else _rnd(g, F, D, s=0.02)
    y0 = gemm(a, w, layout)
    yT = torch.empty(D, T, dtype=BF, device="cuda")
    y1 = gemm(a, w, layout, aux_t=yT)
    assert torch.equal(y0, y1)
    assert torch.equal(yT, y0.t())
    wf = w.float().t() if layout == "nt" else w.float()
    exact = a.float() @ wf
    torch.testing.assert_close(y1.float(), exact, rtol=2e-2, atol=2e-2 * exact.abs().max().item())


def test_transpose_bf16():
    g = torch.Generator().manual_seed(4)
    for R, C in ((64, 64), (8192, 4096), (192, 320)):
        src = _rnd(g, R, C)
        dst = torch.empty(C, R, dtype=BF, device="cuda")
        transpose_bf16(src, dst)
        assert torch.equal(dst, src.t())
    big = _rnd(g, 256, 512)                       # strided views (row strides > width)
    dst = torch.empty(256 + 64, 256, dtype=BF, device="cuda")[:256]
    transpose_bf16(big[:, 128:384], dst)
    assert torch.equal(dst, big[:, 128:384].t())


def test_transposed_outputs_reject_bad_shapes():
    g = torch.Generator().manual_seed(5)
    a, b = _rnd(g, 256, 256), _rnd(g, 192, 256)          # K = 192: not a multiple of the 128-deep step
    with pytest.raises(ValueError):
        gemm(b.t().contiguous(), a[:192], "nn", out_t=True)
    with pytest.raises(ValueError):
        gemm(a, a, "nt", out_t=True, epi="sgd_split")    # transposed fused optimizer: NN / TN only


@pytest.mark.parametrize("variant", ["fused_serial", "fused_wgrad_stream", "grads_fp32", "grads_bf16",
                                     "gated_adamw"])
def test_engine_nn_wgrad_layout_bitwise_tn(variant, monkeypatch):
    """Three layers, three steps: the engine's NN weight-gradient layout (transposed copies from the fwd-2 / dx
    epilogues and the step-start transposes) leaves masters bitwise equal to the TN layout's -- fused split-master SGD
    on the serial backward and on the concurrent weight-gradient stream (off by default with NN, kept for A/B runs),
    and stored (fp32 / bf16) gradients."""
    from dllm.models.ffn import init_ffn_params_device
    from dllm.parallel.engine import FFNTrainer
    from dllm.parallel.mesh import Mesh
    from dllm.utils.config import ModelConfig, TrainConfig
    from dllm.utils.data import DeviceMockData

    monkeypatch.setenv("DLLM_NN_CONCURRENT", "1")   # keep the (A/B-only) concurrent NN path covered
    dev = torch.device("cuda", 0)
    gated = variant == "gated_adamw"    # SwiGLU + fused AdamW on split masters (config 5's kind)
    m = ModelConfig(model_size=2048, ffn_dim=8192, layers=3, act="silu" if gated else "relu", gated=gated)
    out = {}
    for layout in ("tn", "nn", "nn_w1", "nn_w2t"):
        cfg = TrainConfig(model=m, batch_size=1, seq_len=1024, dtype="bf16",
                          grad_dtype="bf16" if variant == "grads_bf16" else "fp32",
                          optimizer="adam" if gated else "sgd", lr=1e-3,
                          wgrad_layout=layout, wgrad_stream=variant == "fused_wgrad_stream",
                          fused_optimizer=variant.startswith("fused") or gated)
        eng = FFNTrainer(cfg, Mesh(), dev)
        assert eng.wgrad_nn == (layout != "tn") and eng.wgrad_nn_w2 == (layout in ("nn", "nn_w2t"))
        assert eng.w2t == (layout == "nn_w2t")
        assert (eng.wg_stream is not None) == (variant == "fused_wgrad_stream")
        eng.load_full_params(init_ffn_params_device(m.D, m.F, m.layers, 7, dev, gated=gated))
        data = DeviceMockData(cfg.tokens, m.D, torch.bfloat16, dev)
        ys = []
        for i in range(3):
            x, dy = data.fill(i)
            ys.append(eng.train_step(x, dy).clone())
        torch.cuda.synchronize()
        # logical [out, in] parameters (nn_w2t stores W2 as W2ᵀ: the flat master's layout differs)
        params = torch.cat([t.reshape(-1) for p in eng.local_params() for t in (p["w1"], p["w2"])])
        out[layout] = (params.clone(), ys)
    bits = lambda t: t.view(torch.int16 if t.dtype == BF else torch.int32)   # noqa: E731 (NaN-safe bitwise)
    for layout in ("nn", "nn_w1", "nn_w2t"):
        assert all(torch.equal(bits(a), bits(b)) for a, b in zip(out["tn"][1], out[layout][1])), layout
        assert torch.equal(bits(out["tn"][0]), bits(out[layout][0])), layout
    assert torch.isfinite(out["nn"][0]).all()


@pytest.mark.parametrize("fused", [True, False])
def test_engine_tn_layout_w2_transposed_storage_bitwise(fused):
    """W2 stored as W2ᵀ under the TN weight-gradient layout (the TN kernels' transposed output maps,
    EPI_STORE_T / EPI_SGDS_T) leaves the same logical parameters and outputs, bit for bit, as row-major storage --
    fused split-master SGD and stored bf16 gradients, 3 layers x 3 steps."""
    from dllm.models.ffn import init_ffn_params_device
    from dllm.parallel.engine import FFNTrainer
    from dllm.parallel.mesh import Mesh
    from dllm.utils.config import ModelConfig, TrainConfig
    from dllm.utils.data import DeviceMockData

    dev = torch.device("cuda", 0)
    m = ModelConfig(model_size=2048, ffn_dim=8192, layers=3, act="relu")
    out = {}
    for storage in ("rowmajor", "transposed"):
        cfg = TrainConfig(model=m, batch_size=1, seq_len=1024, dtype="bf16", grad_dtype="bf16", lr=1e-3,
                          wgrad_layout="tn", w2_storage=storage, fused_optimizer=fused)
        eng = FFNTrainer(cfg, Mesh(), dev)
        assert eng.wgrad_nn is False and eng.w2t == (storage == "transposed")
        eng.load_full_params(init_ffn_params_device(m.D, m.F, m.layers, 7, dev))
        data = DeviceMockData(cfg.tokens, m.D, torch.bfloat16, dev)
        ys = [eng.train_step(*data.fill(i)).clone() for i in range(3)]
        torch.cuda.synchronize()
        params = torch.cat([t.reshape(-1) for p in eng.local_params() for t in (p["w1"], p["w2"])])
        out[storage] = (params, ys)
    bits = lambda t: t.view(torch.int16 if t.dtype == BF else torch.int32)   # noqa: E731
    assert all(torch.equal(bits(a), bits(b)) for a, b in zip(out["rowmajor"][1], out["transposed"][1]))
    assert torch.equal(bits(out["rowmajor"][0]), bits(out["transposed"][0]))
    assert torch.isfinite(out["rowmajor"][0]).all()


def test_engine_w2_transposed_storage_validated_at_construction():
    """Transposed W2 storage with a fused optimizer on an fp32 master (no transposed 'sgd' epilogue) or off the
    256x256 tiles is rejected when the engine is built, not at the first backward."""
    from dllm.parallel.engine import FFNTrainer
    from dllm.parallel.mesh import Mesh
    from dllm.utils.config import ModelConfig, TrainConfig

    dev = torch.device("cuda", 0)
    m = ModelConfig(model_size=2048, ffn_dim=8192, layers=1, act="relu")
    with pytest.raises(ValueError, match="split masters"):
        FFNTrainer(TrainConfig(model=m, batch_size=1, seq_len=1024, dtype="bf16", wgrad_layout="tn",
                               w2_storage="transposed", master="fp32"), Mesh(), dev)
    small = ModelConfig(model_size=2048, ffn_dim=8192 + 224, layers=1, act="relu")
    with pytest.raises(ValueError, match="256x256"):
        FFNTrainer(TrainConfig(model=small, batch_size=1, seq_len=1024, dtype="bf16", wgrad_layout="tn",
                               w2_storage="transposed"), Mesh(), dev)
