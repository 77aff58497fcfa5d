"""224-row MFMA tiles (``gemm_bf16_8ph_m224`` / NN ``gemm_bf16_8ph_pair<.., 224>``) and the transposed-activation TP
layout that uses them (``models/ffn.layer_fwd_t`` / ``layer_bwd_t``, engine ``tmode``).

The MP config splits F = 14336 over 8 GPUs: 1792 rows per rank = 7 x 256 (224 of 256 CUs busy) = 8 x 224.  A 224-row
tile runs the same per-element K loop as a 256-row tile, so its outputs must equal, bit for bit, the first 1792 rows of
the 256-tile kernel on the operand padded to 2048 rows -- for every epilogue.  Plus an exact-integer and an A = I /
asymmetric-B check, the ReLU bitmask in the 224-row tile layout, and the engine step in the transposed layout against
the regular one (reference: the TP worker, train_ffns.py:290-312)."""
import pytest
import torch

from dllm.ops.gemm import gemm, gemm_pair, gemm_path, relu_mask_bytes, set_splitk
from dllm.ops.master import join_master, split_master

pytestmark = pytest.mark.gpu
DEV = "cuda"
M, N, K = 1792, 2048, 1024


def _bf(shape, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16).to(DEV)


def _pad_rows(a, rows=2048):
    out = torch.zeros(rows, a.shape[1], dtype=a.dtype, device=a.device)
    out[:a.shape[0]] = a
    return out


def test_path_selection():
    assert gemm_path(torch.bfloat16, torch.bfloat16, 1792, 8192, 4096, 4096, 4096, 8192) == "mfma_bf16_m224"
    assert gemm_path(torch.bfloat16, torch.bfloat16, 2048, 8192, 4096, 4096, 4096, 8192) == "mfma_bf16"


@pytest.mark.parametrize("layout", ["nt", "nn"])
@pytest.mark.parametrize("epi,out_dtype", [("store", torch.float32), ("store", torch.bfloat16), ("act", torch.bfloat16)])
def test_m224_equals_padded_256(layout, epi, out_dtype):
    a = _bf((M, K), 1)
    b = _bf((N, K) if layout == "nt" else (K, N), 2)
    kw = {"epi": epi, "act": "relu" if epi == "act" else "none"}
    out = torch.empty(M, N, dtype=out_dtype, device=DEV)
    gemm(a, b, layout, out=out, **kw)
    ref = torch.empty(2048, N, dtype=out_dtype, device=DEV)
    old = set_splitk(False)   # the reference: whole 256-row tiles, same per-element K order (no split-K partials)
    try:
        gemm(_pad_rows(a), b, layout, out=ref, **kw)
    finally:
        set_splitk(old)
    torch.cuda.synchronize()
    assert torch.equal(out, ref[:M])
    exact = a.double() @ (b.double().t() if layout == "nt" else b.double())
    if epi == "act":
        exact = exact.clamp_min(0)
    assert ((out.double() - exact).abs().max() / exact.abs().max()).item() < (1e-2 if out_dtype == torch.bfloat16 else 1e-5)


def test_m224_exact_integers_and_identity():
    g = torch.Generator().manual_seed(5)
    a = torch.randint(-3, 4, (M, K), generator=g).to(torch.bfloat16).to(DEV)
    b = torch.randint(-3, 4, (K, N), generator=g).to(torch.bfloat16).to(DEV)
    out = torch.empty(M, N, device=DEV)
    gemm(a, b, "nn", out=out)
    torch.cuda.synchronize()
    assert torch.equal(out, (a.double() @ b.double()).float())
    # A = I (M = K = 1792) with an asymmetric B: NT gives exactly Bᵀ
    eye = torch.eye(M, dtype=torch.bfloat16, device=DEV)
    bb = (torch.arange(N * M, dtype=torch.float32).reshape(N, M) % 127 - 63).to(torch.bfloat16).to(DEV)
    o = torch.empty(M, N, device=DEV)
    gemm(eye, bb, "nt", out=o)
    torch.cuda.synchronize()
    assert torch.equal(o, bb.float().t())


def test_m224_relu_mask_roundtrip():
    """Forward ACT writes the bitmask in the 224-row tile layout; the dgrad reading it equals the dgrad reading the
    stored activation, bit for bit (same convention as the 256-row masks)."""
    x, w1 = _bf((N, K), 3), _bf((M, K), 4)          # hᵀ = W1·xᵀ [M, N] (NT)
    aT = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    mask = torch.empty(relu_mask_bytes(M, N), dtype=torch.uint8, device=DEV)
    gemm(w1, x, "nt", out=aT, epi="act", act="relu", mask=mask)
    w2t, dy = _bf((M, K), 5), _bf((N, K), 6)         # daᵀ = W2ᵀ·dyᵀ ⊙ act'
    d1 = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    d2 = torch.empty_like(d1)
    gemm(w2t, dy, "nt", out=d1, epi="dact", act="relu", aux=aT, mask=mask)
    gemm(w2t, dy, "nt", out=d2, epi="dact", act="relu", aux=aT)
    torch.cuda.synchronize()
    assert torch.equal(d1.view(torch.int16), d2.view(torch.int16))
    assert (aT == 0).float().mean().item() > 0.3   # the mask is exercised


@pytest.mark.parametrize("opt", ["sgd", "sgd_split", "adam_split"])
def test_m224_nn_fused_optimizer_pair(opt):
    """dW2ᵀ = aᵀ·dy and dW1 = daᵀ·x ([1792, D], NN) as one grouped launch of 224-row tiles: each half equals the
    single 224-row GEMM bitwise, and the SGD update equals the stored fp32 gradient applied as the kernel does."""
    T, D = 1024, 4096
    aT, daT = _bf((M, T), 7), _bf((M, T), 8)
    dy, x = _bf((T, D), 9), _bf((T, D), 10)
    g = torch.Generator().manual_seed(11)
    w2t = (torch.randn(M, D, generator=g) * 0.02).to(DEV)
    w1 = (torch.randn(M, D, generator=g) * 0.02).to(DEV)

    def state(w):
        st = {"epi": opt, "lr": 1e-2}
        if opt.endswith("split"):
            hi, lo = split_master(w)
            st.update(out=lo, aux_out=hi)
        else:
            st.update(out=w.clone(), aux_out=w.to(torch.bfloat16))
        if opt.startswith("adam"):
            st.update(opt_m=torch.full_like(w, 1e-3), opt_v=torch.full_like(w, 1e-4), step=2, betas=(0.9, 0.95),
                      eps=1e-8, wd=0.01)
        return st

    p2, p1, s2, s1 = state(w2t), state(w1), state(w2t), state(w1)
    gemm_pair(aT, dy, p2, daT, x, p1, layout="nn")
    gemm(aT, dy, "nn", **s2)
    gemm(daT, x, "nn", **s1)
    torch.cuda.synchronize()
    for p, s in ((p2, s2), (p1, s1)):
        for k in ("out", "aux_out", "opt_m", "opt_v"):
            if k in p:
                eq = torch.equal(p[k].view(torch.int16), s[k].view(torch.int16)) if p[k].dtype != torch.float32 \
                    else torch.equal(p[k], s[k])
                assert eq, (opt, k)
    if opt in ("sgd", "sgd_split"):
        grad = torch.empty(M, D, device=DEV)
        gemm(aT, dy, "nn", out=grad)
        torch.cuda.synchronize()
        step = 1e-2 * grad.double()
        want = w2t.double() - step
        got = p2["out"] if opt == "sgd" else join_master(p2["aux_out"], p2["out"])
        # fp32 rounding of the product and of the sum (relative to the operands: w and lr*g may cancel)
        assert ((got.double() - want).abs() <= 2 ** -22 * (w2t.double().abs() + step.abs()) + 1e-12).all()


def _tp8_engine(tmode: bool, L=2, seed=13):
    from dllm.models.ffn import init_ffn_params_device
    from dllm.parallel.engine import FFNTrainer
    from dllm.parallel.mesh import Mesh
    from dllm.utils.config import ModelConfig, TrainConfig

    cfg = TrainConfig(model=ModelConfig(4096, 1792, L, "relu", False), batch_size=2, seq_len=1024, dtype="bf16",
                      grad_dtype="bf16", wgrad_stream=False, tp_transposed=tmode)
    eng = FFNTrainer(cfg, Mesh(), torch.device(DEV))
    eng.load_full_params(init_ffn_params_device(4096, 1792, L, seed, torch.device(DEV), False))
    return cfg, eng


def test_engine_transposed_layout_matches_regular():
    """The TP8-shard engine (F = 1792) in the transposed layout: same forward output and, after 3 steps, the same
    fp32 masters as the regular layout up to summation order; the exported parameters are in the logical layout."""
    from dllm.utils.data import DeviceMockData

    res = []
    for tmode in (True, False):
        cfg, eng = _tp8_engine(tmode)
        assert eng.tmode == tmode
        data = DeviceMockData(cfg.tokens, 4096, torch.bfloat16, torch.device(DEV))
        ys = []
        for s in range(3):
            x, dy = data.fill(60 + s)
            ys.append(eng.train_step(x, dy).float().clone())
        torch.cuda.synchronize()
        res.append((ys, eng.local_params()))
    (yt, pt), (yr, pr) = res
    for a, b in zip(yt, yr):
        assert ((a - b).abs().max() / b.abs().max()).item() < 2e-2
    for lt, lr in zip(pt, pr):
        for name in ("w1", "w2"):
            assert lt[name].shape == lr[name].shape
            rel = ((lt[name] - lr[name]).abs().max() / lr[name].abs().max()).item()
            assert rel < 1e-3, (name, rel)


def test_engine_transposed_checkpoint_roundtrip(tmp_path):
    from dllm.utils.checkpoint import load_checkpoint, save_checkpoint

    _, eng = _tp8_engine(True, L=1)
    before = [{k: v.clone() for k, v in p.items()} for p in eng.local_params()]
    save_checkpoint(eng, str(tmp_path), step=0)
    _, eng2 = _tp8_engine(True, L=1, seed=99)
    load_checkpoint(eng2, str(tmp_path))
    after = eng2.local_params()
    for b, a in zip(before, after):
        for name in ("w1", "w2"):
            assert torch.equal(b[name], a[name]), name
    # and into the regular layout (the logical [D, F] W2 crosses over)
    _, eng3 = _tp8_engine(False, L=1, seed=98)
    load_checkpoint(eng3, str(tmp_path))
    for b, a in zip(before, eng3.local_params()):
        for name in ("w1", "w2"):
            assert torch.equal(b[name], a[name]), name
