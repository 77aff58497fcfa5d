"""Grouped weight-gradient pairs (``ops.gemm.gemm_pair`` -> ``gemm_bf16_8ph_pair``): two TN GEMMs in one launch of
whole 256x256 tiles, as the MP (TP8) shard's dW2 [D, F/8] | dW1 [F/8, D] run instead of two split-K GEMMs plus their
reduction passes (reference: the TP worker's per-shard weight gradients + SGD, train_ffns.py:306-312).

Each half of the pair must equal the same GEMM run alone on the 8-phase kernel, one tile per block, bitwise, for
every epilogue the weight gradients use (plain fp32 / bf16 store, fused SGD and AdamW on fp32 or split masters); and
the store form must match an fp64 reference, including an A = I / asymmetric-B layout check."""
import pytest
import torch

from dllm.ops.gemm import gemm, gemm_pair, pair_supported, set_splitk
from dllm.ops.master import join_master, split_master

pytestmark = pytest.mark.gpu

# the MP config's TP8 shard at reduced T: dW2 = dyᵀ·a [D, F'] and dW1 = daᵀ·x [F', D] with F' = 1792, D = 4096
D, FL, T = 4096, 1792, 2048


def _ops(seed):
    g = torch.Generator().manual_seed(seed)
    dy = torch.randn(T, D, generator=g).to(torch.bfloat16).cuda()
    a = torch.randn(T, FL, generator=g).to(torch.bfloat16).cuda()
    da = torch.randn(T, FL, generator=g).to(torch.bfloat16).cuda()
    x = torch.randn(T, D, generator=g).to(torch.bfloat16).cuda()
    return dy, a, da, x


def _alone(a, b, kw):
    old = set_splitk(False)   # the reference run: one whole tile per block, no split-K
    try:
        gemm(a, b, "tn", **kw)
    finally:
        set_splitk(old)


def test_pair_supported_for_tp8_shard_only():
    assert pair_supported(((4096, 1792, 8192), (1792, 4096, 8192)))          # 112 + 112 tiles, each would split
    assert not pair_supported(((4096, 16384, 8192), (16384, 4096, 8192)))    # flagship: 1024 tiles each
    assert not pair_supported(((4096, 3584, 8192), (7168, 4096, 8192)))      # gated TP8: 224 + 448 > 256 CUs


@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
def test_pair_store_matches_alone_and_fp64(out_dtype):
    dy, a, da, x = _ops(1)
    o2, o1 = torch.empty(D, FL, dtype=out_dtype, device="cuda"), torch.empty(FL, D, dtype=out_dtype, device="cuda")
    gemm_pair(dy, a, {"out": o2}, da, x, {"out": o1})
    r2, r1 = torch.empty_like(o2), torch.empty_like(o1)
    _alone(dy, a, {"out": r2})
    _alone(da, x, {"out": r1})
    torch.cuda.synchronize()
    assert torch.equal(o2, r2) and torch.equal(o1, r1)
    ref2 = dy.double().t() @ a.double()
    ref1 = da.double().t() @ x.double()
    tol = 2e-2 if out_dtype == torch.bfloat16 else 1e-4
    for o, r in ((o2, ref2), (o1, ref1)):
        err = ((o.double() - r).abs().max() / r.abs().max()).item()
        assert err < tol, err


def test_pair_layout_identity_asymmetric():
    """A = I (K = M) with an asymmetric B: each output must be exactly B (a transposed output or swapped operand map
    would give Bᵀ or garbage), in both halves of the grid."""
    K = 2048
    eye = torch.eye(K, dtype=torch.bfloat16, device="cuda")
    g = torch.Generator().manual_seed(3)
    b0 = (torch.arange(K * 1792, dtype=torch.float32).reshape(K, 1792) % 251 - 125).to(torch.bfloat16).cuda()
    b1 = torch.randint(-8, 8, (K, 1024), generator=g).to(torch.bfloat16).cuda()
    o0 = torch.empty(K, 1792, device="cuda")
    o1 = torch.empty(K, 1024, device="cuda")
    gemm_pair(eye, b0, {"out": o0}, eye, b1, {"out": o1})
    torch.cuda.synchronize()
    assert torch.equal(o0, b0.float()) and torch.equal(o1, b1.float())


@pytest.mark.parametrize("opt", ["sgd", "sgd_split", "adam", "adam_split"])
def test_pair_fused_optimizer_bitwise_alone(opt):
    dy, a, da, x = _ops(2)
    g = torch.Generator().manual_seed(4)
    w2 = (torch.randn(D, FL, generator=g) * 0.02).cuda()
    w1 = (torch.randn(FL, D, generator=g) * 0.02).cuda()

    def state(w):
        st = {}
        if opt.endswith("split"):
            hi, lo = split_master(w)
            st.update(out=lo, aux_out=hi)
        else:
            st.update(out=w.clone(), aux_out=w.to(torch.bfloat16))
        if opt.startswith("adam"):
            st.update(opt_m=torch.full_like(w, 1e-3), opt_v=torch.full_like(w, 1e-4), step=3, betas=(0.9, 0.95),
                      eps=1e-8, wd=0.01)
        st.update(epi=opt, lr=1e-2)
        return st

    p2, p1, s2, s1 = state(w2), state(w1), state(w2), state(w1)
    gemm_pair(dy, a, p2, da, x, p1)
    _alone(dy, a, s2)
    _alone(da, x, s1)
    torch.cuda.synchronize()
    for p, s in ((p2, s2), (p1, s1)):
        for k in ("out", "aux_out", "opt_m", "opt_v"):
            if k in p:
                assert torch.equal(p[k].view(torch.int16) if p[k].dtype == torch.bfloat16 else p[k],
                                   s[k].view(torch.int16) if s[k].dtype == torch.bfloat16 else s[k]), (opt, k)
    if opt == "sgd_split":   # and the update itself is right: fp32 master moved by -lr * grad
        ref = w2.double() - 1e-2 * (dy.double().t() @ a.double())
        got = join_master(p2["aux_out"], p2["out"]).double()
        assert ((got - ref).abs().max() / (w2.double() - ref).abs().max()).item() < 1e-3


def test_engine_tp8_shard_pairs_wgrads():
    """The MP / TP8-shard engine step (F = 1792 per rank) uses the pair and matches the unpaired step closely (the
    unpaired form runs split-K, whose partial sums round differently)."""
    from dllm.models.ffn import init_ffn_params_device
    from dllm.parallel.engine import FFNTrainer
    from dllm.parallel.mesh import Mesh
    from dllm.utils.config import ModelConfig, TrainConfig
    from dllm.utils.data import DeviceMockData

    from dllm.ops.gemm import set_pair_wgrads

    outs = []
    for paired in (True, False):
        old = set_pair_wgrads(paired)
        try:
            cfg = TrainConfig(model=ModelConfig(4096, 1792, 2, "relu", False), batch_size=2, seq_len=1024,
                              dtype="bf16", grad_dtype="bf16", wgrad_stream=False, tp_transposed=False)
            eng = FFNTrainer(cfg, Mesh(), torch.device("cuda"))
            assert eng.pair_wgrads == paired
            eng.load_full_params(init_ffn_params_device(4096, 1792, 2, 9, torch.device("cuda"), False))
            data = DeviceMockData(cfg.tokens, 4096, torch.bfloat16, torch.device("cuda"))
            for s in range(3):
                x, dy = data.fill(40 + s)
                eng.train_step(x, dy)
            torch.cuda.synchronize()
            outs.append(eng.master.clone())
        finally:
            set_pair_wgrads(old)
    assert torch.isfinite(outs[0]).all()
    rel = ((outs[0] - outs[1]).abs().max() / outs[1].abs().max()).item()
    assert rel < 1e-3, rel
