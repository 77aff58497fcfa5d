"""Split fp32 master (bf16 working copy + int16 residual, ops/master.py) on the GPU kernels.

Every form of the SGD update -- the fused weight-gradient epilogue of each bf16 kernel family (256x256 2-stage,
8-phase one tile per block and persistent, 256x128 two-per-CU, split-K reduction, generic odd shapes) and the flat
optimizer kernel -- must leave bitwise the fp32 master the fp32-master form leaves, with the working copy equal to
that master rounded half away from zero.  The engine check: one training step from bf16-representable weights (no
rounding ties at the start) gives bitwise the fp32-master engine's master.
"""
import sys

import pytest
import torch

from dllm.ops.gemm import gemm, set_bf16_variant, set_splitk, set_tiles_per_block
from dllm.ops.master import join_flat, join_master, part_flat, split_master

pytestmark = pytest.mark.gpu


def _pair(M, N, K, seed):
    g = torch.Generator().manual_seed(seed)
    a = torch.randn(K, M, generator=g).to(torch.bfloat16).cuda()
    b = torch.randn(K, N, generator=g).to(torch.bfloat16).cuda()
    w = (torch.randn(M, N, generator=g) * 0.02).cuda()
    return a, b, w


def _check_same_update(a, b, w, lr=1e-2):
    m32, c16 = w.clone(), w.to(torch.bfloat16)
    gemm(a, b, "tn", out=m32, epi="sgd", lr=lr, aux_out=c16)
    hi, lo = split_master(w)
    gemm(a, b, "tn", out=lo, epi="sgd_split", lr=lr, aux_out=hi)
    torch.cuda.synchronize()
    assert torch.equal(join_master(hi, lo).view(torch.int32), m32.view(torch.int32))
    assert torch.equal(hi.view(torch.int16), split_master(m32)[0].view(torch.int16))


@pytest.mark.parametrize("variant,tpb", [("2stage", 1), ("8phase_stagger", 1), ("8phase_stagger", 8), ("pp", 1),
                                         ("pp", 8)])
def test_fused_sgd_split_equals_fp32_master(variant, tpb):
    old_v, old_t = set_bf16_variant(variant), set_tiles_per_block(tpb)
    try:
        a, b, w = _pair(2048, 1536, 1024, 5)   # 48 tiles: persistent grids hold several per block
        _check_same_update(a, b, w)
    finally:
        set_bf16_variant(old_v)
        set_tiles_per_block(old_t)


def test_fused_sgd_split_faulting_shape_of_parked_seam_patch():
    """The shape whose deferred-SGD experiment faulted in round 3 (4096 x 8192 x 4352, tpb 8; parked patch
    experiments/seam_and_defer_sgd.patch) on the SHIPPED persistent fused-SGD path: clean and bitwise equal to the fp32
    master form."""
    old_v, old_t = set_bf16_variant("8phase_stagger"), set_tiles_per_block(8)
    try:
        a, b, w = _pair(4096, 8192, 4352, 12)
        _check_same_update(a, b, w)
    finally:
        set_bf16_variant(old_v)
        set_tiles_per_block(old_t)


def test_fused_sgd_split_splitk_and_generic():
    set_splitk(True)
    a, b, w = _pair(512, 512, 2048, 6)         # 4 tiles -> split-K reduction applies the update
    _check_same_update(a, b, w)
    a, b, w = _pair(200, 136, 96, 7)           # odd shape -> generic kernel
    _check_same_update(a, b, w)


def test_flat_sgd_split_and_join_kernels():
    from dllm.ops.elementwise import sgd_split_step_, sgd_step_

    g = torch.Generator().manual_seed(8)
    n = 1 << 20
    w = (torch.randn(n, generator=g) * 0.02).cuda()
    grad = torch.randn(n, generator=g).to(torch.bfloat16).cuda()
    m32, c16 = w.clone(), w.to(torch.bfloat16)
    sgd_step_(m32, grad, 0.1, copy=c16)
    hi = torch.empty(n, dtype=torch.bfloat16, device="cuda")
    lo = torch.empty(n, dtype=torch.int16, device="cuda")
    part_flat(w, hi, lo)
    h_ref, l_ref = split_master(w)
    assert torch.equal(hi.view(torch.int16), h_ref.view(torch.int16)) and torch.equal(lo, l_ref)
    sgd_split_step_(lo, hi, grad, 0.1)
    assert torch.equal(join_flat(hi, lo).view(torch.int32), m32.view(torch.int32))
    # every 32-bit pattern survives the native split / join
    u = torch.randint(-2**31, 2**31 - 1, (n,), generator=g, dtype=torch.int32).cuda()
    part_flat(u.view(torch.float32), hi, lo)
    assert torch.equal(join_flat(hi, lo).view(torch.int32), u)


@pytest.mark.parametrize("wgrad_stream", [False, True])
def test_engine_split_master_step_equals_fp32(wgrad_stream):
    from dllm.parallel.engine import FFNTrainer
    from dllm.parallel.mesh import Mesh
    from dllm.utils.config import ModelConfig, TrainConfig
    from dllm.utils.data import DeviceMockData

    D, F, L = 512, 2048, 3
    g = torch.Generator().manual_seed(9)
    # bf16-representable weights: both formats start from the same working copy (no rounding ties)
    layers = [{"w1": (torch.randn(F, D, generator=g) * 0.02).bfloat16().float(),
               "w2": (torch.randn(D, F, generator=g) * 0.02).bfloat16().float()} for _ in range(L)]
    outs = []
    for fmt in ("fp32", "split"):
        cfg = TrainConfig(model=ModelConfig(D, F, L), batch_size=2, seq_len=512, dtype="bf16", grad_dtype="bf16",
                          lr=1e-2, master=fmt, wgrad_stream=wgrad_stream)
        eng = FFNTrainer(cfg, Mesh(), torch.device("cuda"))
        assert eng.split == (fmt == "split")
        eng.load_full_params(layers)
        x, dy = DeviceMockData(cfg.tokens, D, torch.bfloat16, torch.device("cuda")).fill(3)
        eng.train_step(x, dy)
        torch.cuda.synchronize()
        outs.append(eng.master.clone())
    assert torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32))


@pytest.mark.parametrize("variant,tpb,shape", [("8phase_stagger", 8, (2048, 1536, 1024)), ("pp", 1, (2048, 1536, 1024)),
                                               ("8phase_stagger", 8, (512, 512, 2048)), ("8phase_stagger", 8,
                                                                                          (200, 136, 96))])
def test_fused_adam_split_matches_fp32_master(variant, tpb, shape):
    """AdamW on a split master (fused epilogue: 8-phase persistent, 256x128, split-K seam, generic) == AdamW on an fp32
    master, to fp32 rounding of the moment math (the two epilogues may contract differently)."""
    M, N, K = shape
    old_v, old_t = set_bf16_variant(variant), set_tiles_per_block(tpb)
    try:
        a, b, w = _pair(M, N, K, 11)
        kw = dict(lr=1e-3, betas=(0.9, 0.95), eps=1e-8, wd=0.01, step=3)
        m0 = torch.full((M, N), 1e-3, device="cuda")
        v0 = torch.full((M, N), 1e-6, device="cuda")
        m32, ma, va = w.clone(), m0.clone(), v0.clone()
        gemm(a, b, "tn", out=m32, epi="adam", aux_out=w.to(torch.bfloat16), opt_m=ma, opt_v=va, **kw)
        hi, lo = split_master(w)
        mb, vb = m0.clone(), v0.clone()
        gemm(a, b, "tn", out=lo, epi="adam_split", aux_out=hi, opt_m=mb, opt_v=vb, **kw)
        torch.cuda.synchronize()
        torch.testing.assert_close(join_master(hi, lo), m32, rtol=1e-6, atol=1e-9)
        torch.testing.assert_close(mb, ma, rtol=1e-6, atol=1e-12)
        torch.testing.assert_close(vb, va, rtol=1e-6, atol=1e-15)
    finally:
        set_bf16_variant(old_v)
        set_tiles_per_block(old_t)


def test_flat_adam_split_kernel():
    from dllm.ops.elementwise import adam_split_step_, adam_step_

    g = torch.Generator().manual_seed(12)
    n = 1 << 18
    w = (torch.randn(n, generator=g) * 0.02).cuda()
    grad = torch.randn(n, generator=g).to(torch.bfloat16).cuda()
    ma, va = torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
    m32 = w.clone()
    adam_step_(m32, grad, ma, va, 1, 1e-3, wd=0.01)
    hi = torch.empty(n, dtype=torch.bfloat16, device="cuda")
    lo = torch.empty(n, dtype=torch.int16, device="cuda")
    part_flat(w, hi, lo)
    mb, vb = torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
    adam_split_step_(lo, hi, grad, mb, vb, 1, 1e-3, wd=0.01)
    torch.testing.assert_close(join_flat(hi, lo), m32, rtol=1e-6, atol=1e-9)
    torch.testing.assert_close(vb, va, rtol=1e-6, atol=1e-15)


def test_engine_high_priority_side_streams_bitwise(monkeypatch):
    """DLLM_SIDE_STREAMS=high (native high-priority wgrad / opt streams, utils/streams.py) changes only where the
    side work is queued: the step's master is bitwise the pool-stream step's."""
    from dllm.parallel.engine import FFNTrainer
    from dllm.parallel.mesh import Mesh
    from dllm.utils.config import ModelConfig, TrainConfig
    from dllm.utils.data import DeviceMockData

    D, F, L = 512, 2048, 3
    g = torch.Generator().manual_seed(13)
    layers = [{"w1": torch.randn(F, D, generator=g) * 0.02, "w2": torch.randn(D, F, generator=g) * 0.02}
              for _ in range(L)]
    outs = []
    # keep the weight-gradient stream in use (dllm.ops re-exports a function named gemm: patch the module itself)
    monkeypatch.setitem(sys.modules["dllm.ops.gemm"]._PAIR, "enabled", False)
    for mode in ("pool", "high", "auto"):
        monkeypatch.setenv("DLLM_SIDE_STREAMS", mode)
        cfg = TrainConfig(model=ModelConfig(D, F, L), batch_size=2, seq_len=512, dtype="bf16", grad_dtype="bf16",
                          lr=1e-2, wgrad_stream=True)
        eng = FFNTrainer(cfg, Mesh(), torch.device("cuda"))
        assert eng.wg_stream is not None
        assert isinstance(eng.wg_stream, torch.cuda.ExternalStream) == (mode != "pool")
        eng.load_full_params(layers)
        x, dy = DeviceMockData(cfg.tokens, D, torch.bfloat16, torch.device("cuda")).fill(3)
        for _ in range(2):
            eng.train_step(x, dy)
        torch.cuda.synchronize()
        outs.append(eng.master.clone())
    assert all(torch.equal(outs[0].view(torch.int32), o.view(torch.int32)) for o in outs[1:])
