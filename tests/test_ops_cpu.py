"""CPU checks of the op layer (torch reference path) and helpers."""
import pytest
import torch

from dllm.models import reference as R
from dllm.models.ffn import deinterleave_w13, init_ffn_layer, interleave_w13, layer_bwd, layer_fwd
from dllm.ops.elementwise import _philox_normal_cpu, adam_step_, philox4x32_10, rng_normal_, sgd_step_
from dllm.ops.gemm import _glu_merge, _glu_split, gemm
from dllm.utils.config import ModelConfig, TrainConfig
from dllm.utils.metrics import flops_per_step


def test_philox_known_answers():
    z = torch.zeros(1, dtype=torch.int64)
    f = torch.full((1,), 0xFFFFFFFF, dtype=torch.int64)
    assert [int(v) for v in philox4x32_10(z, z, z, z, 0, 0)] == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert [int(v) for v in philox4x32_10(f, f, f, f, 0xFFFFFFFF, 0xFFFFFFFF)] == [
        0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]


def test_rng_deterministic_and_normal():
    a = torch.empty(10_001)
    b = torch.empty(10_001)
    rng_normal_(a, seed=4, stream_id=2)
    rng_normal_(b, seed=4, stream_id=2)
    assert torch.equal(a, b)
    c = torch.empty(10_001)
    rng_normal_(c, seed=4, stream_id=3)
    assert not torch.equal(a, c)
    z = _philox_normal_cpu(1 << 18, 11, 0, 1.0)
    assert abs(z.mean().item()) < 1e-2 and abs(z.std().item() - 1.0) < 1e-2


def test_rng_bf16_stream_16bit_uniforms():
    """bf16 draws: 8 normals per Philox call from 16-bit uniforms (u1 = 1 - lo16/2^16, u2 = hi16/2^16), a prefix of a
    longer draw, N(0, 1) moments and tail mass, radius bounded by sqrt(-2 ln 2^-16)."""
    import math

    z = _philox_normal_cpu(1 << 20, 11, 0, 1.0, u16=True)
    assert abs(z.mean().item()) < 5e-3 and abs(z.std().item() - 1.0) < 5e-3
    assert abs((z.abs() > 2).float().mean().item() - 0.0455) < 2e-3
    assert z.abs().max().item() <= math.sqrt(-2 * math.log(2.0 ** -16)) + 1e-4
    c0, _, _, _ = philox4x32_10(torch.zeros(1, dtype=torch.int64), torch.zeros(1, dtype=torch.int64),
                                torch.zeros(1, dtype=torch.int64), torch.zeros(1, dtype=torch.int64), 11, 0)
    w = int(c0[0])
    u1, u2 = 1.0 - (w & 0xFFFF) / 65536.0, (w >> 16) / 65536.0
    assert abs(z[0].item() - math.sqrt(-2 * math.log(u1)) * math.cos(2 * math.pi * u2)) < 1e-5
    a = torch.empty(13, dtype=torch.bfloat16)
    b = torch.empty(1000, dtype=torch.bfloat16)
    rng_normal_(a, seed=5, stream_id=1)
    rng_normal_(b, seed=5, stream_id=1)
    assert torch.equal(a, b[:13])


def test_gemm_layouts_cpu():
    a, b = torch.randn(6, 5), torch.randn(7, 5)
    torch.testing.assert_close(gemm(a, b, "nt"), a @ b.t())
    torch.testing.assert_close(gemm(a, b.t().contiguous(), "nn"), a @ b.t())
    torch.testing.assert_close(gemm(a.t().contiguous(), b.t().contiguous(), "tn"), a @ b.t())
    c = torch.ones(6, 7)
    gemm(a, b, "nt", out=c, alpha=2.0, beta=1.0)
    torch.testing.assert_close(c, 2 * a @ b.t() + 1)


def test_glu_interleave_roundtrip():
    w1, w3 = torch.randn(64, 8), torch.randn(64, 8)
    w13 = interleave_w13(w1, w3)
    assert torch.equal(w13[:16], w1[:16]) and torch.equal(w13[16:32], w3[:16])
    r1, r3 = deinterleave_w13(w13)
    assert torch.equal(r1, w1) and torch.equal(r3, w3)
    h = torch.randn(3, 128)
    g, u = _glu_split(h)
    assert torch.equal(_glu_merge(g, u), h)


def _layer_check(act, gated):
    D, F, T = 16, 64, 32
    gen = torch.Generator().manual_seed(0)
    p = init_ffn_layer(D, F, gen, gated)
    x, dy = torch.randn(T, D, dtype=torch.float64), torch.randn(T, D, dtype=torch.float64)
    p = {k: v.double() for k, v in p.items()}
    w1 = interleave_w13(p["w1"], p["w3"]) if gated else p["w1"]
    R1 = w1.shape[0]
    a = torch.empty(T, F, dtype=torch.float64)
    h = torch.empty(T, R1, dtype=torch.float64)
    y = torch.empty(T, D, dtype=torch.float64)
    layer_fwd(x, w1, p["w2"], act, gated, a, h, y)
    torch.testing.assert_close(y, R.layer_fwd(p, x, act))
    gw1, gw2 = torch.empty_like(w1), torch.empty_like(p["w2"])
    dx = layer_bwd(dy, x, w1, p["w2"], act, gated, a, h, gw1, gw2, torch.empty(T, R1, dtype=torch.float64),
                   torch.empty(T, D, dtype=torch.float64))
    rdx, rg = R.layer_bwd(dy, p, x, act)
    torch.testing.assert_close(dx, rdx)
    torch.testing.assert_close(gw2, rg["w2"])
    if gated:
        g1, g3 = deinterleave_w13(gw1)
        torch.testing.assert_close(g1, rg["w1"])
        torch.testing.assert_close(g3, rg["w3"])
    else:
        torch.testing.assert_close(gw1, rg["w1"])


def test_layer_fwd_bwd_all_variants():
    for act in ("relu", "silu", "gelu"):
        for gated in (False, True):
            _layer_check(act, gated)


def test_autograd_agrees_with_reference_backward():
    """Hand-written backward == torch autograd of the forward (fp64)."""
    for act, gated in (("relu", False), ("gelu", False), ("silu", True)):
        gen = torch.Generator().manual_seed(1)
        p = {k: v.double().requires_grad_() for k, v in init_ffn_layer(8, 32, gen, gated).items()}
        x = torch.randn(10, 8, dtype=torch.float64, requires_grad=True)
        dy = torch.randn(10, 8, dtype=torch.float64)
        y = R.layer_fwd(p, x, act)
        y.backward(dy)
        dx, g = R.layer_bwd(dy, {k: v.detach() for k, v in p.items()}, x.detach(), act)
        torch.testing.assert_close(dx, x.grad)
        for k in p:
            torch.testing.assert_close(g[k], p[k].grad)


def test_optimizers_cpu():
    p, g = torch.randn(8), torch.randn(8)
    q = p.clone()
    sgd_step_(q, g, 0.1)
    torch.testing.assert_close(q, p - 0.1 * g)
    m, v = torch.zeros(8), torch.zeros(8)
    q = p.clone()
    adam_step_(q, g, m, v, 1, 0.01)
    torch.testing.assert_close(q, p - 0.01 * g / (g.abs() + 1e-8), rtol=1e-5, atol=1e-6)


def test_flops_accounting():
    cfg = TrainConfig(model=ModelConfig(4096, 0, 8), batch_size=8, seq_len=1024)
    unit = 2 * 8192 * 4096 * 16384
    assert flops_per_step(cfg, recompute="full", skip_dx0=False) == 8 * 7 * unit  # reference: 7 GEMMs / layer
    assert flops_per_step(cfg) == 8 * 6 * unit - unit


def test_gemm_scheduling_knobs_cpu():
    """Process-wide GEMM knobs round-trip without a GPU (the native library loads on CPU); ReLU-mask sizing."""
    from dllm.ops.gemm import relu_mask_bytes, relu_mask_supported, set_tiles_per_block

    old = set_tiles_per_block(4)
    assert set_tiles_per_block(0) == 4          # <= 1 -> one block per tile
    assert set_tiles_per_block(old) == 1
    assert relu_mask_bytes(8192, 16384) == 32 * 64 * 8192
    assert relu_mask_supported(8192, 16384, 4096)
    assert not relu_mask_supported(8192, 16384, 4096 + 64)    # K % 128: 2-stage kernel, no tile-native mask
    assert not relu_mask_supported(8192, 16384 + 128, 4096)   # N % 256
    assert not relu_mask_supported(512, 512, 2048)            # small grid -> split-K
    assert not relu_mask_supported(8192, 16384, 4096, torch.float32)


def test_engine_cpu_has_no_device_side_buffers():
    from dllm.parallel.engine import FFNTrainer
    from dllm.parallel.mesh import Mesh
    from dllm.utils.config import ModelConfig, TrainConfig

    cfg = TrainConfig(model=ModelConfig(256, 1024, 2, "relu", False), batch_size=1, seq_len=256, dtype="bf16",
                      wgrad_stream=True)
    eng = FFNTrainer(cfg, Mesh(), torch.device("cpu"))
    assert eng.masks is None and eng.wg_stream is None


def test_transposed_outputs_reference_cpu():
    """``out_t`` / ``aux_t`` (the NN weight-gradient layout) on the torch reference: out_t writes Cᵀ, aux_t a
    transposed copy next to the plain store; the NN-layout layer backward equals the TN one."""
    from dllm.models.ffn import NNWgrad
    from dllm.ops.gemm import transpose_bf16

    g = torch.Generator().manual_seed(0)
    T, D, F = 64, 32, 96
    x, da, dy, a = (torch.randn(*s, generator=g) for s in ((T, D), (T, F), (T, D), (T, F)))
    torch.testing.assert_close(gemm(x.t().contiguous(), da, "nn", out_t=True), gemm(da, x, "tn"))
    yT = torch.empty(D, T)
    w2 = torch.randn(D, F, generator=g)
    y = gemm(a, w2, "nt", aux_t=yT)
    assert torch.equal(yT, y.t())
    xt = torch.empty(D, T)
    assert torch.equal(transpose_bf16(x, xt), x.t())
    w1 = torch.randn(F, D, generator=g)
    ref, nn = [], []
    for mode in (None, "nn"):
        gw1, gw2 = torch.zeros(F, D), torch.zeros(D, F)
        dx_t = torch.empty(D, T)
        h = x @ w1.t()
        act = torch.relu(h)
        kw = {} if mode is None else {"nn": NNWgrad(x.t().contiguous(), dy.t().contiguous(), dx_t)}
        dx = layer_bwd(dy, x, w1, w2, "relu", False, act, None, gw1, gw2, torch.empty(T, F), torch.empty(T, D), **kw)
        (ref if mode is None else nn).extend([gw1, gw2, dx])
        if mode == "nn":
            assert torch.equal(dx_t, dx.t())
    for r, n in zip(ref, nn):
        torch.testing.assert_close(n, r)


def test_wgrad_layout_nn_needs_gpu():
    import pytest

    from dllm.parallel.engine import FFNTrainer
    from dllm.parallel.mesh import Mesh

    m = ModelConfig(model_size=256, ffn_dim=512, layers=1)
    for layout, ok in (("auto", True), ("tn", True), ("nn", False)):
        cfg = TrainConfig(model=m, batch_size=1, seq_len=256, wgrad_layout=layout)
        if ok:
            assert not FFNTrainer(cfg, Mesh(), torch.device("cpu")).wgrad_nn
        else:
            with pytest.raises(ValueError, match="wgrad_layout nn"):
                FFNTrainer(cfg, Mesh(), torch.device("cpu"))


def test_raster_band_policies_round_trip():
    """Per-layout raster bands (ops.gemm policy): each setter returns the previous value and clamps to >= 1; the
    default bands are NT 4, NN 8 (profiles/r5/group_m_nn_finite_r5.txt), TN 4."""
    from dllm.ops.gemm import _POLICY, set_group_m_nn, set_group_m_nt, set_group_m_tn

    assert (_POLICY["group_m_nt"], _POLICY["group_m_nn"], _POLICY["group_m_tn"]) == (4, 8, 4)
    for setter, key in ((set_group_m_nt, "group_m_nt"), (set_group_m_nn, "group_m_nn"), (set_group_m_tn, "group_m_tn")):
        old = setter(0)
        try:
            assert _POLICY[key] == 1
            assert setter(16) == 1 and _POLICY[key] == 16
        finally:
            setter(old)
        assert _POLICY[key] == old


def test_rng_out_t_fallback_is_the_transpose():
    """rng_normal_(..., out_t=) off the GPU kernel's domain: the same draw, plus its transpose."""
    from dllm.ops.elementwise import rng_normal_

    a, at = torch.empty(96, 40, dtype=torch.bfloat16), torch.empty(40, 96, dtype=torch.bfloat16)
    rng_normal_(a, seed=3, stream_id=1, scale=0.1, out_t=at)
    b = torch.empty_like(a)
    rng_normal_(b, seed=3, stream_id=1, scale=0.1)
    assert torch.equal(a, b) and torch.equal(at, b.t())
    with pytest.raises(ValueError):
        rng_normal_(a, seed=3, out_t=torch.empty(96, 40, dtype=torch.bfloat16))
