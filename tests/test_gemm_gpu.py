"""Numerics of the hand-written gfx950 GEMM kernels against plain PyTorch fp32/fp64 references.

Covers all three operand layouts (NT fwd, NN dgrad, TN wgrad), every fused epilogue, the three kernel
families (bf16 256² MFMA, fp32 MFMA, generic), exact-integer layout checks (A = I with an asymmetric B,
cdna_hip_programming.md §3), strided views, beta-accumulation and odd shapes.
"""
import os

import pytest
import torch

from dllm.ops.gemm import gemm, gemm_path, set_bf16_variant

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _mk(shape, dtype, seed, scale=1.0, integer=False):
    g = torch.Generator().manual_seed(seed)
    if integer:
        t = torch.randint(-3, 4, shape, generator=g).float()
    else:
        t = torch.randn(shape, generator=g) * scale
    return t.to(dtype)


def _operands(layout, M, N, K, dtype, seed=0, integer=False):
    if layout == "nt":
        a, b = _mk((M, K), dtype, seed, integer=integer), _mk((N, K), dtype, seed + 1, integer=integer)
    elif layout == "nn":
        a, b = _mk((M, K), dtype, seed, integer=integer), _mk((K, N), dtype, seed + 1, integer=integer)
    else:
        a, b = _mk((K, M), dtype, seed, integer=integer), _mk((K, N), dtype, seed + 1, integer=integer)
    return a, b


def _ref(a, b, layout):
    a, b = a.double(), b.double()
    return {"nt": lambda: a @ b.t(), "nn": lambda: a @ b, "tn": lambda: a.t() @ b}[layout]()


@pytest.fixture(params=["2stage", "8phase", "8phase_stagger", "4phase_stagger", "pp"])
def variant(request):
    old = set_bf16_variant(request.param)
    yield request.param
    set_bf16_variant(old)


def test_native_library_is_loaded():
    import dllm._native as nat

    nat.lib()
    maps = open("/proc/self/maps").read()
    assert "_dllm_native.so" in maps
    hip = {l.split()[-1] for l in maps.splitlines() if "libamdhip64" in l}
    assert len(hip) == 1, f"more than one HIP runtime mapped: {hip}"


@pytest.mark.parametrize("layout", ["nt", "nn", "tn"])
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 320), (768, 512, 1024), (512, 512, 128),
                                   (1280, 768, 640)])
def test_bf16_mfma_exact_integers(layout, M, N, K, variant):
    a, b = _operands(layout, M, N, K, torch.bfloat16, seed=M + N + K, integer=True)
    assert gemm_path(torch.bfloat16, torch.float32, M, N, K, a.stride(0), b.stride(0), N) == "mfma_bf16"
    out = gemm(a.to(DEV), b.to(DEV), layout, out_dtype=torch.float32, force="mfma_bf16")
    torch.cuda.synchronize()
    assert torch.equal(out.cpu().double(), _ref(a, b, layout))


@pytest.mark.parametrize("layout", ["nt", "nn", "tn"])
def test_identity_asymmetric(layout, variant):
    n = 256
    eye = torch.eye(n, dtype=torch.bfloat16)
    B = (torch.arange(n * n).reshape(n, n) % 7 - 3).to(torch.bfloat16) * torch.arange(1, n + 1).reshape(n, 1).remainder(5).to(torch.bfloat16)
    out = gemm(eye.to(DEV), B.to(DEV), layout, out_dtype=torch.float32, force="mfma_bf16").cpu()
    want = {"nt": B.t(), "nn": B, "tn": B}[layout].float()
    assert torch.equal(out, want)


@pytest.mark.parametrize("layout", ["nt", "nn", "tn"])
@pytest.mark.parametrize("out_dtype", [torch.bfloat16, torch.float32])
def test_bf16_mfma_random(layout, out_dtype, variant):
    M, N, K = 512, 1024, 768
    a, b = _operands(layout, M, N, K, torch.bfloat16, seed=5)
    out = gemm(a.to(DEV), b.to(DEV), layout, out_dtype=out_dtype, force="mfma_bf16").cpu().double()
    ref = _ref(a, b, layout)
    err = (out - ref).abs().max() / ref.abs().max()
    assert err < (8e-3 if out_dtype == torch.bfloat16 else 1e-5), err


@pytest.mark.parametrize("act", ["relu", "silu", "gelu"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_epilogues_match_torch(act, dtype, variant):
    M, N, K = 256, 512, 256
    force = "mfma_bf16" if dtype == torch.bfloat16 else "mfma_f32"
    x, w1 = _operands("nt", M, N, K, dtype, seed=11)
    # fwd: act with aux_out
    a_cpu = torch.empty(M, N, dtype=dtype)
    h_cpu = torch.empty(M, N, dtype=dtype)
    gemm(x, w1, "nt", out=a_cpu, epi="act", act=act, aux_out=h_cpu)
    a_g = torch.empty(M, N, dtype=dtype, device=DEV)
    h_g = torch.empty(M, N, dtype=dtype, device=DEV)
    gemm(x.to(DEV), w1.to(DEV), "nt", out=a_g, epi="act", act=act, aux_out=h_g, force=force)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    torch.testing.assert_close(h_g.cpu().float(), h_cpu.float(), rtol=tol, atol=tol)
    torch.testing.assert_close(a_g.cpu().float(), a_cpu.float(), rtol=tol, atol=tol)
    # dgrad with act' mask: da = (dy · W2) * act'(h)    (NN)
    dy, w2 = _operands("nn", M, N, 384, dtype, seed=12)  # dy [M, 384], w2 [384, N]
    da_cpu = torch.empty(M, N, dtype=dtype)
    gemm(dy, w2, "nn", out=da_cpu, epi="dact", act=act, aux=h_cpu)
    da_g = torch.empty(M, N, dtype=dtype, device=DEV)
    gemm(dy.to(DEV), w2.to(DEV), "nn", out=da_g, epi="dact", act=act, aux=h_cpu.to(DEV), force=force)
    torch.testing.assert_close(da_g.cpu().float(), da_cpu.float(), rtol=tol, atol=tol * 4)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_gated_epilogues(dtype, variant):
    M, N, K = 256, 512, 256  # N = 2F interleaved
    force = "mfma_bf16" if dtype == torch.bfloat16 else "mfma_f32"
    x, w13 = _operands("nt", M, N, K, dtype, seed=21)
    a_c, h_c = torch.empty(M, N // 2, dtype=dtype), torch.empty(M, N, dtype=dtype)
    gemm(x, w13, "nt", out=a_c, epi="glu", act="silu", aux_out=h_c)
    a_g, h_g = torch.empty(M, N // 2, dtype=dtype, device=DEV), torch.empty(M, N, dtype=dtype, device=DEV)
    gemm(x.to(DEV), w13.to(DEV), "nt", out=a_g, epi="glu", act="silu", aux_out=h_g, force=force)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    torch.testing.assert_close(h_g.cpu().float(), h_c.float(), rtol=tol, atol=tol)
    # act(g)*u amplifies the summation-order error of u by |act(g)| (up to ~70 here): scale atol
    torch.testing.assert_close(a_g.cpu().float(), a_c.float(), rtol=tol, atol=tol * a_c.abs().max().item())
    dy, w2 = _operands("nn", M, N // 2, 256, dtype, seed=22)
    d_c = torch.empty(M, N, dtype=dtype)
    gemm(dy, w2, "nn", out=d_c, epi="dglu", act="silu", aux=h_c)
    d_g = torch.empty(M, N, dtype=dtype, device=DEV)
    gemm(dy.to(DEV), w2.to(DEV), "nn", out=d_g, epi="dglu", act="silu", aux=h_c.to(DEV), force=force)
    torch.testing.assert_close(d_g.cpu().float(), d_c.float(), rtol=tol, atol=tol * d_c.abs().max().item())


@pytest.mark.parametrize("layout", ["nt", "nn", "tn"])
@pytest.mark.parametrize("M,N,K", [(256, 384, 272), (512, 768, 288), (256, 256, 32), (768, 512, 96)])
def test_fp32_mfma_exact_f32(layout, M, N, K):
    """Exact-fp32 MFMA paths: the 128x128 kernel (N % 256 != 0) and the 256x256 LDS-DMA kernel (2-stage ring,
    K permutation; nk = 9 / 1 / 3 cover the ring's prologue and tail)."""
    a, b = _operands(layout, M, N, K, torch.float32, seed=3)
    assert gemm_path(torch.float32, torch.float32, M, N, K, a.stride(0), b.stride(0), N) == "mfma_f32"
    out = gemm(a.to(DEV), b.to(DEV), layout, force="mfma_f32").cpu().double()
    ref = _ref(a, b, layout)
    assert ((out - ref).abs().max() / ref.abs().max()) < 1e-6


@pytest.fixture(params=["mfma_f32", "bf16x6"])
def fp32_mode(request):
    from dllm.ops.gemm import set_fp32_mode

    old = set_fp32_mode(request.param)
    yield request.param
    set_fp32_mode(old)


def test_split3_planes_are_exact():
    """The bf16x6 operand split: the three bf16 parts sum exactly to the fp32 input (normals, wide exponent range,
    signed zeros), an inf/nan lands in part 0 alone, and the six planes follow the A / B pairing in both forms."""
    from dllm.ops.gemm import split3

    g = torch.Generator().manual_seed(4)
    x = torch.randn(64, 96, generator=g) * torch.exp2(torch.randint(-60, 60, (64, 96), generator=g).float())
    x[0, :8] = torch.tensor([0.0, -0.0, 1.0, -1.0, 3.4e38, 1.1754944e-38, float("inf"), float("nan")])
    xd = x.to(DEV)
    for role, order in ((0, (0, 1, 2, 0, 1, 0)), (1, (2, 1, 0, 1, 0, 0))):
        for rows in (False, True):
            s = split3(xd, role, rows).cpu()
            planes = s.view(6, 64, 96) if rows else s.view(64, 6, 96).transpose(0, 1)
            parts = [None] * 3
            for p, q in enumerate(order):
                if parts[q] is None:
                    parts[q] = planes[p].clone()
                assert torch.equal(planes[p].view(torch.int16), parts[q].view(torch.int16)), (role, rows, p)
            tot = parts[0].double() + parts[1].double() + parts[2].double()
            fin = torch.isfinite(x)  # incl. 3.4e38, above the largest finite bf16 (part 0 truncated, not inf)
            assert torch.equal(tot[fin], x.double()[fin])
            assert torch.isinf(parts[0][0, 6].float()) and torch.isnan(parts[0][0, 7].float())
            assert parts[1][0, 6].item() == 0 and parts[2][0, 7].item() == 0


@pytest.mark.parametrize("layout", ["nt", "nn", "tn"])
@pytest.mark.parametrize("M,N,K", [(256, 512, 64), (512, 256, 1024), (768, 512, 4096)])
def test_bf16x6_fp32_accuracy(layout, M, N, K):
    """The split fp32 GEMM (bf16 MFMA, six partial products) carries fp32 accuracy: vs an fp64 reference its error
    is at the fp32 MFMA kernel's level (both sum K fp32 products in an fp32 accumulator)."""
    a, b = _operands(layout, M, N, K, torch.float32, seed=31)
    ref = _ref(a, b, layout)
    split = gemm(a.to(DEV), b.to(DEV), layout, force="bf16x6").cpu().double()
    f32 = gemm(a.to(DEV), b.to(DEV), layout, force="mfma_f32").cpu().double()
    scale = ref.abs().max()
    e_split, e_f32 = (split - ref).abs().max() / scale, (f32 - ref).abs().max() / scale
    assert e_split < 2e-6, e_split
    assert e_split < 3 * e_f32 + 1e-7, (e_split, e_f32)
    # bf16 inputs would be 2-3 orders of magnitude off: the low parts are really used
    lo = gemm(a.to(DEV).bfloat16(), b.to(DEV).bfloat16(), layout, out_dtype=torch.float32).cpu().double()
    assert (lo - ref).abs().max() / scale > 100 * e_split


@pytest.mark.parametrize("epi", ["act", "dact", "sgd", "adam", "glu", "beta"])
def test_fp32_256_epilogues(epi, fp32_mode):
    """The fp32 GEMMs' fused epilogues vs the torch oracle: the 256x256 fp32 MFMA kernel and the bf16x6 split
    path (bf16 8-phase kernel with fp32 outputs); the epilogue code is shared with the bf16 kernels."""
    M, N, K = 512, 512, 256
    layout = {"act": "nt", "dact": "nn", "sgd": "tn", "adam": "tn", "glu": "nt", "beta": "nt"}[epi]
    a, b = _operands(layout, M, N, K, torch.float32, seed=13)
    kw = {}
    out = _mk((M, N // 2 if epi == "glu" else N), torch.float32, 14)
    if epi == "act":
        kw = dict(epi="act", act="gelu", aux_out=torch.zeros(M, N))
    elif epi == "dact":
        kw = dict(epi="dact", act="silu", aux=_mk((M, N), torch.float32, 15))
    elif epi == "glu":
        kw = dict(epi="glu", act="silu", aux_out=torch.zeros(M, N))
    elif epi == "beta":
        kw = dict(beta=0.5, alpha=2.0)
    elif epi in ("sgd", "adam"):
        kw = dict(epi=epi, lr=1e-2)
        if epi == "adam":
            kw.update(step=3, opt_m=torch.full((M, N), 0.01), opt_v=torch.full((M, N), 1e-4))
    want_out = out.clone()
    want_kw = {k: (v.clone() if isinstance(v, torch.Tensor) else v) for k, v in kw.items()}
    gemm(a, b, layout, out=want_out, **want_kw)  # CPU: the torch oracle
    got_kw = {k: (v.to(DEV) if isinstance(v, torch.Tensor) else v) for k, v in kw.items()}
    got_out = out.to(DEV)
    gemm(a.to(DEV), b.to(DEV), layout, out=got_out, **got_kw)
    # summation order differs from torch's (K-permuted exact-fp32 MFMA chain): ~K ulps of the largest value;
    # device GELU/SiLU vs torch's: a few more
    tol = 1e-4 if epi in ("act", "glu") else 1e-5
    torch.testing.assert_close(got_out.cpu(), want_out, rtol=tol, atol=2e-6 * float(want_out.abs().max()) + tol)
    for k, v in got_kw.items():
        if isinstance(v, torch.Tensor) and k in ("aux_out", "opt_m", "opt_v"):
            w = want_kw[k]
            torch.testing.assert_close(v.cpu(), w, rtol=1e-5, atol=1e-6 * float(w.abs().max()) + 1e-12)


@pytest.mark.parametrize("layout", ["nt", "nn", "tn"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("epi", ["store", "act", "dact"])
def test_generic_odd_shapes(layout, dtype, epi):
    if layout == "tn" and epi != "store":
        pytest.skip("activation epilogues: NT / NN only (TN runs the weight gradients)")
    M, N, K = 100, 70, 37
    a, b = _operands(layout, M, N, K, dtype, seed=7)
    aux = _mk((M, N), dtype, 9) if epi == "dact" else None
    out_c = torch.empty(M, N, dtype=dtype)
    gemm(a, b, layout, out=out_c, epi=epi, act="gelu", aux=aux)
    out_g = torch.empty(M, N, dtype=dtype, device=DEV)
    gemm(a.to(DEV), b.to(DEV), layout, out=out_g, epi=epi, act="gelu",
         aux=aux.to(DEV) if aux is not None else None, force="generic")
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    torch.testing.assert_close(out_g.cpu().float(), out_c.float(), rtol=tol, atol=tol)


def test_strided_views_and_beta():
    M, N, K = 256, 512, 256
    big_a = _mk((M, K + 64), torch.bfloat16, 1)
    big_b = _mk((N, K + 128), torch.bfloat16, 2)
    a, b = big_a[:, :K], big_b[:, 64:64 + K]
    c0 = _mk((M, N), torch.float32, 3)
    out = c0.clone().to(DEV)
    gemm(big_a.to(DEV)[:, :K], big_b.to(DEV)[:, 64:64 + K], "nt", out=out, beta=1.0, alpha=0.5,
         force="mfma_bf16")
    ref = 0.5 * _ref(a, b, "nt") + c0.double()
    assert ((out.cpu().double() - ref).abs().max() / ref.abs().max()) < 1e-5


def test_rng_matches_cpu_philox():
    from dllm.ops.elementwise import rng_normal_

    g = torch.empty(4099, device=DEV)
    c = torch.empty(4099)
    rng_normal_(g, seed=123, stream_id=1, scale=0.5)
    rng_normal_(c, seed=123, stream_id=1, scale=0.5)
    torch.testing.assert_close(g.cpu(), c, rtol=1e-4, atol=1e-4)
    # bf16: the 16-bit-uniform stream (8 normals per Philox call, a tail that is not a multiple of 8); the hardware
    # transcendentals and libm may round to neighbouring bf16 values
    gb = torch.empty(4099, device=DEV, dtype=torch.bfloat16)
    cb = torch.empty(4099, dtype=torch.bfloat16)
    rng_normal_(gb, seed=123, stream_id=1, scale=0.5)
    rng_normal_(cb, seed=123, stream_id=1, scale=0.5)
    torch.testing.assert_close(gb.cpu().float(), cb.float(), rtol=2 ** -7, atol=1e-3)
    assert (gb.cpu() == cb).float().mean().item() > 0.95
    big = torch.empty(1 << 22, device=DEV, dtype=torch.bfloat16)
    rng_normal_(big, seed=9)
    f = big.float()
    assert abs(f.mean().item()) < 5e-3 and abs(f.std().item() - 1) < 5e-3


@pytest.mark.parametrize("R,C", [(8192, 4096), (192, 320), (64, 64)])
def test_rng_with_transpose_bitwise(R, C):
    """The one-pass draw + transpose (rng_normal_bf16_t_kernel) is bitwise the flat draw and the transpose kernel."""
    from dllm.ops.elementwise import rng_normal_
    from dllm.ops.gemm import transpose_bf16

    a = torch.empty(R, C, device=DEV, dtype=torch.bfloat16)
    at = torch.full((C, R), 7.0, device=DEV, dtype=torch.bfloat16)
    rng_normal_(a, seed=5, stream_id=1, scale=0.1, out_t=at)
    b = torch.empty_like(a)
    bt = torch.empty_like(at)
    rng_normal_(b, seed=5, stream_id=1, scale=0.1)
    transpose_bf16(b, bt)
    assert torch.equal(a.view(torch.int16), b.view(torch.int16))
    assert torch.equal(at.view(torch.int16), bt.view(torch.int16))
    assert torch.equal(at.view(torch.int16), b.t().contiguous().view(torch.int16))


@pytest.mark.parametrize("n", [8192 * 1792, 4099, 64])
def test_rng_pair_bitwise(n):
    """x and dy in one launch (rng_normal_bf16_pair_kernel) are bitwise the two separate draws, tails included."""
    from dllm.ops.elementwise import rng_normal_, rng_normal_pair_

    a, b = torch.empty(n, device=DEV, dtype=torch.bfloat16), torch.empty(n, device=DEV, dtype=torch.bfloat16)
    rng_normal_pair_(a, b, 11, 0, 1.0, 1, 0.1)
    a1, b1 = torch.empty_like(a), torch.empty_like(b)
    rng_normal_(a1, seed=11, stream_id=0, scale=1.0)
    rng_normal_(b1, seed=11, stream_id=1, scale=0.1)
    assert torch.equal(a.view(torch.int16), a1.view(torch.int16))
    assert torch.equal(b.view(torch.int16), b1.view(torch.int16))


def test_device_data_draws_engine_transposes():
    """DeviceMockData.bind_transposed: the NN layout's layer-0 xᵀ / top dyᵀ come with the batch, the engine skips its
    transposes (tag consumed), and the step is bitwise the engine-transposed one."""
    from dllm.models.ffn import init_ffn_params_device
    from dllm.parallel.engine import FFNTrainer
    from dllm.parallel.mesh import Mesh
    from dllm.utils.config import ModelConfig, TrainConfig
    from dllm.utils.data import DeviceMockData

    dev = torch.device(DEV)

    def run(bind):
        m = ModelConfig(model_size=2048, ffn_dim=8192, layers=2, act="relu")   # NN-layout shapes (no split-K)
        cfg = TrainConfig(model=m, batch_size=1, seq_len=1024, dtype="bf16", optimizer="sgd")
        eng = FFNTrainer(cfg, Mesh(), dev)
        assert eng.wgrad_nn and eng.input_transposes()[0] is not None
        eng.load_full_params(init_ffn_params_device(m.D, m.F, m.layers, 0, dev, scale="fan_in"))
        data = DeviceMockData(cfg.tokens, m.D, torch.bfloat16, dev)
        if bind:
            data.bind_transposed(*eng.input_transposes())
        for s_ in range(3):
            x, dy = data.fill(s_)
            assert (getattr(x, "_dllm_t", None) is eng.xT[0]) == bind
            eng.train_step(x, dy)
            assert getattr(x, "_dllm_t", None) is None
        torch.cuda.synchronize()
        return [t.float().cpu() for layer in eng.gather_full_params() for t in layer.values()]

    from dllm.ops.gemm import set_splitk

    old = set_splitk(False)   # T = 1024: the NN layout's shapes without split-K (as in test_gemm_nnwgrad_gpu.py)
    try:
        ref, got = run(False), run(True)
    finally:
        set_splitk(old)
    for p0, p1 in zip(ref, got):
        assert torch.equal(p0, p1)


@pytest.mark.parametrize("gdt", [torch.float32, torch.bfloat16])
def test_optimizers_match_torch(gdt):
    from dllm.ops.elementwise import adam_step_, sgd_step_

    n = 4096 + 64
    p = torch.randn(n)
    gr = torch.randn(n).to(gdt)
    pg, cg = p.clone().to(DEV), torch.empty(n, dtype=torch.bfloat16, device=DEV)
    sgd_step_(pg, gr.to(DEV), 0.1, copy=cg)
    pc = p.clone()
    sgd_step_(pc, gr, 0.1)
    torch.testing.assert_close(pg.cpu(), pc)
    torch.testing.assert_close(cg.cpu().float(), pc.to(torch.bfloat16).float())
    m, v = torch.zeros(n), torch.zeros(n)
    mg, vg = m.to(DEV), v.to(DEV)
    pa, pag = p.clone(), p.clone().to(DEV)
    for step in (1, 2, 3):
        adam_step_(pa, gr, m, v, step, 1e-3, wd=0.01)
        adam_step_(pag, gr.to(DEV), mg, vg, step, 1e-3, wd=0.01)
    torch.testing.assert_close(pag.cpu(), pa, rtol=1e-5, atol=1e-6)


def test_streams_and_events_overlap():
    """test_torch_cuda_stream.py done with assertions: native GEMMs on several HIP streams, joined by events."""
    streams = [torch.cuda.Stream() for _ in range(4)]
    a = [_mk((256, 256), torch.bfloat16, i).to(DEV) for i in range(4)]
    b = [_mk((256, 256), torch.bfloat16, 10 + i).to(DEV) for i in range(4)]
    outs = [torch.empty(256, 256, dtype=torch.float32, device=DEV) for _ in range(4)]
    cur = torch.cuda.current_stream()
    for s in streams:
        s.wait_stream(cur)
    for i, s in enumerate(streams):
        with torch.cuda.stream(s):
            for _ in range(10):
                gemm(a[i], b[i], "nt", out=outs[i])
    for s in streams:
        cur.wait_stream(s)
    total = sum(outs)
    ref = sum(_ref(x.cpu(), y.cpu(), "nt") for x, y in zip(a, b))
    assert ((total.cpu().double() - ref).abs().max() / ref.abs().max()) < 1e-5


@pytest.mark.parametrize("layout", ["nt", "nn", "tn"])
@pytest.mark.parametrize("epi", ["store", "act", "dact", "glu", "dglu", "store_f32", "sgd", "adam"])
def test_splitk_matches_unsplit(layout, epi):
    """Split-K (fp32 partials + reduction epilogue) on a small tile grid == the single-pass kernel."""
    from dllm.ops.gemm import choose_ksplit, set_splitk

    M, N, K = 512, 512, 2048   # 4 tiles -> split 8
    if epi in ("sgd", "adam") and layout != "tn":
        pytest.skip("optimizer epilogues are weight-gradient (TN) only")
    if epi in ("act", "dact", "glu", "dglu") and layout == "tn":
        pytest.skip("activation epilogues: NT / NN only (TN runs the weight gradients)")
    assert choose_ksplit(M, N, K) > 1
    a, b = _operands(layout, M, N, K, torch.bfloat16, seed=31)
    a, b = a.cuda(), b.cuda()
    res = []
    for split in (False, True):
        set_splitk(split)
        kw = {}
        if epi in ("store", "act", "dact", "glu", "dglu"):
            ncols = {"glu": N // 2, "dglu": 2 * N}.get(epi, N)
            out = torch.zeros(M, ncols, dtype=torch.bfloat16, device="cuda")
            if epi == "act":
                kw = dict(epi="act", act="gelu", aux_out=torch.zeros(M, N, dtype=torch.bfloat16, device="cuda"))
            elif epi == "dact":
                kw = dict(epi="dact", act="silu", aux=_mk((M, N), torch.bfloat16, 5).cuda())
            elif epi == "glu":
                kw = dict(epi="glu", act="silu", aux_out=torch.zeros(M, N, dtype=torch.bfloat16, device="cuda"))
            elif epi == "dglu":
                kw = dict(epi="dglu", act="silu", aux=_mk((M, 2 * N), torch.bfloat16, 6).cuda())
        elif epi == "store_f32":
            out = _mk((M, N), torch.float32, 8).cuda()
            kw = dict(beta=1.0)
        else:
            out = _mk((M, N), torch.float32, 9).cuda()
            kw = dict(epi=epi, lr=1e-3, aux_out=torch.zeros(M, N, dtype=torch.bfloat16, device="cuda"))
            if epi == "adam":
                kw.update(step=2, opt_m=torch.full((M, N), 0.01, device="cuda"),
                          opt_v=torch.full((M, N), 1e-4, device="cuda"))
        gemm(a, b, layout, out=out, **kw)
        torch.cuda.synchronize()
        res.append([out] + [v for v in kw.values() if isinstance(v, torch.Tensor)])
    set_splitk(True)
    for x, y in zip(*res):
        tol = 2e-2 if x.dtype == torch.bfloat16 else 1e-5
        torch.testing.assert_close(x.float(), y.float(), rtol=tol, atol=tol * float(y.float().abs().max() + 1e-30))


@pytest.fixture(params=["8phase_stagger", "pp"])
def family(request):
    """The two persistent-capable bf16 families: 256x256 8-phase (one block per CU) and 256x128 (two per CU)."""
    old = set_bf16_variant(request.param)
    yield request.param
    set_bf16_variant(old)


@pytest.mark.parametrize("tpb", [2, 3, 64])
@pytest.mark.parametrize("layout,epi", [("nt", "act"), ("nt", "store"), ("nn", "dact"), ("nn", "store"),
                                        ("tn", "sgd"), ("tn", "adam"), ("tn", "store_f32"), ("nt", "glu")])
def test_persistent_blocks_bitwise_equal(tpb, layout, epi, family):
    """Persistent blocks (several tiles per block, next tile prefetched under the epilogue) give bitwise the same
    results as one block per tile: same tiles, same K order, same epilogue."""
    from dllm.ops.gemm import set_tiles_per_block

    # 1000 tiles: persistent grids with uneven blocks for every cap (tpb 2: 504 blocks, 496 with two tiles and 8
    # with one; tpb 3 / 64: the makespan-optimal 2 per block, or 4 per block on 256 blocks, 24 of them with 3)
    M, N, K = 6400, 10240, 384
    a, b = _operands(layout, M, N, K, torch.bfloat16, seed=41)
    a, b = a.cuda(), b.cuda()
    res = []
    for t in (1, tpb):
        old = set_tiles_per_block(t)
        try:
            kw = {}
            if epi in ("act", "store", "dact", "glu"):
                out = torch.zeros(M, N // 2 if epi == "glu" else N, dtype=torch.bfloat16, device="cuda")
                if epi == "act":
                    kw = dict(epi="act", act="relu", aux_out=torch.zeros(M, N, dtype=torch.bfloat16, device="cuda"))
                elif epi == "dact":   # ReLU: the persistent instantiation
                    kw = dict(epi="dact", act="relu", aux=_mk((M, N), torch.bfloat16, 5).cuda())
                elif epi == "glu":
                    kw = dict(epi="glu", act="silu", aux_out=torch.zeros(M, N, dtype=torch.bfloat16, device="cuda"))
            elif epi == "store_f32":
                out = _mk((M, N), torch.float32, 8).cuda()
                kw = dict(beta=1.0)
            else:
                out = _mk((M, N), torch.float32, 9).cuda()
                kw = dict(epi=epi, lr=1e-3, aux_out=torch.zeros(M, N, dtype=torch.bfloat16, device="cuda"))
                if epi == "adam":
                    kw.update(step=2, opt_m=torch.full((M, N), 0.01, device="cuda"),
                              opt_v=torch.full((M, N), 1e-4, device="cuda"))
            gemm(a, b, layout, out=out, **kw)
            torch.cuda.synchronize()
            res.append([out] + [v for v in kw.values() if isinstance(v, torch.Tensor)])
        finally:
            set_tiles_per_block(old)
    for x, y in zip(*res):
        assert torch.equal(x, y)


@pytest.mark.parametrize("layout", ["nt", "tn"])
def test_persistent_blocks_splitk_bitwise_equal(layout, family):
    """Persistent blocks over split-K slices (slot = tile x slice) == one block per slice, bitwise."""
    from dllm.ops.gemm import choose_ksplit, set_tiles_per_block

    M, N, K = 512, 512, 2048
    assert choose_ksplit(M, N, K) > 1
    a, b = _operands(layout, M, N, K, torch.bfloat16, seed=43)
    a, b = a.cuda(), b.cuda()
    outs = []
    for t in (1, 2, 5):
        old = set_tiles_per_block(t)
        try:
            outs.append(gemm(a, b, layout, out_dtype=torch.float32))
            torch.cuda.synchronize()
        finally:
            set_tiles_per_block(old)
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])


@pytest.mark.parametrize("tpb", [1, 2])
def test_relu_mask_matches_activation_path(tpb, family):
    """ReLU bitmask written by the forward GEMM and read by the dgrad == dgrad masked by the stored
    activation, bitwise (incl. -0 for negative masked values); forward output unchanged."""
    from dllm.ops.gemm import relu_mask_bytes, relu_mask_supported, set_tiles_per_block

    M, F, D = 4608, 2304, 512   # 162 tiles: one / two per block
    assert relu_mask_supported(M, F, D)
    x, w1 = _operands("nt", M, F, D, torch.bfloat16, seed=51)
    dy, w2 = _operands("nn", M, F, D, torch.bfloat16, seed=52)
    x, w1, dy, w2 = x.cuda(), w1.cuda(), dy.cuda(), w2.cuda()
    old = set_tiles_per_block(tpb)
    try:
        a0 = torch.empty(M, F, dtype=torch.bfloat16, device="cuda")
        gemm(x, w1, "nt", out=a0, epi="act", act="relu")
        da0 = torch.empty(M, F, dtype=torch.bfloat16, device="cuda")
        gemm(dy, w2, "nn", out=da0, epi="dact", act="relu", aux=a0)
        mask = torch.full((relu_mask_bytes(M, F),), 0xA5, dtype=torch.uint8, device="cuda")
        a1 = torch.empty_like(a0)
        gemm(x, w1, "nt", out=a1, epi="act", act="relu", mask=mask)
        da1 = torch.empty_like(da0)
        gemm(dy, w2, "nn", out=da1, epi="dact", act="relu", aux=a1, mask=mask)
        torch.cuda.synchronize()
    finally:
        set_tiles_per_block(old)
    assert torch.equal(a0.view(torch.int16), a1.view(torch.int16))
    assert torch.equal(da0.view(torch.int16), da1.view(torch.int16))
    frac = (a1 != 0).float().mean().item()
    assert 0.3 < frac < 0.7  # the mask really masks


def test_relu_mask_rejected_off_the_8phase_path():
    from dllm.ops.gemm import relu_mask_bytes

    M, N, K = 512, 512, 192   # K % 128 != 0 -> 2-stage kernel: no tile-native mask layout
    x, w = _operands("nt", M, N, K, torch.bfloat16, seed=1)
    mask = torch.empty(relu_mask_bytes(M, N), dtype=torch.uint8, device="cuda")
    with pytest.raises(RuntimeError):
        gemm(x.cuda(), w.cuda(), "nt", out_dtype=torch.bfloat16, epi="act", act="relu", mask=mask)


@pytest.mark.parametrize("layout,M,N,K", [("nt", 4352, 8448, 384), ("nn", 2048, 4096, 1024), ("tn", 2560, 3072, 2048),
                                          ("tn", 512, 512, 2048)])
def test_race_screen_repeated_runs_bitwise(layout, M, N, K, family):
    """Kernel race screen (cdna_hip_programming.md §5 race screens): the LDS-DMA pipeline, the staggered
    barriers and the persistent slot loop must give bitwise-identical results on every run, with random data,
    across persistent (> 2 tiles / CU), one-tile and split-K grids, for both kernel families."""
    a, b = _operands(layout, M, N, K, torch.bfloat16, seed=M + K)
    a, b = a.cuda(), b.cuda()
    first = gemm(a, b, layout, out_dtype=torch.float32)
    outs = [torch.empty_like(first) for _ in range(12)]
    for o in outs:
        gemm(a, b, layout, out=o)
    torch.cuda.synchronize()
    for o in outs:
        assert torch.equal(o, first)
    ref = _ref(a[:256].cpu() if layout != "tn" else a[:, :256].cpu(), b.cpu(), layout)
    got = first[:256].cpu().double()
    assert ((got - ref).abs().max() / ref.abs().max()) < 1e-5



def test_engine_step_launches_no_vendor_gemm():
    """Every GEMM of a bf16 training step is a hand-written kernel: a torch.profiler trace of one engine step shows
    only dllm kernels -- no hipBLASLt (``Cijk_*``) or rocBLAS GEMM (the forward's NT store had been routed
    to hipBLASLt on single-rank meshes)."""
    from torch.profiler import ProfilerActivity, profile

    from dllm.parallel.engine import FFNTrainer
    from dllm.parallel.mesh import Mesh
    from dllm.utils.config import ModelConfig, TrainConfig

    D, F, L, T = 512, 2048, 2, 8192   # K = F >= 8192 was the routed shape class; T = 8192 as in the flagship
    cfg = TrainConfig(model=ModelConfig(D, F, L, "relu", False), batch_size=1, seq_len=T, dtype="bf16",
                      grad_dtype="fp32", lr=1e-3)
    eng = FFNTrainer(cfg, Mesh(), torch.device("cuda"))
    g = torch.Generator().manual_seed(0)
    eng.load_full_params([{"w1": torch.randn(F, D, generator=g) * 0.02, "w2": torch.randn(D, F, generator=g) * 0.02}
                          for _ in range(L)])
    x = torch.randn(T, D, generator=g).to(DEV, torch.bfloat16)
    dy = torch.randn(T, D, generator=g).to(DEV, torch.bfloat16)
    eng.train_step(x, dy)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        eng.train_step(x, dy)
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if e.device_type.name == "CUDA"]
    gemms = [n for n in names if "gemm_bf16" in n]
    assert gemms, names[:20]
    vendor = [n for n in names if n.startswith(("Cijk", "Custom_Cijk")) or "rocblas" in n.lower()]
    assert not vendor, vendor
