"""Single-GPU engine (native kernels end to end) against the pure-torch reference oracle."""
import pytest
import torch

from dllm.models import reference as R
from dllm.models.ffn import init_ffn_layer
from dllm.parallel.engine import FFNTrainer
from dllm.parallel.mesh import Mesh
from dllm.utils.config import ModelConfig, TrainConfig
from dllm.utils.data import reference_mock_data

pytestmark = pytest.mark.gpu


def _setup(D, F, L, T, act, gated, steps, seed=5):
    gen = torch.Generator().manual_seed(seed)
    layers = [init_ffn_layer(D, F, gen, gated) for _ in range(L)]
    seeds = torch.randint(100_000, (steps,), generator=gen)
    batches = list(reference_mock_data(seeds, T, D))
    return layers, batches


@pytest.mark.parametrize("act,gated", [("relu", False), ("silu", False), ("gelu", False), ("silu", True)])
@pytest.mark.parametrize("recompute", ["none", "full"])
def test_fp32_engine_matches_oracle(act, gated, recompute):
    D, F, L, T = 128, 512, 2, 256
    lr = 1.0 if gated else 1e-2  # gated updates are ~100x smaller at this init scale
    layers, batches = _setup(D, F, L, T, act, gated, 3)
    cfg = TrainConfig(model=ModelConfig(D, F, L, act, gated), batch_size=1, seq_len=T, dtype="fp32",
                      grad_dtype="fp32", lr=lr, recompute=recompute, skip_input_grad=False)
    eng = FFNTrainer(cfg, Mesh(), torch.device("cuda"))
    eng.load_full_params(layers)
    for x, dy in batches:
        eng.train_step(x.cuda(), dy.cuda())
    got = eng.gather_full_params()
    # same-precision oracle (fp32 on CPU): only GEMM summation order differs
    want = R.train_single(layers, batches, lr, act)
    for g, w, p0 in zip(got, want, layers):
        for k in g:
            d_got, d_want = g[k].double() - p0[k].double(), w[k].double() - p0[k].double()
            assert d_want.abs().max() > 1e-5
            rel = (d_got - d_want).norm() / d_want.norm()
            assert rel < 2e-3, (k, rel.item())


@pytest.mark.parametrize("act", ["relu", "gelu"])
def test_bf16_engine_matches_mixed_precision_oracle(act):
    """bf16 compute + fp32 master/grad path vs an oracle that rounds at exactly the same points."""
    D, F, L, T, lr = 256, 1024, 2, 512, 1e-2
    layers, batches = _setup(D, F, L, T, act, False, 2)
    cfg = TrainConfig(model=ModelConfig(D, F, L, act, False), batch_size=1, seq_len=T, dtype="bf16",
                      grad_dtype="fp32", lr=lr, skip_input_grad=False)
    eng = FFNTrainer(cfg, Mesh(), torch.device("cuda"))
    eng.load_full_params(layers)
    for x, dy in batches:
        eng.train_step(x.cuda().bfloat16(), dy.cuda().bfloat16())
    got = eng.gather_full_params()
    want = R.train_single_mixed(layers, batches, lr, act)
    for g, w, p0 in zip(got, want, layers):
        for k in g:
            d_got, d_want = g[k].double() - p0[k].double(), w[k].double() - p0[k].double()
            rel = (d_got - d_want).norm() / d_want.norm()
            # ReLU: 1-ulp bf16 differences of layer-0 outputs flip a few layer-1 masks (full-size error
            # on those elements); per-layer exactness is asserted by test_layer_intermediates_gpu_vs_cpu
            assert rel < (6e-2 if act == "relu" else 2e-2), (k, rel.item())


@pytest.mark.parametrize("relu_mask", [True, False])
def test_bf16_relu_stack_teacher_forced(relu_mask):
    """Tight stack-level check of the bf16 ReLU path (the 6 % above is mask flips, not kernel error): the oracle
    backward runs on the engine's OWN stored forward activations (same bf16 values -> same ReLU masks), so what
    is left is accumulation order and the bf16 rounding of da / dx.  Also each layer's stored output against
    a_l . W2^T of the engine's a_l.  One step, 3 layers, fp32 master / fp32 gradients."""
    D, F, L, T, lr = 256, 1024, 3, 512, 1e-2
    layers, batches = _setup(D, F, L, T, "relu", False, 1)
    cfg = TrainConfig(model=ModelConfig(D, F, L, "relu", False), batch_size=1, seq_len=T, dtype="bf16",
                      grad_dtype="fp32", lr=lr, skip_input_grad=False, relu_mask=relu_mask)
    eng = FFNTrainer(cfg, Mesh(), torch.device("cuda"))
    assert (eng.masks is not None) == relu_mask
    eng.load_full_params(layers)
    x, dy = (t.cuda().bfloat16() for t in batches[0])
    eng.train_step(x, dy)
    torch.cuda.synchronize()
    got = eng.gather_full_params()
    W = [{k: v.cuda().bfloat16().float() for k, v in p.items()} for p in layers]
    xs = [x.float()] + [eng.xs[l + 1].float() for l in range(L)]
    As = [eng.acts_a[l].float() for l in range(L)]
    for l in range(L):
        assert torch.equal(As[l], torch.relu(As[l]))
        y = (As[l] @ W[l]["w2"].t()).bfloat16().float()
        assert ((xs[l + 1] - y).abs() > 1e-2 * y.abs() + 1e-6).float().mean() < 1e-3, l  # <= 1-ulp bf16 rounding
    g = dy.float()
    for l in reversed(range(L)):
        da = ((g @ W[l]["w2"]) * (As[l] > 0)).bfloat16().float()
        want = {"w2": layers[l]["w2"].cuda() - lr * (g.t() @ As[l]), "w1": layers[l]["w1"].cuda() - lr * (da.t() @ xs[l])}
        for k in ("w1", "w2"):
            d_got = got[l][k].cuda().double() - layers[l][k].cuda().double()
            d_want = want[k].double() - layers[l][k].cuda().double()
            rel = float((d_got - d_want).norm() / d_want.norm())
            assert rel < 5e-3, (l, k, rel)
        g = (da @ W[l]["w1"]).bfloat16().float()


def test_bf16_gated_engine_tracks_fp32_oracle():
    D, F, L, T, lr = 256, 1024, 2, 512, 1.0
    layers, batches = _setup(D, F, L, T, "silu", True, 2)
    cfg = TrainConfig(model=ModelConfig(D, F, L, "silu", True), batch_size=1, seq_len=T, dtype="bf16",
                      grad_dtype="fp32", lr=lr)
    eng = FFNTrainer(cfg, Mesh(), torch.device("cuda"))
    eng.load_full_params(layers)
    for x, dy in batches:
        eng.train_step(x.cuda().bfloat16(), dy.cuda().bfloat16())
    got = eng.gather_full_params()
    want = R.train_single(layers, [(x.bfloat16().float(), dy.bfloat16().float()) for x, dy in batches], lr, "silu")
    for g, w, p0 in zip(got, want, layers):
        for k in g:
            d_got, d_want = g[k].double() - p0[k].double(), w[k].double() - p0[k].double()
            rel = (d_got - d_want).norm() / d_want.norm()
            assert rel < 5e-2, (k, rel.item())


@pytest.mark.parametrize("act", ["silu", "gelu"])
def test_adam_engine_matches_oracle(act):
    """Fused AdamW (in the weight-gradient GEMM epilogue) vs the fp32 oracle, on smooth activations.  Adam's
    update m/sqrt(v) is a sign-like function of each gradient element, so a gradient that differs only by
    summation order can move single elements by ~lr; with ReLU a mask flip wherever h is within rounding of 0
    (one flip moves a whole dW1 row) then spreads through the next steps, so ReLU + Adam has no elementwise
    oracle at fp32 rounding (the fp32 ReLU engine is checked with SGD above).  Checked: the update norm to 1e-3
    and all but 1 % of elements to 1e-4 relative (measured: 0.5 % after 3 steps)."""
    D, F, L, T, lr = 128, 512, 2, 256, 1e-3
    layers, batches = _setup(D, F, L, T, act, False, 3)
    cfg = TrainConfig(model=ModelConfig(D, F, L, act), batch_size=1, seq_len=T, dtype="fp32", grad_dtype="fp32",
                      lr=lr, optimizer="adam", adam_b2=0.95, skip_input_grad=False)
    eng = FFNTrainer(cfg, Mesh(), torch.device("cuda"))
    eng.load_full_params(layers)
    for x, dy in batches:
        eng.train_step(x.cuda(), dy.cuda())
    got = eng.gather_full_params()
    want = R.train_adam_single(layers, batches, lr, b2=0.95, act=act)
    for g, w, p0 in zip(got, want, layers):
        for k in g:
            dg, dw = g[k].double() - p0[k].double(), w[k].double() - p0[k].double()
            assert (dg - dw).norm() / dw.norm() < 1e-3, k
            assert ((dg - dw).abs() > 1e-4 * dw.abs().max()).double().mean() < 1e-2, k


@pytest.mark.parametrize("act", ["relu", "gelu"])
def test_layer_intermediates_gpu_vs_cpu(act):
    """Every intermediate of one bf16 layer fwd/bwd (a, y, dW2, da, dx, dW1) on the HIP kernels matches the
    CPU path on identical inputs to fp32-summation-order precision."""
    from dllm.models.ffn import layer_bwd, layer_fwd

    D, F, T = 256, 1024, 512
    gen = torch.Generator().manual_seed(5)
    p = init_ffn_layer(D, F, gen)
    x = torch.randn(T, D, generator=gen).bfloat16()
    dy = (0.1 * torch.randn(T, D, generator=gen)).bfloat16()
    w1, w2 = p["w1"].bfloat16(), p["w2"].bfloat16()
    res = {}
    for dev in ("cpu", "cuda"):
        X, DY, W1, W2 = x.to(dev), dy.to(dev), w1.to(dev), w2.to(dev)
        a = torch.empty(T, F, dtype=torch.bfloat16, device=dev)
        h = torch.empty(T, F, dtype=torch.bfloat16, device=dev) if act != "relu" else None
        y = torch.empty(T, D, dtype=torch.bfloat16, device=dev)
        layer_fwd(X, W1, W2, act, False, a, h, y)
        gw1, gw2 = torch.empty(F, D, device=dev), torch.empty(D, F, device=dev)
        da = torch.empty(T, F, dtype=torch.bfloat16, device=dev)
        dx = torch.empty(T, D, dtype=torch.bfloat16, device=dev)
        layer_bwd(DY, X, W1, W2, act, False, a, h, gw1, gw2, da, dx)
        res[dev] = dict(a=a, y=y, gw1=gw1, gw2=gw2, da=da, dx=dx)
    for k, want in res["cpu"].items():
        got = res["cuda"][k].cpu().double()
        rel = ((got - want.double()).norm() / want.double().norm()).item()
        assert rel < 1e-3, (k, rel)
    if act == "relu":
        assert torch.equal(res["cuda"]["a"].cpu() > 0, res["cpu"]["a"] > 0)


@pytest.mark.parametrize("opt", ["sgd", "adam"])
@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_fused_optimizer_epilogue_matches_separate_kernel(opt, dtype):
    D, F, L, T = 256, 1024, 2, 512
    layers, batches = _setup(D, F, L, T, "relu", False, 2)
    out = []
    for fused in (True, False):
        cfg = TrainConfig(model=ModelConfig(D, F, L), batch_size=1, seq_len=T, dtype=dtype, grad_dtype="fp32",
                          lr=1e-3, optimizer=opt, fused_optimizer=fused)
        eng = FFNTrainer(cfg, Mesh(), torch.device("cuda"))
        eng.load_full_params(layers)
        cd = torch.bfloat16 if dtype == "bf16" else torch.float32
        for x, dy in batches:
            eng.train_step(x.cuda().to(cd), dy.cuda().to(cd))
        out.append(eng.gather_full_params())
        assert eng.fused_opt == fused
    for g, w in zip(*out):
        for k in w:
            torch.testing.assert_close(g[k], w[k], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_odd_shapes_and_skipped_input_grad(dtype):
    """Shapes off every MFMA tile grid (generic kernel end to end) with the default skipped layer-0 input
    gradient (layer 0 runs dW1 before dW2; the flat layout follows) against the oracle."""
    D, F, L, T, lr = 96, 384, 3, 200, 1e-2
    layers, batches = _setup(D, F, L, T, "relu", False, 2)
    cfg = TrainConfig(model=ModelConfig(D, F, L), batch_size=1, seq_len=T, dtype=dtype, grad_dtype="fp32", lr=lr)
    assert cfg.skip_input_grad
    eng = FFNTrainer(cfg, Mesh(), torch.device("cuda"))
    assert eng.layer_order(0) == ("w1", "w2") and eng.layer_order(1) == ("w2", "w1")
    eng.load_full_params(layers)
    cd = torch.float32 if dtype == "fp32" else torch.bfloat16
    for x, dy in batches:
        eng.train_step(x.cuda().to(cd), dy.cuda().to(cd))
    got = eng.gather_full_params()
    want = (R.train_single(layers, batches, lr) if dtype == "fp32"
            else R.train_single_mixed(layers, batches, lr))
    for g, w, p0 in zip(got, want, layers):
        for k in g:
            d_got, d_want = g[k].double() - p0[k].double(), w[k].double() - p0[k].double()
            rel = (d_got - d_want).norm() / d_want.norm()
            assert rel < (2e-3 if dtype == "fp32" else 2e-2), (k, rel.item())


def test_relu_mask_engine_bitwise():
    """A bf16 ReLU training step with the 1-bit activation masks == the same step reading the activations."""
    D, F, L, T, lr = 512, 2048, 3, 1024, 1e-2
    layers, batches = _setup(D, F, L, T, "relu", False, 2)
    outs = []
    for use in (False, True):
        cfg = TrainConfig(model=ModelConfig(D, F, L, "relu", False), batch_size=1, seq_len=T, dtype="bf16",
                          grad_dtype="fp32", lr=lr, relu_mask=use)
        eng = FFNTrainer(cfg, Mesh(), torch.device("cuda"))
        assert (eng.masks is not None) == use
        eng.load_full_params(layers)
        for x, dy in batches:
            eng.train_step(x.cuda().bfloat16(), dy.cuda().bfloat16())
        torch.cuda.synchronize()
        outs.append(eng.master.clone())
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("act,gated", [("relu", False), ("gelu", False), ("silu", True)])
def test_wgrad_stream_bitwise(act, gated):
    """Weight-gradient GEMMs on a concurrent stream == the sequential schedule, bitwise (same kernels and
    inputs per GEMM; the stream/event edges order every weight update after its last reader); gated (SwiGLU)
    stacks run the DGLU dgrad on the main stream."""
    from dllm.ops.gemm import set_pair_wgrads

    D, F, L, T, lr = 512, 2048, 4, 1024, 1e-2
    layers, batches = _setup(D, F, L, T, act, gated, 3)
    outs = []
    old_pair = set_pair_wgrads(False)   # these small weight gradients would otherwise run as one grouped launch
    try:
        for ws in (False, True):
            cfg = TrainConfig(model=ModelConfig(D, F, L, act, gated), batch_size=1, seq_len=T, dtype="bf16",
                              grad_dtype="fp32", lr=lr, wgrad_stream=ws)
            eng = FFNTrainer(cfg, Mesh(), torch.device("cuda"))
            assert (eng.wg_stream is not None) == ws
            eng.load_full_params(layers)
            for x, dy in batches:
                eng.train_step(x.cuda().bfloat16(), dy.cuda().bfloat16())
            torch.cuda.synchronize()
            outs.append(eng.master.clone())
    finally:
        set_pair_wgrads(old_pair)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("variant", ["8phase_stagger", "pp"])
def test_wgrad_stream_bitwise_full_size(variant):
    """Race screen of the bench's default schedule at a size where the two streams' grids really overlap: L4 D4096
    F16384 T8192 bf16 (persistent 1024/512-tile GEMMs, ReLU 1-bit masks, fused SGD), 3 steps on device-generated
    data.  The concurrent weight-gradient stream must give bitwise the serial schedule's fp32 masters."""
    from dllm.models.ffn import init_ffn_params_device
    from dllm.ops.gemm import set_bf16_variant
    from dllm.utils.data import DeviceMockData

    D, F, L, T = 4096, 16384, 4, 8192
    old = set_bf16_variant(variant)
    try:
        outs = []
        for ws in (False, True):
            cfg = TrainConfig(model=ModelConfig(D, F, L, "relu", False), batch_size=8, seq_len=1024, dtype="bf16",
                              grad_dtype="bf16", wgrad_stream=ws, wgrad_layout="tn")   # the bench's lr: 1e-2 overflows
            eng = FFNTrainer(cfg, Mesh(), torch.device("cuda"))
            assert (eng.wg_stream is not None) == ws and eng.masks is not None
            eng.load_full_params(init_ffn_params_device(D, F, L, 7, torch.device("cuda"), False))
            init_master = eng.master.clone()
            data = DeviceMockData(T, D, torch.bfloat16, torch.device("cuda"))
            for s in range(3):
                x, dy = data.fill(100 + s)
                eng.train_step(x, dy)
            torch.cuda.synchronize()
            outs.append(eng.master.clone())
            del eng, data
            torch.cuda.empty_cache()
        assert torch.isfinite(outs[0]).all()
        assert not torch.equal(outs[0], init_master), "the steps must move the masters"
        assert torch.equal(outs[0], outs[1])
    finally:
        set_bf16_variant(old)


def test_sizing_plan_matches_wgrad_stream_buffers():
    """utils/sizing.plan with wgrad_stream counts the rotated dgrad / dx buffers the engine really allocates."""
    from dllm.utils.sizing import plan

    cfg = TrainConfig(model=ModelConfig(256, 1024, 3), batch_size=2, seq_len=256, dtype="bf16", grad_dtype="bf16",
                      lr=1e-2, wgrad_stream=True, wgrad_layout="tn")
    eng = FFNTrainer(cfg, Mesh(), torch.device("cuda"))
    assert eng.wg_stream is not None
    p = plan(256, 1024, 3, 512, dtype="bf16", grad_dtype="bf16", wgrad_stream=True)["bytes"]
    nb = lambda t: t.numel() * t.element_size()  # noqa: E731
    assert p["dgrad_buffer"] == sum(nb(t) for t in eng.da_ring)
    assert p["dx_buffers"] == sum(nb(t) for t in eng.dxb)
    # the NN weight-gradient layout (flagship-shaped layer: tile grids large enough for it): serial, transposed copies
    cfg = TrainConfig(model=ModelConfig(2048, 8192, 2), batch_size=1, seq_len=8192, dtype="bf16", grad_dtype="bf16",
                      lr=1e-3, wgrad_stream=True, wgrad_layout="nn_w2t")
    eng = FFNTrainer(cfg, Mesh(), torch.device("cuda"))
    assert eng.wg_stream is None and eng.w2t
    p = plan(2048, 8192, 2, 8192, dtype="bf16", grad_dtype="bf16", wgrad_stream=True, wgrad_layout="nn_w2t")["bytes"]
    copies = list(eng.xT) + list(eng.dxTb) + [eng.dyT_top]
    assert p["nn_transposed_copies"] == sum(nb(t) for t in copies)
    assert p["dx_buffers"] == sum(nb(t) for t in eng.dxb)


def test_overlapped_data_pipeline_bitwise():
    """The bench's one-deep data pipeline (next batch drawn on a side stream under the backward) gives bitwise the
    masters of drawing each batch at the start of its step, with the wgrad stream on."""
    from dllm.models.ffn import init_ffn_params_device
    from dllm.utils.data import DeviceMockData

    D, F, L, T = 512, 2048, 3, 2048
    outs = []
    for overlap in (False, True):
        cfg = TrainConfig(model=ModelConfig(D, F, L, "relu", False), batch_size=2, seq_len=1024, dtype="bf16",
                          grad_dtype="bf16", wgrad_stream=True)
        eng = FFNTrainer(cfg, Mesh(), torch.device("cuda"))
        eng.load_full_params(init_ffn_params_device(D, F, L, 3, torch.device("cuda"), False))
        data = DeviceMockData(T, D, torch.bfloat16, torch.device("cuda"), overlap=overlap)
        assert data.overlap == overlap
        eng.before_backward = data.release
        for s in range(5):
            x, dy = data.fill(50 + s, next_seed=51 + s)
            eng.train_step(x, dy)
        torch.cuda.synchronize()
        outs.append(eng.master.clone())
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(outs[0], outs[1])


def test_overlapped_data_mismatched_seed_bitwise():
    """A fill whose seed differs from the announced next_seed (resume, skipped step, eval fill) waits for the
    in-flight side-stream draw before redrawing, so it returns exactly the synchronous draw of that seed even when
    the side stream is still writing the same slot (the redraw used to race the prefetch)."""
    from dllm.utils.data import DeviceMockData

    T, D = 8192, 4096
    dev = torch.device("cuda")
    ref = DeviceMockData(T, D, torch.bfloat16, dev)
    data = DeviceMockData(T, D, torch.bfloat16, dev, overlap=True)
    for s in range(4):
        x, dy = data.fill(100 + s, next_seed=777)  # announces 777, then asks for 101, 102, ...
        data.release()                             # side stream starts drawing 777 into the other slot
        rx, rdy = ref.fill(100 + s)
        torch.cuda.synchronize()
        assert torch.equal(x, rx) and torch.equal(dy, rdy), s
    x, dy = data.fill(777)                          # the announced seed is still served from the prefetch
    rx, rdy = ref.fill(777)
    torch.cuda.synchronize()
    assert torch.equal(x, rx) and torch.equal(dy, rdy)
