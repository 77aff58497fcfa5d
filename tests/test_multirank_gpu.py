"""Multi-rank engine paths on the GPU: 2-4 processes share cuda:0 and talk through gloo (RCCL refuses two ranks
on one device), so DDP / ZeRO-2 / FSDP / TP / hybrid run with the HIP kernels, the side streams and events of
N > 1 -- real shard offsets, real reduce-scatters and gathers -- instead of the size-1 communicators of the
forced-comm entries.  Checked against the reference oracle (fp32), against each other (bf16, the bench's N > 1
default) and against the serialized schedule (every collective waited and the device synchronised: a missing
stream / event edge shows as a bitwise difference).
"""
import pytest
import torch

from dllm.models import reference as R
from dllm.parallel.launch import build_params, draw_seeds, spawn
from dllm.utils.config import ModelConfig, TrainConfig
from dllm.utils.data import reference_mock_data

pytestmark = pytest.mark.gpu
SEED = 5


def _cfg(D, F, L, T, steps=4, **kw):  # steps divisible by dp (train_ffns.py:175)
    return TrainConfig(model=ModelConfig(D, F, L, "relu", False), batch_size=1, seq_len=T, num_steps=steps,
                       lr=kw.pop("lr", 1e-2), data="cpu_compat", **kw)


def _run(cfg, method, n, port, record=False, **opts):
    o = {"seed": SEED, "init": "cpu_compat", "return_full": True, "tp": opts.pop("tp", n), "device": "cuda"}
    o.update(opts)
    rec = spawn(n, cfg, method, "gloo", port, o, timeout_s=240)
    return rec if record else rec["params"]


def _oracle(cfg, n):
    layers = build_params(cfg, "cpu_compat", SEED, "cpu")
    batches = list(reference_mock_data(draw_seeds(cfg, SEED), cfg.tokens, cfg.model.D))
    if n == 1:
        return R.train_single(layers, batches, cfg.lr, cfg.model.act)
    return R.train_data_parallel(layers, batches, n, cfg.lr, cfg.model.act)


def _close(got, want, rtol, atol):
    for g, w in zip(got, want):
        for k in w:
            torch.testing.assert_close(torch.as_tensor(g[k]).float(), torch.as_tensor(w[k]).float(),
                                       rtol=rtol, atol=atol)


def _equal(a, b):
    return all(torch.equal(torch.as_tensor(x[k]), torch.as_tensor(y[k])) for x, y in zip(a, b) for k in x)


@pytest.mark.parametrize("method,n,opts", [(2, 2, {}), (6, 2, {}), (3, 2, {}), (4, 2, {}),
                                           (5, 4, {"tp": 2, "hybrid_dp_mode": "fsdp"})],
                         ids=["ddp", "zero2", "fsdp", "tp", "fsdp2xtp2"])
def test_fp32_methods_match_oracle(method, n, opts, free_port):
    """fp32 (bf16x6 GEMMs) on 2 / 4 ranks of one GPU vs the reference algorithm on the CPU."""
    cfg = _cfg(256, 512, 2, 256, dtype="fp32", grad_dtype="fp32")
    got = _run(cfg, method, n, free_port, **dict(opts))
    _close(got, _oracle(cfg, 1 if method == 4 else 2), rtol=1e-4, atol=1e-6)


def test_bf16_data_parallel_methods_agree(free_port):
    """bf16 compute and bf16 gradient collectives (the bench's N > 1 path) at a size that runs the 8-phase
    persistent kernels with ReLU masks: DDP (all-reduce), ZeRO-2 (reduce-scatter, sharded update, all-gather)
    and FSDP (gathered weights) on 2 ranks sum the same two bf16 gradients, so their masters are equal."""
    cfg = _cfg(1024, 4096, 2, 2048, dtype="bf16", grad_dtype="bf16", lr=1e-3)
    ddp = _run(cfg, 2, 2, free_port)
    zero = _run(cfg, 6, 2, free_port + 1)
    fsdp = _run(cfg, 3, 2, free_port + 2)
    # two-rank sums are order-free and every update is the same elementwise kernel: bitwise equal
    # (profiles/r3/pytest_multirank_gpu_r3.txt)
    assert _equal(ddp, zero) and _equal(ddp, fsdp)


@pytest.mark.parametrize("method", [6, 3], ids=["zero2", "fsdp"])
def test_overlapped_equals_serialized(method, free_port):
    """Race screen of the N > 1 schedules with real streams: the overlapped step (side-stream shard updates,
    prefetched gathers, in-loop reduce-scatters) is bitwise the serialized one."""
    base = dict(dtype="bf16", grad_dtype="bf16", lr=1e-3)
    over = _run(_cfg(1024, 4096, 2, 2048, **base), method, 2, free_port)
    ser = _run(_cfg(1024, 4096, 2, 2048, debug_sync=True, **base), method, 2, free_port + 1)
    assert _equal(over, ser)


def test_tp_transposed_layout_two_ranks_and_checkpoint_crossing(free_port, tmp_path):
    """the transposed-activation TP layout (tmode: W2 stored transposed, 224-row tiles, NN fused optimizer)
    on a real 2-rank TP group (gloo on cuda:0), F_loc = 1792.  Its masters match the row-major layout's after the same
    steps, and a sharded checkpoint written by one layout resumes in the other (both directions)."""
    base = dict(dtype="bf16", grad_dtype="bf16", lr=1e-3)
    D, F, L, T = 256, 3584, 2, 512                 # F / tp = 1792 = 8 x 224 -> tmode
    t_on = _cfg(D, F, L, T, tp_transposed=True, **base)
    t_off = _cfg(D, F, L, T, tp_transposed=False, **base)
    on = _run(t_on, 4, 2, free_port)
    off = _run(t_off, 4, 2, free_port + 1)
    _close(on, off, rtol=2e-2, atol=1e-4)          # bf16 working copies: GEMM order may differ by one rounding
    for i, (src, dst) in enumerate(((t_on, t_off), (t_off, t_on))):
        d = str(tmp_path / f"ck{i}")
        # 2 of the 4 steps in the source layout, checkpointed sharded; the other 2 resumed in the other layout
        _run(src, 4, 2, free_port + 2 + 2 * i, ckpt_dir=d, ckpt_format="sharded", stop_after=2)
        resumed = _run(dst, 4, 2, free_port + 3 + 2 * i, resume=d)
        _close(resumed, on, rtol=2e-2, atol=1e-4)


def test_nn_weight_gradient_layout_two_ranks_and_checkpoint_crossing(free_port, tmp_path):
    """The NN weight-gradient layout (nn_w2t: W2 stored transposed, transposed xᵀ / dyᵀ copies, stored gradients
    through the transposed map) on 2 real DDP / ZeRO-2 / FSDP ranks: bitwise the TN layout's masters; a sharded ZeRO
    checkpoint written in one layout resumes in the other (both directions).  Shapes large enough that no GEMM of the
    layer takes split-K (the engine's condition for the NN layout)."""
    base = dict(dtype="bf16", grad_dtype="bf16", lr=1e-3)
    D, F, L, T = 2048, 8192, 2, 8192
    nn = _cfg(D, F, L, T, wgrad_layout="nn_w2t", **base)
    tn = _cfg(D, F, L, T, wgrad_layout="tn", **base)
    port = free_port
    ref = {}
    for method in (2, 6, 3):                       # DDP, ZeRO-2, FSDP
        ra = _run(nn, method, 2, port, record=True)
        rb = _run(tn, method, 2, port + 1, record=True)
        port += 2
        assert ra["layout"]["wgrad_nn_w2"] and ra["layout"]["w2t"] and not rb["layout"]["wgrad_nn"]
        assert _equal(ra["params"], rb["params"]), method
        ref[method] = rb["params"]
    for i, (src, dst) in enumerate(((nn, tn), (tn, nn))):
        d = str(tmp_path / f"ck{i}")
        _run(src, 6, 2, port, ckpt_dir=d, ckpt_format="sharded", stop_after=2)
        resumed = _run(dst, 6, 2, port + 1, resume=d)
        port += 2
        assert _equal(resumed, ref[6]), i
