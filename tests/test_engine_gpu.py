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
    D, F, L, T, lr = 128, 512, 2, 256, 1e-2
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


@pytest.mark.parametrize("act,gated", [("relu", False), ("silu", True)])
def test_bf16_engine_tracks_oracle(act, gated):
    D, F, L, T, lr = 256, 1024, 2, 512, 1e-2
    layers, batches = _setup(D, F, L, T, act, gated, 2)
    cfg = TrainConfig(model=ModelConfig(D, F, L, act, gated), batch_size=1, seq_len=T, dtype="bf16",
                      grad_dtype="fp32", lr=lr)
    eng = FFNTrainer(cfg, Mesh(), torch.device("cuda"))
    eng.load_full_params(layers)
    for x, dy in batches:
        eng.train_step(x.cuda().bfloat16(), dy.cuda().bfloat16())
    got = eng.gather_full_params()
    want = R.train_single(layers, [(x.bfloat16().float(), dy.bfloat16().float()) for x, dy in batches], lr, act)
    for g, w, p0 in zip(got, want, layers):
        for k in g:
            d_got, d_want = g[k].double() - p0[k].double(), w[k].double() - p0[k].double()
            rel = (d_got - d_want).norm() / d_want.norm()
            assert rel < 5e-2, (k, rel.item())


def test_adam_engine_matches_oracle():
    D, F, L, T, lr = 128, 512, 2, 256, 1e-3
    layers, batches = _setup(D, F, L, T, "relu", False, 3)
    cfg = TrainConfig(model=ModelConfig(D, F, L), batch_size=1, seq_len=T, dtype="fp32", grad_dtype="fp32",
                      lr=lr, optimizer="adam", adam_b2=0.95, skip_input_grad=False)
    eng = FFNTrainer(cfg, Mesh(), torch.device("cuda"))
    eng.load_full_params(layers)
    for x, dy in batches:
        eng.train_step(x.cuda(), dy.cuda())
    got = eng.gather_full_params()
    want = R.train_adam_single(layers, batches, lr, b2=0.95)
    for g, w in zip(got, want):
        for k in g:
            torch.testing.assert_close(g[k], w[k], rtol=1e-4, atol=2e-5)
