"""HIP-graph captured training step == eager step (bitwise: every kernel is deterministic)."""
import pytest
import torch

from dllm.models.ffn import init_ffn_params_device
from dllm.ops.elementwise import rng_normal_, rng_normal_devseed_
from dllm.parallel.engine import FFNTrainer
from dllm.parallel.mesh import Mesh
from dllm.utils.config import ModelConfig, TrainConfig
from dllm.utils.data import DeviceMockData
from dllm.utils.graphs import GraphedStep

pytestmark = pytest.mark.gpu


def test_devseed_rng_matches_host_seed():
    a = torch.empty(4096, device="cuda", dtype=torch.bfloat16)
    b = torch.empty_like(a)
    rng_normal_(a, seed=77, stream_id=1, scale=0.1)
    rng_normal_devseed_(b, torch.tensor([77], device="cuda"), stream_id=1, scale=0.1)
    assert torch.equal(a, b)


def _engine():
    m = ModelConfig(256, 1024, 3)
    cfg = TrainConfig(model=m, batch_size=2, seq_len=256, dtype="bf16", lr=1e-2)
    eng = FFNTrainer(cfg, Mesh(), torch.device("cuda"))
    eng.load_full_params(init_ffn_params_device(m.D, m.F, m.layers, 3, "cuda"))
    return eng, cfg


def test_graphed_step_equals_eager():
    eng_a, cfg = _engine()
    g = GraphedStep(eng_a, cfg.tokens, cfg.model.D)
    # the capture warm-up ran 2 eager steps: replay the same on the eager engine
    eng_b, _ = _engine()
    data = DeviceMockData(cfg.tokens, cfg.model.D, torch.bfloat16, torch.device("cuda"))
    for s in (-1, -2):
        eng_b.train_step(*data.fill(s % (2**64)))
    for seed in (11, 12, 13):
        g.step(seed)
        eng_b.train_step(*data.fill(seed))
    torch.cuda.synchronize()
    assert torch.equal(eng_a.master, eng_b.master)
    assert torch.equal(eng_a.copy, eng_b.copy)
