"""Data pipeline (utils/data.py) on the CPU: the overlapped device pipeline degrades to synchronous draws without a
GPU, and the engine calls its ``before_backward`` hook once per step, before any backward work."""
import torch

from dllm.parallel.engine import FFNTrainer
from dllm.parallel.mesh import Mesh
from dllm.utils.config import ModelConfig, TrainConfig
from dllm.utils.data import DeviceMockData


def test_device_data_overlap_is_off_without_gpu():
    d = DeviceMockData(64, 32, torch.float32, torch.device("cpu"), overlap=True)
    assert not d.overlap and d.depth == 0
    x, dy = d.fill(7, next_seed=8)
    d.release()  # no-op
    x0, dy0 = x.clone(), dy.clone()
    x, dy = DeviceMockData(64, 32, torch.float32, torch.device("cpu")).fill(7)
    assert torch.equal(x, x0) and torch.equal(dy, dy0)


def test_before_backward_hook_runs_once_per_step():
    cfg = TrainConfig(model=ModelConfig(32, 64, 2), batch_size=2, seq_len=16, dtype="fp32", lr=1e-3)
    eng = FFNTrainer(cfg, Mesh(), torch.device("cpu"))
    calls = []
    eng.before_backward = lambda: calls.append(eng.step_count)
    data = DeviceMockData(cfg.tokens, 32, torch.float32, torch.device("cpu"))
    for s in range(3):
        eng.train_step(*data.fill(s))
    assert calls == [1, 2, 3]


def test_size1_inplace_collectives_move_nothing(monkeypatch):
    """comm._moves: an in-place collective on a size-1 communicator launches no kernel (the observer counts it but
    does not time it); out-of-place or multi-rank ones move data."""
    from dllm.parallel import comm

    t, o = torch.zeros(8), torch.zeros(8)
    monkeypatch.setattr(comm, "_group_size", lambda g: 1)
    assert not comm._moves(None, t, t) and comm._moves(None, o, t)
    monkeypatch.setattr(comm, "_group_size", lambda g: 2)
    assert comm._moves(None, t, t)


def test_bind_transposed_draws_and_tags_the_transposes(monkeypatch):
    """bind_transposed: the batch arrives with xᵀ / dyᵀ written into the bound buffers and tagged (the engine's
    train_step consumes the tag); the overlap pipeline and DLLM_DRAW_T=0 leave the transposes to the engine."""
    d = DeviceMockData(64, 32, torch.bfloat16, torch.device("cpu"))
    xt, dyt = torch.empty(32, 64, dtype=torch.bfloat16), torch.empty(32, 64, dtype=torch.bfloat16)
    d.bind_transposed(xt, dyt)
    x, dy = d.fill(5)
    assert x._dllm_t is xt and dy._dllm_t is dyt
    assert torch.equal(xt, x.t()) and torch.equal(dyt, dy.t())
    ref_x, ref_dy = DeviceMockData(64, 32, torch.bfloat16, torch.device("cpu")).fill(5)
    assert torch.equal(x, ref_x) and torch.equal(dy, ref_dy)       # same values as the unbound draw
    d.bind_transposed(xt, None)
    x, dy = d.fill(6)
    assert x._dllm_t is xt and dy._dllm_t is None
    monkeypatch.setenv("DLLM_DRAW_T", "0")
    d.bind_transposed(xt, dyt)
    x, _ = d.fill(7)
    assert x._dllm_t is None
    o = DeviceMockData(64, 32, torch.bfloat16, torch.device("cpu"), overlap=True)   # (CPU: overlap is off anyway)
    monkeypatch.delenv("DLLM_DRAW_T")
    o.bind_transposed(xt, dyt)
    x, _ = o.fill(8)
    assert x._dllm_t is xt
