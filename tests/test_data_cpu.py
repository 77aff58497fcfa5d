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
