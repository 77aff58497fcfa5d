"""utils/streams.py: the side-stream placement knob (DLLM_SIDE_STREAMS) and the engine's use of it off the GPU."""
import pytest
import torch

from dllm.utils import streams


def test_mode_default_and_validation(monkeypatch):
    monkeypatch.delenv("DLLM_SIDE_STREAMS", raising=False)
    assert streams.mode() == "role" and streams.high_priority("fsdp")
    assert not streams.high_priority("wgrad") and not streams.high_priority("opt")
    monkeypatch.setenv("DLLM_SIDE_STREAMS", "pool")
    assert not streams.high_priority("fsdp")
    monkeypatch.setenv("DLLM_SIDE_STREAMS", "auto")
    assert streams.high_priority("wgrad") and not streams.high_priority("opt") and not streams.high_priority("fsdp")
    monkeypatch.setenv("DLLM_SIDE_STREAMS", "high")
    assert streams.mode() == "high" and streams.high_priority("opt")
    monkeypatch.setenv("DLLM_SIDE_STREAMS", "masked")
    with pytest.raises(ValueError):
        streams.mode()


def test_engine_has_no_side_streams_on_cpu(monkeypatch):
    from dllm.parallel.engine import FFNTrainer
    from dllm.parallel.mesh import Mesh
    from dllm.utils.config import ModelConfig, TrainConfig

    monkeypatch.setenv("DLLM_SIDE_STREAMS", "high")   # never reaches the native library off the GPU
    cfg = TrainConfig(model=ModelConfig(64, 128, 2), batch_size=1, seq_len=64, dtype="fp32", grad_dtype="fp32")
    eng = FFNTrainer(cfg, Mesh(), torch.device("cpu"))
    assert eng._side_stream("opt") is None and eng.wg_stream is None
