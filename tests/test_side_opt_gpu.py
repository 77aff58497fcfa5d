"""Side-stream optimizer (TrainConfig.side_optimizer): wgrad GEMMs store gradients, a low-occupancy SGD
kernel on its own stream applies the update, the forward waits per weight.  Same result as the
unfused single-device path (bitwise: same kernels' arithmetic on the same stored gradients)."""
import pytest
import torch

from dllm.models.ffn import init_ffn_layer
from dllm.parallel.engine import FFNTrainer
from dllm.parallel.mesh import Mesh
from dllm.utils.config import ModelConfig, TrainConfig
from dllm.utils.data import reference_mock_data

pytestmark = pytest.mark.gpu


def _train(side, fused, dtype="bf16", opt="sgd", master="fp32"):
    D, F, L, T = 256, 1024, 3, 512
    gen = torch.Generator().manual_seed(5)
    layers = [init_ffn_layer(D, F, gen) for _ in range(L)]
    batches = list(reference_mock_data(torch.randint(100_000, (4,), generator=gen), T, D))
    cfg = TrainConfig(model=ModelConfig(D, F, L), batch_size=1, seq_len=T, dtype=dtype, grad_dtype=dtype,
                      lr=1e-2 if opt == "sgd" else 1e-3, optimizer=opt, side_optimizer=side, fused_optimizer=fused,
                      master=master)   # the capped SGD side kernel: fp32 master
    dev = torch.device("cuda", 0)
    eng = FFNTrainer(cfg, Mesh.build(1, 1, device=dev), dev)
    assert eng.side_opt == (side != 0)
    eng.load_full_params(layers)
    cd = torch.bfloat16 if dtype == "bf16" else torch.float32
    for x, dy in batches:
        eng.train_step(x.to(dev, cd), dy.to(dev, cd))
    out = eng.local_params()
    torch.cuda.synchronize()
    return [{k: v.cpu().clone() for k, v in p.items()} for p in out]


@pytest.mark.parametrize("blocks", [4, 32])
def test_side_optimizer_matches_unfused(blocks):
    a = _train(blocks, fused=False)
    b = _train(0, fused=False)
    for pa, pb in zip(a, b):
        for k in pa:
            assert torch.equal(pa[k], pb[k]), k



@pytest.mark.parametrize("opt", ["sgd", "adam"])
def test_whole_chip_side_optimizer_matches_unfused(opt):
    """side_optimizer < 0: stored gradients, each weight's flat update (split masters, SGD / AdamW) on the side stream
    with the whole chip -- bitwise the serial unfused update (the same flat kernel on the same gradients)."""
    a = _train(-1, fused=False, opt=opt, master="split")
    b = _train(0, fused=False, opt=opt, master="split")
    for pa, pb in zip(a, b):
        for k in pa:
            assert torch.equal(pa[k], pb[k]), k
