"""Debug: fp32 engine (SGD, unfused), one step: layer-0 intermediates vs CPU recomputation from the engine's own inputs."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch
import dllm  # noqa
from dllm.parallel.engine import FFNTrainer
from dllm.parallel.mesh import Mesh
from dllm.utils.config import ModelConfig, TrainConfig
from test_engine_gpu import _setup

def rep(name, got, want):
    got, want = got.cpu(), want.cpu()
    d = (got - want).abs()
    bad = d > 1e-5 * want.abs().max() + 1e-8
    idx = bad.nonzero()[:5].tolist()
    print(f"{name:10s} max|d| {d.max():.3e} ref {want.abs().max():.3e} nbad {int(bad.sum())} first {idx}", flush=True)

D, F, L, T, lr = 128, 512, 2, 256, 1e-3
layers, batches = _setup(D, F, L, T, "relu", False, 3)
cfg = TrainConfig(model=ModelConfig(D, F, L), batch_size=1, seq_len=T, dtype="fp32", grad_dtype="fp32",
                  lr=lr, optimizer="sgd", skip_input_grad=False, fused_optimizer=False)
eng = FFNTrainer(cfg, Mesh(), torch.device("cuda"))
eng.load_full_params(layers)
x, dy = batches[0]
xg, dyg = x.cuda(), dy.cuda()
eng.train_step(xg, dyg)
torch.cuda.synchronize()
W1 = [layers[l]["w1"] for l in range(L)]; W2 = [layers[l]["w2"] for l in range(L)]
a0 = torch.relu(x @ W1[0].t()); y0 = a0 @ W2[0].t()
rep("a0", eng.acts_a[0], a0)
rep("y0", eng.xs[1], y0)
a1 = torch.relu(eng.xs[1].cpu() @ W1[1].t())
rep("a1", eng.acts_a[1], a1)
# backward of layer 1 from the engine's own tensors
da1 = (dy @ W2[1]) * (eng.acts_a[1].cpu() > 0)
dx1 = da1 @ W1[1]
rep("dW2_1", eng.grad_view(1, "w2"), dy.t() @ eng.acts_a[1].cpu())
rep("dW1_1", eng.grad_view(1, "w1"), da1.t() @ eng.xs[1].cpu())
rep("dx1", eng.dxb[1], dx1)
da0 = (eng.dxb[1].cpu() @ W2[0]) * (eng.acts_a[0].cpu() > 0)
rep("da0", eng.da, da0)
rep("dW2_0", eng.grad_view(0, "w2"), eng.dxb[1].cpu().t() @ eng.acts_a[0].cpu())
rep("dW1_0", eng.grad_view(0, "w1"), eng.da.cpu().t() @ x)
rep("dW1_0b", eng.grad_view(0, "w1"), da0.t() @ x)
