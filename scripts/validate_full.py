"""Full-size validation of the flagship training step against an independent torch (hipBLASLt) step.

Runs ONE step of the bench configuration (L8 D4096 F16384 ReLU, T=8192, bf16 compute, fp32 master, SGD)
through the engine (native kernels, fused optimizer) and through plain torch ops with the same rounding
points, then compares the weight updates of every layer.  Also reports the fraction of zero activations
(ReLU sparsity: the reason the end-to-end clock, and TFLOP/s, runs above the dense-random microbench).
"""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import dllm  # noqa
from dllm.models.ffn import init_ffn_params_device
from dllm.parallel.engine import FFNTrainer
from dllm.parallel.mesh import Mesh
from dllm.utils.config import ModelConfig, TrainConfig
from dllm.utils.data import DeviceMockData

L = int(os.environ.get("VAL_LAYERS", "8"))
D, F, T, lr = 4096, 16384, 8192, 1.0
dev = torch.device("cuda")
m = ModelConfig(D, F, L)
cfg = TrainConfig(model=m, batch_size=8, seq_len=1024, dtype="bf16", grad_dtype="fp32", lr=lr)
eng = FFNTrainer(cfg, Mesh(), dev)
params = init_ffn_params_device(D, F, L, 1234, dev)
eng.load_full_params(params)
data = DeviceMockData(T, D, torch.bfloat16, dev)
x, dy = data.fill(777)
x, dy = x.clone(), dy.clone()
eng.train_step(x, dy)
torch.cuda.synchronize()
zero_frac = [float((eng.acts_a[l] == 0).float().mean()) for l in range(L)]
got = eng.local_params()

# independent torch step (bf16 storage at the same points, fp32 accumulation)
W = [{k: v.to(torch.bfloat16) for k, v in p.items()} for p in params]
xs, As = [x], []
for l in range(L):
    a = torch.relu(xs[-1] @ W[l]["w1"].t())
    As.append(a)
    xs.append(a @ W[l]["w2"].t())
g = dy
res = {}
for l in reversed(range(L)):
    da = (g @ W[l]["w2"]) * (As[l] > 0)
    gw2 = g.float().t() @ As[l].float()
    gw1 = da.float().t() @ xs[l].float()
    new = {"w1": params[l]["w1"] - lr * gw1, "w2": params[l]["w2"] - lr * gw2}
    for k in ("w1", "w2"):
        d_got = got[l][k] - params[l][k]
        d_ref = new[k] - params[l][k]
        res[f"L{l}.{k}"] = float((d_got - d_ref).norm() / d_ref.norm())
    if l > 0:
        g = da @ W[l]["w1"]
worst = max(res.values())
print(json.dumps({"layers": L, "worst_rel_update_err": worst, "per_tensor": res, "relu_zero_frac": zero_frac}))
assert worst < 2e-2, worst
print("validate_full OK")
