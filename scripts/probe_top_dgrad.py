"""Why the top layer's dgrad runs ~25 % longer than the others in the flagship step (rocprofv3 timeline): time the
same NT dgrad GEMM (da = dy·W2 ⊙ ReLU mask, W2 stored transposed) with the step's mock dL/dy (0.1·N(0,1)) as dy and
with a computed input gradient (the dx a lower layer's dgrad receives), same weights and mask."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dllm  # noqa: E402,F401
from dllm.models.ffn import init_ffn_params_device  # noqa: E402
from dllm.ops.gemm import gemm  # noqa: E402
from dllm.parallel.engine import FFNTrainer  # noqa: E402
from dllm.parallel.mesh import Mesh  # noqa: E402
from dllm.utils.config import ModelConfig, TrainConfig  # noqa: E402
from dllm.utils.data import DeviceMockData  # noqa: E402


def timeit(fn, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def stats(t):
    f = t.float()
    nz = (t != 0).float().mean().item()
    return f"std {f.std().item():.4f} nonzero {nz:.3f} |x|<2^-10 {(f.abs() < 2**-10).float().mean().item():.3f}"


def main():
    dev = torch.device("cuda", 0)
    m = ModelConfig(model_size=4096, ffn_dim=16384, layers=8, act="relu")
    cfg = TrainConfig(model=m, batch_size=8, seq_len=1024, dtype="bf16", grad_dtype="bf16", optimizer="sgd")   # the reference lr (1e-5)
    eng = FFNTrainer(cfg, Mesh(), dev)
    eng.load_full_params(init_ffn_params_device(m.D, m.F, m.layers, 1, dev))
    data = DeviceMockData(cfg.tokens, m.D, torch.bfloat16, dev)
    for i in range(3):
        x, dy = data.fill(i)
        eng.train_step(x, dy)
    torch.cuda.synchronize()
    L = m.layers
    w2 = eng.copy_view(L - 1, "w2")
    a, mask = eng.acts_a[L - 1], eng._mask(L - 1)
    dx = eng.dxb[(1) % len(eng.dxb)]                     # a computed input gradient of this step
    da = torch.empty_like(a)
    lay = "nt" if eng.w2s else "nn"
    print("mock dy :", stats(dy), flush=True)
    print("dx      :", stats(dx), flush=True)
    print("x (input):", stats(x), flush=True)
    scaled = (dx.float() * (dy.float().std() / dx.float().std())).to(torch.bfloat16)
    res = {"mock dy": [], "computed dx": [], "dx rescaled to dy's std": [], "x (N(0,1))": []}
    for _ in range(5):
        for k, A in (("mock dy", dy), ("computed dx", dx), ("dx rescaled to dy's std", scaled), ("x (N(0,1))", x)):
            res[k].append(timeit(lambda: gemm(A, w2, lay, out=da, epi="dact", act="relu", aux=a, mask=mask)))
    for k, v in res.items():
        print(f"{k:26s} {statistics.median(v):7.1f} us", flush=True)


if __name__ == "__main__":
    main()
