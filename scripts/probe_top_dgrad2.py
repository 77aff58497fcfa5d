"""Isolated dgrad (NT, W2 stored transposed, ReLU mask) with the weights and masks of different layers of a trained
flagship stack: which operand makes the top layer's dgrad slow?"""
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


def main():
    dev = torch.device("cuda", 0)
    m = ModelConfig(model_size=4096, ffn_dim=16384, layers=8, act="relu")
    cfg = TrainConfig(model=m, batch_size=8, seq_len=1024, dtype="bf16", grad_dtype="bf16", optimizer="sgd")
    eng = FFNTrainer(cfg, Mesh(), dev)
    eng.load_full_params(init_ffn_params_device(m.D, m.F, m.layers, 1, dev))
    data = DeviceMockData(cfg.tokens, m.D, torch.bfloat16, dev)
    for i in range(3):
        x, dy = data.fill(i)
        eng.train_step(x, dy)
    torch.cuda.synchronize()
    lay = "nt" if eng.w2s else "nn"
    dx = eng.dxb[1].clone()
    da = torch.empty_like(eng.acts_a[0])
    for l in range(8):
        msk = eng._mask(l)
        dens = None
        a = eng.acts_a[l]
        dens = (a != 0).float().mean().item()
        print(f"layer {l}: activation density {dens:.3f}  |W2| std {eng.copy_view(l, 'w2').float().std().item():.4f}",
              flush=True)
    res = {}
    for _ in range(3):
        for lw in (7, 6, 3, 0):
            for lm in (7, 3):
                k = (lw, lm)
                res.setdefault(k, []).append(timeit(lambda: gemm(dx, eng.copy_view(lw, "w2"), lay, out=da, epi="dact",
                                                                 act="relu", aux=eng.acts_a[lm], mask=eng._mask(lm))))
    for (lw, lm), v in res.items():
        print(f"W2 of layer {lw}, mask of layer {lm}: {statistics.median(v):7.1f} us", flush=True)
    res2 = []
    for _ in range(3):
        res2.append(timeit(lambda: gemm(dx, eng.copy_view(7, "w2"), lay, out=da)))
    print(f"plain store (no mask), W2 of layer 7: {statistics.median(res2):7.1f} us", flush=True)


if __name__ == "__main__":
    main()
