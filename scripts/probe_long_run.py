"""Long-run behaviour of the flagship stack on the reference's mock objective (fresh random dL/dy every step, SGD at
lr 1e-5), fan-in init: weight / output statistics every 20 steps, for the TN weight-gradient layout, the NN layout,
and the NN layout with the transposes drawn with the batch.  All three are bitwise the same step (GPU tests), so they
must agree here too; the question is when the weights stop being finite and why (bench.py reports ``finite``).

    python scripts/probe_long_run.py [--steps 240] [--every 20]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dllm  # noqa: E402,F401
from dllm.models.ffn import init_ffn_params_device  # noqa: E402
from dllm.parallel.engine import FFNTrainer  # noqa: E402
from dllm.parallel.mesh import Mesh  # noqa: E402
from dllm.utils.config import ModelConfig, TrainConfig  # noqa: E402
from dllm.utils.data import DeviceMockData  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=240)
    ap.add_argument("--every", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    m = ModelConfig(model_size=4096, ffn_dim=16384, layers=8, act="relu")
    for layout, bind in (("tn", False), ("auto", False), ("auto", True)):
        cfg = TrainConfig(model=m, batch_size=8, seq_len=1024, dtype="bf16", grad_dtype="bf16", optimizer="sgd",
                          wgrad_layout=layout)
        eng = FFNTrainer(cfg, Mesh(), dev)
        eng.load_full_params(init_ffn_params_device(m.D, m.F, m.layers, 1, dev, scale="fan_in"))
        data = DeviceMockData(cfg.tokens, m.D, torch.bfloat16, dev)
        if bind:
            data.bind_transposed(*eng.input_transposes())
        print(f"layout {layout} bind {bind}: wgrad_nn {eng.wgrad_nn} w2t {eng.w2t} lr {cfg.lr}", flush=True)
        for i in range(a.steps):
            x, dy = data.fill(10_000 + i)
            y = eng.train_step(x, dy)
            if (i + 1) % a.every == 0 or i < 2:
                torch.cuda.synchronize()
                ps = eng.local_params()
                st = [(p["w1"].float().abs().max().item(), p["w2"].float().abs().max().item()) for p in ps]
                yf = y.float()
                print(f"  step {i + 1:4d}: y std {yf.std().item():.4g} max {yf.abs().max().item():.4g} finite "
                      f"{bool(torch.isfinite(yf).all())} copy finite {bool(torch.isfinite(eng.copy).all())}; max|w1|/|w2| "
                      f"L0 {st[0][0]:.4g}/{st[0][1]:.4g} L4 {st[4][0]:.4g}/{st[4][1]:.4g} L7 {st[7][0]:.4g}/{st[7][1]:.4g}",
                      flush=True)
        del eng, data
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
