"""Weights' statistics over the first steps of the flagship stack, TN vs NN weight-gradient layouts (a sanity check:
the master must stay finite and move by ~lr-sized steps)."""
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
    dev = torch.device("cuda", 0)
    m = ModelConfig(model_size=4096, ffn_dim=16384, layers=8, act="relu")
    for layout in ("tn", "auto"):
        cfg = TrainConfig(model=m, batch_size=8, seq_len=1024, dtype="bf16", grad_dtype="bf16", optimizer="sgd",
                          wgrad_layout=layout)
        eng = FFNTrainer(cfg, Mesh(), dev)
        eng.load_full_params(init_ffn_params_device(m.D, m.F, m.layers, 1, dev))
        data = DeviceMockData(cfg.tokens, m.D, torch.bfloat16, dev)
        print(f"layout {layout}: wgrad_nn {eng.wgrad_nn} w2t {eng.w2t} lr {cfg.lr}", flush=True)
        for i in range(4):
            x, dy = data.fill(i)
            y = eng.train_step(x, dy)
            torch.cuda.synchronize()
            ps = eng.local_params()
            s = [(p["w1"].float().std().item(), p["w2"].float().std().item()) for p in ps]
            print(f"  step {i}: y std {y.float().std().item():.4g} finite {bool(torch.isfinite(y).all())}; "
                  f"w1/w2 std L0 {s[0][0]:.4g}/{s[0][1]:.4g} L7 {s[7][0]:.4g}/{s[7][1]:.4g}", flush=True)
        del eng, data
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
