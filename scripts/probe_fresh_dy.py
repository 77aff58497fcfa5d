"""In the flagship step the top layer's dgrad (reading the step's mock dL/dy, drawn ~28 ms earlier) runs ~150 us
longer than the other layers' (reading a dx the previous GEMM just wrote).  Probe: rewrite dL/dy right before the
backward (FFNTrainer.before_backward, a 64 MB device copy) so it is as freshly written as a computed dx, and compare
step times, interleaved."""
import os
import statistics
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
    cfg = TrainConfig(model=m, batch_size=8, seq_len=1024, dtype="bf16", grad_dtype="bf16", optimizer="sgd")
    eng = FFNTrainer(cfg, Mesh(), dev)
    eng.load_full_params(init_ffn_params_device(m.D, m.F, m.layers, 1, dev))
    data = DeviceMockData(cfg.tokens, m.D, torch.bfloat16, dev)
    dy_buf = torch.empty(cfg.tokens, m.D, dtype=torch.bfloat16, device=dev)
    src = {}

    def fresh():
        dy_buf.copy_(src["dy"])

    def run(mode, steps=20):
        eng.before_backward = fresh if mode == "fresh" else None
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for i in range(steps + 3):
            if i == 3:
                torch.cuda.synchronize()
                s.record()
            x, dy = data.fill(i)
            src["dy"] = dy
            dy_buf.copy_(dy)          # both modes pay one copy at the step start
            eng.train_step(x, dy_buf)
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / steps

    res = {"copy at step start only": [], "fresh": []}
    for _ in range(4):
        res["copy at step start only"].append(run("start"))
        res["fresh"].append(run("fresh"))
    for k, v in res.items():
        print(f"{k:26s} {statistics.median(v):.3f} ms  ({', '.join(f'{t:.3f}' for t in v)})", flush=True)


if __name__ == "__main__":
    main()
