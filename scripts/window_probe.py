"""Where a short timed window loses time: runs the TP8-shard MP step (or any single-device FFN stack) and times windows
of K steps the way bench.py does (synchronise, K steps, synchronise), with a GPU event at every step boundary, for
several K.  Prints per window: wall ms/step, the first step's GPU time, the median step's GPU time and the delay from
the window's start to the first GPU event (host launch latency).

    python scripts/window_probe.py [--ffn_dim 1792 --layers 1]"""
import argparse
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dllm  # noqa: E402,F401
from dllm.models.ffn import init_ffn_params_device  # noqa: E402
from dllm.parallel.engine import FFNTrainer  # noqa: E402
from dllm.parallel.mesh import Mesh  # noqa: E402
from dllm.utils.config import ModelConfig, TrainConfig  # noqa: E402
from dllm.utils.data import DeviceMockData  # noqa: E402
from dllm.utils.streams import reserve_compute_queue  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model_size", type=int, default=4096)
    ap.add_argument("--ffn_dim", type=int, default=1792)
    ap.add_argument("--layers", type=int, default=1)
    ap.add_argument("--windows", default="5,10,20,50,100")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    reserve_compute_queue(dev)
    cfg = TrainConfig(model=ModelConfig(a.model_size, a.ffn_dim, a.layers, "relu", False), batch_size=8, seq_len=1024,
                      dtype="bf16", grad_dtype="bf16")
    eng = FFNTrainer(cfg, Mesh(), dev)
    eng.load_full_params(init_ffn_params_device(a.model_size, a.ffn_dim, a.layers, 1, dev, False))
    data = DeviceMockData(cfg.tokens, a.model_size, torch.bfloat16, dev)
    seed = 0
    for _ in range(20):
        x, dy = data.fill(seed)
        eng.train_step(x, dy)
        seed += 1
    for k in [int(v) for v in a.windows.split(",")]:
        torch.cuda.synchronize()
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(k + 1)]
        t0 = time.perf_counter()
        t0_ev = torch.cuda.Event(enable_timing=True)
        for i in range(k):
            evs[i].record()
            x, dy = data.fill(seed)
            eng.train_step(x, dy)
            seed += 1
        evs[k].record()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        gpu = [evs[i].elapsed_time(evs[i + 1]) for i in range(k)]
        del t0_ev
        print(f"K={k:4d}: wall {wall / k:.4f} ms/step, GPU first step {gpu[0]:.4f} ms, median {statistics.median(gpu):.4f},"
              f" GPU sum {sum(gpu):.3f} ms vs wall {wall:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
