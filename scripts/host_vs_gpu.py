"""Is a forced-communicator step host-bound?  Runs a method's engine (N=1, size-1 communicators) and records, per
step, the host time to enqueue it (train_step returning) and the GPU time between step-boundary events, without any
synchronisation inside the timed loop.  If the host's enqueue time per step approaches the GPU's step time, the GPU
waits for the host somewhere in the step (idle gaps in a kernel trace), whatever the collectives themselves cost.

    python scripts/host_vs_gpu.py --method fsdp [--layers 8 --ffn_dim 16384 --steps 12] [--elide]"""
import argparse
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dllm  # noqa: E402,F401
from dllm.models.ffn import init_ffn_params_device  # noqa: E402
from dllm.parallel import comm  # noqa: E402
from dllm.parallel.engine import FFNTrainer  # noqa: E402
from dllm.parallel.mesh import Mesh, init_distributed  # noqa: E402
from dllm.utils.config import ModelConfig, TrainConfig  # noqa: E402
from dllm.utils.data import DeviceMockData  # noqa: E402
from dllm.utils.streams import reserve_compute_queue  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--method", default="fsdp", choices=["ddp", "zero", "fsdp", "hybrid"])
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--model_size", type=int, default=4096)
    ap.add_argument("--ffn_dim", type=int, default=16384)
    ap.add_argument("--gated", action="store_true")
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--elide", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    reserve_compute_queue(dev)
    os.environ.setdefault("LOCAL_RANK", "0")
    init_distributed("nccl", 0, 1, "127.0.0.1", 29500 + os.getpid() % 500)
    dp_mode = "fsdp" if a.method == "hybrid" else a.method
    cfg = TrainConfig(model=ModelConfig(a.model_size, a.ffn_dim, a.layers, "silu" if a.gated else "relu", a.gated),
                      batch_size=8, seq_len=1024, dtype="bf16", grad_dtype="bf16", dp_mode=dp_mode, force_comm=True,
                      comm_backend="torch")
    mesh = Mesh.build(1, 1, force=True, comm_backend="torch", device=dev)
    eng = FFNTrainer(cfg, mesh, dev)
    eng.load_full_params(init_ffn_params_device(a.model_size, a.ffn_dim, a.layers, 1, dev, a.gated,
                                                scale="fan_in" if a.gated else 2e-2))
    data = DeviceMockData(cfg.tokens, a.model_size, torch.bfloat16, dev)
    comm.set_elide(a.elide)
    for s in range(3):
        x, dy = data.fill(s)
        eng.train_step(x, dy)
    torch.cuda.synchronize()
    evs, host = [], []
    t0 = time.perf_counter()
    for s in range(a.steps):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        evs.append(ev)
        x, dy = data.fill(100 + s)
        eng.train_step(x, dy)
        host.append(time.perf_counter())
    ev = torch.cuda.Event(enable_timing=True)
    ev.record()
    evs.append(ev)
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    gpu = [evs[i].elapsed_time(evs[i + 1]) for i in range(a.steps)]
    hostd = [(host[i] - (host[i - 1] if i else t0)) * 1e3 for i in range(a.steps)]
    print(f"{a.method} L{a.layers} elide={a.elide}: GPU ms/step median {statistics.median(gpu):.3f}, host enqueue "
          f"ms/step median {statistics.median(hostd):.3f} (total host {t_host * 1e3:.1f} ms for {a.steps} steps, "
          f"GPU {sum(gpu):.1f} ms)", flush=True)
    print("  host per step:", [round(v, 2) for v in hostd], flush=True)
    comm.set_elide(False)
    mesh.destroy()


if __name__ == "__main__":
    main()
