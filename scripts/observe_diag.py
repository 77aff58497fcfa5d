"""Comm-observer diagnostics: run a communicating method at N=1 over size-1 communicators for a few steps under the
CommObserver and print the raw intervals of the last step (collective issue -> completion per role, GEMM begin ->
end) next to the summary, so the observer's overlap can be checked against a rocprofv3 trace of the same run.

    python scripts/observe_diag.py --method zero [--steps 3] [--layers 8]

Same-run check against the kernel trace (scripts/gpu_runs/r3_obs.sh):
    rocprofv3 --kernel-trace -d gpurun_out/obs_zero -o run -- python3 scripts/observe_diag.py --method zero
    python scripts/rocpd_stats.py gpurun_out/obs_zero/run_results.db --overlap copyBuffer,nccl,rccl \
        --step_marker 'rng_normal_kernel<unsigned short>' --from_marker 3
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dllm  # noqa: E402,F401
from dllm.models.ffn import init_ffn_params_device  # noqa: E402
from dllm.parallel.engine import FFNTrainer  # noqa: E402
from dllm.parallel.mesh import Mesh, init_distributed  # noqa: E402
from dllm.utils.config import ModelConfig, TrainConfig  # noqa: E402
from dllm.utils.data import DeviceMockData  # noqa: E402
from dllm.utils.observe import CommObserver  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--method", default="zero", choices=["ddp", "zero", "fsdp"])
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--comm", default="torch")
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29611")
    init_distributed("nccl", 0, 1)
    dev = torch.device("cuda", 0)
    m = ModelConfig(4096, 16384, a.layers)
    cfg = TrainConfig(model=m, batch_size=8, seq_len=1024, dtype="bf16", grad_dtype="bf16", dp_mode=a.method,
                      force_comm=True, comm_backend=a.comm, lr=1e-5)
    mesh = Mesh.build(1, 1, force=True, comm_backend=a.comm, device=dev)
    eng = FFNTrainer(cfg, mesh, dev)
    eng.load_full_params(init_ffn_params_device(m.D, m.F, m.layers, 1, dev, False))
    data = DeviceMockData(cfg.tokens, m.D, torch.bfloat16, dev)
    for s in range(2):
        eng.train_step(*data.fill(s))
    torch.cuda.synchronize()
    with CommObserver(dev, dict(mesh.groups)) as obs:
        for s in range(a.steps):
            eng.train_step(*data.fill(10 + s))
    summ = obs.summary(a.steps)
    per_role, gemms = obs.intervals()
    t_last = gemms[-(len(gemms) // a.steps)][0] if gemms else 0.0
    print(json.dumps(summ))
    print("last step (ms since observation start):")
    ev = [(s, e, f"GEMM") for s, e in gemms if s >= t_last]
    for r, iv in per_role.items():
        ev += [(s, e, r) for s, e in iv if s >= t_last]
    for s, e, what in sorted(ev):
        print(f"  {what:6s} {s:9.3f} -> {e:9.3f}  ({(e - s) * 1e3:8.1f} us)")
    mesh.destroy()
    torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
