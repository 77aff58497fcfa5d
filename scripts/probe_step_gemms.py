"""Per-GEMM HIP-event times inside the flagship step (models/ffn's gemm wrapped; no synchronisation added), to study
the top layer's slow dgrad.  --dup: run the first dgrad of every backward twice (the first result discarded), to see
whether the slowness belongs to the first dgrad after the forward or to that layer's data."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dllm  # noqa: E402,F401
import dllm.models.ffn as ffn  # noqa: E402
from dllm.models.ffn import init_ffn_params_device  # noqa: E402
from dllm.parallel.engine import FFNTrainer  # noqa: E402
from dllm.parallel.mesh import Mesh  # noqa: E402
from dllm.utils.config import ModelConfig, TrainConfig  # noqa: E402
from dllm.utils.data import DeviceMockData  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dup", action="store_true")
    ap.add_argument("--steps", type=int, default=6)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    m = ModelConfig(model_size=4096, ffn_dim=16384, layers=8, act="relu")
    cfg = TrainConfig(model=m, batch_size=8, seq_len=1024, dtype="bf16", grad_dtype="bf16", optimizer="sgd")
    eng = FFNTrainer(cfg, Mesh(), dev)
    eng.load_full_params(init_ffn_params_device(m.D, m.F, m.layers, 1, dev))
    data = DeviceMockData(cfg.tokens, m.D, torch.bfloat16, dev)
    inner = ffn.gemm
    rec = []
    state = {"first_dact": True}

    def timed(*args, **kw):
        if a.dup and kw.get("epi") == "dact" and state["first_dact"]:
            state["first_dact"] = False
            s0, e0 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s0.record()
            inner(*args, **kw)
            e0.record()
            rec.append(("dact (duplicate, discarded)", s0, e0))
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        out = inner(*args, **kw)
        e.record()
        name = f"{args[2]} {kw.get('epi', 'store')}{' out_t' if kw.get('out_t') else ''}{' +copy' if kw.get('aux_t') is not None else ''}"
        rec.append((name, s, e))
        return out

    ffn.gemm = timed
    for i in range(a.steps):
        rec.clear()
        state["first_dact"] = True
        x, dy = data.fill(i)
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        eng.train_step(x, dy)
        t1.record()
    torch.cuda.synchronize()
    print(f"step {t0.elapsed_time(t1):.3f} ms (dup={a.dup})", flush=True)
    for name, s, e in rec:
        print(f"  {name:34s} {s.elapsed_time(e) * 1e3:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
