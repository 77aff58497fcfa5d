"""Debug aid: run the engine with wgrad_layout tn and nn side by side for a few steps and report the first tensors
that differ (outputs per step, masters per weight, the transposed copies against their sources)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dllm  # noqa: E402,F401
from dllm.models.ffn import init_ffn_params_device  # noqa: E402
from dllm.ops.gemm import set_splitk  # noqa: E402
from dllm.parallel.engine import FFNTrainer  # noqa: E402
from dllm.parallel.mesh import Mesh  # noqa: E402
from dllm.utils.config import ModelConfig, TrainConfig  # noqa: E402
from dllm.utils.data import DeviceMockData  # noqa: E402


def main():
    D, F, L, T = (int(v) for v in (sys.argv[1:5] if len(sys.argv) > 4 else (512, 1024, 3, 1024)))
    variant = sys.argv[5] if len(sys.argv) > 5 else "fused_serial"
    set_splitk(False)
    dev = torch.device("cuda", 0)
    m = ModelConfig(model_size=D, ffn_dim=F, layers=L, act="relu")
    engs = {}
    for layout in ("tn", "nn"):
        cfg = TrainConfig(model=m, batch_size=1, seq_len=T, dtype="bf16", grad_dtype="fp32", optimizer="sgd", lr=0.05,
                          wgrad_layout=layout, wgrad_stream=variant == "fused_wgrad_stream",
                          fused_optimizer=variant.startswith("fused"))
        eng = FFNTrainer(cfg, Mesh(), dev)
        eng.load_full_params(init_ffn_params_device(D, F, L, 7, dev))
        engs[layout] = eng
        print(layout, "wgrad_nn", eng.wgrad_nn, "pair", eng.pair_wgrads, "wg_stream", eng.wg_stream is not None,
              flush=True)
    data = DeviceMockData(T, D, torch.bfloat16, dev)
    for i in range(3):
        x, dy = data.fill(i)
        ys = {k: e.train_step(x, dy).clone() for k, e in engs.items()}
        torch.cuda.synchronize()
        print(f"step {i}: y equal {torch.equal(ys['tn'], ys['nn'])}", flush=True)
        e = engs["nn"]
        for l in range(L):
            print(f"  xT[{l}] == xs[{l}].t(): {torch.equal(e.xT[l], e.xs[l].t())}", flush=True)
        for l in range(L):
            for n in ("w1", "w2"):
                a_, b_ = engs["tn"].copy_view(l, n), e.copy_view(l, n)
                if not torch.equal(a_, b_):
                    d = (a_.float() - b_.float()).abs()
                    print(f"  copy {l}.{n} differs: max {d.max().item():.3e} count {(d > 0).sum().item()}", flush=True)


if __name__ == "__main__":
    main()
