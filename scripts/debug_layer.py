"""Compare every intermediate of the engine's bf16 layer fwd/bwd on GPU with the CPU mixed oracle."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import dllm  # noqa
from dllm.models.ffn import init_ffn_layer, layer_fwd, layer_bwd
from dllm.ops.gemm import set_bf16_variant

def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm()).item(), (a - b).abs().max().item()

for variant in ("2stage", "8phase_stagger"):
    set_bf16_variant(variant)
    for act in ("relu", "gelu"):
        D, F, T = 256, 1024, 512
        gen = torch.Generator().manual_seed(5)
        p = init_ffn_layer(D, F, gen)
        x = torch.randn(T, D, generator=gen).bfloat16()
        dy = (0.1 * torch.randn(T, D, generator=gen)).bfloat16()
        w1, w2 = p["w1"].bfloat16(), p["w2"].bfloat16()
        res = {}
        for dev in ("cpu", "cuda"):
            X, DY, W1, W2 = x.to(dev), dy.to(dev), w1.to(dev), w2.to(dev)
            a = torch.empty(T, F, dtype=torch.bfloat16, device=dev)
            h = torch.empty(T, F, dtype=torch.bfloat16, device=dev) if act != "relu" else None
            y = torch.empty(T, D, dtype=torch.bfloat16, device=dev)
            layer_fwd(X, W1, W2, act, False, a, h, y)
            gw1 = torch.empty(F, D, device=dev); gw2 = torch.empty(D, F, device=dev)
            da = torch.empty(T, F, dtype=torch.bfloat16, device=dev)
            dx = torch.empty(T, D, dtype=torch.bfloat16, device=dev)
            layer_bwd(DY, X, W1, W2, act, False, a, h, gw1, gw2, da, dx)
            torch.cuda.synchronize()
            res[dev] = dict(a=a, y=y, gw1=gw1, gw2=gw2, da=da, dx=dx)
        print(variant, act, {k: rel(res["cuda"][k], res["cpu"][k]) for k in res["cpu"]}, flush=True)
        if act == "relu":
            a_g, a_c = res["cuda"]["a"].cpu(), res["cpu"]["a"]
            print("  a zero-mask mismatches:", ((a_g > 0) != (a_c > 0)).sum().item(),
                  " da mask mismatch:", ((res["cuda"]["da"].cpu() != 0) != (res["cpu"]["da"] != 0)).sum().item())
