"""The TP8 shard's transposed-layout forward GEMM y = (aᵀ)ᵀ·W2ᵀ ([8192, 4096], K = F/8 = 1792, TN) and dx-shaped
products: native TN kernel vs torch.matmul (hipBLASLt) on the same operands; median of rounds.

    python scripts/bench_tn_small_k.py"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dllm  # noqa: E402,F401
from dllm.ops.gemm import gemm  # noqa: E402


def timeit(fn, iters=20):
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
    g = torch.Generator().manual_seed(0)
    for F, T, D in ((1792, 8192, 4096), (3584, 8192, 4096)):
        aT = torch.randn(F, T, generator=g).to(torch.bfloat16).cuda()
        w2t = torch.randn(F, D, generator=g).to(torch.bfloat16).cuda()
        y = torch.empty(T, D, dtype=torch.bfloat16, device="cuda")
        nat, lib = [], []
        for _ in range(5):
            nat.append(timeit(lambda: gemm(aT, w2t, "tn", out=y)))
            lib.append(timeit(lambda: torch.matmul(aT.t(), w2t, out=y)))
        fl = 2 * T * D * F
        n, l = statistics.median(nat), statistics.median(lib)
        print(f"TN [T {T}, D {D}] K = {F}: native {n:.1f} us ({fl / n / 1e6:.0f} TF), hipBLASLt {l:.1f} us "
              f"({fl / l / 1e6:.0f} TF)", flush=True)


if __name__ == "__main__":
    main()
