"""How much do CU-occupying side-stream kernels (a stand-in for RCCL channel workgroups during an
overlapped collective) slow the GEMMs down?

    python experiments/interference.py [--cus 0,8,16,32,64] [--usec 3000]

A side stream keeps `c` CUs busy (experiments/occupy.hip, built here into its own .so: one 96-KiB-LDS wave per CU,
spinning) for the whole
timed window while the main stream runs a GEMM back to back.  The ideal slowdown is 256/(256-c); anything
above that is tile-wave quantisation / dispatch interference.  Also reports torch.matmul (hipBLASLt).
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dllm  # noqa: E402,F401
from dllm.ops.gemm import gemm  # noqa: E402



def _occupier() -> ctypes.CDLL:
    here = os.path.dirname(os.path.abspath(__file__))
    src, so = os.path.join(here, "occupy.hip"), os.path.join(here, "_occupy.so")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.run(["hipcc", "-O3", "-fPIC", "-shared", "--offload-arch=gfx950", src, "-o", so], check=True)
    lib = ctypes.CDLL(so)
    lib.dllm_occupy_cus.restype = ctypes.c_int
    lib.dllm_occupy_cus.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=8192)
    ap.add_argument("--D", type=int, default=4096)
    ap.add_argument("--F", type=int, default=16384)
    ap.add_argument("--cus", default="0,8,16,32,64")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--json", default="")
    ap.add_argument("--tpb", type=int, default=2, help="tiles per persistent GEMM block (1 = off)")
    ap.add_argument("--min_bpc", type=int, default=1, help="minimum persistent blocks per CU")
    a = ap.parse_args()
    from dllm.ops.gemm import set_min_blocks_per_cu, set_tiles_per_block

    set_tiles_per_block(a.tpb)
    set_min_blocks_per_cu(a.min_bpc)
    occ = _occupier()
    T, D, F = a.T, a.D, a.F
    bf, dev = torch.bfloat16, "cuda"
    x = torch.randn(T, D, device=dev, dtype=bf)
    w1 = torch.randn(F, D, device=dev, dtype=bf) * 0.02
    w2 = torch.randn(D, F, device=dev, dtype=bf) * 0.02
    h = torch.randn(T, F, device=dev, dtype=bf)
    out_tf = torch.empty(T, F, device=dev, dtype=bf)
    out_td = torch.empty(T, D, device=dev, dtype=bf)
    dy = torch.randn(T, D, device=dev, dtype=bf)
    g = torch.empty(D, F, device=dev, dtype=bf)
    cases = {
        "fwd1 NT act (2048 tiles)": lambda: gemm(x, w1, "nt", out=out_tf, epi="act", act="relu"),
        "fwd2 NT (512 tiles)": lambda: gemm(h, w2, "nt", out=out_td),
        "wgrad TN bf16 (1024 tiles)": lambda: gemm(dy, h, "tn", out=g),
        "dx-shape NN (512 tiles)": lambda: gemm(h, w1, "nn", out=out_td),
    }
    side = torch.cuda.Stream()
    res = {}
    for name, fn in cases.items():
        res[name] = {}
        fn()
        torch.cuda.synchronize()
        for c in [int(v) for v in a.cus.split(",")]:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            # estimate the window: iters * ~1.5 ms, cover it generously
            if c:
                with torch.cuda.stream(side):
                    rc = occ.dllm_occupy_cus(c, 2000 + 2000 * a.iters, side.cuda_stream)
                    assert rc == 0, rc
                torch.cuda._sleep(2_000_000)  # let the occupiers land before the GEMMs start
            s.record()
            for _ in range(a.iters):
                fn()
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / a.iters
            base = res[name].get(0, ms)
            res[name][c] = ms
            ideal = 256 / (256 - c)
            print(f"{name:28s} occupied CUs {c:3d}: {ms*1e3:8.1f} us  slowdown x{ms/base:.3f} (ideal x{ideal:.3f})",
                  flush=True)
    if a.json:
        json.dump(res, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
