"""Round-2 4-wave / 4-stage NT GEMM prototype (experiments/gemm_w4b.hip) vs the production 8-phase kernel and
torch.matmul (hipBLASLt) on the FFN's NT shapes, random N(0,1) bf16 operands, interleaved rounds."""
import ctypes
import os
import statistics
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dllm  # noqa: E402,F401
from dllm.ops.gemm import gemm  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def lib(tag="", defines=()):
    src, so = os.path.join(HERE, "gemm_w4b.hip"), os.path.join(HERE, f"_w4b{tag}.so")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.run(["hipcc", "-O3", "-std=c++20", "-fPIC", "-shared", "--offload-arch=gfx950",
                        *[f"-D{d}" for d in defines], src, "-o", so], check=True)
    L = ctypes.CDLL(so)
    L.dllm_gemm_w4b.restype = ctypes.c_int
    L.dllm_gemm_w4b.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p,
                                ctypes.c_long, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    return L


def timeit(fn, it=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


VARIANTS = {"": (), "_n5": ("W4B_NST=5",), "_r4": ("W4B_RD_EVERY=4",)}


def main(build_only=False):
    libs = {t: lib(t, d) for t, d in VARIANTS.items()}
    if build_only:
        return
    for tag, L in libs.items():
        print(f"== variant {tag or 'default'} {VARIANTS[tag]}", flush=True)
        run(L)


def run(L):
    st = torch.cuda.current_stream().cuda_stream
    gm = int(os.environ.get("W4B_GROUP_M", "4"))
    for (M, N, K) in [(512, 512, 256), (8192, 16384, 4096), (8192, 4096, 16384), (8192, 8192, 8192)]:
        a = torch.randn(M, K, device="cuda").bfloat16()
        b = torch.randn(N, K, device="cuda").bfloat16()
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        rc = L.dllm_gemm_w4b(a.data_ptr(), K, b.data_ptr(), K, c.data_ptr(), N, M, N, K, gm, st)
        assert rc == 0, rc
        torch.cuda.synchronize()
        ref = (a.float() @ b.float().t())
        err = ((c.float() - ref).abs().max() / ref.abs().max()).item()
        print(f"M{M} N{N} K{K}: w4b rel err {err:.2e}", flush=True)
        if M < 4096:
            continue
        c2 = torch.empty_like(c)
        f = 2 * M * N * K
        tw, t8, tt = [], [], []
        for _ in range(3):
            tw.append(timeit(lambda: L.dllm_gemm_w4b(a.data_ptr(), K, b.data_ptr(), K, c.data_ptr(), N, M, N, K, gm, st)))
            t8.append(timeit(lambda: gemm(a, b, "nt", out=c2)))
            tt.append(timeit(lambda: torch.matmul(a, b.t())))
        print(f"   w4b {f / statistics.median(tw) / 1e9:6.0f} TF  8ph {f / statistics.median(t8) / 1e9:6.0f} TF  "
              f"torch {f / statistics.median(tt) / 1e9:6.0f} TF", flush=True)


if __name__ == "__main__":
    main(build_only="--build" in sys.argv)
