"""Prototype check: 4-wave 128x128-per-wave NT GEMM (csrc/gemm_w4.hip) vs the 8-phase kernel vs
hipBLASLt on the forward FFN shapes, random bf16, numerics against torch."""
import ctypes
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dllm  # noqa: E402,F401
from dllm import _native  # noqa: E402
from dllm.ops.gemm import gemm  # noqa: E402

c_long, c_int, c_void_p = ctypes.c_long, ctypes.c_int, ctypes.c_void_p
_native.register_optional("dllm_gemm_w4_proto", c_int,
                          [c_void_p, c_long, c_void_p, c_long, c_void_p, c_long, c_int, c_int, c_int, c_int, c_void_p])


def w4(a, b, out, group_m=4):
    M, K = a.shape
    N = b.shape[0]
    rc = _native.lib().dllm_gemm_w4_proto(a.data_ptr(), K, b.data_ptr(), K, out.data_ptr(), N, M, N, K, group_m,
                                           torch.cuda.current_stream().cuda_stream)
    assert rc == 0, rc
    return out


def timeit(fn, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    bf = torch.bfloat16
    for (M, N, K) in [(512, 512, 256), (8192, 16384, 4096), (8192, 4096, 16384), (8192, 8192, 8192)]:
        a = torch.randn(M, K, device="cuda", dtype=bf)
        b = torch.randn(N, K, device="cuda", dtype=bf)
        o1 = torch.empty(M, N, device="cuda", dtype=bf)
        o2 = torch.empty(M, N, device="cuda", dtype=bf)
        w4(a, b, o1)
        ref = (a.float() @ b.float().t())
        err = ((o1.float() - ref).norm() / ref.norm()).item()
        print(f"M{M} N{N} K{K}: w4 rel err {err:.2e}", flush=True)
        assert err < 1e-2, err
        if M < 4096:
            continue
        fl = 2 * M * N * K
        res = {"w4": [], "8ph": [], "torch": []}
        for _ in range(3):
            res["w4"].append(timeit(lambda: w4(a, b, o1)))
            res["8ph"].append(timeit(lambda: gemm(a, b, "nt", out=o2)))
            res["torch"].append(timeit(lambda: torch.matmul(a, b.t(), out=o2)))
        print("   " + "  ".join(f"{k} {fl / statistics.median(v) / 1e9:.0f} TF" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
