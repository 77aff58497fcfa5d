"""Deferred fused split-master SGD (csrc/gemm_kernels.h DEFER): a persistent block parks each finished tile's
accumulators and applies the update under its next tile's main loop.  It must leave bitwise what the plain EPI_SGDS
epilogue leaves, whatever the number of tiles per block, and run to run."""
import pytest
import torch

from dllm.ops.gemm import gemm, set_defer_sgd, set_tiles_per_block
from dllm.ops.master import join_master, split_master

pytestmark = pytest.mark.gpu


def _run(a, b, w, defer, tpb, lr=1e-2):
    old_d, old_t = set_defer_sgd(defer), set_tiles_per_block(tpb)
    try:
        hi, lo = split_master(w)
        gemm(a, b, "tn", out=lo, epi="sgd_split", lr=lr, aux_out=hi)
        torch.cuda.synchronize()
        return hi, lo
    finally:
        set_defer_sgd(old_d)
        set_tiles_per_block(old_t)


# persistent grids (> 256 tiles): 2, 3, 4 tiles per block; K from the 17-iteration minimum to the flagship's 8192
@pytest.mark.parametrize("M,N,K,tpb", [(4096, 8192, 4352, 8), (4096, 12288, 4352, 3), (6400, 10240, 2176, 64),
                                       (4096, 16384, 8192, 8)])
def test_deferred_sgd_bitwise_equals_epilogue(M, N, K, tpb):
    g = torch.Generator().manual_seed(M + N + K)
    a = torch.randn(K, M, generator=g).to(torch.bfloat16).cuda()
    b = torch.randn(K, N, generator=g).to(torch.bfloat16).cuda()
    w = (torch.randn(M, N, generator=g) * 0.02).cuda()
    h0, l0 = _run(a, b, w, False, tpb)
    for _ in range(3):   # bitwise run to run (race screen of the counted waits)
        h1, l1 = _run(a, b, w, True, tpb)
        assert torch.equal(h0.view(torch.int16), h1.view(torch.int16)) and torch.equal(l0, l1)
    # and it is the fp32-master update
    m32 = w.clone()
    gemm(a, b, "tn", out=m32, epi="sgd", lr=1e-2)
    assert torch.equal(join_master(h1, l1).view(torch.int32), m32.view(torch.int32))


def test_deferred_sgd_kernel_is_used():
    from torch.profiler import ProfilerActivity, profile

    M, N, K = 4096, 8192, 4352
    a = torch.randn(K, M, device="cuda").to(torch.bfloat16)
    b = torch.randn(K, N, device="cuda").to(torch.bfloat16)
    hi, lo = split_master(torch.randn(M, N, device="cuda") * 0.02)
    gemm(a, b, "tn", out=lo, epi="sgd_split", lr=1e-3, aux_out=hi)
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        gemm(a, b, "tn", out=lo, epi="sgd_split", lr=1e-3, aux_out=hi)
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if "gemm_bf16_8ph" in e.name]
    assert names and all("true, false, true>" in n for n in names), names
