"""dllm.api primitives and trainers on the GPU: the HIP kernels behind the reference-compatible names,
against fp32 torch formulas of the reference (train_ffns.py:41-70)."""
import pytest
import torch

from dllm import api
from dllm.models import reference as R

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype,T,D", [(torch.float32, 256, 128), (torch.bfloat16, 512, 256), (torch.float32, 40, 24)])
def test_layer_bkwd_matches_reference_formulas(dtype, T, D):
    F = 4 * D
    g = torch.Generator()
    g.manual_seed(1)
    w1, w2 = (p.cuda().to(dtype) for p in api.init_tlayer_ffn(D, F, g))
    x = torch.randn(T, D, generator=g).cuda().to(dtype)
    dy = (0.1 * torch.randn(T, D, generator=g)).cuda().to(dtype)
    dx, (dw1, dw2) = api.tlayer_ffn_bkwd(dy, [w1, w2], x)
    xf, dyf, w1f, w2f = x.float(), dy.float(), w1.float(), w2.float()
    h = xf @ w1f.t()
    a = torch.where(h <= 0, 0, h)
    if dtype == torch.bfloat16:
        a = a.bfloat16().float()
    da = (dyf @ w2f).masked_fill(h <= 0, 0)
    if dtype == torch.bfloat16:
        da = da.bfloat16().float()
    tol = dict(rtol=2e-2, atol=2e-3) if dtype == torch.bfloat16 else dict(rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(dw2.float(), dyf.t() @ a, **tol)
    torch.testing.assert_close(dw1.float(), da.t() @ xf, **tol)
    torch.testing.assert_close(dx.float(), da @ w1f, **tol)
    y = api.tlayer_ffn_fwd([w1, w2], x)
    torch.testing.assert_close(y.float(), a @ w2f.t(), **tol)


def test_train_1gpu_matches_oracle():
    D, F, T, L = 128, 512, 256, 2
    g = torch.Generator()
    g.manual_seed(4)
    layers = [api.init_tlayer_ffn(D, F, g) for _ in range(L)]
    seeds = torch.tensor([1, 2, 3])
    out = api.train_1gpu(layers, seeds, T, D, lr=1e-2)
    assert out[0][0].is_cuda
    ref = R.train_single([{"w1": a.clone(), "w2": b.clone()} for a, b in layers],
                         list(api.mock_data(seeds, T, D)), 1e-2)
    for l in range(L):
        torch.testing.assert_close(out[l][0].cpu(), ref[l]["w1"], rtol=1e-4, atol=1e-6)
        torch.testing.assert_close(out[l][1].cpu(), ref[l]["w2"], rtol=1e-4, atol=1e-6)
