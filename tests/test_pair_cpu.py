"""``layer_bwd(..., pair_wgrads=True)`` (the grouped weight-gradient schedule: da, dx, dW2 | dW1) on CPU: the same
gradients as the default schedule, dx computed before W1's update, and the hooks fired in the flat layout's
completion order (layer 0 without dx: W1 first)."""
import torch

from dllm.models.ffn import layer_bwd


def _layer(seed, T=64, D=32, F=48):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(T, D, generator=g, dtype=torch.float64)
    w1 = torch.randn(F, D, generator=g, dtype=torch.float64) * 0.1
    w2 = torch.randn(D, F, generator=g, dtype=torch.float64) * 0.1
    dy = torch.randn(T, D, generator=g, dtype=torch.float64)
    h = x @ w1.t()
    a = torch.relu(h)
    return x, w1, w2, dy, a, h


class _Rec:
    def __init__(self):
        self.ev = []

    def after_w2(self):
        self.ev.append("w2")

    def after_w1(self):
        self.ev.append("w1")

    def after_dx(self, dx):
        self.ev.append("dx")


def test_pair_schedule_same_grads_and_hook_order():
    for need_dx in (True, False):
        outs = []
        for pair in (False, True):
            x, w1, w2, dy, a, h = _layer(1)
            gw1, gw2 = torch.empty_like(w1), torch.empty_like(w2)
            da = torch.empty_like(h)
            dxo = torch.empty_like(x) if need_dx else None
            rec = _Rec()
            dx = layer_bwd(dy, x, w1, w2, "relu", False, a, h, gw1, gw2, da, dxo, rec, pair_wgrads=pair)
            outs.append((gw1, gw2, dx, rec.ev))
        (g1a, g2a, dxa, eva), (g1b, g2b, dxb, evb) = outs
        assert torch.equal(g1a, g1b) and torch.equal(g2a, g2b)
        if need_dx:
            assert torch.equal(dxa, dxb)
            assert evb == ["dx", "w2", "w1"]
        else:
            assert dxb is None and evb == ["w1", "w2"] == eva


def test_pair_schedule_fused_sgd_reads_old_w1_for_dx():
    """With fused updates the pair runs after dx, so dx uses the pre-update W1 (as the default schedule does)."""
    x, w1, w2, dy, a, h = (t.float() for t in _layer(2))
    ref = layer_bwd(dy, x, w1.clone(), w2.clone(), "relu", False, a, h, torch.empty_like(w1), torch.empty_like(w2),
                    torch.empty_like(h), torch.empty_like(x))
    w1f, w2f = w1.clone(), w2.clone()
    dx = layer_bwd(dy, x, w1f, w2f, "relu", False, a, h, {"out": w1f, "epi": "sgd", "lr": 0.1},
                   {"out": w2f, "epi": "sgd", "lr": 0.1}, torch.empty_like(h), torch.empty_like(x), pair_wgrads=True)
    assert torch.allclose(dx, ref, rtol=0, atol=1e-6)
    assert not torch.equal(w1f, w1)


def test_transposed_activation_layer_matches_reference_layer():
    """layer_fwd_t / layer_bwd_t (activations [F, T], W2 stored as W2ᵀ) compute the reference layer's y, dx, dW1, dW2
    (train_ffns.py:54-70) -- checked in fp64 on CPU against layer_fwd / layer_bwd."""
    from dllm.models.ffn import layer_bwd_t, layer_fwd, layer_fwd_t

    x, w1, w2, dy, a, h = _layer(3)
    T, F = a.shape
    D = x.shape[1]
    y = torch.empty(T, D, dtype=torch.float64)
    layer_fwd(x, w1, w2, "relu", False, torch.empty(T, F, dtype=torch.float64), None, y)
    yt = torch.empty_like(y)
    aT = torch.empty(F, T, dtype=torch.float64)
    layer_fwd_t(x, w1, w2.t().contiguous(), "relu", aT, None, yt)
    assert torch.allclose(yt, y, rtol=1e-12, atol=1e-12) and torch.allclose(aT.t(), a)
    gw1, gw2 = torch.empty_like(w1), torch.empty_like(w2)
    dx = layer_bwd(dy, x, w1, w2, "relu", False, a, None, gw1, gw2, torch.empty_like(h), torch.empty_like(x))
    gw1t, gw2t = torch.empty_like(w1), torch.empty(F, D, dtype=torch.float64)
    rec = _Rec()
    dxt = layer_bwd_t(dy, x, w1, w2.t().contiguous(), "relu", aT, None, gw1t, gw2t, torch.empty(F, T, dtype=torch.float64),
                      torch.empty_like(x), rec)
    assert torch.allclose(dxt, dx, rtol=1e-12, atol=1e-12)
    assert torch.allclose(gw1t, gw1, rtol=1e-12, atol=1e-12) and torch.allclose(gw2t.t(), gw2, rtol=1e-12, atol=1e-12)
    assert rec.ev == ["dx", "w2", "w1"]
