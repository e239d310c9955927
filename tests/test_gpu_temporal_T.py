"""GPU parity of the temporal attention layer over the whole sequence-length range: the one-wave matrix-core
kernels (v4, T <= 32), the workgroup-per-unit matrix-core kernels (v5, 32 < T <= 128 with head_dim 16/32: C3's
T = 64, C5's T = 128) and the VALU v3 kernels (other head widths).
The layer (AsymmetricTemporalAttention, temporal_attention.py:624-1217) against the fp64 oracle
(oracle/tagan_oracle.py temporal_attention), forward and every gradient; tolerance 1e-4 fp32."""
import pytest
import torch

import golden_io as G
import oracle

pytestmark = pytest.mark.gpu

OUT_ATOL, OUT_RTOL = 1e-4, 1e-4
GRAD_ATOL, GRAD_RTOL = 1e-4, 1e-4    # north_star: 1e-4 fp32 (observed errors: profiles/parity_errors_r02.json)


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import tagan_amd  # noqa: F401
    return torch.device("cuda:0")


def _layer(H, heads, causal, dev, seed):
    from tagan_amd.layers import AsymmetricTemporalAttention
    torch.manual_seed(seed)
    mod = AsymmetricTemporalAttention(H, heads, dropout=0.0, causal=causal).to(dev).train()
    with torch.no_grad():   # non-trivial LayerNorm affine parameters
        for n, p in mod.named_parameters():
            if "layer_norm" in n:
                p.add_(0.1 * torch.randn_like(p))
    return mod


@pytest.mark.parametrize("T,H,heads,causal", [
    (1, 64, 4, False), (10, 64, 4, False), (16, 128, 4, False), (20, 64, 4, True), (32, 128, 8, False),
    (32, 128, 4, True),                                  # matrix-core (v4) range: T <= 32, d in {16, 32}
    (8, 64, 4, False), (33, 128, 8, False), (64, 128, 8, True), (65, 256, 16, False),
    (100, 128, 8, False), (128, 256, 16, False), (128, 128, 4, True),
    (48, 256, 8, False), (64, 256, 8, True),            # d = 32 in the 4-wave v5 range (C3: T = 64)
])
def test_temporal_layer_T_sweep(dev, T, H, heads, causal):
    mod = _layer(H, heads, causal, dev, seed=T)
    g = torch.Generator().manual_seed(T)
    B = 20
    x = torch.randn(B, T, H, generator=g)
    gy = torch.randn(B, T, H, generator=g)
    xd = x.to(dev).requires_grad_(True)
    out = mod(xd)
    (out * gy.to(dev)).sum().backward()
    P = {"m." + k: v.detach().cpu().double().requires_grad_(v.is_floating_point())
         for k, v in mod.state_dict().items()}
    x64 = x.double().requires_grad_(True)
    ref = oracle.temporal_attention(x64, P, "m", heads, cls="asym", causal=causal)
    G.assert_close("out", out, ref, OUT_ATOL, OUT_RTOL)
    (ref * gy.double()).sum().backward()
    G.assert_close("grad x", xd.grad, x64.grad, GRAD_ATOL, GRAD_RTOL)
    for n, p in mod.named_parameters():
        if P["m." + n].grad is not None:
            G.assert_close("grad " + n, p.grad, P["m." + n].grad, GRAD_ATOL, GRAD_RTOL)


def test_temporal_layer_T128_bf16(dev):
    """bf16 activation storage at T = 128 (the C5 shape) against the fp32 path of the same layer;
    tolerance 2e-2 relative on outputs, 8e-2 on gradients with a floor of 1 % of the largest gradient
    norm (k_linear.bias has an analytically zero gradient: softmax is shift-invariant per query)."""
    from tagan_amd.fused import precision
    T, H, heads = 128, 256, 16
    mod = _layer(H, heads, False, dev, seed=5)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(12, T, H, generator=g).to(dev)
    gy = torch.randn(12, T, H, generator=g).to(dev)
    res = {}
    for mode in ("fp32", "bf16"):
        mod.zero_grad(set_to_none=True)
        xi = x.clone().requires_grad_(True)
        with precision(mode):
            out = mod(xi)
            (out.float() * gy).sum().backward()
        res[mode] = (out.float().detach(), xi.grad.detach(), {n: p.grad.detach().clone()
                                                              for n, p in mod.named_parameters()
                                                              if p.grad is not None})
    def rel(a, b):
        return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))
    assert rel(res["bf16"][0], res["fp32"][0]) < 2e-2
    assert rel(res["bf16"][1], res["fp32"][1]) < 2e-2
    top = max(float(gr.norm()) for gr in res["fp32"][2].values())
    for n, gr in res["fp32"][2].items():
        gb = res["bf16"][2][n]
        assert float((gb - gr).norm()) <= 8e-2 * max(float(gr.norm()), 1e-2 * top), n
