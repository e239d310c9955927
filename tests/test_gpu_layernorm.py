"""GPU parity of the fused LayerNorm kernels (csrc/layernorm.hip) against a plain PyTorch fp64
restatement of the reference's chain  LN(dropout(proj) + identity)  (geometric_attention.py:586-596,
temporal_attention.py:1190-1200) and the skip branch  y + LN_s(x)  (model.py:258-262).

Ragged row counts (not a multiple of the rows one wave handles) pin the dead-row handling of the
multi-row-group waves; every supported width H is covered.  Dropout cannot match torch's RNG, so
with p > 0 the kept mask is read back from the saved LN input and the backward is checked to use
the same mask (dropped entries get zero gradient, kept ones the 1/(1-p) scale)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

ATOL, RTOL = 2e-5, 1e-4
HS = (32, 64, 128, 256, 512)
MS = (1, 3, 7, 130, 1001)


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import tagan_amd  # noqa: F401
    return torch.device("cuda:0")


def _inputs(dev, M, H, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed * 7919 + M * 31 + H)
    t = lambda *s: torch.randn(*s, generator=g).to(dev)  # noqa: E731
    return t(M, H), t(M, H), t(H), 1.0 + 0.1 * t(H), t(H), t(M, H), t(M, H)


def _ref_ln(x, w, b, eps):
    x = x.double()
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return (x - mu) / torch.sqrt(var + eps) * w.double() + b.double()


@pytest.mark.parametrize("H", HS)
@pytest.mark.parametrize("M", MS)
def test_add_layernorm_fwd_bwd(dev, M, H):
    from tagan_amd.fused import ln_bwd, ln_fwd
    a, b, a_bias, gamma, beta, dy, dres = _inputs(dev, M, H)
    y, s, mean, rstd = ln_fwd(a, b, 0.0, 0, gamma, beta, 1e-5, True, a_bias=a_bias)
    # fp64 autograd reference
    ad, bd = (a + a_bias).double().requires_grad_(), b.double().requires_grad_()
    gd, btd = gamma.double().requires_grad_(), beta.double().requires_grad_()
    yr = _ref_ln(ad + bd, gd, btd, 1e-5)
    torch.testing.assert_close(y.double(), yr.detach(), atol=ATOL, rtol=RTOL)
    torch.testing.assert_close(s.double(), (ad + bd).detach(), atol=2e-6, rtol=1e-6)
    (yr * dy.double()).sum().backward()
    ds, da, dg, dbt, dsa = ln_bwd(s, mean, rstd, gamma, dy, dres, 0.0, 0, True, True, True)
    torch.testing.assert_close(da.double(), ad.grad, atol=ATOL, rtol=RTOL)
    torch.testing.assert_close(ds.double(), bd.grad + dres.double(), atol=ATOL, rtol=RTOL)
    tol = dict(atol=ATOL * max(1, M) ** 0.5, rtol=RTOL)
    torch.testing.assert_close(dg.double(), gd.grad, **tol)
    torch.testing.assert_close(dbt.double(), btd.grad, **tol)
    torch.testing.assert_close(dsa.double(), ad.grad.sum(0), **tol)


@pytest.mark.parametrize("H", HS)
@pytest.mark.parametrize("M", (3, 1001))
def test_skip_layernorm_fwd(dev, M, H):
    from tagan_amd.fused import ln_skip_fwd
    a, b, a_bias, gamma, beta, _, _ = _inputs(dev, M, H, seed=1)
    gs, bs = 1.0 - 0.05 * gamma, 0.5 * beta
    y, s, mean, rstd, (mean_s, rstd_s) = ln_skip_fwd(a, b, 0.0, 0, gamma, beta, 1e-5, gs, bs, 1e-6, a_bias=a_bias)
    ref = _ref_ln(a + a_bias + b, gamma, beta, 1e-5) + _ref_ln(b, gs, bs, 1e-6)
    torch.testing.assert_close(y.double(), ref, atol=2 * ATOL, rtol=RTOL)
    torch.testing.assert_close(mean_s.double(), b.double().mean(-1), atol=1e-6, rtol=1e-5)


@pytest.mark.parametrize("M", (7, 1001))
def test_layernorm_dropout_mask_shared(dev, M):
    from tagan_amd.fused import ln_bwd, ln_fwd
    H, p, seed = 128, 0.25, 12345
    a, _, _, gamma, beta, dy, _ = _inputs(dev, M, H, seed=2)
    b = torch.zeros_like(a)                                  # s = dropout(a) exactly
    y, s, mean, rstd = ln_fwd(a, b, p, seed, gamma, beta, 1e-5, True)
    drop = s == 0                                            # a is N(0,1): exact zeros are dropped entries
    torch.testing.assert_close(s[~drop], a[~drop] / (1 - p), atol=1e-6, rtol=1e-6)
    frac = drop.double().mean().item()
    assert abs(frac - p) < 0.05 + 3 / (M * H) ** 0.5
    y2, s2, _, _ = ln_fwd(a, b, p, seed, gamma, beta, 1e-5, True)
    assert torch.equal(y, y2) and torch.equal(s, s2)         # deterministic in the seed
    ds, da, _, _, _ = ln_bwd(s, mean, rstd, gamma, dy, None, p, seed, True, True, False)
    assert torch.all(da[drop] == 0)
    torch.testing.assert_close(da[~drop], ds[~drop] / (1 - p), atol=1e-6, rtol=1e-5)


@pytest.mark.parametrize("H", [128, 256])
@pytest.mark.parametrize("M", MS + (320000,))
@pytest.mark.parametrize("da_bf16", [False, True])
def test_skip_bwd_fused_equals_two_passes(dev, M, da_bf16, H):
    """tagan_layernorm_skip_bwd (the skip block's LN2 + LN_s backward in one pass) against the two-pass chain it
    replaces (LN2's backward, then LN_s's with that ds as dres), with dropout: the same dropout decisions (da zero
    exactly where the chain's is) and the same values to fp32 rounding -- the compiler contracts the fused pass's
    multiply-adds differently (observed 1 ulp), so the bound is 4 ulp of the tensor's scale, not bit equality."""
    from tagan_amd.fused import ln_bwd, ln_skip_bwd, ln_skip_fwd
    a, b, ab, g2, b2, _, dy = _inputs(dev, M, H, seed=11)
    gs, bs = 1.0 + 0.1 * torch.randn(H, device=dev), 0.1 * torch.randn(H, device=dev)
    y, s, mean, rstd, (ms, rss) = ln_skip_fwd(a, b, 0.1, 99, g2, b2, 1e-5, gs, bs, 1e-5, a_bias=ab)
    dt = torch.bfloat16 if da_bf16 else torch.float32
    ds1, da1, dg1, db1, dsa1 = ln_bwd(s, mean, rstd, g2, dy, None, 0.1, 99, True, True, True, da_dtype=dt)
    ds1, _, dgs1, dbs1, _ = ln_bwd(b, ms, rss, gs, dy, ds1, 0.0, 0, True, False, False)
    ds2, da2, dg2, db2, dsa2, dgs2, dbs2 = ln_skip_bwd(s, mean, rstd, g2, b, ms, rss, gs, dy, 0.1, 99, da_dtype=dt)
    for n, x1, x2 in (("ds", ds1, ds2), ("da", da1, da2), ("dgamma", dg1, dg2), ("dbeta", db1, db2),
                      ("dsum_a", dsa1, dsa2), ("dgamma_s", dgs1, dgs2), ("dbeta_s", dbs1, dbs2)):
        err = float((x1.double() - x2.double()).abs().max())
        scale = max(1.0, float(x1.double().abs().max()))
        if n in ("ds", "da"):   # elementwise: a few fp32 ulp (one bf16 ulp where da is stored in bf16)
            tol = (2.0 ** -7 if x1.dtype == torch.bfloat16 else 8 * 2.0 ** -23) * scale
        else:                   # column sums over M rows of those elements
            tol = 1e-5 * scale
        assert err <= tol, (n, err, tol)
    assert torch.equal(da1 == 0, da2 == 0)
