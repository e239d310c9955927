"""GPU parity of the fused projection kernels (csrc/proj_gemm.hip) against plain PyTorch fp64 restatements
of the reference's per-layer chain  layer_norm1 -> q/k/v Linears  and  out Linear -> output_dropout ->
+ residual -> layer_norm2  (geometric_attention.py:541-596, temporal_attention.py:985-1200), their
backward (autograd of the same fp64 graph), and the skip branch  y + LN_s(x)  (model.py:258-262).

Row counts that are not a multiple of the 128 rows of a workgroup (and fewer than one wave's 32) pin the
dead-row handling.  Dropout cannot match torch's RNG: with p > 0 the kept mask is read back from the
saved LN input s (s - x = dropped-or-scaled projection), and checked to be the mask of the standalone
LayerNorm kernel (same counter hash: stream = row, counter = column)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

H = 128
MS = (1, 31, 333, 1000, 4099)
ATOL, RTOL = 1e-4, 1e-4


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import tagan_amd  # noqa: F401
    return torch.device("cuda:0")


def _t(g, dev, *s, scale=1.0):
    return (scale * torch.randn(*s, generator=g, dtype=torch.float64)).to(dev)


def _ln(x, w, b, eps=1e-5):
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return (x - mu) / torch.sqrt(var + eps) * w + b


def _close(got, want, atol=ATOL, rtol=RTOL, msg=""):
    torch.testing.assert_close(got.double(), want.double(), atol=atol, rtol=rtol, msg=msg)


@pytest.mark.parametrize("M", MS)
def test_ln_qkv_fwd(dev, M):
    from tagan_amd.fused import proj_ln_qkv
    g = torch.Generator().manual_seed(M)
    x = _t(g, dev, M, H, scale=3.0) + 0.5
    lw, lb = 1.0 + 0.1 * _t(g, dev, H), 0.1 * _t(g, dev, H)
    w, b = _t(g, dev, 3 * H, H, scale=H ** -0.5), 0.1 * _t(g, dev, 3 * H)
    qkv, h_aug, mean, rstd = proj_ln_qkv(x.float(), lw.float(), lb.float(), 1e-5, w.float(), b.float(), True)
    h = _ln(x, lw, lb)
    _close(h_aug[:, :H], h, msg="h")
    _close(h_aug[:, H:], torch.tensor([1.0, 0, 0, 0], device=dev).expand(M, 4), atol=0, rtol=0, msg="ones")
    _close(qkv, h @ w.t() + b, msg="qkv")
    _close(mean, x.mean(-1), msg="mean")
    _close(rstd, 1 / torch.sqrt(x.var(-1, unbiased=False) + 1e-5), msg="rstd")
    qkv2, none, _, _ = proj_ln_qkv(x.float(), lw.float(), lb.float(), 1e-5, w.float(), b.float(), False)
    assert none is None and torch.equal(qkv, qkv2)


@pytest.mark.parametrize("skip", [False, True])
@pytest.mark.parametrize("M", MS)
def test_proj_ln_fwd(dev, M, skip):
    from tagan_amd.fused import proj_ln_out
    g = torch.Generator().manual_seed(100 + M)
    c, x = _t(g, dev, M, H), _t(g, dev, M, H, scale=2.0)
    w, b = _t(g, dev, H, H, scale=H ** -0.5), 0.1 * _t(g, dev, H)
    lw, lb = 1.0 + 0.1 * _t(g, dev, H), 0.1 * _t(g, dev, H)
    sw, sb = (1.0 + 0.1 * _t(g, dev, H), 0.1 * _t(g, dev, H)) if skip else (None, None)
    f = lambda t: None if t is None else t.float()  # noqa: E731
    y, s, mean, rstd, st = proj_ln_out(c.float(), w.float(), b.float(), x.float(), 0.0, 0, lw.float(), lb.float(),
                                       1e-5, f(sw), f(sb), 1e-5)
    sref = c @ w.t() + b + x
    yref = _ln(sref, lw, lb) + (_ln(x, sw, sb) if skip else 0)
    _close(s, sref, msg="s")
    _close(y, yref, msg="y")
    _close(mean, sref.mean(-1), msg="mean")
    if skip:
        _close(st[0], x.mean(-1), msg="mean_s")
        _close(st[1], 1 / torch.sqrt(x.var(-1, unbiased=False) + 1e-5), msg="rstd_s")


def test_proj_ln_fwd_dropout_matches_ln_kernel(dev):
    """The fused epilogue draws the standalone LayerNorm kernel's mask (stream = row, counter = column)."""
    from tagan_amd.fused import ln_fwd, proj_ln_out
    M, p, seed = 1000, 0.3, 12345
    g = torch.Generator().manual_seed(7)
    c, x = _t(g, dev, M, H).float(), _t(g, dev, M, H).float()
    w, b = _t(g, dev, H, H, scale=H ** -0.5).float(), 0.1 * _t(g, dev, H).float()
    lw, lb = torch.ones(H, device=dev), torch.zeros(H, device=dev)
    y, s, mean, rstd, _ = proj_ln_out(c, w, b, x, p, seed, lw, lb, 1e-5)
    o = (c.double() @ w.double().t() + b.double()).float()
    y2, s2, _, _ = ln_fwd(o, x, p, seed, lw, lb, 1e-5, True)
    kept = (s - x).abs() > 0
    kept2 = (s2 - x).abs() > 0
    assert torch.equal(kept, kept2)
    frac = kept.float().mean().item()
    assert abs(frac - (1 - p)) < 0.01
    _close(s, s2, msg="s")
    _close(y, y2, msg="y")


@pytest.mark.parametrize("K", [H, 3 * H])
@pytest.mark.parametrize("kmajor", [True, False])
@pytest.mark.parametrize("M", (31, 1000))
def test_proj_gemm(dev, M, K, kmajor):
    from tagan_amd.fused import proj_mm
    g = torch.Generator().manual_seed(K + M)
    a = _t(g, dev, M, K)
    w = _t(g, dev, K, H, scale=K ** -0.5) if kmajor else _t(g, dev, H, K, scale=K ** -0.5)
    out = proj_mm(a.float(), w.float(), kmajor)
    _close(out, a @ (w if kmajor else w.t()), msg="gemm")


@pytest.mark.parametrize("K", [H, 3 * H])
@pytest.mark.parametrize("M", MS)
def test_proj_ln_bwd(dev, M, K):
    """dx, dgamma, dbeta of  LN(x) -> Linear(K_out = K)  against fp64 autograd (da = d(Linear output))."""
    from tagan_amd.fused import proj_ln_bwd
    g = torch.Generator().manual_seed(300 + M + K)
    x = (_t(g, dev, M, H, scale=2.0) + 0.3).requires_grad_()
    lw = (1.0 + 0.1 * _t(g, dev, H)).requires_grad_()
    lb = (0.1 * _t(g, dev, H)).requires_grad_()
    w = _t(g, dev, K, H, scale=H ** -0.5)
    da, dres = _t(g, dev, M, K), _t(g, dev, M, H)
    h = _ln(x, lw, lb)
    (h @ w.t()).backward(da)
    mean = x.detach().mean(-1).float()
    rstd = (1 / torch.sqrt(x.detach().var(-1, unbiased=False) + 1e-5)).float()
    dx, dg, db = proj_ln_bwd(da.float(), w.float(), x.detach().float(), mean, rstd, lw.detach().float(), dres.float())
    _close(dx, x.grad + dres, msg="dx")
    tol = dict(atol=ATOL * max(1, M) ** 0.5, rtol=RTOL)
    _close(dg, lw.grad, msg="dgamma", **tol)
    _close(db, lb.grad, msg="dbeta", **tol)
    dx2, _, _ = proj_ln_bwd(da.float(), w.float(), x.detach().float(), mean, rstd, lw.detach().float(), dres.float())
    assert torch.equal(dx, dx2)


@pytest.mark.parametrize("subset", ["all", "out,dc", "qkv,dh"])
def test_block_fused_vs_unfused(dev, subset):
    """One geometric attention block through AttnBlockFn with the fused kernels (a TAGAN_PROJ subset) against the
    TAGAN_PROJ=0 path (hipBLASLt + separate LayerNorm kernels), forward and every gradient, fp32, dropout on."""
    import tagan_amd.fused as fu
    from tagan_amd import TAGANConfig  # noqa: F401
    from tagan_amd.kernels import build_graph
    from tagan_amd.layers.graph_attention import TAGANGraphAttention
    torch.manual_seed(3)
    layer = TAGANGraphAttention(hidden_dim=H, num_heads=8, dropout=0.1).to(dev).train()
    N, E = 3000, 20000
    gen = torch.Generator().manual_seed(11)
    x = torch.randn(N, H, generator=gen).to(dev).requires_grad_()
    ei = torch.randint(0, N, (2, E), generator=gen).to(dev)
    graph = build_graph([ei], [N])
    dy = torch.randn(N, H, generator=gen).to(dev)
    res = {}
    saved = (fu.PROJ, fu.PROJ_SET)
    for proj in (True, False):
        fu.PROJ_SET = ({"qkv", "out", "dc", "dh"} if subset == "all" else set(subset.split(","))) if proj else set()
        fu.PROJ = bool(fu.PROJ_SET)
        try:
            torch.manual_seed(99)
            y = layer.forward_graph(x, graph)
            layer.zero_grad()
            x.grad = None
            y.backward(dy)
            res[proj] = (y.detach().clone(), x.grad.clone(),
                         {k: p.grad.clone() for k, p in layer.named_parameters() if p.grad is not None})
        finally:
            fu.PROJ, fu.PROJ_SET = saved
    y1, dx1, g1 = res[True]
    y0, dx0, g0 = res[False]
    _close(y1, y0, msg="y")
    _close(dx1, dx0, msg="dx")
    assert g1.keys() == g0.keys()
    for k in g1:
        _close(g1[k], g0[k], atol=1e-4 * max(1.0, g0[k].abs().max().item()), msg=k)
