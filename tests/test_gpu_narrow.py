"""GPU parity of the narrow-input projection (csrc/narrow.hip, the node embedding of model.py:233) against a
plain PyTorch fp64 restatement y = x·Wᵀ + b, dW = dyᵀ·x, db = Σ dy.

The kernels are exact-f32 MFMA chains (one rounding per product, k-ordered), so the bound is the fp32 summation
bound: |err| <= c · u · Σ|terms| with u = 2⁻²⁴ and c the chain length (K for y, the rows for dW / db, plus the
ordered partial folds).  Ragged row counts pin the dead-row handling (the 16-row forward tiles, the 4-row backward
groups, the per-workgroup row ranges); a column view of a wider buffer pins the row stride; two runs must be
bitwise equal (fixed-order partials)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

U = 2.0 ** -24


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import tagan_amd  # noqa: F401
    return torch.device("cuda:0")


def _run(dev, M, K, N, ldx=None, bias=True, seed=0):
    from tagan_amd.kernels import NarrowLinearFn
    g = torch.Generator(device="cpu").manual_seed(seed * 1009 + M * 7 + K * 3 + N)
    ldx = ldx or K
    xb = torch.randn(M, ldx, generator=g).to(dev)
    x = xb[:, :K]
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(dev).requires_grad_(True)
    b = torch.randn(N, generator=g).to(dev).requires_grad_(True) if bias else None
    dy = torch.randn(M, N, generator=g).to(dev)
    y = NarrowLinearFn.apply(x, w, b)
    y.backward(dy)
    return x, w, b, dy, y.detach(), w.grad.detach().clone(), (b.grad.detach().clone() if bias else None)


def _check(got, ref, absterm, chain, what):
    bound = (chain + 2) * U * absterm + 1e-30
    err = (got.double() - ref).abs()
    worst = (err / bound).max().item()
    assert worst <= 1.0, f"{what}: worst error / bound = {worst:.3g}"


@pytest.mark.parametrize("M,K,N", [(1, 27, 128), (15, 27, 128), (17, 27, 128), (1001, 27, 128), (4099, 16, 64),
                                   (2050, 27, 256), (333, 5, 64), (129, 31, 64), (320000, 27, 128)])
def test_narrow_linear_vs_fp64(dev, M, K, N):
    x, w, b, dy, y, dw, db = _run(dev, M, K, N)
    xd, wd, bd, dyd = x.double(), w.detach().double(), b.detach().double(), dy.double()
    _check(y, xd @ wd.t() + bd, (xd.abs() @ wd.abs().t()) + bd.abs(), K, "y")
    _check(dw, dyd.t() @ xd, dyd.abs().t() @ xd.abs(), M, "dW")
    _check(db, dyd.sum(0), dyd.abs().sum(0), M, "db")


def test_narrow_linear_strided_no_bias(dev):
    x, w, b, dy, y, dw, _ = _run(dev, 777, 27, 128, ldx=40, bias=False)
    xd, wd, dyd = x.double(), w.detach().double(), dy.double()
    _check(y, xd @ wd.t(), xd.abs() @ wd.abs().t(), 27, "y (row stride 40, no bias)")
    _check(dw, dyd.t() @ xd, dyd.abs().t() @ xd.abs(), 777, "dW (row stride 40)")


def test_narrow_linear_reproducible(dev):
    a = _run(dev, 50001, 27, 128, seed=3)
    c = _run(dev, 50001, 27, 128, seed=3)
    for u, v, name in zip(a[4:], c[4:], ("y", "dW", "db")):
        assert torch.equal(u, v), f"{name} differs between two identical runs"


def test_embedding_falls_back_off_the_supported_widths(dev):
    from tagan_amd import kernels
    x = torch.randn(100, 27, device=dev)
    w = torch.randn(32, 27, device=dev, requires_grad=True)
    y = kernels.embed_linear(x, w, None)
    assert not type(y.grad_fn).__name__.startswith("NarrowLinearFn")
    torch.testing.assert_close(y, x @ w.t(), rtol=1e-5, atol=1e-5)


def test_embedding_uses_narrow_kernel(dev):
    from tagan_amd import kernels
    x = torch.randn(100, 27, device=dev)
    w = torch.randn(128, 27, device=dev, requires_grad=True)
    y = kernels.embed_linear(x, w, None)
    assert y.grad_fn is not None and type(y.grad_fn).__name__.startswith("NarrowLinearFn")
