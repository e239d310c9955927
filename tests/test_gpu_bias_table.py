"""GPU parity of the temporal bias-table kernels (csrc/params.hip; temporal_attention.py:732-790): the forward
against the layer's one-hot gather GEMMs (the CPU path of AsymmetricTemporalAttention._bias_table), bitwise; the
table gradients against fp64 sums over the clamped diagonals."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import tagan_amd  # noqa: F401
    return torch.device("cuda:0")


def _ref(K, R, T, W, m):
    delta = torch.arange(-(T - 1), T)
    a = torch.nn.functional.one_hot(torch.clamp(delta + W, 0, 2 * W), 2 * W + 1).double()
    a = a * ((delta >= -W) & (delta <= W)).unsqueeze(-1).double()
    tab = a @ K.double()
    if R is not None:
        r = torch.nn.functional.one_hot(torch.clamp(delta + m, 0, 2 * m), 2 * m + 1).double()
        tab = r @ R.double() + tab
    return tab.t()


@pytest.mark.parametrize("T,heads,W,m,rel", [(2, 4, 5, 32, True), (10, 4, 5, 32, True), (32, 8, 5, 32, True),
                                             (128, 16, 5, 32, True), (64, 8, 3, 8, False), (1, 2, 5, 32, True)])
def test_bias_table(dev, T, heads, W, m, rel):
    from tagan_amd.kernels import BiasTableFn
    g = torch.Generator().manual_seed(T * 131 + heads)
    K = torch.randn(2 * W + 1, heads, generator=g)
    R = torch.randn(2 * m + 1, heads, generator=g) if rel else None
    Kd = K.to(dev).requires_grad_(True)
    Rd = R.to(dev).requires_grad_(True) if rel else None
    tab = BiasTableFn.apply(Kd, Rd, T, W, m)
    ref = _ref(K, R, T, W, m)
    # the forward is the same fp32 add of two gathered entries as the gather-GEMM form: bitwise
    assert torch.equal(tab.cpu(), ref.float())
    gout = torch.randn(heads, 2 * T - 1, generator=g)
    tab.backward(gout.to(dev))
    Kr = K.double().requires_grad_(True)
    Rr = R.double().requires_grad_(True) if rel else None
    _ref(Kr, Rr, T, W, m).backward(gout.double().t().t())
    torch.testing.assert_close(Kd.grad.cpu().double(), Kr.grad, rtol=1e-6, atol=1e-6)
    if rel:
        torch.testing.assert_close(Rd.grad.cpu().double(), Rr.grad, rtol=1e-5, atol=1e-5)
