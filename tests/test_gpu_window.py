"""TemporalSkipConnection's window aggregation kernel (csrc/window.hip, WindowFn) against the reference's own
per-step formulation (temporal_propagation.py:868-925: slice the ±w window, stack, mean / max / sum) in fp32
torch, forward and gradient: every mode, windows wider than T, T = 1, ragged H, and ties under max (gradient to
the first maximum in window order, as torch.max over the stacked window)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import tagan_amd  # noqa: F401
    return torch.device("cuda:0")


def _ref(x, w, agg):
    T = x.shape[0]
    out = []
    for t in range(T):
        win = torch.stack([x[i] for i in range(max(0, t - w), min(T, t + w + 1))], 0)
        out.append(win.mean(0) if agg == "mean" else win.max(0)[0] if agg == "max" else win.sum(0))
    return torch.stack(out, 0)


@pytest.mark.parametrize("agg", ["mean", "max", "sum"])
@pytest.mark.parametrize("T,N,H,w", [(16, 300, 64, 3), (5, 17, 12, 8), (1, 9, 4, 2), (40, 1000, 128, 1),
                                     (7, 33, 10, 2)])    # H % 4 != 0: the device pooling form
def test_window_vs_reference_loop(dev, agg, T, N, H, w):
    from tagan_amd.layers.temporal_propagation import window_aggregate
    g = torch.Generator().manual_seed(T * 7 + w)
    x0 = torch.randn(T, N, H, generator=g).to(dev)
    dy = torch.randn(T, N, H, generator=g).to(dev)
    x1 = x0.clone().requires_grad_()
    y1 = window_aggregate(x1, w, agg)
    (y1 * dy).sum().backward()
    x2 = x0.clone().requires_grad_()
    y2 = _ref(x2, w, agg)
    (y2 * dy).sum().backward()
    torch.testing.assert_close(y1, y2, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(x1.grad, x2.grad, atol=1e-5, rtol=1e-5)


def test_window_max_ties_first_wins(dev):
    from tagan_amd.layers.temporal_propagation import window_aggregate
    x = torch.zeros(6, 3, 4, device=dev)
    x[2] = 1.0
    x[3] = 1.0          # tie with step 2 in every window that holds both
    x1 = x.clone().requires_grad_()
    window_aggregate(x1, 2, "max").sum().backward()
    x2 = x.clone().requires_grad_()
    _ref(x2, 2, "max").sum().backward()
    torch.testing.assert_close(x1.grad, x2.grad)


def test_window_zero_is_identity(dev):
    from tagan_amd.layers.temporal_propagation import window_aggregate
    x = torch.randn(4, 5, 8, device=dev)
    assert window_aggregate(x, 0, "max") is x
