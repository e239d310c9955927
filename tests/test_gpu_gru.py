"""The GRU recurrence kernel (csrc/gru.hip, GRUSeqFn) against the per-step Python recurrence of the same module
(TAGAN_GRU_KERNEL=0: the reference's TemporalGRUCell step, temporal_propagation.py:475-551, on torch GEMMs), at
widths and lengths beyond the G6 goldens (which test_gpu_tprop.py checks against the reference itself):
forward states and every gradient (input, W_x, W_h, biases, both LayerNorms), time-aware and bidirectional."""
import pytest
import torch

pytestmark = pytest.mark.gpu

ATOL, RTOL = 1e-4, 1e-4


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import tagan_amd  # noqa: F401
    return torch.device("cuda:0")


def _run(layer, xt, ts, dy, kernel):
    import tagan_amd.layers.temporal_propagation as tp
    prev = tp.USE_GRU_KERNEL
    tp.USE_GRU_KERNEL = kernel
    try:
        x = xt.clone().requires_grad_()
        layer.zero_grad(set_to_none=True)
        y = layer.forward_time_major(x, ts)
        (y * dy).sum().backward()
        return y.detach(), x.grad, {k: p.grad.clone() for k, p in layer.named_parameters() if p.grad is not None}
    finally:
        tp.USE_GRU_KERNEL = prev


@pytest.mark.parametrize("H,T,N,bidir,timed,ln", [
    (128, 16, 1000, False, True, True),
    (64, 12, 777, True, True, True),
    (256, 6, 300, False, False, True),
    (64, 9, 500, False, True, False),
    (32, 20, 129, True, False, True),
])
def test_gru_kernel_vs_python_steps(dev, H, T, N, bidir, timed, ln):
    from tagan_amd.layers.temporal_propagation import TemporalEvolutionLayer
    torch.manual_seed(H + T)
    layer = TemporalEvolutionLayer(H, H, dropout=0.0, time_aware=True, bidirectional=bidir, use_layer_norm=ln).to(dev)
    with torch.no_grad():   # non-trivial LayerNorm affine parameters
        for n, p in layer.named_parameters():
            if "layer_norm" in n:
                p.add_(0.1 * torch.randn_like(p))
    g = torch.Generator().manual_seed(7)
    xt = torch.randn(T, N, H, generator=g).to(dev)
    dy = torch.randn(T, N, H, generator=g).to(dev)
    ts = (torch.rand(N, T, generator=g).cumsum(1) * 3.0).to(dev) if timed else None
    y1, dx1, g1 = _run(layer, xt, ts, dy, True)
    y0, dx0, g0 = _run(layer, xt, ts, dy, False)
    torch.testing.assert_close(y1, y0, atol=ATOL, rtol=RTOL)
    torch.testing.assert_close(dx1, dx0, atol=ATOL, rtol=RTOL)
    assert g1.keys() == g0.keys()
    for k in g0:
        scale = max(1.0, float(g0[k].abs().max()))
        torch.testing.assert_close(g1[k], g0[k], atol=ATOL * scale, rtol=RTOL, msg=k)


def test_gru_kernel_dropout_reproducible(dev):
    """With dropout the kernel's counter-hash mask is the same in forward and backward and across runs with the
    same seed (no torch RNG involved): two identical runs agree bitwise."""
    from tagan_amd.layers.temporal_propagation import TemporalEvolutionLayer
    torch.manual_seed(1)
    layer = TemporalEvolutionLayer(64, 64, dropout=0.2, time_aware=False).to(dev).train()
    g = torch.Generator().manual_seed(3)
    xt = torch.randn(8, 400, 64, generator=g).to(dev)
    dy = torch.randn(8, 400, 64, generator=g).to(dev)
    outs = []
    for _ in range(2):
        torch.manual_seed(42)
        outs.append(_run(layer, xt, None, dy, True))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    torch.manual_seed(43)
    other = _run(layer, xt, None, dy, True)
    assert not torch.equal(other[0], outs[0][0])
