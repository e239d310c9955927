"""Graph-feature pooling kernel (csrc/pool.hip) vs the reference's view(T,-1,H) pooling (model.py:377-427)
expressed in torch fp64, on strided time-major inputs; and the TAGAN-level path."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("T,N,H", [(32, 10000, 128), (5, 13, 64), (7, 3, 32), (6, 6, 64), (10, 500, 256), (3, 1, 8)])
def test_pool_matches_reference_view(T, N, H):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from tagan_amd.kernels import pool_time_major
    g = torch.Generator().manual_seed(T * 1000 + N)
    base = torch.randn(T, N, H + 8, generator=g)           # strided rows: a view with ld_row = H + 8
    x = base[:, :, :H].cuda().requires_grad_(True)
    out = pool_time_major(x)
    ref_in = base[:, :, :H].double().requires_grad_(True)
    ref = ref_in.transpose(0, 1).reshape(T, N, H).mean(1)  # node-major flat rows [t*N, (t+1)*N)
    assert torch.allclose(out.double().cpu(), ref, atol=1e-5, rtol=1e-5)
    go = torch.randn(T, H, generator=g)
    (out * go.cuda()).sum().backward()
    (ref * go.double()).sum().backward()
    assert torch.allclose(x.grad.double().cpu(), ref_in.grad, atol=1e-7, rtol=1e-5)


@pytest.mark.parametrize("M,N", [(320000, 384), (1000, 128), (7, 4), (12345, 1024), (64, 36)])
def test_colsum_matches_fp64(M, N):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from tagan_amd.kernels import colsum
    g = torch.Generator().manual_seed(M + N)
    base = torch.randn(M, N + 4, generator=g)
    got = colsum(base[:, :N].cuda())                      # row stride N + 4
    want = base[:, :N].double().sum(0)
    assert torch.allclose(got.double().cpu(), want, atol=1e-6 * M ** 0.5, rtol=1e-5)
    again = colsum(base[:, :N].cuda())
    assert torch.equal(got, again)                        # ordered partials: bitwise reproducible
