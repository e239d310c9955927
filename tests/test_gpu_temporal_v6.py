"""The head-group-slab temporal kernels (v6: T <= 32, head_dim 16/32; Q | K | V | dO of GH heads streamed through
one LDS slab per workgroup) against the one-wave-per-head v4 kernels on every input they take (bias table, dense
bias, keep-mask, causal, dropout, fp32/bf16 storage, both layouts, both group widths, row counts below 8 and above
the 1024 row groups).  Same per-head arithmetic in the same order, so the results must agree bitwise except for
the bias-table / QKV-bias partial sums, which fold rows per workgroup: tolerance 2e-5 (fp32)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import tagan_amd  # noqa: F401
    return torch.device("cuda:0")


def _run(dev, qkv, T, R, time_major, heads, mask, p, seed, bt, bd, dctx, monkeypatch, v6, gh):
    from tagan_amd.fused import TemporalCore
    monkeypatch.setenv("TAGAN_TATTN_V6", v6)
    monkeypatch.setenv("TAGAN_V6_GH", gh)
    core = TemporalCore(T, R, time_major, heads, mask, p, seed)
    out, saved = core.fwd(qkv, bt, bd)
    dqkv, dbt, dbd, dsum = core.bwd(qkv, out, saved, dctx, bt is not None, bd is not None, want_bias_sum=True)
    torch.cuda.synchronize()
    return [out, saved[0], dqkv] + [t for t in (dbt, dbd, dsum) if t is not None]


@pytest.mark.parametrize("gh", ["8", "4", "2"])
@pytest.mark.parametrize("T,H,heads,time_major,p,causal,masked,dense,dtype,R", [
    (32, 128, 8, True, 0.1, False, False, False, torch.float32, 37),    # C2 layer
    (32, 128, 8, True, 0.1, False, False, False, torch.bfloat16, 37),   # C2 bf16 mode
    (16, 128, 4, True, 0.1, False, False, False, torch.float32, 37),    # C4 (d = 32)
    (10, 64, 4, False, 0.3, True, False, False, torch.float32, 37),     # C1, causal
    (23, 64, 2, False, 0.0, False, True, True, torch.float32, 37),      # explicit mask + time-aware bias
    (32, 64, 2, True, 0.2, True, True, False, torch.float32, 37),       # d = 32, mask + causal + dropout
    (32, 128, 8, True, 0.1, False, False, False, torch.float32, 5),     # rows < 8
    (16, 128, 8, True, 0.1, False, False, False, torch.float32, 2061),  # > 1024 rows: several rows per workgroup
    (24, 96, 6, True, 0.1, False, False, False, torch.float32, 41),     # 6 heads: GH = 2 whatever is asked
])
def test_v6_matches_v4(dev, monkeypatch, gh, T, H, heads, time_major, p, causal, masked, dense, dtype, R):
    from tagan_amd.kernels import TemporalMask
    g = torch.Generator(device=dev).manual_seed(T * 7 + heads)
    shape = (T, R, 3 * H) if time_major else (R, T, 3 * H)
    qkv = torch.randn(*shape, device=dev, generator=g).to(dtype).reshape(-1, 3 * H)
    dctx = torch.randn(T * R, H, device=dev, generator=g).to(dtype)
    bt = 0.3 * torch.randn(heads, 2 * T - 1, device=dev, generator=g)
    bd = 0.2 * torch.randn(R, heads, T, T, device=dev, generator=g) if dense else None
    mask = TemporalMask(causal=causal)
    if masked:
        keep = (torch.rand(R, heads, T, T, device=dev, generator=g) > 0.3)
        keep[..., 0] = True
        mask = TemporalMask(causal=causal, keep=keep.to(torch.uint8).contiguous(), bstride=heads * T * T,
                            hstride=T * T)
    a = _run(dev, qkv, T, R, time_major, heads, mask, p, 4321, bt, bd, dctx, monkeypatch, "2", gh)
    b = _run(dev, qkv, T, R, time_major, heads, mask, p, 4321, bt, bd, dctx, monkeypatch, "0", gh)
    assert len(a) == len(b)
    tol = 2e-5 if dtype == torch.float32 else 2e-2
    for name, x, y in zip(["out", "lse", "dqkv", "dbias_table", "dbias_dense", "dsum_qkv"], a, b):
        x, y = x.float(), y.float()
        err = (x - y).abs().max().item()
        assert err <= tol * max(1.0, y.abs().max().item()), "%s: max |v6 - v4| = %g" % (name, err)
