"""The matrix-core temporal kernels (v4, T <= 32, head_dim 16/32) against the VALU v3 kernels on
every input the kernels take: folded bias table, dense (time-aware) bias, explicit keep-mask,
causal flag, attention dropout (the same counter-hash mask: stream row*heads+h, counter i*T+j),
fp32 and bf16 storage, row-major and time-major layouts.  Both are fp32 math; they differ only in
summation order (and v4's exact two-pass softmax vs v3's online one): tolerance 2e-5 (fp32)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import tagan_amd  # noqa: F401
    return torch.device("cuda:0")


def _run(dev, qkv, T, R, time_major, heads, mask, p, seed, bt, bd, dctx, monkeypatch, v4):
    from tagan_amd.fused import TemporalCore
    monkeypatch.setenv("TAGAN_TATTN_V4", "1" if v4 else "0")
    core = TemporalCore(T, R, time_major, heads, mask, p, seed)
    out, saved = core.fwd(qkv, bt, bd)
    dqkv, dbt, dbd = core.bwd(qkv, out, saved, dctx, bt is not None, bd is not None)
    torch.cuda.synchronize()
    return [out, saved[0], dqkv] + [t for t in (dbt, dbd) if t is not None]


@pytest.mark.parametrize("T,H,heads,time_major,p,causal,masked,dense,dtype,R", [
    (32, 128, 8, True, 0.1, False, False, False, torch.float32, 37),    # C2 layer
    (32, 128, 8, True, 0.1, False, False, False, torch.bfloat16, 37),   # C2 bf16 mode
    (16, 128, 4, True, 0.1, False, False, False, torch.float32, 37),    # C4 (d = 32)
    (10, 64, 4, False, 0.3, True, False, False, torch.float32, 37),     # C1, causal (T == heads rule)
    (23, 64, 2, False, 0.0, False, True, True, torch.float32, 37),      # explicit mask + time-aware bias
    (32, 64, 2, True, 0.2, True, True, False, torch.float32, 37),       # d = 32, mask + causal + dropout
    (32, 128, 8, True, 0.1, False, False, False, torch.float32, 5),     # rows < 8: plain wave map
    (16, 128, 8, True, 0.1, False, False, False, torch.float32, 2061),  # > 1024 rows: several rows per wave
])
def test_v4_matches_v3(dev, monkeypatch, T, H, heads, time_major, p, causal, masked, dense, dtype, R):
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
        keep[..., 0] = True                                      # no fully masked query row
        mask = TemporalMask(causal=causal, keep=keep.to(torch.uint8).contiguous(), bstride=heads * T * T,
                            hstride=T * T)
    seed = 1234567
    a = _run(dev, qkv, T, R, time_major, heads, mask, p, seed, bt, bd, dctx, monkeypatch, True)
    b = _run(dev, qkv, T, R, time_major, heads, mask, p, seed, bt, bd, dctx, monkeypatch, False)
    tol = 2e-5 if dtype == torch.float32 else 2e-2
    names = ["out", "lse", "dqkv", "dbias_table", "dbias_dense"]
    for name, x, y in zip(names, a, b):
        x, y = x.float(), y.float()
        err = (x - y).abs().max().item()
        scale = max(1.0, y.abs().max().item())
        assert err <= tol * scale, "%s: max |v4 - v3| = %g (scale %g)" % (name, err, scale)


def test_v4_qkv_bias_sum(dev, monkeypatch):
    """The matrix-core backward also returns Σ over rows and steps of dq | dk | dv (the QKV projection's bias
    gradient, summed in-kernel in a fixed order) -- against the sum of the returned dqkv; the VALU path
    declines (None) and the caller reduces dqkv itself."""
    from tagan_amd.fused import TemporalCore
    from tagan_amd.kernels import TemporalMask
    T, H, heads, R = 32, 128, 8, 45
    g = torch.Generator(device=dev).manual_seed(11)
    qkv = torch.randn(T * R, 3 * H, device=dev, generator=g)
    dctx = torch.randn(T * R, H, device=dev, generator=g)
    bt = 0.3 * torch.randn(heads, 2 * T - 1, device=dev, generator=g)
    core = TemporalCore(T, R, True, heads, TemporalMask(causal=False), 0.1, 99)
    monkeypatch.setenv("TAGAN_TATTN_V4", "1")
    out, saved = core.fwd(qkv, bt, None)
    dqkv, dbt, _, dsum = core.bwd(qkv, out, saved, dctx, True, False, want_bias_sum=True)
    torch.cuda.synchronize()
    assert dsum is not None and dsum.shape == (3 * H,)
    ref = dqkv.double().sum(0)
    err = (dsum.double() - ref).abs().max().item()
    assert err <= 1e-4 * max(1.0, ref.abs().max().item()), err
    monkeypatch.setenv("TAGAN_TATTN_V4", "0")
    *_, dsum3 = core.bwd(qkv, out, saved, dctx, True, False, want_bias_sum=True)
    assert dsum3 is None
