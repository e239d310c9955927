"""The workgroup-per-unit matrix-core temporal kernels (v5: T in (32, 128] -- C3's T = 64, C5's T = 128 -- and,
with TAGAN_TATTN_V5=2, T in (16, 32]) against the VALU v3 kernels (T > 32) and the one-wave v4 kernels (T <= 32)
on every input the kernels take: folded bias table (from registers at TT <= 4, from LDS at TT = 8), dense
(time-aware) bias, explicit keep-mask, causal flag, attention dropout (same counter-hash mask), fp32 and bf16
storage, both layouts, fewer than 8 rows and many rows per workgroup, the 160 KB LDS case (T = 128, d = 32).
All are fp32 math and differ only in summation order: tolerance 2e-5 (fp32), 2e-2 (bf16 storage)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import tagan_amd  # noqa: F401
    return torch.device("cuda:0")


def _run(dev, qkv, T, R, time_major, heads, mask, p, seed, bt, bd, dctx, monkeypatch, v4, v5):
    from tagan_amd.fused import TemporalCore
    monkeypatch.setenv("TAGAN_TATTN_V4", v4)
    monkeypatch.setenv("TAGAN_TATTN_V5", v5)
    core = TemporalCore(T, R, time_major, heads, mask, p, seed)
    out, saved = core.fwd(qkv, bt, bd)
    dqkv, dbt, dbd = core.bwd(qkv, out, saved, dctx, bt is not None, bd is not None)
    torch.cuda.synchronize()
    return [out, saved[0], dqkv] + [t for t in (dbt, dbd) if t is not None]


def _inputs(dev, T, H, heads, time_major, causal, masked, dense, dtype, R):
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
    return qkv, dctx, bt, bd, mask


CASES = [
    (64, 256, 8, True, 0.1, False, False, False, torch.float32, 37),     # C3 layer (d = 32, 4 waves)
    (128, 256, 16, True, 0.1, False, False, False, torch.float32, 37),   # C5 layer (d = 16, 8 waves, LDS bias)
    (128, 256, 16, True, 0.1, False, False, False, torch.bfloat16, 37),  # C5 bf16 mode
    (128, 256, 8, True, 0.1, False, False, False, torch.float32, 21),    # d = 32 at 8 waves: 160 KB of LDS
    (48, 64, 2, False, 0.0, False, True, True, torch.float32, 29),       # mask + time-aware bias, padded tile
    (100, 128, 8, True, 0.2, True, True, False, torch.float32, 19),      # causal + mask + dropout, 8 waves
    (40, 128, 8, True, 0.1, False, False, False, torch.float32, 5),      # rows < 8: plain map
    (64, 128, 8, True, 0.1, False, False, False, torch.float32, 2061),   # > 1024 rows: several per workgroup
]


@pytest.mark.parametrize("T,H,heads,time_major,p,causal,masked,dense,dtype,R", CASES)
def test_v5_matches_v3(dev, monkeypatch, T, H, heads, time_major, p, causal, masked, dense, dtype, R):
    qkv, dctx, bt, bd, mask = _inputs(dev, T, H, heads, time_major, causal, masked, dense, dtype, R)
    a = _run(dev, qkv, T, R, time_major, heads, mask, p, 1234567, bt, bd, dctx, monkeypatch, "1", "1")
    b = _run(dev, qkv, T, R, time_major, heads, mask, p, 1234567, bt, bd, dctx, monkeypatch, "0", "0")
    tol = 2e-5 if dtype == torch.float32 else 2e-2
    for name, x, y in zip(["out", "lse", "dqkv", "dbias_table", "dbias_dense"], a, b):
        x, y = x.float(), y.float()
        err = (x - y).abs().max().item()
        scale = max(1.0, y.abs().max().item())
        assert err <= tol * scale, "%s: max |v5 - v3| = %g (scale %g)" % (name, err, scale)


@pytest.mark.parametrize("T,H,heads,time_major,p,causal,masked,dense,dtype,R", [
    (32, 128, 8, True, 0.1, False, False, False, torch.float32, 37),     # C2 layer
    (20, 64, 2, False, 0.1, True, True, True, torch.float32, 23),        # d = 32, everything on
])
def test_v5_matches_v4_at_T32(dev, monkeypatch, T, H, heads, time_major, p, causal, masked, dense, dtype, R):
    qkv, dctx, bt, bd, mask = _inputs(dev, T, H, heads, time_major, causal, masked, dense, dtype, R)
    a = _run(dev, qkv, T, R, time_major, heads, mask, p, 77, bt, bd, dctx, monkeypatch, "1", "2")
    b = _run(dev, qkv, T, R, time_major, heads, mask, p, 77, bt, bd, dctx, monkeypatch, "1", "0")
    for name, x, y in zip(["out", "lse", "dqkv", "dbias_table", "dbias_dense"], a, b):
        err = (x - y).abs().max().item()
        assert err <= 2e-5 * max(1.0, y.abs().max().item()), "%s: max |v5 - v4| = %g" % (name, err)


def test_v5_deterministic_and_qkv_bias_sum(dev, monkeypatch):
    """Bitwise identical reruns (no atomics anywhere), and the in-kernel Σ dq | dk | dv against the sum of the
    returned dqkv at the C3 shape."""
    from tagan_amd.fused import TemporalCore
    from tagan_amd.kernels import TemporalMask
    monkeypatch.setenv("TAGAN_TATTN_V5", "1")
    T, H, heads, R = 64, 256, 8, 300
    g = torch.Generator(device=dev).manual_seed(5)
    qkv = torch.randn(T * R, 3 * H, device=dev, generator=g)
    dctx = torch.randn(T * R, H, device=dev, generator=g)
    bt = 0.3 * torch.randn(heads, 2 * T - 1, device=dev, generator=g)
    core = TemporalCore(T, R, True, heads, TemporalMask(causal=False), 0.1, 99)
    res = []
    for _ in range(2):
        out, saved = core.fwd(qkv, bt, None)
        res.append((out, *core.bwd(qkv, out, saved, dctx, True, False, want_bias_sum=True)))
    torch.cuda.synchronize()
    for x, y in zip(res[0], res[1]):
        if x is not None:
            assert torch.equal(x, y)
    dqkv, dsum = res[0][1], res[0][4]
    assert dsum is not None and dsum.shape == (3 * H,)
    ref = dqkv.double().sum(0)
    err = (dsum.double() - ref).abs().max().item()
    assert err <= 1e-4 * max(1.0, ref.abs().max().item()), err


@pytest.mark.parametrize("T,H,heads,dtype", [(64, 256, 8, torch.float32), (128, 256, 16, torch.float32),
                                             (128, 256, 16, torch.bfloat16), (48, 128, 8, torch.float32)])
def test_v5_keep_bits_match_counter_hash(dev, monkeypatch, T, H, heads, dtype):
    """The keep-bit cache (the forward stores each element's dropout decision, the backward reads it instead of
    re-evaluating the counter hash) gives the results of the hash path (the forward bitwise, the backward to fp32
    rounding), and is used exactly where it is meant to be: written at p > 0 on the v5 path at T = 128, not at p = 0,
    not with a causal mask or an explicit mask (tagan_temporal_attn_keep_bytes)."""
    import ctypes
    from tagan_amd import _lib, fused, kernels
    from tagan_amd.kernels import TemporalMask
    monkeypatch.setenv("TAGAN_TATTN_V5", "1")
    R = 45
    qkv, dctx, bt, _, mask = _inputs(dev, T, H, heads, True, False, False, False, dtype, R)
    a = _run(dev, qkv, T, R, True, heads, mask, 0.1, 4242, bt, None, dctx, monkeypatch, "1", "1")
    core = fused.TemporalCore(T, R, True, heads, mask, 0.1, 4242)
    out, saved = core.fwd(qkv, bt, None)
    fast = T == 128   # the cache is used at 8 tiles only (T = 64: 4 tiles; T = 48 pads its tiles: the general path)
    assert (saved[-1] is not None) == fast, "the fast shape at p > 0 stores keep bits"
    monkeypatch.setattr(fused, "_keep_cache", lambda *args: (None, 0, ctypes.c_int32(0)))
    b = _run(dev, qkv, T, R, True, heads, mask, 0.1, 4242, bt, None, dctx, monkeypatch, "1", "1")
    for name, x, y in zip(["out", "lse", "dqkv", "dbias_table"], a, b):
        if name in ("out", "lse"):   # the forward is the same arithmetic with or without storing the bits
            assert torch.equal(x, y), name
        else:   # the cached backward applies 1 / (1 - p) to its outputs instead of per element: fp32 rounding apart
            x, y = x.float(), y.float()
            tol = (2e-6 if dtype == torch.float32 else 8e-3) * max(1.0, y.abs().max().item())
            assert (x - y).abs().max().item() <= tol, name
    L = _lib.lib()
    d = H // heads
    assert L.tagan_temporal_attn_keep_bytes(R, T, heads, d, 0, 0, 0, 0.1) == (R * heads * (T // 16) * 64 * 4
                                                                             if fast else 0)
    assert L.tagan_temporal_attn_keep_bytes(R, T, heads, d, 0, 0, 0, 0.0) == 0
    assert L.tagan_temporal_attn_keep_bytes(R, T, heads, d, 1, 0, 0, 0.1) == 0
    assert L.tagan_temporal_attn_keep_bytes(R, T, heads, d, 0, 1, 0, 0.1) == 0
    assert L.tagan_temporal_attn_keep_bytes(R, 32, heads, d, 0, 0, 0, 0.1) == 0   # v4 / v6 range
    assert kernels._keep_cache(R, T, heads, d, TemporalMask(causal=True), None, 0.1, dev)[0] is None


def test_temporal_dropout_mask_matches_restatement(dev):
    """The post-dropout attention weights of the general kernel are zero exactly where the numpy restatement of the
    pair-word mask (tests/test_abi.py::_temporal_keep) drops; every other kernel generation is held to the general
    one by the comparisons above, so this pins the mask of them all."""
    import numpy as np
    from test_abi import _temporal_keep
    from tagan_amd.kernels import TemporalAttnFn, TemporalMask
    T, H, heads, R, p, seed = 24, 64, 4, 7, 0.3, 987654321
    g = torch.Generator(device=dev).manual_seed(1)
    qkv = torch.randn(R, T, 3 * H, device=dev, generator=g)
    _, attn = TemporalAttnFn.apply(qkv, None, None, False, heads, TemporalMask(), p, seed, True)
    torch.cuda.synchronize()
    stream = (np.arange(R, dtype=np.uint64)[:, None] * heads + np.arange(heads, dtype=np.uint64)[None, :])
    ctr = (np.arange(T, dtype=np.uint32)[:, None] * T + np.arange(T, dtype=np.uint32)[None, :])
    keep = _temporal_keep(seed, stream[:, :, None, None], ctr[None, None], p)
    got = (attn != 0).cpu().numpy()
    assert got.shape == keep.shape
    assert (got == keep).all(), "%d of %d decisions differ" % ((got != keep).sum(), keep.size)
    assert 0.6 < keep.mean() < 0.8
