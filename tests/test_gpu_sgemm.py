"""Streaming projection GEMMs (csrc/stream_gemm.hip) through the C-ABI, against fp64 products of the same inputs.

fp32 mode (three bf16 planes per operand, six plane products): the kernels' error against fp64 must stay within
2x the error torch's own fp32 GEMM makes on the same product (normwise), and within 1e-6 of max|ref| elementwise —
i.e. fp32-GEMM accuracy (the products of the attention blocks at H = 128 and their transposes).  bf16 mode (one
plane): within 1e-2 normwise of the fp64 product of the bf16-rounded operands' source values (bf16 rounding of two
operands, fp32 accumulation).  Weight gradients must be bitwise reproducible (fixed-order partial sums).
Edge cases: ragged row counts (not a multiple of any tile, fewer rows than one tile, zero rows), row strides wider
than the row, column views, no bias."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import tagan_amd  # noqa: F401
    return torch.device("cuda:0")


def _nerr(x, ref):
    return float((x.double() - ref).norm() / ref.norm().clamp_min(1e-300))


def _merr(x, ref):
    return float((x.double() - ref).abs().max() / ref.abs().max().clamp_min(1e-300))


# (N, K, kmajor): QKV forward, out-projection forward, out-projection input gradient, QKV input gradient at every
# hidden width BASELINE names (H = 128: C2 / C4, H = 256: C3 / C5, H = 64: C1); (256, 768, True) in fp32 runs as two
# K = 384 halves, the second accumulating into C
NT_SHAPES = [(3 * H, H, False) for H in (128, 256, 64)] + [(H, H, False) for H in (128, 256, 64)] + \
            [(H, H, True) for H in (128, 256, 64)] + [(H, 3 * H, True) for H in (128, 256, 64)]
ROWS = [1, 15, 33, 1000, 40961]


@pytest.mark.parametrize("N,K,kmajor", NT_SHAPES)
@pytest.mark.parametrize("M", ROWS)
def test_nt_fp32_planes(N, K, kmajor, M):
    dev = _dev()
    from tagan_amd import stream_gemm as sg
    g = torch.Generator(device=dev).manual_seed(M * 7 + N + K)
    a = torch.randn(M, K, device=dev, generator=g)
    w = torch.randn(K, N, device=dev, generator=g) if kmajor else torch.randn(N, K, device=dev, generator=g)
    w = w / K ** 0.5
    bias = torch.randn(N, device=dev, generator=g)
    B = w.t() if kmajor else w                        # [N, K]
    c = sg.nt(a, sg.wprep(w, kmajor, 3), N, 3, bias=bias)
    ref = a.double() @ B.double().t() + bias.double()
    ct = a @ B.t() + bias
    assert _nerr(c, ref) <= 2 * _nerr(ct, ref) + 1e-7, (_nerr(c, ref), _nerr(ct, ref))
    assert _merr(c, ref) <= 1e-6


def test_nt_strided_and_zero_rows():
    dev = _dev()
    from tagan_amd import stream_gemm as sg
    g = torch.Generator(device=dev).manual_seed(3)
    big = torch.randn(777, 200, device=dev, generator=g)
    a = big[:, 8:136]                                  # row stride 200, 16-byte aligned start
    w = torch.randn(384, 128, device=dev, generator=g) / 128 ** 0.5
    wp = sg.wprep(w, False, 3)
    out = torch.full((777, 400), 7.0, device=dev)
    sg.nt(a, wp, 384, 3, out=out[:, :384])
    ref = a.double() @ w.double().t()
    assert _merr(out[:, :384], ref) <= 1e-6
    assert bool((out[:, 384:] == 7.0).all())           # nothing written past the N columns
    z = sg.nt(torch.empty(0, 128, device=dev), wp, 384, 3)
    assert z.shape == (0, 384)


@pytest.mark.parametrize("N,K", [(384, 128), (128, 128), (768, 256), (256, 256), (192, 64), (64, 64)])
@pytest.mark.parametrize("M", ROWS + [0])
def test_tn_fp32_planes(N, K, M):
    dev = _dev()
    from tagan_amd import stream_gemm as sg
    g = torch.Generator(device=dev).manual_seed(M + 11 * N)
    dy = torch.randn(M, N, device=dev, generator=g)
    x = torch.randn(M, K, device=dev, generator=g)
    dw, db = sg.tn(dy, x, 3)
    if M == 0:
        assert bool((dw == 0).all()) and bool((db == 0).all())
        return
    ref = dy.double().t() @ x.double()
    refb = dy.double().sum(0)
    dwt = dy.t() @ x
    assert _nerr(dw, ref) <= 2 * _nerr(dwt, ref) + 1e-7, (_nerr(dw, ref), _nerr(dwt, ref))
    assert _merr(db, refb) <= 2e-6
    dw2, db2 = sg.tn(dy, x, 3)
    assert torch.equal(dw, dw2) and torch.equal(db, db2)   # fixed-order reduction


def test_tn_column_views():
    """dW of a column block of dqkv against a column view of another tensor (row strides 3H and 2H)."""
    dev = _dev()
    from tagan_amd import stream_gemm as sg
    g = torch.Generator(device=dev).manual_seed(9)
    dq = torch.randn(5000, 384, device=dev, generator=g)
    xx = torch.randn(5000, 256, device=dev, generator=g)
    dw = torch.zeros(128, 200, device=dev)
    _, db = sg.tn(dq[:, 128:256], xx[:, 128:], 3, dw=dw[:, 40:168])
    ref = dq[:, 128:256].double().t() @ xx[:, 128:].double()
    assert _merr(dw[:, 40:168], ref) <= 1e-6
    assert bool((dw[:, :40] == 0).all()) and bool((dw[:, 168:] == 0).all())
    assert _merr(db, dq[:, 128:256].double().sum(0)) <= 2e-6


@pytest.mark.parametrize("H", [128, 256, 64])
@pytest.mark.parametrize("store", ["fp32", "bf16"])
def test_bf16_plane(store, H):
    """One-plane products of a block at width H: QKV forward, its input gradient (K = 3H) and both weight
    gradients."""
    dev = _dev()
    from tagan_amd import stream_gemm as sg
    g = torch.Generator(device=dev).manual_seed(21 + H)
    dt = torch.bfloat16 if store == "bf16" else torch.float32
    a = torch.randn(3001, H, device=dev, generator=g).to(dt)
    w = torch.randn(3 * H, H, device=dev, generator=g) / H ** 0.5
    bias = torch.randn(3 * H, device=dev, generator=g)
    c = sg.nt(a, sg.wprep(w, False, 1), 3 * H, 1, bias=bias, out_dtype=dt)
    ref = a.double() @ w.double().t() + bias.double()
    assert c.dtype == dt
    assert _nerr(c, ref) < 1e-2
    dq = torch.randn(3001, 3 * H, device=dev, generator=g).to(dt)
    dh = sg.nt(dq, sg.wprep(w, True, 1), H, 1)
    assert _nerr(dh, dq.double() @ w.double()) < 1e-2
    dw, db = sg.tn(dq, a, 1)
    assert _nerr(dw, dq.double().t() @ a.double()) < 1e-2
    assert _nerr(db, dq.double().sum(0)) < 1e-2
    dw2, db2 = sg.tn(dq[:, :H], a, 1)
    assert _nerr(dw2, dq[:, :H].double().t() @ a.double()) < 1e-2


def test_split_k_accumulates_exactly_twice():
    """The K = 768 three-plane product (two K = 384 halves, the second accumulating into C) equals the sum of the
    two half products computed separately, up to one fp32 rounding per element."""
    dev = _dev()
    from tagan_amd import stream_gemm as sg
    g = torch.Generator(device=dev).manual_seed(77)
    dq = torch.randn(4099, 768, device=dev, generator=g)
    w = torch.randn(768, 256, device=dev, generator=g) / 768 ** 0.5      # dh = dq·w: B = wᵀ (k-major)
    full = sg.nt(dq, sg.wprep(w, True, 3), 256, 3)
    lo = sg.nt(dq[:, :384], sg.wprep(w[:384], True, 3), 256, 3)
    hi = sg.nt(dq[:, 384:], sg.wprep(w[384:], True, 3), 256, 3)
    assert (full - (lo + hi)).abs().max() <= 1e-6 * full.abs().max()
    ref = dq.double() @ w.double()
    assert _merr(full, ref) <= 1e-6


def test_unsupported_shape_reported():
    _dev()
    from tagan_amd import stream_gemm as sg
    assert not sg.supported(96, 64, 3)
    assert not sg.tn_supported(96, 64, 3)
    assert not sg.supported(768, 1536, 3) and not sg.tn_supported(1536, 512, 3)
    with pytest.raises(RuntimeError):
        sg.nt(torch.randn(10, 64, device="cuda"), torch.empty(96 * 64 * 3, dtype=torch.bfloat16, device="cuda"),
              96, 3)


@pytest.mark.parametrize("H", [128, 256, 64])
@pytest.mark.parametrize("planes", [1, 3])
def test_wprep_block_equals_single_preps(planes, H):
    """tagan_sgemm_wprep_block's four operands are bitwise the four tagan_sgemm_wprep calls they stand for."""
    dev = _dev()
    from tagan_amd import stream_gemm as sg
    g = torch.Generator(device=dev).manual_seed(31)
    wq = torch.randn(3 * H, H, device=dev, generator=g)
    wo = torch.randn(H, H, device=dev, generator=g)
    got = sg.wprep_block(wq, wo, planes)
    want = (sg.wprep(wq, False, planes), sg.wprep(wo, False, planes), sg.wprep(wo, True, planes),
            sg.wprep(wq, True, planes))
    for a, b in zip(got, want):
        assert torch.equal(a, b)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("M", [320_000, 3_200_000])
@pytest.mark.parametrize("H", [128, 256])
@pytest.mark.parametrize("form", ["plain", "lnx"])
def test_one_plane_tn_reproducible_at_scale(form, H, M):
    """The one-plane weight gradients of the bf16 activation mode (C5) at C2 / C5-share row counts, where the
    next tile's loads are issued chunk by chunk during the stash (TAGAN_SG_TN_ILOAD) and each workgroup runs many
    tiles: three calls bitwise equal, and within 1e-2 normwise of fp64.  "lnx": the LN-recomputing form (x fp32)."""
    dev = _dev()
    from tagan_amd import stream_gemm as sg
    g = torch.Generator(device=dev).manual_seed(M % 9973 + H)
    dq = torch.randn(M, 3 * H, device=dev, generator=g).to(torch.bfloat16)
    if form == "plain":
        x = torch.randn(M, H, device=dev, generator=g).to(torch.bfloat16)
        runs = [sg.tn(dq, x, 1) for _ in range(3)]
        xr = x
    else:
        if not sg.ln_supported(H, 1, True, "in"):
            pytest.skip("no LN1-prologue kernels at H=%d" % H)
        x = 0.3 + torch.randn(M, H, device=dev, generator=g)
        ln_w = 1.0 + 0.1 * torch.randn(H, device=dev, generator=g)
        ln_b = 0.1 * torch.randn(H, device=dev, generator=g)
        x64 = x.double()
        mean = x64.mean(1)
        rstd = 1.0 / torch.sqrt(((x64 - mean[:, None]) ** 2).mean(1) + 1e-5)
        runs = [sg.tn_ln(dq, x, ln_w, ln_b, mean.float(), rstd.float(), 1) for _ in range(3)]
        xr = None
        del x64
    for dw, db in runs[1:]:
        assert torch.equal(dw, runs[0][0]) and torch.equal(db, runs[0][1])
    ref = torch.zeros(3 * H, H, device=dev, dtype=torch.float64)
    for r0 in range(0, M, 400_000):
        d = dq[r0:r0 + 400_000].double()
        if xr is not None:
            xx = xr[r0:r0 + 400_000].double()
        else:
            xc = x[r0:r0 + 400_000].double()
            xx = (xc - mean[r0:r0 + 400_000, None]) * rstd[r0:r0 + 400_000, None] * ln_w.double() + ln_b.double()
        ref += d.t() @ xx
    assert _nerr(runs[0][0], ref) < 1e-2
    assert _nerr(runs[0][1], dq.double().sum(0)) < 1e-2
