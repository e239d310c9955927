"""LayerNorm-fused projection GEMMs (csrc/stream_gemm.hip MODE_LN_IN / MODE_LN_OUT / MODE_LN_BWD and the LN-recomputing
weight gradient) through the C-ABI, against fp64 restatements of the unfused chain they replace:

  LN1 + QKV projection        geometric_attention.py:541-548 / temporal_attention.py:985-990
  out-projection + dropout + residual + LN2 (+ skip LN)  geometric_attention.py:586-596, model.py:258-262
  their backward (LN1 backward after the QKV input gradient; the QKV weight gradient of h = LN1(x)).

fp32 mode (three bf16 planes): outputs within 2e-5 of max|ref| elementwise and 1e-5 normwise (fp32-GEMM accuracy
on O(1) LayerNorm outputs).  bf16 planes: within 1e-2 normwise.  The dropout mask of the out-projection epilogue
must be the standalone LayerNorm kernel's (same hash, stream = row, counter = column): checked by running both on
the same inputs.  Statistics (mean, rstd) to 1e-5 relative.  dgamma / dbeta are fixed-order sums (bitwise
reproducible).  Rows: ragged counts (1, 15, 33, 1000, 40961)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

H = 128
ROWS = [1, 15, 33, 1000, 40961]


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import tagan_amd  # noqa: F401
    return torch.device("cuda:0")


def _nerr(x, ref):
    return float((x.double() - ref).norm() / ref.norm().clamp_min(1e-300))


def _merr(x, ref):
    return float((x.double() - ref).abs().max() / ref.abs().max().clamp_min(1e-300))


def _ln64(x, g, b, eps):
    x = x.double()
    m = x.mean(1, keepdim=True)
    v = ((x - m) ** 2).mean(1, keepdim=True)
    rs = 1.0 / torch.sqrt(v + eps)
    return (x - m) * rs * g.double() + b.double(), m[:, 0], rs[:, 0]


def _params(dev, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    ln_w = 1.0 + 0.1 * torch.randn(H, device=dev, generator=g)
    ln_b = 0.1 * torch.randn(H, device=dev, generator=g)
    return g, ln_w, ln_b


@pytest.mark.parametrize("M", ROWS)
@pytest.mark.parametrize("planes,store", [(3, "fp32"), (1, "bf16"), (1, "fp32")])
@pytest.mark.parametrize("Hw", [128, 256])
def test_ln_in_qkv(M, planes, store, Hw):
    """LN1 in the QKV projection's prologue (16 lanes per row at H = 128, 32 at H = 256) and the LN-recomputing
    weight gradient."""
    dev = _dev()
    from tagan_amd import stream_gemm as sg
    H = Hw
    if not sg.ln_supported(H, planes, store == "bf16", "in"):
        pytest.skip("no LN1-prologue kernel at this width / precision")
    g = torch.Generator(device=dev).manual_seed(M + planes + H)
    ln_w = 1.0 + 0.1 * torch.randn(H, device=dev, generator=g)
    ln_b = 0.1 * torch.randn(H, device=dev, generator=g)
    x = 0.5 + 2.0 * torch.randn(M, H, device=dev, generator=g)
    w = torch.randn(3 * H, H, device=dev, generator=g) / H ** 0.5
    bias = torch.randn(3 * H, device=dev, generator=g)
    dt = torch.bfloat16 if store == "bf16" else torch.float32
    out, mean, rstd = sg.nt_ln_in(x, ln_w, ln_b, 1e-5, sg.wprep(w, False, planes), 3 * H, planes, bias=bias,
                                  out_dtype=dt)
    h, m64, rs64 = _ln64(x, ln_w, ln_b, 1e-5)
    ref = h @ w.double().t() + bias.double()
    assert out.dtype == dt
    assert _merr(mean, m64) <= 1e-5 and _merr(rstd, rs64) <= 1e-5
    if planes == 3:
        assert _merr(out, ref) <= 2e-5 and _nerr(out, ref) <= 1e-5, (_merr(out, ref), _nerr(out, ref))
    else:
        assert _nerr(out, ref) < 1e-2
    # the weight gradient of h = LN(x), h recomputed from x and the statistics just written
    dq = torch.randn(M, 3 * H, device=dev, generator=g).to(dt)
    dw, db = sg.tn_ln(dq, x, ln_w, ln_b, mean, rstd, planes)
    refw = dq.double().t() @ h
    if planes == 3:
        assert _merr(dw, refw) <= 2e-5, _merr(dw, refw)
    else:
        assert _nerr(dw, refw) < 1e-2
    # db: Σ dq through dq's planes (one bf16 plane of an fp32 dq rounds it: bf16-gemm mode)
    assert _merr(db, dq.double().sum(0)) <= (2e-6 if planes == 3 else 1e-3 if store == "bf16" else 1e-2)
    dw2, db2 = sg.tn_ln(dq, x, ln_w, ln_b, mean, rstd, planes)
    assert torch.equal(dw, dw2) and torch.equal(db, db2)


def test_ln_in_recompute_matches_stored_h():
    """The weight gradient over the recomputed h equals the plain weight gradient over a stored LN(x) computed with
    the same statistics (bf16 plane: the same rounding of the same fp32 value)."""
    dev = _dev()
    from tagan_amd import stream_gemm as sg
    g, ln_w, ln_b = _params(dev, 5)
    M = 5000
    x = torch.randn(M, H, device=dev, generator=g)
    w = torch.randn(3 * H, H, device=dev, generator=g) / H ** 0.5
    _, mean, rstd = sg.nt_ln_in(x, ln_w, ln_b, 1e-5, sg.wprep(w, False, 1), 3 * H, 1, out_dtype=torch.bfloat16)
    # fma(t, g, b) with t = (x - m) rs in fp32: the fp64 t·g + b rounded once to fp32 (t·g is exact in fp64)
    t = (x - mean[:, None]) * rstd[:, None]
    h = (t.double() * ln_w.double() + ln_b.double()).float()
    dq = torch.randn(M, 3 * H, device=dev, generator=g).to(torch.bfloat16)
    dw_a, _ = sg.tn_ln(dq, x, ln_w, ln_b, mean, rstd, 1)
    dw_b, _ = sg.tn(dq, h.to(torch.bfloat16), 1)
    assert _merr(dw_a, dw_b.double()) <= 1e-5


@pytest.mark.parametrize("M", ROWS)
@pytest.mark.parametrize("planes,store,Hw", [(3, "fp32", 128), (1, "bf16", 128), (1, "bf16", 256), (1, "fp32", 256)])
@pytest.mark.parametrize("skip", [False, True])
def test_ln_out(M, planes, store, Hw, skip):
    """Out-projection + dropout + residual + LN2 (+ skip LN) epilogue; H = 256 on the one-plane row-owner kernel."""
    dev = _dev()
    from tagan_amd import stream_gemm as sg
    H = Hw
    g = torch.Generator(device=dev).manual_seed(100 + M + planes + H)
    ln_w = 1.0 + 0.1 * torch.randn(H, device=dev, generator=g)
    ln_b = 0.1 * torch.randn(H, device=dev, generator=g)
    dt = torch.bfloat16 if store == "bf16" else torch.float32
    a = torch.randn(M, H, device=dev, generator=g).to(dt)
    res = torch.randn(M, H, device=dev, generator=g)
    w = torch.randn(H, H, device=dev, generator=g) / H ** 0.5
    bias = torch.randn(H, device=dev, generator=g)
    gs = bs = None
    if skip:
        gs = 1.0 + 0.1 * torch.randn(H, device=dev, generator=g)
        bs = 0.1 * torch.randn(H, device=dev, generator=g)
    y, s, mean, rstd, sk = sg.nt_ln_out(a, sg.wprep(w, False, planes), planes, bias, res, 0.0, 0, ln_w, ln_b, 1e-5,
                                        gs, bs, 1e-5)
    s64 = a.double() @ w.double().t() + bias.double() + res.double()
    y64, m64, rs64 = _ln64(s64, ln_w, ln_b, 1e-5)
    if skip:
        ys, ms64, rss64 = _ln64(res, gs, bs, 1e-5)
        y64 = y64 + ys
        assert _merr(sk[0], ms64) <= 1e-5 and _merr(sk[1], rss64) <= 1e-5
    tol = (2e-5, 1e-5) if planes == 3 else (5e-2, 1e-2)
    assert _merr(s, s64) <= tol[0] and _nerr(s, s64) <= tol[1], (_merr(s, s64), _nerr(s, s64))
    assert _merr(y, y64) <= tol[0] and _nerr(y, y64) <= tol[1], (_merr(y, y64), _nerr(y, y64))
    # the mean against the row's scale (a near-zero mean of a single row has no relative accuracy to speak of)
    mtol = 1e-5 if planes == 3 else 1e-2
    assert float((mean.double() - m64).abs().max()) <= mtol * max(1.0, float(m64.abs().max()))
    assert _merr(rstd, rs64) <= mtol


@pytest.mark.parametrize("skip", [False, True])
def test_ln_out_dropout_matches_layernorm_kernel(skip):
    """The epilogue's dropout decisions and LayerNorm equal the standalone chain on the same o = a·Wᵀ."""
    dev = _dev()
    from tagan_amd import stream_gemm as sg
    from tagan_amd.fused import ln_fwd, ln_skip_fwd
    g, ln_w, ln_b = _params(dev, 77)
    M = 3001
    a = torch.randn(M, H, device=dev, generator=g)
    res = torch.randn(M, H, device=dev, generator=g)
    w = torch.randn(H, H, device=dev, generator=g) / H ** 0.5
    bias = torch.randn(H, device=dev, generator=g)
    gs = 1.0 + 0.1 * torch.randn(H, device=dev, generator=g) if skip else None
    bs = 0.1 * torch.randn(H, device=dev, generator=g) if skip else None
    wp = sg.wprep(w, False, 3)
    y, s, mean, rstd, sk = sg.nt_ln_out(a, wp, 3, bias, res, 0.1, 1234, ln_w, ln_b, 1e-5, gs, bs, 1e-5)
    o = sg.nt(a, wp, H, 3)
    if skip:
        y2, s2, m2, r2, sk2 = ln_skip_fwd(o, res, 0.1, 1234, ln_w, ln_b, 1e-5, gs, bs, 1e-5, a_bias=bias)
    else:
        y2, s2, m2, r2 = ln_fwd(o, res, 0.1, 1234, ln_w, ln_b, 1e-5, True, a_bias=bias)
    dropped = (s - res).abs() < 1e-30
    dropped2 = (s2 - res).abs() < 1e-30
    assert torch.equal(dropped, dropped2)
    assert 0.05 < float(dropped.float().mean()) < 0.15
    assert _merr(s, s2.double()) <= 1e-5 and _merr(y, y2.double()) <= 1e-5
    assert _merr(mean, m2.double()) <= 1e-5 and _merr(rstd, r2.double()) <= 1e-5


@pytest.mark.parametrize("M", ROWS)
@pytest.mark.parametrize("planes,store", [(1, "fp32"), (1, "bf16")])
@pytest.mark.parametrize("with_dres", [True, False])
def test_ln_bwd(M, planes, store, with_dres):
    dev = _dev()
    from tagan_amd import stream_gemm as sg
    g, ln_w, ln_b = _params(dev, 300 + M + planes)
    dt = torch.bfloat16 if store == "bf16" else torch.float32
    x = 0.3 + torch.randn(M, H, device=dev, generator=g)
    _, m64, rs64 = _ln64(x, ln_w, ln_b, 1e-5)
    mean, rstd = m64.float(), rs64.float()
    dq = torch.randn(M, 3 * H, device=dev, generator=g).to(dt)
    wq = torch.randn(3 * H, H, device=dev, generator=g) / H ** 0.5          # nn.Linear weight [3H, H]
    dres = torch.randn(M, H, device=dev, generator=g) if with_dres else None
    dx, dg, db = sg.nt_ln_bwd(dq, sg.wprep(wq, True, planes), planes, x, mean, rstd, ln_w, dres)
    dh = dq.double() @ wq.double()
    xh = (x.double() - mean.double()[:, None]) * rstd.double()[:, None]
    gd = dh * ln_w.double()
    c1 = (gd * xh).mean(1, keepdim=True)
    c2 = gd.mean(1, keepdim=True)
    ref = rstd.double()[:, None] * (gd - c1 * xh - c2)
    if with_dres:
        ref = ref + dres.double()
    rdg = (dh * xh).sum(0)
    rdb = dh.sum(0)
    if planes == 3:
        assert _merr(dx, ref) <= 2e-5 and _nerr(dx, ref) <= 1e-5, (_merr(dx, ref), _nerr(dx, ref))
        assert _merr(dg, rdg) <= 2e-5 and _merr(db, rdb) <= 2e-5
    else:
        assert _nerr(dx, ref) < 1e-2 and _nerr(dg, rdg) < 1e-2 and _nerr(db, rdb) < 1e-2
    dx2, dg2, db2 = sg.nt_ln_bwd(dq, sg.wprep(wq, True, planes), planes, x, mean, rstd, ln_w, dres)
    assert torch.equal(dx, dx2) and torch.equal(dg, dg2) and torch.equal(db, db2)


def _ln2_ref(dy, s, ln_w, c, w_o, skip):
    """fp64 LN2 backward (p_drop = 0) + the out-projection gradients: dres, dc, dw_o, db_o, dg, db, dgs, dbs."""
    _, m64, rs64 = _ln64(s, ln_w, ln_w, 1e-5)
    d = dy.double()
    xh = (s.double() - m64[:, None]) * rs64[:, None]
    gd = d * ln_w.double()
    o = rs64[:, None] * (gd - (gd * xh).mean(1, keepdim=True) * xh - gd.mean(1, keepdim=True))
    dres = o.clone()
    dgs = dbs = None
    if skip is not None:
        xs, gs = skip
        _, ms, rss = _ln64(xs, gs, gs, 1e-5)
        xsh = (xs.double() - ms[:, None]) * rss[:, None]
        gsd = d * gs.double()
        dres = dres + rss[:, None] * (gsd - (gsd * xsh).mean(1, keepdim=True) * xsh - gsd.mean(1, keepdim=True))
        dgs, dbs = (d * xsh).sum(0), d.sum(0)
    cd = c.double()
    return dres, o @ w_o.double(), o.t() @ cd, o.sum(0), (d * xh).sum(0), d.sum(0), dgs, dbs


@pytest.mark.parametrize("M", ROWS)
@pytest.mark.parametrize("planes,store", [(3, "fp32"), (1, "bf16"), (1, "fp32")])
@pytest.mark.parametrize("skip", [False, True])
def test_ln2_bwd_out(M, planes, store, skip):
    """tagan_ln2_bwd_out (LN2 backward + dC + dW_o + db_o in one pass) against fp64 (no dropout)."""
    dev = _dev()
    from tagan_amd import stream_gemm as sg
    if not sg.ln2_bwd_out_supported(H, planes, store == "bf16"):
        pytest.skip("no kernel")
    g, ln_w, _ = _params(dev, 500 + M + planes)
    dt = torch.bfloat16 if store == "bf16" else torch.float32
    s = 0.2 + torch.randn(M, H, device=dev, generator=g)
    dy = torch.randn(M, H, device=dev, generator=g)
    c = torch.randn(M, H, device=dev, generator=g).to(dt)
    w_o = torch.randn(H, H, device=dev, generator=g) / H ** 0.5
    _, m64, rs64 = _ln64(s, ln_w, ln_w, 1e-5)
    sk = ref_sk = None
    if skip:
        xs = torch.randn(M, H, device=dev, generator=g)
        gs = 1.0 + 0.1 * torch.randn(H, device=dev, generator=g)
        _, ms, rss = _ln64(xs, gs, gs, 1e-5)
        sk, ref_sk = (xs, ms.float(), rss.float(), gs), (xs, gs)
    out = sg.ln2_bwd_out(dy, s, m64.float(), rs64.float(), ln_w, 0.0, 0, c, sg.wprep(w_o, True, planes), planes,
                         skip=sk)
    ref = _ln2_ref(dy, s, ln_w, c, w_o, ref_sk)
    names = ["dres", "dc", "dw_o", "db_o", "dgamma", "dbeta", "dgamma_s", "dbeta_s"]
    for name, got, want in zip(names, out, ref):
        if want is None:
            assert got is None, name
            continue
        if planes == 3 or name in ("dres", "dgamma", "dbeta", "dgamma_s", "dbeta_s"):
            assert _merr(got, want) <= 2e-5 and _nerr(got, want) <= 1e-5, (name, _merr(got, want), _nerr(got, want))
        else:   # one bf16 plane of do (and c) in the products
            assert _nerr(got, want) < 1e-2, (name, _nerr(got, want))
    again = sg.ln2_bwd_out(dy, s, m64.float(), rs64.float(), ln_w, 0.0, 0, c, sg.wprep(w_o, True, planes), planes,
                           skip=sk)
    for name, a, b in zip(names, out, again):
        assert (a is None and b is None) or torch.equal(a, b), name   # fixed-order sums: bitwise reproducible


@pytest.mark.parametrize("planes,store", [(3, "fp32"), (1, "bf16")])
def test_ln2_bwd_out_reproducible_at_c2_rows(planes, store):
    """320,000 rows (many tiles per workgroup, where a first form's LN sums came out nondeterministic,
    profiles/r5d_ln2_probe.txt): five calls bitwise equal, dgamma within fp32 accuracy of fp64."""
    dev = _dev()
    from tagan_amd import stream_gemm as sg
    g, ln_w, _ = _params(dev, 31)
    M = 320000
    dt = torch.bfloat16 if store == "bf16" else torch.float32
    s = 0.2 + torch.randn(M, H, device=dev, generator=g)
    dy = torch.randn(M, H, device=dev, generator=g)
    c = torch.randn(M, H, device=dev, generator=g).to(dt)
    w_o = torch.randn(H, H, device=dev, generator=g) / H ** 0.5
    xs = torch.randn(M, H, device=dev, generator=g)
    gs = 1.0 + 0.1 * torch.randn(H, device=dev, generator=g)
    _, m64, rs64 = _ln64(s, ln_w, ln_w, 1e-5)
    _, ms, rss = _ln64(xs, gs, gs, 1e-5)
    wp = sg.wprep(w_o, True, planes)
    runs = [sg.ln2_bwd_out(dy, s, m64.float(), rs64.float(), ln_w, 0.1, 99, c, wp, planes,
                           skip=(xs, ms.float(), rss.float(), gs)) for _ in range(5)]
    for r in runs[1:]:
        for a, b in zip(runs[0], r):
            assert torch.equal(a, b)
    xh = (s.double() - m64[:, None]) * rs64[:, None]
    assert _merr(runs[0][4], (dy.double() * xh).sum(0)) <= 2e-5


@pytest.mark.parametrize("skip", [False, True])
def test_ln2_bwd_out_matches_unfused_chain_with_dropout(skip):
    """Same dropout decisions as the standalone LayerNorm backward (stream = row, counter = column), so the fused
    pass equals tagan_layernorm_bwd [+ skip] -> tagan_sgemm_nt -> tagan_sgemm_tn on the same inputs."""
    dev = _dev()
    from tagan_amd import stream_gemm as sg
    from tagan_amd.fused import ln_bwd, ln_skip_bwd
    g, ln_w, _ = _params(dev, 91)
    M = 5003
    s = torch.randn(M, H, device=dev, generator=g)
    dy = torch.randn(M, H, device=dev, generator=g)
    c = torch.randn(M, H, device=dev, generator=g)
    w_o = torch.randn(H, H, device=dev, generator=g) / H ** 0.5
    _, m64, rs64 = _ln64(s, ln_w, ln_w, 1e-5)
    mean, rstd = m64.float(), rs64.float()
    wp = sg.wprep(w_o, True, 3)
    if skip:
        xs = torch.randn(M, H, device=dev, generator=g)
        gs = 1.0 + 0.1 * torch.randn(H, device=dev, generator=g)
        _, ms, rss = _ln64(xs, gs, gs, 1e-5)
        ms, rss = ms.float(), rss.float()
        dres0, do0, dg0, db0, dbo0, dgs0, dbs0 = ln_skip_bwd(s, mean, rstd, ln_w, xs, ms, rss, gs, dy, 0.1, 4321)
        got = sg.ln2_bwd_out(dy, s, mean, rstd, ln_w, 0.1, 4321, c, wp, 3, skip=(xs, ms, rss, gs))
    else:
        dres0, do0, dg0, db0, dbo0 = ln_bwd(s, mean, rstd, ln_w, dy, None, 0.1, 4321, True, True, True)
        dgs0 = dbs0 = None
        got = sg.ln2_bwd_out(dy, s, mean, rstd, ln_w, 0.1, 4321, c, wp, 3)
    dc0 = sg.nt(do0, wp, H, 3)
    dw0 = sg.tn(do0, c, 3, want_db=False)[0]
    want = [dres0, dc0, dw0, dbo0, dg0, db0, dgs0, dbs0]
    dropped = float((do0 == 0).float().mean())
    assert 0.05 < dropped < 0.15
    for name, a, b in zip(["dres", "dc", "dw_o", "db_o", "dgamma", "dbeta", "dgamma_s", "dbeta_s"], got, want):
        if b is None:
            assert a is None
            continue
        assert _merr(a, b.double()) <= 2e-5, (name, _merr(a, b.double()))


@pytest.mark.parametrize("M", [5003, 40961])
@pytest.mark.parametrize("store", ["bf16", "fp32"])
@pytest.mark.parametrize("skip", [False, True])
def test_ln2_bwd_out_256_matches_unfused_chain(skip, store, M):
    """H = 256, one plane (k_ln2_bwd_out256: two column groups): the same values as the unfused chain -- LN2 backward
    [+ skip] (tagan_layernorm_bwd / _skip_bwd), then tagan_sgemm_nt (dC) and tagan_sgemm_tn (dW_o) on its do -- with
    dropout: the same do (bf16-rounded operand of both products), fp32 sums in another order (column sums: 1e-5
    sqrt(M / 1000) of the tensor's scale; dres per element; dc per element to one bf16 ulp: do is a bf16 operand of
    its product in both, and the two fp32 row maths may round it differently where they differ by an fp32 ulp)."""
    dev = _dev()
    from tagan_amd import stream_gemm as sg
    from tagan_amd.fused import ln_bwd, ln_skip_bwd
    W = 256
    if not sg.ln2_bwd_out_supported(W, 1, store == "bf16"):
        pytest.skip("no H = 256 fused LN2 backward")
    g = torch.Generator(device=dev).manual_seed(256 + M)
    ln_w = 1.0 + 0.1 * torch.randn(W, device=dev, generator=g)
    dt = torch.bfloat16 if store == "bf16" else torch.float32
    s = torch.randn(M, W, device=dev, generator=g)
    dy = torch.randn(M, W, device=dev, generator=g)
    c = torch.randn(M, W, device=dev, generator=g).to(dt)
    w_o = torch.randn(W, W, device=dev, generator=g) / W ** 0.5
    x = s.double()
    m64 = x.mean(1)
    rs64 = 1.0 / torch.sqrt(((x - m64[:, None]) ** 2).mean(1) + 1e-5)
    mean, rstd = m64.float(), rs64.float()
    wp = sg.wprep(w_o, True, 1)
    if skip:
        xs = torch.randn(M, W, device=dev, generator=g)
        gs = 1.0 + 0.1 * torch.randn(W, device=dev, generator=g)
        xx = xs.double()
        ms = xx.mean(1)
        rss = 1.0 / torch.sqrt(((xx - ms[:, None]) ** 2).mean(1) + 1e-5)
        ms, rss = ms.float(), rss.float()
        dres0, do0, dg0, db0, dbo0, dgs0, dbs0 = ln_skip_bwd(s, mean, rstd, ln_w, xs, ms, rss, gs, dy, 0.1, 4321,
                                                             da_dtype=dt)
        got = sg.ln2_bwd_out(dy, s, mean, rstd, ln_w, 0.1, 4321, c, wp, 1, skip=(xs, ms, rss, gs))
    else:
        dres0, do0, dg0, db0, dbo0 = ln_bwd(s, mean, rstd, ln_w, dy, None, 0.1, 4321, True, True, True, da_dtype=dt)
        dgs0 = dbs0 = None
        got = sg.ln2_bwd_out(dy, s, mean, rstd, ln_w, 0.1, 4321, c, wp, 1)
    dc0 = sg.nt(do0, wp, W, 1, out_dtype=dt)
    dw0 = sg.tn(do0, c, 1, want_db=False)[0]
    want = [dres0, dc0, dw0, dbo0, dg0, db0, dgs0, dbs0]
    assert 0.05 < float((do0 == 0).float().mean()) < 0.15
    for name, a, b in zip(["dres", "dc", "dw_o", "db_o", "dgamma", "dbeta", "dgamma_s", "dbeta_s"], got, want):
        if b is None:
            assert a is None
            continue
        if name == "dres":           # per element, fp32
            tol = 2e-5
        elif name == "dc":           # per element: a 1-ulp fp32 difference in do can flip its bf16 operand rounding
            tol = 2.0 ** -7
        else:                        # column sums over M rows in another fp32 order: grows like sqrt(M)
            tol = 1e-5 * (M / 1000) ** 0.5
        assert a.dtype == b.dtype, name
        assert _merr(a, b.double()) <= tol, (name, _merr(a, b.double()))
    again = sg.ln2_bwd_out(dy, s, mean, rstd, ln_w, 0.1, 4321, c, wp, 1, skip=(xs, ms, rss, gs) if skip else None)
    for a, b in zip(got, again):
        assert (a is None and b is None) or torch.equal(a, b)


@pytest.mark.timeout(300)
def test_ln2_bwd_out_256_reproducible_at_scale():
    """3.2M rows (a quarter of the C5 one-rank share), bf16 activations, skip form, dropout: three calls bitwise
    equal (fixed-order partials in both column groups), dgamma within fp32 accuracy of fp64."""
    dev = _dev()
    from tagan_amd import stream_gemm as sg
    W, M = 256, 3_200_000
    if not sg.ln2_bwd_out_supported(W, 1, True):
        pytest.skip("no H = 256 fused LN2 backward")
    g = torch.Generator(device=dev).manual_seed(77)
    ln_w = 1.0 + 0.1 * torch.randn(W, device=dev, generator=g)
    gs = 1.0 + 0.1 * torch.randn(W, device=dev, generator=g)
    s = 0.2 + torch.randn(M, W, device=dev, generator=g)
    dy = torch.randn(M, W, device=dev, generator=g)
    c = torch.randn(M, W, device=dev, generator=g).to(torch.bfloat16)
    xs = torch.randn(M, W, device=dev, generator=g)
    w_o = torch.randn(W, W, device=dev, generator=g) / W ** 0.5

    def stats(t):
        m = torch.empty(M, device=dev, dtype=torch.float64)
        r = torch.empty(M, device=dev, dtype=torch.float64)
        for a in range(0, M, 400_000):
            x = t[a:a + 400_000].double()
            m[a:a + 400_000] = x.mean(1)
            r[a:a + 400_000] = 1.0 / torch.sqrt(((x - m[a:a + 400_000, None]) ** 2).mean(1) + 1e-5)
        return m, r
    m64, rs64 = stats(s)
    ms, rss = stats(xs)
    wp = sg.wprep(w_o, True, 1)
    runs = [sg.ln2_bwd_out(dy, s, m64.float(), rs64.float(), ln_w, 0.1, 5, c, wp, 1,
                           skip=(xs, ms.float(), rss.float(), gs)) for _ in range(3)]
    for r in runs[1:]:
        for a, b in zip(runs[0], r):
            assert torch.equal(a, b)
    ref = torch.zeros(W, device=dev, dtype=torch.float64)
    for a in range(0, M, 400_000):
        xh = (s[a:a + 400_000].double() - m64[a:a + 400_000, None]) * rs64[a:a + 400_000, None]
        ref += (dy[a:a + 400_000].double() * xh).sum(0)
    assert _merr(runs[0][4], ref) <= 2e-5


def test_ln_supported_shapes():
    _dev()
    from tagan_amd import stream_gemm as sg
    for op in ("in", "out", "bwd"):
        assert sg.ln_supported(128, 1, True, op) and sg.ln_supported(128, 1, False, op)
        assert sg.ln_supported(128, 3, False, op) == (op != "bwd")   # the three-plane LN1-backward form is not built
        # H = 256: the LN1 prologue and, one-plane, the LN2 epilogue ("out"); LN1's backward stays standalone there
        # (the three-plane H = 256 LN1 prologue lost its A/B and is not built)
        assert not sg.ln_supported(256, 3, False, op)
        assert sg.ln_supported(256, 1, True, op) == (op in ("in", "out"))
