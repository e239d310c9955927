"""GPU parity: the HIP path (through the C-ABI) against the reference's golden vectors
and against the CPU oracle.  Tolerance: 1e-4 fp32 (north_star), written per check.

Run on an MI355X:  python -m pytest tests -m gpu -q
"""
import pytest
import torch

import golden_io as G
import oracle

pytestmark = pytest.mark.gpu

OUT_ATOL, OUT_RTOL = 1e-4, 1e-4      # forward values
GRAD_ATOL, GRAD_RTOL = 1e-4, 1e-4    # north_star: 1e-4 fp32 (observed errors: profiles/parity_errors_r02.json)


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import tagan_amd  # noqa: F401
    return torch.device("cuda:0")


def _load(module, sd, dev):
    module.load_state_dict({k: v for k, v in sd.items()}, strict=True)
    return module.to(dev).train()


# ----------------------------------------------------------------------------- CSR builder
def _check_csr(dev, counts, eis):
    from tagan_amd.kernels import build_graph
    graph = build_graph([e.to(dev) for e in eis], counts, cpos=True)
    nnz = graph.nnz_host()
    cols, off = [], 0
    rp_all = [0]
    for n, ei in zip(counts, eis):
        rp, c = oracle.csr_from_edge_index(ei, n)
        cols.append(c + off)
        rp_all.extend((rp[1:] + rp_all[-1]).tolist())
        off += n
    want_col = torch.cat(cols)
    assert nnz == want_col.numel()
    assert graph.rowptr.cpu().tolist() == rp_all
    assert torch.equal(graph.col[:nnz].cpu().long(), want_col)
    # CSC is the transpose with edge ids pointing back into the CSR, rows ascending in each column
    src = torch.repeat_interleave(torch.arange(off), torch.tensor(rp_all).diff())
    eid = graph.csc_eid[:nnz].cpu().long()
    crow = graph.csc_row[:nnz].cpu().long()
    assert torch.equal(src[eid], crow)
    ccol = torch.repeat_interleave(torch.arange(off), graph.csc_ptr.cpu().long().diff())
    assert torch.equal(want_col[eid], ccol)
    same = ccol[1:] == ccol[:-1]
    assert torch.all(crow.diff()[same] > 0)
    # the CSR -> CSC position map written by the same build when asked for: the inverse of csc_eid
    cpos = graph.csr_cpos[:nnz].cpu().long()
    assert torch.equal(cpos[eid], torch.arange(nnz))
    return graph


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_csr_build_matches_oracle(dev, seed):
    g = torch.Generator().manual_seed(seed)
    counts = [1, 7, 50, 3, 200]
    eis = []
    for n in counts:
        E = int(torch.randint(0, 4 * n + 1, (1,), generator=g))
        eis.append(torch.randint(-n, n, (2, E), generator=g))      # negatives wrap like torch indexing
    _check_csr(dev, counts, eis)


def test_csr_build_wide_keys(dev):
    """N x (largest snapshot) >= 2^32 takes the 64-bit sort keys (a 70,000-node snapshot); the other CSR
    tests (and C1/C2) run on 32-bit keys."""
    g = torch.Generator().manual_seed(5)
    counts = [70_000, 3, 5_000]
    eis = [torch.randint(-n, n, (2, 4 * n), generator=g) for n in counts]
    assert sum(counts) * max(counts) >= 2 ** 32
    _check_csr(dev, counts, eis)


def test_csr_build_hub_buckets(dev):
    """Power-law hubs overflow the small LDS bucket finish: a row with ~40k raw out-edges (duplicates included:
    beyond the 16k-key LDS of the big-bucket kernel -> its global-memory sort) and columns with ~5k and ~12k
    distinct in-neighbours (the big kernel's LDS path and, past 8k pairs, its global path), next to ordinary
    buckets in the same launch; then the same graph again (the device-side big-bucket lists are reset)."""
    g = torch.Generator().manual_seed(11)
    n0, n1 = 20_000, 3_000
    hub_out = torch.stack([torch.full((40_000,), 5), torch.randint(0, n0, (40_000,), generator=g)])
    hub_in = torch.stack([torch.randperm(n0, generator=g)[:12_000], torch.full((12_000,), 7)])
    mid_in = torch.stack([torch.randint(0, n0, (6_000,), generator=g), torch.full((6_000,), 9000)])
    rest = torch.randint(0, n0, (2, 60_000), generator=g)
    ei0 = torch.cat([hub_out, hub_in, mid_in, rest], 1)
    ei0 = ei0[:, torch.randperm(ei0.shape[1], generator=g)]
    ei1 = torch.randint(0, n1, (2, 9_000), generator=g)
    g1 = _check_csr(dev, [n0, n1], [ei0, ei1])
    g2 = _check_csr(dev, [n0, n1], [ei0, ei1])
    for a, b in ((g1.rowptr, g2.rowptr), (g1.col, g2.col), (g1.csc_row, g2.csc_row), (g1.csc_eid, g2.csc_eid)):
        n = g1.nnz_host()
        assert torch.equal(a[:n], b[:n])        # bitwise deterministic


def test_csr_build_rejects_out_of_range(dev):
    from tagan_amd.kernels import build_graph
    with pytest.raises(IndexError):
        build_graph([torch.tensor([[0, 1], [1, 5]], device=dev)], [5])


# ----------------------------------------------------------------------------- layer units vs goldens
@pytest.mark.parametrize("case", G.case_names("gat_"))
def test_graph_attention_golden(dev, case):
    from tagan_amd.layers import TAGANGraphAttention
    meta, t = G.load(case)
    torch.manual_seed(0)
    layer = _load(TAGANGraphAttention(meta["H"], meta["heads"], 0.0, meta["metric"], True,
                                      meta["learnable_distance"]), G.state_dict(t), dev)
    x = t["in.x"].to(dev).requires_grad_(True)
    out = layer(x, t["in.edge_index"].to(dev))
    G.assert_close("out", out, t["out"], OUT_ATOL, OUT_RTOL)
    (out * t["in.grad_out"].to(dev)).sum().backward()
    G.assert_close("grad x", x.grad, t["grad.x"], GRAD_ATOL, GRAD_RTOL)
    params = dict(layer.named_parameters())
    for name, g in G.grads(t).items():
        G.assert_close("grad " + name, params[name].grad, g, GRAD_ATOL, GRAD_RTOL)


@pytest.mark.parametrize("case", G.case_names("geo_"))
def test_geometric_attention_golden(dev, case):
    from tagan_amd.layers import GeometricAttention
    meta, t = G.load(case)
    mod = _load(GeometricAttention(meta["H"], meta["heads"], 0.0, meta["metric"], True), G.state_dict(t), dev)
    x = t["in.x"].to(dev).requires_grad_(True)
    mask = t.get("in.mask")
    bias = t.get("in.bias")
    out = mod(x, mask.to(dev) if mask is not None else None, bias.to(dev) if bias is not None else None)
    G.assert_close("out", out, t["out"], OUT_ATOL, OUT_RTOL)
    (out * t["in.grad_out"].to(dev)).sum().backward()
    G.assert_close("grad x", x.grad, t["grad.x"], GRAD_ATOL, GRAD_RTOL)
    params = dict(mod.named_parameters())
    for name, g in G.grads(t).items():
        G.assert_close("grad " + name, params[name].grad, g, GRAD_ATOL, GRAD_RTOL)


@pytest.mark.parametrize("case", G.case_names("tatt_"))
def test_temporal_attention_golden(dev, case):
    from tagan_amd.layers import AsymmetricTemporalAttention, TemporalAttention
    meta, t = G.load(case)
    cls = AsymmetricTemporalAttention if meta["cls"] == "AsymmetricTemporalAttention" else TemporalAttention
    mod = _load(cls(**meta["ctor"]), G.state_dict(t), dev)
    if meta.get("eval"):
        mod.eval()
    if meta["x_kind"] == "list":
        xs = [t["in.x.%d" % i].to(dev).requires_grad_(True) for i in range(meta["T"])]
        x_in = xs
    else:
        xs = [t["in.x"].to(dev).requires_grad_(True)]
        x_in = xs[0]
    kw = {}
    if "in.mask" in t:
        kw["attention_mask"] = t["in.mask"].to(dev)
    if "in.time_stamps" in t:
        kw["time_stamps"] = t["in.time_stamps"].to(dev)
    if meta["with_attn"]:
        kw["return_attention_weights"] = True
    res = mod(x_in, **kw)
    out, attn = res if meta["with_attn"] else (res, None)
    G.assert_close("out", out, t["out"], OUT_ATOL, OUT_RTOL)
    if attn is not None:
        G.assert_close("attn", attn, t["out.attn"], OUT_ATOL, OUT_RTOL)
    (out * t["in.grad_out"].to(dev)).sum().backward()
    for i, xi in enumerate(xs):
        key = "grad.x.%d" % i if meta["x_kind"] == "list" else "grad.x"
        G.assert_close(key, xi.grad, t[key], GRAD_ATOL, GRAD_RTOL)
    params = dict(mod.named_parameters())
    for name, g in G.grads(t).items():
        G.assert_close("grad " + name, params[name].grad, g, GRAD_ATOL, GRAD_RTOL)


# ----------------------------------------------------------------------------- end to end vs goldens
@pytest.mark.parametrize("case", G.case_names("e2e_"))
def test_tagan_golden(dev, case):
    from tagan_amd import TAGAN, TAGANConfig
    meta, t = G.load(case)
    cfg = TAGANConfig(**dict(meta["config"], device="cuda"))
    model = _load(TAGAN(cfg), G.state_dict(t), dev)
    if meta.get("eval"):
        model.eval()
    seq = G.sequence(meta, t, dev)
    seq = [(x.requires_grad_(True), ei, ea, ids) for x, ei, ea, ids in seq]
    labels = G.labels(meta, t, dev)
    with torch.set_grad_enabled(not meta.get("eval", False)):
        out = model(seq, labels=labels, return_attention_weights=meta.get("return_attention_weights", False))
    G.assert_close("logits", out["logits"], t["out.logits"], OUT_ATOL, OUT_RTOL)
    G.assert_close("predictions", out["predictions"], t["out.predictions"], OUT_ATOL, OUT_RTOL)
    if meta.get("return_attention_weights"):
        G.assert_close("tattn", out["temporal_attention_weights"], t["out.temporal_attention_weights"],
                       OUT_ATOL, OUT_RTOL)
        assert out["geometric_attention_weights"] == [{"node_attention": None}] * meta["n_geo_attn_weights"]
    if "out.loss" not in t:
        assert out["loss"] is None
        return
    G.assert_close("loss", out["loss"].reshape(1), t["out.loss"], OUT_ATOL, OUT_RTOL)
    out["loss"].backward()
    want = G.grads(t)
    for name, p in model.named_parameters():
        if name in want:
            G.assert_close("grad " + name, p.grad, want[name], GRAD_ATOL, GRAD_RTOL)
        else:
            assert p.grad is None or float(p.grad.abs().max()) == 0.0, name
    for i, (x, _, _, _) in enumerate(seq):
        G.assert_close("grad x.%d" % i, x.grad, t["grad.x.%d" % i], GRAD_ATOL, GRAD_RTOL)


# ----------------------------------------------------------------------------- larger shapes vs oracle
def _rand_seq(counts, F, De, epn, seed):
    g = torch.Generator().manual_seed(seed)
    seq = []
    for n in counts:
        seq.append((torch.randn(n, F, generator=g), torch.randint(0, n, (2, epn * n), generator=g),
                    torch.randn(epn * n, De, generator=g), list(range(n))))
    return seq


@pytest.mark.parametrize("learnable,H,heads,counts", [
    (False, 128, 8, [700, 650, 720, 690, 700, 710]),       # C2 architecture (euclidean), ragged N
    (True, 128, 8, [600] * 8),                              # scaled-dot metric
    (False, 256, 16, [300] * 16),                           # C5 head geometry (d=16, T=heads -> causal)
    (False, 128, 4, [400] * 5),                             # C4 head geometry (d=32)
])
def test_tagan_vs_oracle_medium(dev, learnable, H, heads, counts):
    from tagan_amd import TAGAN, TAGANConfig
    F_, De = 27, 2
    cfg = TAGANConfig(hidden_dim=H, num_heads=heads, node_feature_dim=F_, edge_feature_dim=De,
                      use_edge_features=True, output_dim=1, loss_type="bce", dropout=0.0,
                      learnable_distance=learnable, device="cuda")
    torch.manual_seed(3)
    model = TAGAN(cfg).to(dev).train()
    seq = _rand_seq(counts, F_, De, 10, 4)
    labels = torch.tensor([1.0])
    out = model([(x.to(dev), ei.to(dev), ea.to(dev), ids) for x, ei, ea, ids in seq], labels=labels.to(dev))
    out["loss"].backward()
    P = {k: v.detach().cpu().double().requires_grad_(v.is_floating_point())
         for k, v in model.state_dict().items()}
    seq64 = [(x.double(), ei, ea.double(), ids) for x, ei, ea, ids in seq]
    ref = oracle.tagan_forward(P, cfg.to_dict(), seq64, labels.double())
    G.assert_close("logits", out["logits"], ref["logits"], OUT_ATOL, OUT_RTOL)
    G.assert_close("loss", out["loss"].reshape(1), ref["loss"].reshape(1), OUT_ATOL, OUT_RTOL)
    ref["loss"].backward()
    for name, p in model.named_parameters():
        if P[name].grad is not None:
            G.assert_close("grad " + name, p.grad, P[name].grad, GRAD_ATOL, GRAD_RTOL)


# ----------------------------------------------------------------------------- determinism / dropout
def test_deterministic_with_dropout(dev):
    from tagan_amd import TAGAN, TAGANConfig
    cfg = TAGANConfig(hidden_dim=128, num_heads=8, node_feature_dim=27, edge_feature_dim=2, use_edge_features=True,
                      output_dim=1, loss_type="bce", dropout=0.1, device="cuda")
    seq = [(x.to(dev), ei.to(dev), ea.to(dev), ids) for x, ei, ea, ids in _rand_seq([500] * 6, 27, 2, 10, 9)]
    grads = []
    for _ in range(2):
        torch.manual_seed(11)
        model = TAGAN(cfg).to(dev).train()
        torch.manual_seed(12)
        out = model(seq, labels=torch.tensor([1.0], device=dev))
        out["loss"].backward()
        grads.append(torch.cat([p.grad.flatten() for p in model.parameters() if p.grad is not None]))
    assert torch.equal(grads[0], grads[1]), "backward is not bitwise reproducible"
    assert torch.isfinite(grads[0]).all()


# ----------------------------------------------------------------------------- chunked work decomposition
def _hub_graph(n, seed):
    """Random graph plus a hub (node 0 <-> everyone): rows and columns far longer than one chunk."""
    g = torch.Generator().manual_seed(seed)
    ei = torch.randint(0, n, (2, 4 * n), generator=g)
    hub = torch.stack([torch.zeros(n, dtype=torch.long), torch.arange(n)])
    return torch.cat([ei, hub, hub.flip(0)], 1)


@pytest.mark.parametrize("cold", [False, True])
@pytest.mark.parametrize("metric", list(oracle.METRICS))
@pytest.mark.parametrize("chunk", [4, 16, 128])
def test_geo_kernel_chunked_vs_oracle(dev, metric, chunk, cold, monkeypatch):
    """Multi-chunk rows/columns (merge passes) against the float64 oracle edge-softmax.  ``cold``: the batch
    classified cache-cold (TAGAN_GEO_COLD=1; C3-C5 are): launch block order and the fp32 forward with 4 features
    per lane instead of 8."""
    monkeypatch.setenv("TAGAN_GEO_COLD", "1" if cold else "0")
    from tagan_amd import _lib
    from tagan_amd.kernels import GeoAttnFn, build_graph
    counts = [300, 257]
    H, heads = 128, 8
    eis = [_hub_graph(n, 5 + i) for i, n in enumerate(counts)]
    graph = build_graph([e.to(dev) for e in eis], counts, chunk=chunk)
    N = sum(counts)
    g = torch.Generator().manual_seed(1)
    qkv = (torch.randn(N, 3 * H, generator=g) * 0.5)
    param = torch.linspace(0.7, 1.3, heads) if metric in ("gaussian_kernel", "rbf_kernel") else None
    x = qkv.to(dev).requires_grad_(True)
    pd = param.to(dev).requires_grad_(True) if param is not None else None
    out = GeoAttnFn.apply(x, pd, graph, _lib.METRIC_IDS[metric], heads, 0.0, 0)
    gout = torch.randn(N, H, generator=g)
    (out * gout.to(dev)).sum().backward()
    # oracle: block-diagonal CSR of the same snapshots, float64
    rps, cols, off = [], [], 0
    for n, ei in zip(counts, eis):
        rp, c = oracle.csr_from_edge_index(ei, n)
        rps.append(rp[:-1] + (sum(len(x) for x in cols)))
        cols.append(c + off)
        off += n
    rowptr = torch.cat(rps + [torch.tensor([sum(len(x) for x in cols)])])
    col = torch.cat(cols)
    q64 = qkv.double().requires_grad_(True)
    p64 = param.double().requires_grad_(True) if param is not None else None
    P = {"m.distance_param": p64} if p64 is not None else {}
    d = H // heads
    q = q64[:, :H].view(1, N, heads, d).transpose(1, 2)
    k = q64[:, H:2 * H].view(1, N, heads, d).transpose(1, 2)
    v = q64[:, 2 * H:].view(1, N, heads, d).transpose(1, 2)
    ctx = oracle.tagan_oracle._sparse_context(q, k, v, metric, P, "m", p64 is not None, None, (rowptr, col))
    ref = ctx.transpose(1, 2).reshape(N, H)
    (ref * gout.double()).sum().backward()
    G.assert_close("out", out, ref, OUT_ATOL, OUT_RTOL)
    G.assert_close("dqkv", x.grad, q64.grad, GRAD_ATOL, GRAD_RTOL)
    if param is not None:
        G.assert_close("dparam", pd.grad, p64.grad, 1e-3, 1e-3)


def test_geo_kernel_dropout_matches_regenerated_mask(dev):
    """Dropout on attention weights: the kernel's counter-based mask, regenerated on the host, reproduces it."""
    import numpy as np
    from tagan_amd import _lib
    from tagan_amd.kernels import GeoAttnFn, build_graph
    from test_abi import _drop_uniform
    n, H, heads, p, seed = 400, 64, 4, 0.3, 987654321
    ei = _hub_graph(n, 3)
    graph = build_graph([ei.to(dev)], [n], chunk=16)
    g = torch.Generator().manual_seed(2)
    qkv = torch.randn(n, 3 * H, generator=g) * 0.5
    x = qkv.to(dev).requires_grad_(True)
    out = GeoAttnFn.apply(x, None, graph, 0, heads, p, seed)
    gout = torch.randn(n, H, generator=g)
    (out * gout.to(dev)).sum().backward()
    rowptr, col = oracle.csr_from_edge_index(ei, n)
    E = col.numel()
    u = _drop_uniform(seed, np.arange(heads, dtype=np.uint64)[None, :], np.arange(E, dtype=np.uint32)[:, None])
    keep = torch.from_numpy((u >= p).astype(np.float64)) / (1 - p)
    q64 = qkv.double().requires_grad_(True)
    d = H // heads
    src = torch.repeat_interleave(torch.arange(n), rowptr.diff())
    qf, kf, vf = (q64[:, i * H:(i + 1) * H].view(n, heads, d) for i in range(3))
    s = -torch.sqrt(((qf[src] - kf[col]) ** 2).sum(-1) + 1e-8)
    m = torch.full((n, heads), float("-inf"), dtype=torch.float64).scatter_reduce(
        0, src[:, None].expand(-1, heads), s, reduce="amax")
    e = torch.exp(s - m[src])
    a = e / torch.zeros(n, heads, dtype=torch.float64).index_add(0, src, e)[src]
    ref = torch.zeros(n, heads, d, dtype=torch.float64).index_add(0, src, (a * keep)[:, :, None] * vf[col])
    ref = ref.reshape(n, H)
    (ref * gout.double()).sum().backward()
    G.assert_close("out", out, ref, OUT_ATOL, OUT_RTOL)
    G.assert_close("dqkv", x.grad, q64.grad, GRAD_ATOL, GRAD_RTOL)


@pytest.mark.parametrize("chunk", [4, 64])
def test_chunk_order_is_a_length_sorted_permutation_and_results_do_not_depend_on_it(dev, chunk, monkeypatch):
    """tagan_chunk_order: a permutation of the real chunks, windows of 2^ORDER_BITS segments in order,
    longest chunk first inside a window; the edge kernels give bitwise-identical outputs and gradients
    in that order and in plain row order (every chunk's output / partial slot is fixed by its index)."""
    from tagan_amd import kernels
    from tagan_amd.kernels import GeoAttnFn, build_graph
    monkeypatch.setattr(kernels, "ORDER_BITS", 6)     # several windows at this size
    counts = [300, 257, 190]
    eis = [_hub_graph(n, 11 + i) for i, n in enumerate(counts)]
    N, H, heads = sum(counts), 64, 4
    g = torch.Generator().manual_seed(3)
    qkv = torch.randn(N, 3 * H, generator=g) * 0.5
    gout = torch.randn(N, H, generator=g).to(dev)
    res = []
    for flag in ("1", "0"):
        monkeypatch.setenv("TAGAN_CHUNK_ORDER", flag)
        graph = build_graph([e.to(dev) for e in eis], counts, chunk=chunk)
        if flag == "1":
            for chunks, order, ptr_ in ((graph.row_chunks, graph.row_order, graph.rowptr),
                                        (graph.col_chunks, graph.col_order, graph.csc_ptr)):
                n_ch = int(chunks[5][0])
                o = order[:n_ch].cpu().long()
                assert torch.equal(o.sort().values, torch.arange(n_ch))
                seg, beg = chunks[1][:n_ch].cpu().long(), chunks[2][:n_ch].cpu().long()
                cnt = torch.minimum(torch.full_like(seg, chunk), ptr_.cpu().long()[seg + 1] - beg)
                key = (seg[o] >> 6) * 256 + (255 - cnt[o])
                assert bool((key[1:] >= key[:-1]).all())
        else:
            assert graph.row_order is None
        x = qkv.to(dev).requires_grad_(True)
        out = GeoAttnFn.apply(x, None, graph, 0, heads, 0.1, 77)
        (out * gout).sum().backward()
        res.append((out.detach(), x.grad))
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1])


@pytest.mark.parametrize("metric", ["euclidean", "cosine_similarity", "manhattan", "gaussian_kernel"])
@pytest.mark.parametrize("chunk", [4, 64])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_geo_backward_orders_are_bitwise_identical(dev, metric, chunk, dtype):
    """Column-first backward (node pass -> CSC pass storing dS per edge -> CSR pass from dS, gathering K only)
    against the row-first order (graph without nnz_cap): same delta, same dS bits, so dq, dk, dv and the metric
    parameter gradient are bitwise identical, with dropout, hub rows split over many chunks, and bf16 storage."""
    from tagan_amd import _lib
    from tagan_amd.fused import GeoCore
    from tagan_amd.kernels import build_graph
    counts = [300, 257]
    eis = [_hub_graph(n, 21 + i) for i, n in enumerate(counts)]
    N, H, heads = sum(counts), 128, 8
    g = torch.Generator().manual_seed(4)
    qkv = (torch.randn(N, 3 * H, generator=g) * 0.5).to(dev, dtype)
    gout = torch.randn(N, H, generator=g).to(dev, dtype)
    param = torch.linspace(0.7, 1.3, heads).to(dev) if metric == "gaussian_kernel" else None
    graph = build_graph([e.to(dev) for e in eis], counts, chunk=chunk)
    assert graph.nnz_cap > 0
    core = GeoCore(graph, _lib.METRIC_IDS[metric], heads, 0.1, 1234)
    L = _lib.lib()
    res = []
    for mode in (1, 0):                                # column-first, then row-first
        prev = L.tagan_geo_set_bwd_order(mode)
        try:
            out, saved = core.fwd(qkv, param, None)
            dqkv, dprm, _ = core.bwd(qkv, out, saved, gout, param is not None, False)
            torch.cuda.synchronize()
        finally:
            L.tagan_geo_set_bwd_order(prev)
        res.append((out, dqkv, dprm))
    assert torch.equal(res[0][0], res[1][0])
    assert torch.isfinite(res[0][1].float()).all()
    assert torch.equal(res[0][1], res[1][1])
    if param is not None:
        assert torch.equal(res[0][2], res[1][2])


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_geo_block_order_does_not_change_results(dev, dtype, monkeypatch):
    """The edge chunk kernels' block order (geo_attn.hip geo_xcd_mode: 0 launch order, 1 XCD eighths of the
    capacity-sized grid, 2 XCD eighths of the valid blocks; chosen by working set) only decides WHICH workgroup runs a
    chunk: every chunk's output / partial slot is fixed by its index, so outputs and gradients are bitwise identical
    in all three orders, with hub rows over many chunks, dropout and both storage types."""
    from tagan_amd import _lib
    from tagan_amd.fused import GeoCore
    from tagan_amd.kernels import build_graph
    counts = [300, 257, 190]
    eis = [_hub_graph(n, 31 + i) for i, n in enumerate(counts)]
    N, H, heads = sum(counts), 128, 8
    g = torch.Generator().manual_seed(5)
    qkv = (torch.randn(N, 3 * H, generator=g) * 0.5).to(dev, dtype)
    gout = torch.randn(N, H, generator=g).to(dev, dtype)
    graph = build_graph([e.to(dev) for e in eis], counts, chunk=16)
    core = GeoCore(graph, _lib.METRIC_IDS["euclidean"], heads, 0.1, 4321)
    res = []
    for mode in ("0", "1", "2"):
        monkeypatch.setenv("TAGAN_GEO_XCD", mode)
        out, saved = core.fwd(qkv, None, None)
        dqkv, _, _ = core.bwd(qkv, out, saved, gout, False, False)
        torch.cuda.synchronize()
        res.append((out, dqkv))
    assert torch.isfinite(res[0][1].float()).all()
    for out, dqkv in res[1:]:
        assert torch.equal(out, res[0][0])
        assert torch.equal(dqkv, res[0][1])
