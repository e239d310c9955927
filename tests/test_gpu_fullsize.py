"""Correctness at every BASELINE.json workload at its full size.

* C2 (10k nodes, 100k Zipf(1.1) edges/snapshot, 32 snapshots, H=128, 8 heads) — the bench's own
  workload (``synthetic.make_sequence("c2", seed=1000)``, dropout 0): the whole TAGAN forward + backward
  through the HIP path against the fp64 CPU oracle (logits, loss, every parameter gradient, every
  d(node features)) at the north_star's 1e-4 (model.py:158-473, graph_attention.py:96-105,
  geometric_attention.py:378-401, temporal_attention.py:985-1205).
* C3 / C4 / C5 (100k-1M nodes, 2M-20M edges per snapshot) are far beyond what the oracle can run
  whole, so at full size they are checked through properties plus sampled-row oracle comparisons:
    - the device CSR of two snapshots equals the host ``unique`` of their edges, bit for bit
      (64-bit sort keys at C4: N·N_snapshot ≥ 2³²);
    - the per-row softmax of the edge kernel sums to 1 on sampled rows;
    - geometric layer 0 (+ the skip LayerNorm) on 2,048 sampled query rows against the fp64 oracle
      run on exactly those rows and their gathered neighbours, forward and backward (the output
      gradient is non-zero only on the sampled rows, so every gradient is a function of them alone);
    - the temporal attention on 2,048 sampled node rows against the fp64 oracle on their T-windows,
      forward and backward (T = 64 / 16 / 128 rows of 100k / 1M / 100k nodes);
    - the whole model, forward + backward with dropout 0.1, finite and bitwise reproducible.
  C5 is the 8-GPU snapshot-sharded configuration: its geometric stage is checked on one rank's share
  (128 / 8 = 16 snapshots of 100k nodes), its temporal stage at the full T = 128 over all 100k rows.

Observed errors land in $TAGAN_PARITY_LOG (profiles/parity_errors_r02.json).
"""
import pytest
import torch
import torch.nn.functional as F

import golden_io as G
import oracle

pytestmark = pytest.mark.gpu

OUT_ATOL, OUT_RTOL = 1e-4, 1e-4
GRAD_ATOL, GRAD_RTOL = 1e-4, 1e-4
# normwise relative error bound of each gradient tensor: the element-wise atol is vacuous for the tiny
# gradients of a scalar loss over 10^5-10^7 rows, so every tensor is also held to 1e-4 in norm
NORM_REL = 1e-4
# analytically zero gradients (fp32 noise against fp64 noise): scaled-dot attention is invariant to a shift
# of k by a per-head constant, so d(k bias) = 0 exactly (temporal_attention.py:1006 scores = q·kᵀ/√d)
ZERO_GRADS = ("temporal_attention.k_linear.bias",)
# ill-conditioned in ANY fp32 implementation (written exception): the attention-pool bias gradient
# is Σ_t dscore_t·(1 - tanh²)·w₂ where the softmax backward makes Σ_t dscore_t = 0 (classification.py:856-966),
# so it is a small difference of larger terms.  The CPU fp32 oracle itself lands at 1.72e-4 normwise vs fp64 on
# this exact tensor at C2 (tools/fp32_conditioning.py -> profiles/r2_fp32_conditioning.json); the HIP path is
# held to 2x that in norm and to the full 1e-4 element-wise bound.
COND_GRADS = {"classification_head.classification_head.attention.0.bias": 3.5e-4}
SAMPLE = 2048


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import tagan_amd  # noqa: F401
    return torch.device("cuda:0")


def _free():
    import gc
    import sys
    # a failed test's traceback (sys.last_traceback, kept by pytest) pins its frames and their 10-100 GB of
    # device tensors: drop it so one failure does not turn every later full-size test into an OOM
    sys.last_type = sys.last_value = sys.last_traceback = None
    gc.collect()
    torch.cuda.empty_cache()


@pytest.fixture(autouse=True)
def _clean_device():
    _free()
    yield
    _free()


def _p64(module, prefix=""):
    return {prefix + k: v.detach().cpu().double().requires_grad_(v.is_floating_point())
            for k, v in module.state_dict().items()}


def _close_grad(name, got, want):
    G.assert_close(name, got, want, GRAD_ATOL, GRAD_RTOL)
    if any(name.endswith(z) for z in ZERO_GRADS):
        return
    nr = G.normwise_rel(got, want)
    bound = next((b for k, b in COND_GRADS.items() if name.endswith(k)), NORM_REL)
    assert nr <= bound, "%s: normwise rel %.3e" % (name, nr)


def _unit_grad(shape, gen, dev):
    """Upstream gradient on the sampled rows, normalised to unit Frobenius norm -- the scale of a mean-reduced
    loss over those rows.  With an O(1)-per-element randn upstream gradient summed over 10^5 rows x T, every
    parameter gradient is ~10^2-10^3 in size and an absolute 1e-4 bound becomes a 10^-7 relative one, tighter
    than fp32 rounding of the result itself; the normwise check (scale-free) is unchanged by this."""
    g = torch.randn(*shape, generator=gen, dtype=torch.float64)
    return (g / g.norm()).float().to(dev)


def _segments(rp, rows):
    """Flat CSR positions of the given rows: (positions, owner index into rows, counts)."""
    beg, cnt = rp[rows], rp[rows + 1] - rp[rows]
    owner = torch.repeat_interleave(torch.arange(rows.numel(), device=rows.device), cnt)
    start = torch.cumsum(cnt, 0) - cnt
    pos = beg[owner] + torch.arange(owner.numel(), device=rows.device) - start[owner]
    return pos, owner, cnt


# ----------------------------------------------------------------------------- C2 whole model
_C2_REF = {}


def _c2_oracle(model, seq, labels, cfg):
    """The fp64 oracle on the C2 workload (logits, loss, every parameter and input gradient), computed once per
    session: the fp32 and the bf16 tests share it (same seeds, same weights)."""
    if "ref" not in _C2_REF:
        P = _p64(model)
        seq64 = [(x.detach().cpu().double().requires_grad_(True), ei.cpu(), None, ids) for x, ei, _, ids in seq]
        ref = oracle.tagan_forward(P, cfg.to_dict(), seq64, labels.cpu().double())
        ref["loss"].backward()
        _C2_REF["ref"] = ({"logits": ref["logits"].detach(), "loss": ref["loss"].detach()},
                          {k: (None if v.grad is None else v.grad.detach()) for k, v in P.items()},
                          [x64.grad.detach() for x64, _, _, _ in seq64])
    return _C2_REF["ref"]


def _c2_run(dev, precision):
    from tagan_amd import TAGAN, synthetic
    cfg = synthetic.config_for("c2", dropout=0.0)
    torch.manual_seed(0)
    model = TAGAN(cfg, precision=precision).to(dev).train()
    seq = synthetic.make_sequence("c2", dev, seed=1000)
    seq = [(x.clone().requires_grad_(True), ei, ea, ids) for x, ei, ea, ids in seq]
    labels = torch.tensor([1.0], device=dev)
    out = model(seq, labels=labels)
    out["loss"].backward()
    return cfg, model, seq, labels, out


@pytest.mark.timeout(900)
def test_c2_full_model_vs_oracle(dev):
    cfg, model, seq, labels, out = _c2_run(dev, "fp32")
    ref, pgrad, xgrad = _c2_oracle(model, seq, labels, cfg)
    G.assert_close("logits", out["logits"], ref["logits"], OUT_ATOL, OUT_RTOL)
    G.assert_close("loss", out["loss"].reshape(1), ref["loss"].reshape(1), OUT_ATOL, OUT_RTOL)
    n_checked = 0
    for name, p in model.named_parameters():
        if pgrad[name] is not None:
            _close_grad("grad " + name, p.grad, pgrad[name])
            n_checked += 1
        else:
            assert p.grad is None or float(p.grad.abs().max()) == 0.0, name
    assert n_checked >= 30
    for t, ((x, _, _, _), g64) in enumerate(zip(seq, xgrad)):
        _close_grad("grad x.%d" % t, x.grad, g64)


# bf16 mode (BASELINE's C2 dtype; fused.py "bf16": activations stored in bf16 between kernels, fp32 math and
# accumulation inside every kernel, bf16 GEMM operands) against the same fp64 oracle.  Tolerance per tensor t,
# derived from the bf16 roundings on its dependency path:
#     bound_t = SAFETY * U_RMS * max(kappa_t, 1)
#   U_RMS   = 2^-8 / sqrt(3): RMS relative error of one round-to-nearest store to bf16 (8 significant bits, error
#             uniform within half an ulp);
#   kappa_t = sqrt(sum_s kappa_{t,s}^2) over the 24 store sites s of the mode (per attention block: h = LN1(x),
#             Q|K|V, the attention output, the rounded W_qkv and W_o, d(out-projection output), d(context),
#             dQ|dK|dV), kappa_{t,s} = t's relative condition number for elementwise relative perturbations at s:
#             measured on this workload by tools/bf16_conditioning.py with the fp64 oracle (16 draws of every site
#             perturbed at once, tests/golden/bf16_conditioning.json "kappa_rss"); to first order the normwise
#             error of t has RMS U_RMS * kappa_t;
#   SAFETY  = 4: a 4-sigma tail of that error;
#   max(., 1): the head's scalar-like gradients (classifier biases, the loss) measure up to 4.5 U_RMS * kappa_t on
#             the GPU, more than the first-order model predicts for them (profiles/r4j_parity_errors.json): their
#             kappa is floored at one rounding's worth.
# Written exceptions: the analytically zero gradients (golden_io.ANALYTIC_ZERO: noise on both sides, checked to be
# zero) and the ill-conditioned attention-pool bias (COND_GRADS: its fp32 oracle already carries a 1.7e-4
# normwise error, i.e. a ~2900x amplification of fp32 rounding -- at bf16 precision that tensor has no correct
# digits in ANY bf16 implementation; it is held to the element-wise bound only).
U_RMS = 2.0 ** -8 / 3 ** 0.5
SAFETY = 4.0


def _kappa():
    import json
    import os
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "bf16_conditioning.json")) as f:
        return json.load(f)["kappa_rss"]


def _bf16_bound(kappa, key):
    return SAFETY * U_RMS * max(kappa[key], 1.0)


@pytest.mark.timeout(900)
def test_c2_bf16_vs_oracle(dev):
    cfg, model, seq, labels, out = _c2_run(dev, "bf16")
    # the oracle runs on the fp32 master weights (the same initialisation as the fp32 test)
    ref, pgrad, xgrad = _c2_oracle(model, seq, labels, cfg)
    kappa = _kappa()
    for key, got, want in (("logits", out["logits"], ref["logits"]),
                           ("loss", out["loss"].reshape(1), ref["loss"].reshape(1))):
        bound_out = _bf16_bound(kappa, key)
        nr = G.normwise_rel(got, want)
        G.ERRORS.setdefault("test_c2_bf16_vs_oracle", {})[key] = [nr, bound_out]
        assert nr <= bound_out, "%s: bf16 normwise %.3e > %.3e" % (key, nr, bound_out)
    n_checked = 0
    worst = (0.0, None)
    for name, p in model.named_parameters():
        if pgrad[name] is None:
            continue
        n_checked += 1
        if G.declared_zero("grad " + name) and float(pgrad[name].abs().max()) <= GRAD_ATOL:
            assert float(p.grad.abs().max()) <= 1e-3, name    # bf16 noise around an exact zero
            continue
        if any(name.endswith(k) for k in COND_GRADS):
            G.assert_close("grad " + name, p.grad, pgrad[name], GRAD_ATOL, GRAD_RTOL, norm_rtol=float("inf"))
            continue
        bound = _bf16_bound(kappa, "grad " + name)
        nr = G.normwise_rel(p.grad, pgrad[name])
        G.ERRORS.setdefault("test_c2_bf16_vs_oracle", {})["grad " + name] = [nr, bound]
        worst = max(worst, (nr / bound, name))
        assert nr <= bound, "grad %s: bf16 normwise %.3e > %.3e" % (name, nr, bound)
    assert n_checked >= 30
    bound_x = _bf16_bound(kappa, "grad x")
    for t, ((x, _, _, _), g64) in enumerate(zip(seq, xgrad)):
        nr = G.normwise_rel(x.grad, g64)
        G.ERRORS.setdefault("test_c2_bf16_vs_oracle", {})["grad x.%d" % t] = [nr, bound_x]
        assert nr <= bound_x, "grad x.%d: bf16 normwise %.3e > %.3e" % (t, nr, bound_x)
    print("bf16 C2: worst normwise / bound = %.3f (%s)" % worst)


# ----------------------------------------------------------------------------- C3 / C5 geometry, whole model
# The full T / hidden / heads of C3 (T 64, H 256, 8 heads) and C5 (T 128, H 256, 16 heads) with the node count cut
# (degree kept at 20) so the fp64 oracle runs the whole model: every layer (both geometric layers on the H = 256
# stream GEMMs, the v5 temporal kernel, pooling, head, loss) forward and backward against it at the north_star's
# 1e-4, like the C2 test above.
GEOMETRY = {"c3": (1500, 30_000), "c5": (800, 16_000)}


@pytest.mark.timeout(900)
@pytest.mark.parametrize("name", ["c3", "c5"])
def test_geometry_whole_model_vs_oracle(dev, name):
    from tagan_amd import synthetic
    nodes, edges = GEOMETRY[name]
    cfg, model = _model(name, dev)
    seq = synthetic.make_sequence(name, dev, seed=2024, nodes=nodes, edges=edges)
    seq = [(x.clone().requires_grad_(True), ei, ea, ids) for x, ei, ea, ids in seq]
    labels = torch.tensor([1.0], device=dev)
    out = model(seq, labels=labels)
    out["loss"].backward()
    P = _p64(model)
    seq64 = [(x.detach().cpu().double().requires_grad_(True), ei.cpu(), None, ids) for x, ei, _, ids in seq]
    ref = oracle.tagan_forward(P, cfg.to_dict(), seq64, labels.cpu().double())
    ref["loss"].backward()
    G.assert_close("%s logits" % name, out["logits"], ref["logits"].detach(), OUT_ATOL, OUT_RTOL)
    G.assert_close("%s loss" % name, out["loss"].reshape(1), ref["loss"].detach().reshape(1), OUT_ATOL, OUT_RTOL)
    n_checked = 0
    for pname, p in model.named_parameters():
        want = P[pname].grad
        if want is not None:
            _close_grad("grad " + pname, p.grad, want)
            n_checked += 1
        else:
            assert p.grad is None or float(p.grad.abs().max()) == 0.0, pname
    assert n_checked >= 30
    for t, ((x, _, _, _), (x64, _, _, _)) in enumerate(zip(seq, seq64)):
        _close_grad("grad x.%d" % t, x.grad, x64.grad)


# ----------------------------------------------------------------------------- C3-C5 sampled checks
FULL = {
    # name: snapshots on this GPU for the geometric stage (C5: one rank's share of the 8-GPU shard)
    "c3": 64, "c4": 16, "c5": 16,
}


def _model(name, dev, dropout=0.0, precision="fp32"):
    from tagan_amd import TAGAN, synthetic
    cfg = synthetic.config_for(name, dropout=dropout)
    torch.manual_seed(0)
    model = TAGAN(cfg, precision=precision).to(dev).train()
    with torch.no_grad():   # non-trivial LayerNorm affine parameters (init is 1 / 0)
        g = torch.Generator(device=dev).manual_seed(3)
        for n, p in model.named_parameters():
            if "layer_norm" in n:
                p.add_(0.1 * torch.randn(p.shape, device=dev, generator=g))
    return cfg, model


def _sample_rows(graph, n_total, k, gen):
    """k random query rows plus the longest CSR row (a hub: multi-chunk merge path)."""
    deg = graph.rowptr[1:] - graph.rowptr[:-1]
    hub = int(torch.argmax(deg))
    rows = torch.randint(0, n_total, (k - 1,), generator=gen).to(graph.rowptr.device)
    return torch.unique(torch.cat([rows, torch.tensor([hub], device=rows.device)]))


def _local_csr(graph, rows):
    """CSR over U = rows ∪ neighbours(rows) in local ids: the sampled rows keep their full neighbour list,
    every other node of U only its self-loop (its output is not checked and gets a zero gradient)."""
    pos, own, _ = _segments(graph.rowptr.long(), rows)
    nbr = graph.col[pos].long()
    U = torch.unique(torch.cat([rows, nbr]))
    loc = torch.searchsorted(U, rows)
    owner = loc[own]
    lnbr = torch.searchsorted(U, nbr)
    is_row = torch.zeros(U.numel(), dtype=torch.bool, device=U.device)
    is_row[loc] = True
    others = (~is_row).nonzero().flatten()
    src = torch.cat([owner, others])
    dst = torch.cat([lnbr, others])
    key = torch.sort(src * U.numel() + dst).values
    src, dst = key // U.numel(), key % U.numel()
    rowptr = torch.zeros(U.numel() + 1, dtype=torch.long, device=U.device)
    rowptr[1:] = torch.cumsum(torch.bincount(src, minlength=U.numel()), 0)
    return U, loc, rowptr.cpu(), dst.cpu()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("name", ["c3", "c4", "c5"])
def test_fullsize_csr_softmax_and_geometric_rows(dev, name):
    from tagan_amd import _lib, synthetic
    from tagan_amd.kernels import build_graph, geo_edge_alpha
    N, E, T, H, heads = synthetic.CONFIGS[name][:5]
    Tg = FULL[name]
    cfg, model = _model(name, dev)
    seq = synthetic.make_sequence(name, dev, seed=1000, snapshots=Tg)
    graph = build_graph([ei for _, ei, _, _ in seq], [N] * Tg)
    # (1) device CSR of two snapshots == host unique of their edges (bit-exact)
    for t in (0, Tg - 1):
        rp, col = oracle.csr_from_edge_index(seq[t][1].cpu(), N)
        rp_gpu = graph.rowptr[t * N:(t + 1) * N + 1].cpu().long()
        assert torch.equal(rp_gpu - rp_gpu[0], rp), "rowptr of snapshot %d" % t
        assert torch.equal(graph.col[int(rp_gpu[0]):int(rp_gpu[-1])].cpu().long() - t * N, col), "col %d" % t
    x_cat = torch.cat([x for x, _, _, _ in seq])
    del seq
    gen = torch.Generator().manual_seed(7)
    rows = _sample_rows(graph, N * Tg, SAMPLE, gen)
    layer = model.geometric_attention_layers[0]
    ga = layer.geometric_attention
    with torch.no_grad():
        h0 = F.linear(x_cat, model.node_embedding.weight, model.node_embedding.bias)
    del x_cat
    # (2) per-row softmax sums to 1 on the sampled rows (edge kernel's alpha output, dropout 0)
    with torch.no_grad():
        hn = F.layer_norm(h0, (H,), ga.layer_norm1.weight, ga.layer_norm1.bias, ga.layer_norm1.eps)
        w = torch.cat([ga.q_linear.weight, ga.k_linear.weight, ga.v_linear.weight])
        b = torch.cat([ga.q_linear.bias, ga.k_linear.bias, ga.v_linear.bias])
        qkv = torch.addmm(b, hn, w.t())
        del hn
        alpha = geo_edge_alpha(qkv, graph, _lib.METRIC_IDS["euclidean"], heads)
        del qkv
        pos, seg, _ = _segments(graph.rowptr.long(), rows)
        sums = torch.zeros(rows.numel(), heads, device=dev, dtype=torch.float64).index_add_(
            0, seg, alpha[pos].double())
        del alpha
    G.assert_close("softmax row sums", sums, torch.ones_like(sums), 1e-5, 0.0)
    _free()
    # (3) geometric layer 0 (+ skip LN) on the sampled rows vs the fp64 oracle on their neighbourhoods
    h0.requires_grad_(True)
    y = layer.forward_graph(h0, graph, skip_ln=model.skip_layer_norm)
    gy = torch.zeros_like(y)
    gy[rows] = _unit_grad((rows.numel(), H), gen, dev)
    (y * gy).sum().backward()
    U, loc, rowptr_l, col_l = _local_csr(graph, rows)
    P = _p64(model)
    hl = h0.detach()[U].cpu().double().requires_grad_(True)
    sub = "geometric_attention_layers.0.geometric_attention"
    ref = oracle.geometric_attention(hl.unsqueeze(0), P, sub, heads, "euclidean", True, False,
                                     mode="sparse", csr=(rowptr_l, col_l)).squeeze(0)
    ref = ref + F.layer_norm(hl, (H,), P["skip_layer_norm.weight"], P["skip_layer_norm.bias"], 1e-5)
    lc = loc.cpu()
    G.assert_close("layer0 rows", y.detach()[rows], ref[lc], OUT_ATOL, OUT_RTOL)
    gl = torch.zeros(U.numel(), H, dtype=torch.float64)
    gl[lc] = gy[rows].cpu().double()
    (ref * gl).sum().backward()
    _close_grad("layer0 dx (rows + neighbours)", h0.grad[U], hl.grad)
    assert float(h0.grad.index_fill_(0, U, 0.0).abs().max()) == 0.0, "gradient outside the sampled neighbourhoods"
    for n, p in list(layer.named_parameters()) + [("skip." + k, v) for k, v in
                                                  model.skip_layer_norm.named_parameters()]:
        key = ("geometric_attention_layers.0." + n) if not n.startswith("skip.") else "skip_layer_norm." + n[5:]
        _close_grad("grad " + key, p.grad, P[key].grad)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("name", ["c3", "c4", "c5"])
def test_fullsize_temporal_rows(dev, name):
    """The temporal stage at full T over all N node rows; 2,048 sampled rows vs the fp64 oracle."""
    from tagan_amd import synthetic
    N, E, T, H, heads = synthetic.CONFIGS[name][:5]
    cfg, model = _model(name, dev)
    ta = model.temporal_attention
    g = torch.Generator(device=dev).manual_seed(11)
    xt = torch.randn(T, N, H, device=dev, generator=g).requires_grad_(True)
    out, _ = ta.forward_time_major(xt, True, False)
    gen = torch.Generator().manual_seed(5)
    rows = torch.unique(torch.randint(0, N, (SAMPLE - 1,), generator=gen).to(dev))
    rows = torch.unique(torch.cat([rows, torch.tensor([N - 1], device=dev)]))
    gy = torch.zeros_like(out)
    gy[:, rows] = _unit_grad((T, rows.numel(), H), gen, dev)
    (out * gy).sum().backward()
    P = _p64(ta, "temporal_attention.")
    x64 = xt.detach()[:, rows].permute(1, 0, 2).cpu().double().requires_grad_(True)
    ref = oracle.temporal_attention(x64, P, "temporal_attention", heads, cls="asym",
                                    causal=cfg.causal_attention, relative_position_bias=cfg.asymmetric_temporal_bias,
                                    asymmetric_window_size=cfg.window_size, attention_mask=torch.ones(T, T))
    G.assert_close("temporal rows", out.detach()[:, rows].permute(1, 0, 2), ref, OUT_ATOL, OUT_RTOL)
    (ref * gy[:, rows].permute(1, 0, 2).cpu().double()).sum().backward()
    _close_grad("temporal dx rows", xt.grad[:, rows].permute(1, 0, 2), x64.grad)
    assert float(xt.grad.index_fill_(1, rows, 0.0).abs().max()) == 0.0, "gradient outside the sampled rows"
    for n, p in ta.named_parameters():
        key = "temporal_attention." + n
        if P[key].grad is not None:
            _close_grad("grad " + key, p.grad, P[key].grad)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("name,precision", [("c3", "fp32"), ("c4", "fp32"), ("c5", "fp32"), ("c5", "bf16")])
def test_fullsize_model_finite_and_reproducible(dev, name, precision):
    """Whole TAGAN forward + backward at full size (C5: one rank's 16-snapshot share), training mode with
    the config's dropout 0.1: finite loss and gradients, and a second run with the same seeds is bitwise
    identical (atomic-free, fixed-order reductions; counter-based dropout).  C5 also in the bf16 activation mode
    (BASELINE's C5 dtype), whose one-plane stream GEMMs and weight gradients the fp32 run does not reach."""
    from tagan_amd import synthetic
    N = synthetic.CONFIGS[name][0]
    cfg, model = _model(name, dev, dropout=0.1, precision=precision)
    seq = synthetic.make_sequence(name, dev, seed=1000, snapshots=FULL[name])
    labels = torch.tensor([1.0], device=dev)
    runs = []
    for _ in range(2):
        model.zero_grad(set_to_none=True)
        torch.manual_seed(123)
        out = model(seq, labels=labels)
        out["loss"].backward()
        runs.append((out["loss"].detach().clone(), out["logits"].detach().clone(),
                     {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}))
        del out
        _free()
    (l0, z0, g0), (l1, z1, g1) = runs
    assert torch.isfinite(l0).all() and torch.isfinite(z0).all()
    assert len(g0) >= 30 and all(bool(torch.isfinite(v).all()) for v in g0.values())
    assert torch.equal(l0, l1) and torch.equal(z0, z1)
    assert sorted(g0) == sorted(g1)
    for n in g0:
        assert torch.equal(g0[n], g1[n]), "gradient of %s is not bitwise reproducible at %s" % (n, name)
    assert N * FULL[name] >= 1_600_000
