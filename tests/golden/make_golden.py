"""Mint golden vectors for the TAGAN hot path from the reference itself.

CONTAINER-ONLY TOOL.  It imports the read-only reference checkout at
``/root/reference`` (``src.tagan``), runs it on seeded inputs and writes small
fixtures next to this file:

    <case>.pt    tensors only (load with ``torch.load(..., weights_only=True)``)
    <case>.json  metadata: config kwargs, input layout, reference file:line anchors

It never runs on the GPU box (the reference does not travel) and nothing in the
product imports it.  Import hygiene follows SURVEY.md §8c: bytecode writing off,
scratch cwd (``debug_utils`` creates ``./debug_output`` on import), stdout/stderr
swallowed (the reference prints on every call), dropout = 0 for value parity.

Cases (SURVEY.md §8c G1–G5):
  e2e_*        TAGAN.forward + loss.backward (model.py:158-473) — inputs, state_dict,
               per-snapshot geometric outputs, temporal output, graph_features,
               logits, loss, every parameter grad and d(node features).
  gat_*        TAGANGraphAttention (graph_attention.py:61-133) per distance metric,
               duplicate edges / explicit self-loops / isolated nodes.
  geo_*        GeometricAttention standalone (dense mask, no mask, geometric_bias).
  tatt_*       AsymmetricTemporalAttention / TemporalAttention (temporal_attention.py).
  membank_*    NodeMemoryBank.update/get_states/update_state/decay_all traces.
  ingest_dict_* TAGAN.forward on the reference's snapshot DICTS (model.py:187-230; the format of
               preprocess_social_media.py:374-389): global user ids, a variable node count per snapshot,
               edge_attr absent or present, timestep keys — inputs from tagan_amd.synthetic.make_social_snapshots.
  tprop_*      TemporalPropagation's intended compute (G6): TemporalEvolutionLayer (GRU over T,
               time-aware / bidirectional), TemporalSkipConnection (mean/max/sum windows),
               TemporalGatingUnit, and the full forward with tensor masks — reachable only with a
               fixture-time ``NodeMemoryBank.__len__`` (the shipped class has none, so
               temporal_propagation.py:1505 raises TypeError).

Usage:  python tests/golden/make_golden.py [case-prefix ...]
"""
import contextlib
import io
import json
import os
import sys
import tempfile

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True

import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def _import_reference():
    if not os.path.isdir(REF):
        raise SystemExit("reference checkout not present; golden fixtures are committed")
    sys.path.insert(0, REF)
    cwd = os.getcwd()
    scratch = tempfile.mkdtemp(prefix="tagan_golden_")
    os.chdir(scratch)
    try:
        with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
            from src.tagan.model import TAGAN
            from src.tagan.utils.config import TAGANConfig
            from src.tagan.layers.graph_attention import TAGANGraphAttention
            from src.tagan.layers.geometric_attention import GeometricAttention
            from src.tagan.layers.temporal_attention import (
                TemporalAttention, AsymmetricTemporalAttention)
            from src.tagan.utils.memory_bank import NodeMemoryBank
            from src.tagan.layers.temporal_propagation import (
                TemporalPropagation, TemporalEvolutionLayer, TemporalSkipConnection, TemporalGatingUnit)
    finally:
        os.chdir(cwd)
    return dict(TAGAN=TAGAN, TAGANConfig=TAGANConfig, TAGANGraphAttention=TAGANGraphAttention,
                GeometricAttention=GeometricAttention, TemporalAttention=TemporalAttention,
                AsymmetricTemporalAttention=AsymmetricTemporalAttention,
                NodeMemoryBank=NodeMemoryBank, TemporalPropagation=TemporalPropagation,
                TemporalEvolutionLayer=TemporalEvolutionLayer, TemporalSkipConnection=TemporalSkipConnection,
                TemporalGatingUnit=TemporalGatingUnit)


def quiet(fn, *a, **k):
    with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
        return fn(*a, **k)


def save(case, tensors, meta):
    tensors = {k: (v.detach().contiguous().clone() if isinstance(v, torch.Tensor) else v)
               for k, v in tensors.items()}
    torch.save(tensors, os.path.join(HERE, case + ".pt"))
    with open(os.path.join(HERE, case + ".json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    nbytes = sum(v.numel() * v.element_size() for v in tensors.values() if isinstance(v, torch.Tensor))
    print(f"  {case}: {len(tensors)} tensors, {nbytes/1e6:.2f} MB")


# --------------------------------------------------------------------------- inputs
def make_sequence(n_list, F, De, seed, edges_per_node=2, zipf=False):
    """Seeded snapshot list in the reference's tuple format (model.py:187-230).

    Mirrors example.py:35-48: x ~ N(0,1), edge_index ~ U{0..N-1} (duplicates and
    self-loops allowed), edge_attr ~ N(0,1), node ids a permutation.
    """
    g = torch.Generator().manual_seed(seed)
    seq = []
    for N in n_list:
        x = torch.randn(N, F, generator=g)
        E = edges_per_node * N
        ei = torch.randint(0, N, (2, E), generator=g)
        ea = torch.randn(E, De, generator=g) if De > 0 else None
        ids = torch.randperm(N, generator=g).tolist()
        seq.append((x, ei, ea, ids))
    return seq


def make_edge_case_sequence(F, De, seed):
    """Edge cases of the adjacency semantics (graph_attention.py:96-105: adj[src, dst] = 1 over the edge list, then
    + eye(N)): a one-node snapshot and a twelve-node one without edges (self-loops only), duplicate edges, explicit
    self-loops and negative indices (torch indexing wraps them), a star hub (every node <-> node 0), a complete
    graph, and a plain random snapshot; ragged N throughout."""
    g = torch.Generator().manual_seed(seed)
    seq = []

    def snap(N, ei):
        x = torch.randn(N, F, generator=g)
        ea = torch.randn(ei.shape[1], De, generator=g)
        return (x, ei, ea, torch.randperm(N, generator=g).tolist())

    seq.append(snap(1, torch.zeros(2, 0, dtype=torch.int64)))
    seq.append(snap(12, torch.zeros(2, 0, dtype=torch.int64)))
    base = torch.randint(0, 40, (2, 60), generator=g)
    loops = torch.arange(0, 40, 4).repeat(2, 1)
    neg = torch.randint(-40, 0, (2, 10), generator=g)
    seq.append(snap(40, torch.cat([base, base[:, :20], loops, neg], 1)))
    j = torch.arange(1, 64)
    seq.append(snap(64, torch.cat([torch.stack([torch.zeros_like(j), j]), torch.stack([j, torch.zeros_like(j)])], 1)))
    a = torch.arange(24)
    seq.append(snap(24, torch.stack([a.repeat_interleave(24), a.repeat(24)])))
    seq.append(snap(37, torch.randint(0, 37, (2, 74), generator=g)))
    return seq


def seq_tensors(seq):
    t = {}
    for i, (x, ei, ea, ids) in enumerate(seq):
        t[f"in.x.{i}"] = x
        t[f"in.edge_index.{i}"] = ei
        if ea is not None:
            t[f"in.edge_attr.{i}"] = ea
        t[f"in.node_ids.{i}"] = torch.tensor(ids, dtype=torch.int64)
    return t


# --------------------------------------------------------------------------- e2e
def e2e_case(R, case, cfg_kw, n_list, seed, labels, with_attn=False, store_intermediate=True, seq_fn=None):
    cfg_kw = dict(cfg_kw)
    cfg_kw.setdefault("device", "cpu")
    cfg_kw.setdefault("dropout", 0.0)
    torch.manual_seed(seed)
    cfg = quiet(R["TAGANConfig"], **cfg_kw)
    model = quiet(R["TAGAN"], cfg)
    model.train()
    F = cfg.node_feature_dim
    De = cfg.edge_feature_dim
    seq = (seq_fn or (lambda: make_sequence(n_list, F, De if De > 0 else 8, seed + 1)))()
    n_list = [x.shape[0] for x, _, _, _ in seq]
    seq = [(x.clone().requires_grad_(True), ei, ea, ids) for (x, ei, ea, ids) in seq]

    geo_out, temporal_out, gf = [], [], []
    h1 = model.geometric_attention_layers[-1].register_forward_hook(
        lambda m, i, o: geo_out.append((o[0] if isinstance(o, tuple) else o).detach().clone()))
    h2 = model.temporal_attention.register_forward_hook(
        lambda m, i, o: temporal_out.append((o[0] if isinstance(o, tuple) else o).detach().clone()))
    h3 = model.classification_head.register_forward_hook(
        lambda m, i, o: gf.append(i[0].detach().clone()))
    out = quiet(model, seq, labels=labels, return_attention_weights=with_attn)
    h1.remove(); h2.remove(); h3.remove()
    loss = out["loss"]
    quiet(loss.backward)

    t = {}
    t.update(seq_tensors([(x.detach(), ei, ea, ids) for (x, ei, ea, ids) in seq]))
    for k, v in model.state_dict().items():
        t["sd." + k] = v
    if labels is not None:
        t["in.labels"] = labels
    for name, p in model.named_parameters():
        if p.grad is not None:
            t["grad." + name] = p.grad
    for i, (x, _, _, _) in enumerate(seq):
        t[f"grad.x.{i}"] = x.grad
    if store_intermediate:
        for i, o in enumerate(geo_out):
            t[f"out.geo.{i}"] = o
        t["out.temporal"] = temporal_out[0]
    t["out.graph_features"] = gf[0]
    t["out.logits"] = out["logits"]
    t["out.predictions"] = out["predictions"]
    t["out.loss"] = loss.detach().reshape(1)
    if with_attn:
        t["out.temporal_attention_weights"] = out["temporal_attention_weights"]
    meta = dict(kind="e2e", config=cfg_kw, n_list=list(n_list), seed=seed,
                T=len(n_list), labels=None if labels is None else labels.tolist(),
                labels_dtype=None if labels is None else str(labels.dtype),
                return_attention_weights=with_attn,
                n_geo_attn_weights=len(out.get("geometric_attention_weights", []) or []),
                grad_none=[n for n, p in model.named_parameters() if p.grad is None],
                anchors=["src/tagan/model.py:158-473", "src/tagan/layers/graph_attention.py:61-133",
                         "src/tagan/layers/geometric_attention.py:332-598",
                         "src/tagan/layers/temporal_attention.py:904-1205"])
    save(case, t, meta)


# --------------------------------------------------------------------------- layer units
METRICS = ["euclidean", "squared_euclidean", "manhattan", "cosine_similarity", "cosine_distance",
           "dot_product", "scaled_dot_product", "gaussian_kernel", "rbf_kernel"]


def gat_graph(N, seed):
    """Graph with duplicate edges, explicit self-loops and isolated nodes."""
    g = torch.Generator().manual_seed(seed)
    src = torch.randint(0, N - 4, (3 * N,), generator=g)   # last 4 nodes isolated (self-loop only)
    dst = torch.randint(0, N - 4, (3 * N,), generator=g)
    dup = torch.stack([src[:N // 2], dst[:N // 2]])           # duplicates
    loops = torch.arange(0, N - 4, 3).repeat(2, 1)             # explicit self-loops
    ei = torch.cat([torch.stack([src, dst]), dup, loops], dim=1)
    return ei


def gat_case(R, case, metric, learnable, N=24, H=32, heads=4, seed=7):
    torch.manual_seed(seed)
    layer = R["TAGANGraphAttention"](hidden_dim=H, num_heads=heads, dropout=0.0,
                                     distance_metric=metric, use_layer_norm=True,
                                     learnable_distance=learnable)
    if learnable and metric in ("gaussian_kernel", "rbf_kernel"):
        with torch.no_grad():   # per-head distinct parameters so a head mix-up is visible
            layer.geometric_attention.distance_param.copy_(torch.linspace(0.6, 1.4, heads))
    layer.train()
    g = torch.Generator().manual_seed(seed + 1)
    x = (torch.randn(N, H, generator=g) * 0.7).requires_grad_(True)
    ei = gat_graph(N, seed + 2)
    out = quiet(layer, x, ei)
    gout = torch.randn(out.shape, generator=g)
    quiet((out * gout).sum().backward)
    t = {"in.x": x.detach(), "in.edge_index": ei, "in.grad_out": gout, "out": out, "grad.x": x.grad}
    for k, v in layer.state_dict().items():
        t["sd." + k] = v
    for n, p in layer.named_parameters():
        if p.grad is not None:
            t["grad." + n] = p.grad
    meta = dict(kind="gat", metric=metric, learnable_distance=learnable, N=N, H=H, heads=heads,
                anchors=["src/tagan/layers/graph_attention.py:61-133",
                         "src/tagan/layers/geometric_attention.py:15-225,332-598"])
    save(case, t, meta)


def geo_case(R, case, mode, B=2, S=12, H=32, heads=4, seed=11, metric="euclidean"):
    torch.manual_seed(seed)
    mod = R["GeometricAttention"](hidden_dim=H, num_heads=heads, dropout=0.0,
                                  distance_metric=metric, use_layer_norm=True)
    mod.train()
    g = torch.Generator().manual_seed(seed + 1)
    x = torch.randn(B, S, H, generator=g).requires_grad_(True)
    mask = bias = None
    if mode in ("mask", "mask_bias"):
        mask = (torch.rand(B, S, S, generator=g) < 0.4).float()
        mask = torch.clamp(mask + torch.eye(S).unsqueeze(0), max=1.0)
    if mode == "badmask":
        mask = torch.ones(B, S + 1, S + 1)
    if mode in ("bias", "mask_bias"):
        bias = torch.randn(B, S, S, generator=g) * 0.5
    out = quiet(mod, x, mask, bias)
    gout = torch.randn(out.shape, generator=g)
    quiet((out * gout).sum().backward)
    t = {"in.x": x.detach(), "in.grad_out": gout, "out": out, "grad.x": x.grad}
    if mask is not None:
        t["in.mask"] = mask
    if bias is not None:
        t["in.bias"] = bias
    for k, v in mod.state_dict().items():
        t["sd." + k] = v
    for n, p in mod.named_parameters():
        if p.grad is not None:
            t["grad." + n] = p.grad
    meta = dict(kind="geo", mode=mode, metric=metric, B=B, S=S, H=H, heads=heads,
                anchors=["src/tagan/layers/geometric_attention.py:474-598"])
    save(case, t, meta)


def tatt_case(R, case, cls, ctor_kw, x_kind, B=5, T=6, H=32, heads=4, seed=21,
              mask_kind=None, with_time=False, with_attn=False):
    torch.manual_seed(seed)
    kw = dict(hidden_dim=H, num_heads=heads, dropout=0.0)
    kw.update(ctor_kw)
    mod = R[cls](**kw)
    # TimeEncoding keeps its own default dropout=0.1 (temporal_attention.py:696-701),
    # so the time-aware case is minted in eval mode to stay deterministic.
    mod.train(not with_time)
    g = torch.Generator().manual_seed(seed + 1)
    t = {}
    if x_kind == "list":
        n_list = [B - (i % 3) for i in range(T)]           # ragged -> zero padding (temporal_attention.py:948-964)
        xs = [torch.randn(n, H, generator=g).requires_grad_(True) for n in n_list]
        x_in = xs
        for i, xi in enumerate(xs):
            t[f"in.x.{i}"] = xi.detach()
    else:
        n_list = None
        xs = [torch.randn(B, T, H, generator=g).requires_grad_(True)]
        x_in = xs[0]
        t["in.x"] = xs[0].detach()
    mask = None
    if mask_kind == "ones_TT":
        mask = torch.ones(T, T)
    elif mask_kind == "rand_BTT":
        mask = (torch.rand(B, T, T, generator=g) < 0.6).float()
        mask = torch.clamp(mask + torch.eye(T).unsqueeze(0), max=1.0)
    elif mask_kind == "bad":
        mask = torch.ones(T + 1, T + 2)
    if mask is not None:
        t["in.mask"] = mask
    kwargs = {}
    if mask is not None:
        kwargs["attention_mask"] = mask
    if with_time:
        ts = torch.cumsum(torch.rand(B, T, generator=g) * 3.0, dim=1)
        t["in.time_stamps"] = ts
        kwargs["time_stamps"] = ts
    if with_attn:
        kwargs["return_attention_weights"] = True
    res = quiet(mod, x_in, **kwargs)
    out, attn = (res if with_attn else (res, None))
    gout = torch.randn(out.shape, generator=g)
    quiet((out * gout).sum().backward)
    t.update({"in.grad_out": gout, "out": out})
    if attn is not None:
        t["out.attn"] = attn
    for i, xi in enumerate(xs):
        t[f"grad.x.{i}" if x_kind == "list" else "grad.x"] = xi.grad
    for k, v in mod.state_dict().items():
        t["sd." + k] = v
    for n, p in mod.named_parameters():
        if p.grad is not None:
            t["grad." + n] = p.grad
    meta = dict(kind="tatt", cls=cls, ctor=kw, x_kind=x_kind, eval=with_time, B=B, T=T, H=H, heads=heads,
                n_list=n_list, mask_kind=mask_kind, with_time=with_time, with_attn=with_attn,
                anchors=["src/tagan/layers/temporal_attention.py:309-621,624-1205"])
    save(case, t, meta)


# --------------------------------------------------------------------------- temporal propagation (G6)
def tprop_case(R, case, kind, ctor_kw, B=7, T=6, H=32, seed=31, with_time=True):
    torch.manual_seed(seed)
    kw = dict(dropout=0.0)
    kw.update(ctor_kw)
    g = torch.Generator().manual_seed(seed + 1)
    t = {}
    kwargs = {}
    ts = None
    if with_time:
        ts = torch.cumsum(torch.rand(B, T, generator=g) * 3.0, dim=1)
        t["in.time_stamps"] = ts
    if kind == "gating":
        mod = R["TemporalGatingUnit"](input_dim=H, **kw)
        cur = torch.randn(B, H, generator=g).requires_grad_(True)
        prev = torch.randn(B, H, generator=g).requires_grad_(True)
        xs = [cur, prev]
        out = quiet(mod, cur, prev)
        t["in.current"], t["in.previous"] = cur.detach(), prev.detach()
        outs = [out]
    else:
        xs = [torch.randn(B, H, generator=g).requires_grad_(True) for _ in range(T)]
        for i, xi in enumerate(xs):
            t[f"in.x.{i}"] = xi.detach()
        if kind == "evolution":
            mod = R["TemporalEvolutionLayer"](input_dim=H, hidden_dim=H, **kw)
            outs = quiet(mod, xs, ts)
        elif kind == "skip":
            mod = R["TemporalSkipConnection"](input_dim=H, **kw)
            outs = quiet(mod, xs)
        else:   # full TemporalPropagation.forward, tensor masks, bank with a fixture-time __len__
            NMB = R["NodeMemoryBank"]
            had = "__len__" in NMB.__dict__
            NMB.__len__ = lambda self: len(self.node_states)
            try:
                mod = R["TemporalPropagation"](input_dim=H, hidden_dim=H, **kw)
                bank = NMB(hidden_dim=H)
                masks = [torch.ones(B) for _ in range(T)]
                outs, _bank = quiet(mod, xs, masks, ts, bank)
            finally:
                if not had:
                    del NMB.__len__
    gouts = [torch.randn(o.shape, generator=g) for o in outs]
    quiet(sum((o * go).sum() for o, go in zip(outs, gouts)).backward)
    for i, (o, go) in enumerate(zip(outs, gouts)):
        t[f"out.{i}"] = o
        t[f"in.grad_out.{i}"] = go
    for i, xi in enumerate(xs):
        t[f"grad.x.{i}"] = xi.grad
    for k, v in mod.state_dict().items():
        t["sd." + k] = v
    for n, p in mod.named_parameters():
        if p.grad is not None:
            t["grad." + n] = p.grad
    meta = dict(kind="tprop", module=kind, ctor=kw, B=B, T=T, H=H, with_time=with_time,
                anchors=["src/tagan/layers/temporal_propagation.py:402-558,561-765,768-957,960-1075,1078-1522"])
    save(case, t, meta)


# --------------------------------------------------------------------------- memory bank
def membank_case(R, case, seed=5, H=8, decay=0.8, max_inactivity=3):
    g = torch.Generator().manual_seed(seed)
    bank = R["NodeMemoryBank"](hidden_dim=H, decay_factor=decay, max_inactivity=max_inactivity)
    ops = []
    t = {}
    # timesteps with gaps (reappearance after 1..5 steps), duplicates in one call, pruning
    schedule = [
        ("update", [1, 2, 3, 4], 0), ("update", [1, 2, 5], 1), ("update", [3, 5, 6], 2),
        ("update", [1, 6, 6, 7], 3),                 # duplicate id 6 in one call
        ("get_states", [2, 8, 9], None),             # 8, 9 unknown -> zeros inserted
        ("update", [2, 4, 8], 5),                    # 4 reappears after 5 steps (maybe pruned)
        ("update_state", [9], 6), ("decay_all", [], None),
        ("update", [1, 2, 3, 4, 5, 6, 7, 8, 9, 10], 9), ("update", [10, 3], 10),
        ("update", [], 11), ("update", [2, 2, 2], 12),
    ]
    for k, (op, ids, ts) in enumerate(schedule):
        rec = dict(op=op, ids=ids, t=ts)
        if op in ("update", "update_state"):
            st = torch.randn(len(ids), H, generator=g)
            t[f"op{k}.states"] = st
            if op == "update":
                quiet(bank.update, ids, st, ts)
            else:
                quiet(bank.update_state, ids[0], st[0], ts)
        elif op == "get_states":
            r = quiet(bank.get_states, ids)
            t[f"op{k}.result"] = r
        elif op == "decay_all":
            quiet(bank.decay_all)
        keys = sorted(bank.node_states.keys())
        rec["keys"] = keys
        rec["inactivity"] = {str(i): bank.inactivity_counter[i] for i in sorted(bank.inactivity_counter)}
        rec["last_seen"] = {str(i): bank.last_seen[i] for i in sorted(bank.last_seen)}
        rec["frequency"] = {str(i): bank.frequency[i] for i in sorted(bank.frequency)}
        rec["size"] = bank.size
        if keys:
            t[f"op{k}.bank_states"] = torch.stack([bank.node_states[i] for i in keys])
        ops.append(rec)
    meta = dict(kind="membank", H=H, decay_factor=decay, max_inactivity=max_inactivity, ops=ops,
                anchors=["src/tagan/utils/memory_bank.py:65-244"])
    save(case, t, meta)


# --------------------------------------------------------------------------- main
def main(prefixes):
    R = _import_reference()
    torch.set_num_threads(8)
    base = dict(hidden_dim=64, num_heads=4, node_feature_dim=16, edge_feature_dim=8,
                use_edge_features=True, output_dim=1, loss_type="bce")
    lab1 = torch.tensor([1.0])
    cases = []
    # G1
    nv = [30, 44, 37, 50, 41, 33, 48, 35, 46, 39]
    cases.append(("e2e_c1mini_euclid", lambda: e2e_case(R, "e2e_c1mini_euclid", base, nv, 100, lab1)))
    cases.append(("e2e_c1mini_sdp", lambda: e2e_case(R, "e2e_c1mini_sdp", dict(base, learnable_distance=True), nv, 101, lab1)))
    cases.append(("e2e_c1full_euclid", lambda: e2e_case(R, "e2e_c1full_euclid", base, [500] * 10, 42, lab1,
                                                        store_intermediate=False)))
    cases.append(("e2e_c1full_sdp", lambda: e2e_case(R, "e2e_c1full_sdp", dict(base, learnable_distance=True),
                                                     [500] * 10, 43, torch.tensor([0.0]), store_intermediate=False)))
    # G2
    cases.append(("e2e_T_eq_heads", lambda: e2e_case(R, "e2e_T_eq_heads", base, [14, 20, 17, 12], 102, lab1)))
    cases.append(("e2e_ce_out2", lambda: e2e_case(R, "e2e_ce_out2", dict(base, output_dim=2, loss_type="ce"),
                                                  [18, 22, 20, 25, 19], 103, torch.tensor([1]))))
    cases.append(("e2e_batch3", lambda: e2e_case(R, "e2e_batch3", base, [20, 24, 21, 26, 23], 104,
                                                 torch.tensor([1.0, 0.0, 1.0]))))
    cases.append(("e2e_N_eq_T", lambda: e2e_case(R, "e2e_N_eq_T", base, [6] * 6, 105, lab1)))
    cases.append(("e2e_noln", lambda: e2e_case(R, "e2e_noln", dict(base, use_layer_norm=False),
                                               [18, 22, 20, 25, 19], 106, lab1)))
    cases.append(("e2e_causal", lambda: e2e_case(R, "e2e_causal", dict(base, causal_attention=True),
                                                 [18, 22, 20, 25, 19, 21, 23], 107, lab1)))
    cases.append(("e2e_h128", lambda: e2e_case(R, "e2e_h128", dict(base, hidden_dim=128, num_heads=8,
                                                                   node_feature_dim=27, edge_feature_dim=2),
                                               [40, 36, 44, 38, 42, 40, 37, 41], 108, lab1)))
    cases.append(("e2e_attnw", lambda: e2e_case(R, "e2e_attnw", base, [16, 19, 17, 15, 18], 109, lab1,
                                                with_attn=True)))
    cases.append(("e2e_nolabels", lambda: e2e_case_nolabel(R)))
    cases.append(("e2e_T1", lambda: e2e_case(R, "e2e_T1", base, [25], 113, lab1)))
    cases.append(("e2e_T2", lambda: e2e_case(R, "e2e_T2", base, [19, 23], 114, torch.tensor([0.0]))))
    edge_seq = (lambda: make_edge_case_sequence(16, 8, 111))
    cases.append(("e2e_edgecases", lambda: e2e_case(R, "e2e_edgecases", base, None, 110, lab1, seq_fn=edge_seq)))
    cases.append(("e2e_edgecases_sdp", lambda: e2e_case(R, "e2e_edgecases_sdp", dict(base, learnable_distance=True),
                                                        None, 112, lab1, seq_fn=edge_seq)))
    # ingestion: dict snapshots with global ids, variable N, edge_attr absent / present
    soc = dict(base, node_feature_dim=27, edge_feature_dim=2)
    cases.append(("ingest_dict_social", lambda: ingest_dict_case(R, "ingest_dict_social", soc, 6, 60, 150, 120,
                                                                 False)))
    cases.append(("ingest_dict_social_ea", lambda: ingest_dict_case(
        R, "ingest_dict_social_ea", dict(soc, hidden_dim=128, num_heads=8), 5, 80, 240, 121, True)))
    # G3
    for m in METRICS:
        for learn in (False, True):
            if learn and m not in ("gaussian_kernel", "rbf_kernel", "scaled_dot_product"):
                continue
            name = f"gat_{m}{'_learn' if learn else ''}"
            cases.append((name, (lambda m=m, learn=learn, name=name: gat_case(R, name, m, learn))))
    for mode in ("mask", "nomask", "bias", "mask_bias", "badmask"):
        cases.append((f"geo_{mode}", (lambda mode=mode: geo_case(R, f"geo_{mode}", mode))))
    cases.append(("geo_sdp_mask", lambda: geo_case(R, "geo_sdp_mask", "mask", metric="scaled_dot_product")))
    # G4
    A = "AsymmetricTemporalAttention"
    cases.append(("tatt_asym_list", lambda: tatt_case(R, "tatt_asym_list", A, {}, "list", mask_kind="ones_TT")))
    cases.append(("tatt_asym_list_Teqh", lambda: tatt_case(R, "tatt_asym_list_Teqh", A, {}, "list", T=4,
                                                           mask_kind="ones_TT", with_attn=True)))
    cases.append(("tatt_asym_tensor_causal", lambda: tatt_case(R, "tatt_asym_tensor_causal", A, dict(causal=True),
                                                               "tensor")))
    cases.append(("tatt_asym_tensor_nomask", lambda: tatt_case(R, "tatt_asym_tensor_nomask", A,
                                                               dict(relative_position_bias=False), "tensor", T=9)))
    cases.append(("tatt_asym_randmask", lambda: tatt_case(R, "tatt_asym_randmask", A, {}, "tensor",
                                                          mask_kind="rand_BTT")))
    cases.append(("tatt_asym_badmask", lambda: tatt_case(R, "tatt_asym_badmask", A, {}, "tensor", mask_kind="bad")))
    cases.append(("tatt_asym_longT", lambda: tatt_case(R, "tatt_asym_longT", A, dict(asymmetric_window_size=3),
                                                       "tensor", B=3, T=40, mask_kind="ones_TT")))
    cases.append(("tatt_asym_time", lambda: tatt_case(R, "tatt_asym_time", A, {}, "tensor", with_time=True)))
    cases.append(("tatt_base_causal", lambda: tatt_case(R, "tatt_base_causal", "TemporalAttention",
                                                        dict(causal=True), "tensor", mask_kind="ones_TT")))
    cases.append(("tatt_base_list", lambda: tatt_case(R, "tatt_base_list", "TemporalAttention", {}, "list",
                                                      mask_kind="rand_BTT")))
    # G5
    cases.append(("membank_trace", lambda: membank_case(R, "membank_trace")))
    # G6
    cases.append(("tprop_evolution", lambda: tprop_case(R, "tprop_evolution", "evolution", {})))
    cases.append(("tprop_evolution_notime", lambda: tprop_case(R, "tprop_evolution_notime", "evolution",
                                                               dict(use_layer_norm=False), with_time=False)))
    cases.append(("tprop_evolution_bidir", lambda: tprop_case(R, "tprop_evolution_bidir", "evolution",
                                                              dict(bidirectional=True))))
    for agg in ("mean", "max", "sum"):
        cases.append((f"tprop_skip_{agg}", (lambda agg=agg: tprop_case(
            R, f"tprop_skip_{agg}", "skip", dict(window_size=2, aggregation=agg), with_time=False))))
    cases.append(("tprop_gating", lambda: tprop_case(R, "tprop_gating", "gating", {}, with_time=False)))
    cases.append(("tprop_full", lambda: tprop_case(R, "tprop_full", "full", dict(window_size=2))))
    cases.append(("tprop_full_bidir_notime", lambda: tprop_case(
        R, "tprop_full_bidir_notime", "full", dict(window_size=1, bidirectional=True, aggregation="max"),
        T=5, with_time=False)))
    for name, fn in cases:
        if prefixes and not any(name.startswith(p) for p in prefixes):
            continue
        print(name)
        fn()


def ingest_dict_case(R, case, cfg_kw, T, users, edges, seed, with_edge_attr):
    """TAGAN.forward + backward on dict snapshots (model.py:187-230) — the ingestion golden."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from tagan_amd.synthetic import make_social_snapshots   # our generator (CPU only, no GPU code)
    cfg_kw = dict(cfg_kw, device="cpu", dropout=0.0)
    torch.manual_seed(seed)
    cfg = quiet(R["TAGANConfig"], **cfg_kw)
    model = quiet(R["TAGAN"], cfg)
    model.train()
    seq = make_social_snapshots(T, users, edges, seed=seed + 1, with_edge_attr=with_edge_attr)
    for snap in seq:
        snap["x"] = snap["x"].clone().requires_grad_(True)
    labels = torch.tensor([1.0])
    out = quiet(model, seq, labels=labels)
    quiet(out["loss"].backward)
    t = {}
    for i, snap in enumerate(seq):
        t[f"in.x.{i}"] = snap["x"].detach()
        t[f"in.edge_index.{i}"] = snap["edge_index"]
        t[f"in.node_ids.{i}"] = torch.tensor(snap["node_ids"], dtype=torch.int64)
        if "edge_attr" in snap:
            t[f"in.edge_attr.{i}"] = snap["edge_attr"]
        t[f"grad.x.{i}"] = snap["x"].grad
    t["in.timestep"] = torch.tensor([snap["timestep"] for snap in seq], dtype=torch.float64)
    t["in.labels"] = labels
    for k, v in model.state_dict().items():
        t["sd." + k] = v
    for name, p in model.named_parameters():
        if p.grad is not None:
            t["grad." + name] = p.grad
    t["out.logits"] = out["logits"]
    t["out.predictions"] = out["predictions"]
    t["out.loss"] = out["loss"].detach().reshape(1)
    n_list = [int(snap["x"].shape[0]) for snap in seq]
    meta = dict(kind="e2e", format="dict", config=cfg_kw, n_list=n_list, seed=seed, T=T, users=users,
                edges=edges, with_edge_attr=with_edge_attr, labels=[1.0], labels_dtype=str(labels.dtype),
                anchors=["src/tagan/model.py:158-473 (dict snapshots :187-230)",
                         "preprocess_social_media.py:297-315, 374-389"])
    save(case, t, meta)


def e2e_case_nolabel(R):
    """labels=None: loss is None, batch_size stays 1 (model.py:379-446); store logits only."""
    cfg_kw = dict(hidden_dim=64, num_heads=4, node_feature_dim=16, edge_feature_dim=8,
                  use_edge_features=True, output_dim=3, loss_type="ce", device="cpu", dropout=0.0)
    torch.manual_seed(110)
    cfg = quiet(R["TAGANConfig"], **cfg_kw)
    model = quiet(R["TAGAN"], cfg)
    model.eval()
    seq = make_sequence([15, 18, 16], 16, 8, 111)
    with torch.no_grad():
        out = quiet(model, seq)
    t = seq_tensors(seq)
    for k, v in model.state_dict().items():
        t["sd." + k] = v
    t["out.logits"] = out["logits"]
    t["out.predictions"] = out["predictions"]
    meta = dict(kind="e2e", config=cfg_kw, n_list=[15, 18, 16], seed=110, T=3, labels=None,
                labels_dtype=None, eval=True, return_attention_weights=False,
                anchors=["src/tagan/model.py:158-473"])
    save("e2e_nolabels", t, meta)


if __name__ == "__main__":
    main(sys.argv[1:])
