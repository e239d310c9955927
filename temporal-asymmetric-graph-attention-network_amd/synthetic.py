"""Seeded synthetic temporal graphs for the benchmark configs.

No datasets are available offline, so the shapes of the reference's inputs are
reproduced instead:
  * ``example``       — example.py:35-48: x~N(0,1), edge_index~U{0..N-1}
                        (duplicates and self-loops allowed), edge_attr~N(0,1).
  * ``social``        — synthetic_social_media_data.py/preprocess_social_media.py
                        shapes: F=27 node features, De=2 edge features, reply
                        edges parent-author -> reply-author with Zipf(1.1) user
                        activity (power-law degrees), same user set every snapshot.
Generated directly on the target device (inputs resident in HBM before timing).

``make_social_snapshots`` is the ingestion-shaped variant: the reference's snapshot DICTS
(preprocess_social_media.py:297-315, 374-389; model.py:187-230) with global user ids, a variable
active-user count per snapshot, local edge indices and optional edge_attr.

Degree law and unique edges (``social``): both endpoints of each reply edge are drawn from the same
Zipf(alpha = 1.1) user-activity law p(u) ∝ rank(u)^-1.1, so in- and out-degrees are power-law and hub pairs
repeat; the reference's adjacency is a SET (graph_attention.py:96-105), so what the kernels see is the
unique (src, dst) count plus one self-loop per node.  At C2 (10,000 users, 100,000 edges per snapshot)
that is 52.8k unique edges + 10k self-loops = 62.8k CSR entries per snapshot (2,011,143 over the 32
snapshots, measured on the GPU by tagan_csr_build; ``unique_edges`` computes it on the host);
``uniform`` (C3-C5) keeps ≈ E unique edges (E/N² ≪ 1).
"""
from typing import List, Sequence, Tuple

import torch

CONFIGS = {
    # name: (nodes, edges/snapshot, snapshots, hidden, heads, F, De, generator)
    "c1": (500, 1000, 10, 64, 4, 16, 8, "example"),
    "c2": (10_000, 100_000, 32, 128, 8, 27, 2, "social"),
    "c3": (100_000, 2_000_000, 64, 256, 8, 27, 2, "uniform"),
    "c4": (1_000_000, 20_000_000, 16, 128, 4, 27, 2, "uniform"),
    "c5": (100_000, 2_000_000, 128, 256, 16, 27, 2, "uniform"),
}


def make_sequence(name: str, device, seed: int = 42, snapshots: int = None,
                  nodes: int = None, edges: int = None) -> List[Tuple]:
    N, E, T, _H, _h, F, De, kind = CONFIGS[name]
    N = nodes or N
    E = edges or E
    T = snapshots or T
    g = torch.Generator(device=device).manual_seed(seed)
    seq = []
    if kind == "social":
        ranks = torch.randperm(N, generator=g, device=device).to(torch.float32) + 1.0
        activity = ranks.pow(-1.1)
    # the snapshots' node features and edges are row / column slices of one [T·N, F] and one [2, T·E] buffer (the
    # batched layout of ingest.SnapshotBatch), so the model's concatenations are views, not copies
    x_all = torch.empty(T * N, F, device=device)
    ei_all = torch.empty(2, T * E, dtype=torch.int64, device=device)
    for t in range(T):
        x = x_all[t * N:(t + 1) * N]
        x.copy_(torch.randn(N, F, generator=g, device=device))
        if kind == "social":
            src = torch.multinomial(activity, E, replacement=True, generator=g)
            dst = torch.multinomial(activity, E, replacement=True, generator=g)
            ei = torch.stack([src, dst])
        else:
            ei = torch.randint(0, N, (2, E), generator=g, device=device)
        ei_all[:, t * E:(t + 1) * E] = ei
        ea = torch.randn(E, De, generator=g, device=device)
        seq.append((x, ei_all[:, t * E:(t + 1) * E], ea, list(range(N)) if N <= 100_000 else torch.arange(N)))
    return seq


def take(seq: List[Tuple], t0: int, t1: int) -> List[Tuple]:
    """Snapshots [t0, t1) of a ``make_sequence`` sequence repacked into buffers of their own (one [ΣN, F] and one
    [2, ΣE] buffer again, so the model's concatenations stay views): a rank's block of a sharded sequence then does
    not keep the whole sequence's buffers alive."""
    part = seq[t0:t1]
    if not part:
        return []
    x_all = torch.cat([x for x, _, _, _ in part], 0)
    ei_all = torch.cat([ei for _, ei, _, _ in part], 1)
    out, r, c = [], 0, 0
    for x, ei, ea, ids in part:
        n, e = x.shape[0], ei.shape[1]
        out.append((x_all[r:r + n], ei_all[:, c:c + e], ea.clone() if ea is not None else None, ids))
        r += n
        c += e
    return out


def config_for(name: str, **over):
    from .utils.config import TAGANConfig
    N, E, T, H, h, F, De, _ = CONFIGS[name]
    kw = dict(hidden_dim=H, num_heads=h, node_feature_dim=F, edge_feature_dim=De, use_edge_features=True,
              output_dim=1, loss_type="bce", dropout=0.1, device="cuda")
    kw.update(over)
    return TAGANConfig(**kw)


def unique_edges(edge_index: torch.Tensor, num_nodes: int) -> int:
    """|unique (src, dst)| of one snapshot (the reference's set adjacency, before self-loops)."""
    key = edge_index[0].to(torch.int64) * num_nodes + edge_index[1].to(torch.int64)
    return int(torch.unique(key).numel())


def make_social_snapshots(T: int, users: int, edges: int, seed: int = 42, alpha: float = 1.1,
                          active: Tuple[float, float] = (0.6, 0.9), feature_dim: int = 27,
                          with_edge_attr: bool = True, device="cpu") -> List[dict]:
    """Reference-shaped snapshot dicts {x, edge_index, edge_attr, node_ids, timestep}.

    Per snapshot t: a Zipf(alpha)-weighted sample (without replacement) of round(users * U(active)) active
    users, their GLOBAL ids (user ids 1000 + permuted rank, as the preprocessing's user_id column) in
    node_ids, x = [activity, age/100, post_count/10, 16-d text embedding, 8-d interest one-hot]
    (feature_dim = 27, preprocess_social_media.py:297-309), ``edges`` reply edges parent-author ->
    reply-author drawn from the active users' activity law (LOCAL indices into x; duplicates and self
    replies allowed), edge_attr [E, 2] = (controversial flag, 1.0) (:312-315), timestep = t * 3600.0."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    rank = torch.randperm(users, generator=g).to(torch.float64) + 1.0
    activity = rank.pow(-alpha)
    user_id = 1000 + torch.randperm(users, generator=g)
    age = torch.randint(18, 70, (users,), generator=g).to(torch.float32)
    seq = []
    for t in range(T):
        frac = active[0] + (active[1] - active[0]) * float(torch.rand(1, generator=g))
        n = max(2, int(round(users * frac)))
        act = torch.multinomial(activity, n, replacement=False, generator=g)       # active users this window
        w = activity[act]
        src = torch.multinomial(w, edges, replacement=True, generator=g)
        dst = torch.multinomial(w, edges, replacement=True, generator=g)
        posts = torch.bincount(src, minlength=n).to(torch.float32)
        x = torch.zeros(n, feature_dim)
        x[:, 0] = (w / w.max()).to(torch.float32)
        x[:, 1] = age[act] / 100.0
        x[:, 2] = posts / 10.0
        emb = torch.randn(n, 16, generator=g)
        x[:, 3:19] = emb / emb.norm(dim=1, keepdim=True)
        x[torch.arange(n), 19 + torch.randint(0, feature_dim - 19, (n,), generator=g)] = 1.0
        snap = {"x": x.to(device), "edge_index": torch.stack([src, dst]).to(device),
                "node_ids": user_id[act].tolist(), "timestep": t * 3600.0}
        if with_edge_attr:
            ea = torch.ones(edges, 2)
            ea[:, 0] = (torch.rand(edges, generator=g) < 0.2).to(torch.float32)
            snap["edge_attr"] = ea.to(device)
        seq.append(snap)
    return seq
