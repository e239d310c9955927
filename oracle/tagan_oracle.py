"""TEST INFRASTRUCTURE ONLY — torch-CPU restatement of TAGAN's hot path.

This is the parity checker for the HIP implementation in ``tagan_amd`` and the
``cpu_baseline`` leg of ``bench.py``.  It is never imported by the product.
It restates, functionally (parameters come in as a flat ``state_dict``-keyed
mapping), the behaviour of the reference at
MaLoskins/Temporal-Asymmetric-Graph-Attention-Network @ 2025-04-18:

  * ``csr_from_edge_index``  — the dense adjacency of graph_attention.py:96-105
    (``adj[src,dst]=1; adj += eye``) expressed as its CSR: the de-duplicated set
    {(src,dst)} ∪ {(i,i)}, rows = src = query (SURVEY.md header fact 3).
  * ``pair_score``          — DistanceMetric (geometric_attention.py:15-225) and
    its use in _get_attention_weights (:351-469): distances are negated.
  * ``geometric_attention`` — GeometricAttention.forward (:518-598) incl. mask
    handling (:474-507) and the post-softmax ``geometric_bias`` (:567-575).
    ``mode='dense_faithful'`` keeps the reference's per-(head,node) loop and dense
    N×N mask (its cost model); ``'dense'`` vectorises it; ``'sparse'`` is a CSR
    edge-softmax (identical values, O(E) memory).
  * ``temporal_attention``  — TemporalAttention.forward (temporal_attention.py:400-621)
    and AsymmetricTemporalAttention.forward (:904-1205) incl. list padding
    (:928-976), relative-position / asymmetric-kernel bias (:732-790, :1010-1027),
    time-aware bias + time mask (:122-220, :792-903, :1030-1070) and the mask
    quirks (:1072-1170): a [T,T] all-ones mask becomes causal only when T == heads.
  * ``tagan_forward``       — TAGAN.forward (model.py:158-473): per-snapshot
    embedding + geometric layers (+skip LN after layer 0), the TemporalPropagation
    identity fallback (temporal_propagation.py:1287/1505 always raise; model.py:302-309),
    temporal attention with the default ones(T,T) mask (model.py:335-375),
    the un-permuted ``view(T,-1,H)`` pooling (model.py:377-427), the head
    (classification.py:856-966) and the loss (model.py:433-446,
    classification.py:401-592).
"""
import math
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F

METRICS = ("euclidean", "squared_euclidean", "manhattan", "cosine_similarity", "cosine_distance",
           "dot_product", "scaled_dot_product", "gaussian_kernel", "rbf_kernel")

TAGANParams = Dict[str, torch.Tensor]


def _ln(x, P, name):
    return F.layer_norm(x, (x.shape[-1],), P[name + ".weight"], P[name + ".bias"], 1e-5)


def _lin(x, P, name):
    return F.linear(x, P[name + ".weight"], P.get(name + ".bias"))


# ----------------------------------------------------------------------------- graph
def csr_from_edge_index(edge_index: torch.Tensor, num_nodes: int):
    """Dense adjacency (graph_attention.py:96-105) as a CSR over unique (src,dst)+self-loops.

    Negative indices wrap like torch advanced indexing; out-of-range ones raise.
    Returns (rowptr[N+1], col[nnz]) int64, rows sorted, columns ascending.
    """
    N = int(num_nodes)
    ei = edge_index.to(torch.int64)
    src, dst = ei[0], ei[1]
    src = torch.where(src < 0, src + N, src)
    dst = torch.where(dst < 0, dst + N, dst)
    if src.numel() and (int(src.min()) < 0 or int(src.max()) >= N or int(dst.min()) < 0 or int(dst.max()) >= N):
        raise IndexError("edge_index out of range for %d nodes" % N)
    loops = torch.arange(N, dtype=torch.int64)
    keys = torch.unique(torch.cat([src * N + dst, loops * N + loops]))
    rows = keys // N
    col = keys % N
    rowptr = torch.zeros(N + 1, dtype=torch.int64)
    rowptr[1:] = torch.cumsum(torch.bincount(rows, minlength=N), 0)
    return rowptr, col


def pair_score(metric: str, q: torch.Tensor, k: torch.Tensor, param=None) -> torch.Tensor:
    """Similarity of broadcast pairs q[...,d] vs k[...,d] (geometric_attention.py:15-225, :351-469)."""
    d = q.shape[-1]
    if metric == "scaled_dot_product":
        return (q * k).sum(-1) / math.sqrt(d)
    if metric == "dot_product":
        return (q * k).sum(-1)
    if metric in ("cosine_similarity", "cosine_distance"):
        qn = torch.norm(q, p=2, dim=-1, keepdim=True)
        kn = torch.norm(k, p=2, dim=-1, keepdim=True)
        qn = torch.where(qn == 0, torch.ones_like(qn) * 1e-8, qn)
        kn = torch.where(kn == 0, torch.ones_like(kn) * 1e-8, kn)
        cos = torch.clamp((q * k).sum(-1) / (qn * kn).squeeze(-1), -1.0, 1.0)
        return cos if metric == "cosine_similarity" else -(1.0 - cos)
    if metric == "euclidean":
        return -torch.sqrt(((q - k) ** 2).sum(-1) + 1e-8)
    if metric == "squared_euclidean":
        return -((q - k) ** 2).sum(-1)
    if metric == "manhattan":
        return -torch.abs(q - k).sum(-1)
    if metric == "gaussian_kernel":
        sigma = 1.0 if param is None else param
        return torch.exp(-((q - k) ** 2).sum(-1) / (2 * sigma ** 2))
    if metric == "rbf_kernel":
        gamma = 1.0 if param is None else param
        return torch.exp(-gamma * ((q - k) ** 2).sum(-1))
    raise ValueError("Unknown distance metric: %s" % metric)


def _metric_param(P, name, metric, learnable, h):
    if learnable and metric in ("gaussian_kernel", "rbf_kernel"):
        return P[name + ".distance_param"][h]
    return None


def _dense_scores(q, k, metric, P, name, learnable, faithful):
    B, h, S, d = q.shape
    if metric == "scaled_dot_product":
        return torch.matmul(q, k.transpose(-2, -1)) / math.sqrt(d)
    if faithful:
        scores = torch.zeros(B, h, S, S, dtype=q.dtype)
        for hh in range(h):
            prm = _metric_param(P, name, metric, learnable, hh)
            for i in range(S):
                scores[:, hh, i] = pair_score(metric, q[:, hh, i].unsqueeze(1), k[:, hh], prm)
        return scores
    per_head = []
    for hh in range(h):
        prm = _metric_param(P, name, metric, learnable, hh)
        per_head.append(pair_score(metric, q[:, hh, :, None, :], k[:, hh, None, :, :], prm))
    return torch.stack(per_head, 1)


def geometric_attention(x, P: TAGANParams, name: str, num_heads: int, metric: str,
                        use_layer_norm=True, learnable=False, attention_mask=None,
                        geometric_bias=None, mode="dense", csr=None):
    """GeometricAttention.forward (geometric_attention.py:518-598); x [B,S,H]."""
    if metric == "mahalanobis":
        raise ValueError("Unknown distance metric: mahalanobis")   # get_metric at construction (:206-225, :306)
    B, S, H = x.shape
    d = H // num_heads
    identity = x
    hx = _ln(x, P, name + ".layer_norm1") if use_layer_norm else x
    q = _lin(hx, P, name + ".q_linear").view(B, S, num_heads, d).transpose(1, 2)
    k = _lin(hx, P, name + ".k_linear").view(B, S, num_heads, d).transpose(1, 2)
    v = _lin(hx, P, name + ".v_linear").view(B, S, num_heads, d).transpose(1, 2)
    if mode == "sparse" and geometric_bias is None:
        ctx = _sparse_context(q, k, v, metric, P, name, learnable, attention_mask, csr)
    else:
        scores = _dense_scores(q, k, metric, P, name, learnable, mode == "dense_faithful")
        if attention_mask is not None:
            if attention_mask.shape[-2:] != scores.shape[-2:]:
                em = torch.ones(B, 1, S, S, dtype=scores.dtype)
            else:
                em = attention_mask.unsqueeze(1)
            scores = scores.masked_fill(em == 0, float("-inf"))
        w = F.softmax(scores, dim=-1)
        if geometric_bias is not None:
            w = F.softmax(w + geometric_bias.unsqueeze(1), dim=-1)
        ctx = torch.matmul(w, v)
    ctx = ctx.transpose(1, 2).reshape(B, S, H)
    out = _lin(ctx, P, name + ".output_proj") + identity
    if use_layer_norm:
        out = _ln(out, P, name + ".layer_norm2")
    return out


def _sparse_context(q, k, v, metric, P, name, learnable, attention_mask, csr):
    """Edge-softmax over the CSR of the mask: identical values to the dense masked softmax."""
    B, h, S, d = q.shape
    if csr is None:
        if attention_mask is None or attention_mask.shape[-2:] != (S, S):
            m = torch.ones(B, S, S, dtype=torch.bool)
        else:
            m = (attention_mask != 0).expand(B, S, S)
        b, i, j = m.nonzero(as_tuple=True)
        src, dst = b * S + i, b * S + j
    else:
        rowptr, col = csr
        src = torch.repeat_interleave(torch.arange(rowptr.numel() - 1), rowptr[1:] - rowptr[:-1])
        dst = col
    Nt = B * S
    qf = q.transpose(1, 2).reshape(Nt, h, d)
    kf = k.transpose(1, 2).reshape(Nt, h, d)
    vf = v.transpose(1, 2).reshape(Nt, h, d)
    per_head = []
    for hh in range(h):
        prm = _metric_param(P, name, metric, learnable, hh)
        per_head.append(pair_score(metric, qf[src, hh], kf[dst, hh], prm))
    s = torch.stack(per_head, 1)                                     # [E', h]
    m = torch.full((Nt, h), float("-inf"), dtype=s.dtype).scatter_reduce(
        0, src[:, None].expand(-1, h), s, reduce="amax", include_self=True)
    p = torch.exp(s - m[src])
    l = torch.zeros(Nt, h, dtype=s.dtype).index_add(0, src, p)
    a = p / l[src]
    ctx = torch.zeros(Nt, h, d, dtype=q.dtype).index_add(0, src, a[:, :, None] * vf[dst])
    return ctx.view(B, S, h, d).transpose(1, 2)


def graph_attention(x, edge_index, P, name, num_heads, metric, use_layer_norm=True,
                    learnable=False, mode="sparse"):
    """TAGANGraphAttention.forward (graph_attention.py:61-133); x [N,H] -> [N,H]."""
    N = x.shape[0]
    sub = name + ".geometric_attention"
    if mode == "sparse":
        csr = csr_from_edge_index(edge_index, N)
        out = geometric_attention(x.unsqueeze(0), P, sub, num_heads, metric, use_layer_norm,
                                  learnable, mode="sparse", csr=csr)
    else:
        adj = torch.zeros(N, N, dtype=x.dtype)
        adj[edge_index[0], edge_index[1]] = 1
        adj = adj + torch.eye(N, dtype=x.dtype)
        out = geometric_attention(x.unsqueeze(0), P, sub, num_heads, metric, use_layer_norm,
                                  learnable, attention_mask=adj.unsqueeze(0), mode=mode)
    return out.squeeze(0)


# ----------------------------------------------------------------------------- temporal
def time_basis_bias(time_stamps, P, name, num_heads, hidden_dim):
    """_compute_time_based_attention via TimeEncoding 'basis' (temporal_attention.py:122-220, :792-871)."""
    B, T = time_stamps.shape
    diffs = (time_stamps.unsqueeze(2) - time_stamps.unsqueeze(1)).reshape(B * T * T, 1)
    diffs = torch.nan_to_num(diffs, nan=0.0)
    tmin, tmax = diffs.min(), diffs.max()
    if tmax > tmin and (tmax - tmin) > 1e-7:
        tn = (diffs - tmin) / (tmax - tmin)
    else:
        tn = torch.zeros_like(diffs)
    mu = P[name + ".time_encoding.basis_mu"]
    sigma = P[name + ".time_encoding.basis_sigma"]
    if float(sigma.detach().min()) < 1e-7:
        sigma = torch.clamp(sigma, min=1e-7)
    expo = torch.clamp(-(((tn.unsqueeze(-1) - mu) ** 2) / (2 * sigma ** 2)), -88.0, 88.0)
    basis = torch.nan_to_num(torch.exp(expo), nan=0.0)
    enc = torch.nan_to_num(_lin(basis, P, name + ".time_encoding.basis_proj"), nan=0.0)
    enc = enc.view(B, T, T, hidden_dim)
    return _lin(enc, P, name + ".time_q_proj").permute(0, 3, 1, 2)


def _stack_list(x_list):
    """List of [N_t,H] -> zero-padded [N_max,T,H] (temporal_attention.py:928-976)."""
    xs = [t[0] if isinstance(t, list) and len(t) > 0 else t for t in x_list]
    n_max = max(t.shape[0] for t in xs)
    padded = [torch.cat([t, torch.zeros(n_max - t.shape[0], t.shape[1], dtype=t.dtype)], 0)
              if t.shape[0] < n_max else t for t in xs]
    return torch.stack(padded, 0).permute(1, 0, 2)


class MaskBroadcastError(RuntimeError):
    """Raised where the reference's layer raises after a mask broadcast (h == 1 < T)."""


def _asym_mask(attention_mask, time_mask, scores, heads, causal_ctor):
    """Effective mask logic of AsymmetricTemporalAttention.forward (temporal_attention.py:1041-1170).

    Returns a boolean 'keep' tensor broadcastable to scores, or None (no masking).
    """
    B, h, T, _ = scores.shape
    if time_mask is not None:
        if attention_mask is None:
            attention_mask = time_mask
        elif isinstance(attention_mask, torch.Tensor) and attention_mask.shape[-2:] == time_mask.shape[-2:]:
            attention_mask = attention_mask * time_mask
    keep = None
    if causal_ctor:
        keep = torch.tril(torch.ones(T, T, dtype=torch.bool)).unsqueeze(0)
    if attention_mask is None:
        return keep, False
    if isinstance(attention_mask, list):
        L = len(attention_mask)
        attention_mask = torch.ones(B, L, L)
    if attention_mask.shape[-1] != T or attention_mask.shape[-2] != T:
        em = torch.tril(torch.ones(T, T)).expand(B, heads, T, T)
    else:
        em = attention_mask.unsqueeze(1)
        if bool(torch.all(em == 1.0)):
            em = em * torch.tril(torch.ones(T, T))
    if em.numel() == 0:
        return keep, False
    try:
        shape = torch.broadcast_shapes(em.shape, scores.shape)
    except RuntimeError:
        return keep, False                     # masked_fill raises; the layer swallows it (:1164-1170)
    if tuple(shape) != tuple(scores.shape):
        return keep, True                      # masked_fill broadcasts up; reshape at :1187 raises
    k2 = (em != 0)
    keep = k2 if keep is None else (keep & k2)
    return keep, False


def _base_mask(attention_mask, scores, heads, causal_ctor):
    """Mask logic of TemporalAttention.forward (temporal_attention.py:501-588)."""
    B, h, T, _ = scores.shape
    keep = torch.tril(torch.ones(T, T, dtype=torch.bool)).unsqueeze(0) if causal_ctor else None
    if attention_mask is None:
        return keep
    if isinstance(attention_mask, list):
        try:
            attention_mask = torch.stack(attention_mask, 0)
        except Exception:
            attention_mask = torch.ones(T, T)
    ms = attention_mask.shape
    em = torch.ones(B, 1, T, T)
    if len(ms) == 2:
        if ms[0] == T and ms[1] == T:
            em = attention_mask.unsqueeze(0).unsqueeze(0).expand(B, heads, -1, -1)
        elif ms[0] == T and causal_ctor:
            em = em * torch.tril(torch.ones(T, T)).unsqueeze(0).unsqueeze(0)
    elif len(ms) == 3 and ms[0] == B and ms[1] == ms[2]:
        em = attention_mask.unsqueeze(1)
    try:
        shape = torch.broadcast_shapes(em.shape, scores.shape)
        if tuple(shape) != tuple(scores.shape):
            return keep
    except RuntimeError:
        return keep
    k2 = em != 0
    return k2 if keep is None else keep & k2


def temporal_attention(x, P, name, num_heads, cls="asym", causal=False, use_layer_norm=True,
                       relative_position_bias=True, max_relative_position=32,
                       asymmetric_window_size=5, time_aware=True, use_time_masks=True,
                       time_stamps=None, attention_mask=None, return_attention_weights=False):
    """(Asymmetric)TemporalAttention.forward; x [B,S,H] or list of [N_t,H]."""
    if isinstance(x, list):
        x = _stack_list(x)
    B, T, H = x.shape
    d = H // num_heads
    identity = x
    hx = _ln(x, P, name + ".layer_norm1") if use_layer_norm else x
    q = _lin(hx, P, name + ".q_linear").view(B, T, num_heads, d).transpose(1, 2)
    k = _lin(hx, P, name + ".k_linear").view(B, T, num_heads, d).transpose(1, 2)
    v = _lin(hx, P, name + ".v_linear").view(B, T, num_heads, d).transpose(1, 2)
    scores = torch.matmul(q, k.transpose(-2, -1)) / math.sqrt(d)
    if cls == "asym":
        pos = torch.arange(T)
        rel = pos.unsqueeze(1) - pos.unsqueeze(0)
        if relative_position_bias:
            idx = torch.clamp(rel + max_relative_position, 0, 2 * max_relative_position)
            scores = scores + P[name + ".relative_pos_table"][idx].permute(2, 0, 1).unsqueeze(0)
        W = asymmetric_window_size
        kv = P[name + ".asymmetric_kernel"][torch.clamp(rel + W, 0, 2 * W)]
        kv = kv * ((rel >= -W) & (rel <= W)).unsqueeze(-1).to(kv.dtype)
        scores = scores + kv.permute(2, 0, 1).unsqueeze(0)
        time_mask = None
        if time_aware and time_stamps is not None:
            scores = scores + time_basis_bias(time_stamps, P, name, num_heads, H)
            if use_time_masks:
                time_mask = (torch.abs(time_stamps.unsqueeze(2) - time_stamps.unsqueeze(1)) <= 10.0).to(x.dtype)
        keep, explode = _asym_mask(attention_mask, time_mask, scores, num_heads, causal)
        if explode:
            raise MaskBroadcastError("mask broadcast enlarges the score tensor (reference raises at reshape)")
    else:
        keep = _base_mask(attention_mask, scores, num_heads, causal)
    if keep is not None:
        scores = scores.masked_fill(~keep, float("-inf"))
    w = F.softmax(scores, dim=-1)
    ctx = torch.matmul(w, v).transpose(1, 2).reshape(B, T, H)
    out = _lin(ctx, P, name + ".output_proj") + identity
    if use_layer_norm:
        out = _ln(out, P, name + ".layer_norm2")
    return (out, w) if return_attention_weights else out


# ----------------------------------------------------------------------------- head + loss
def classification_head(gf, P, use_layer_norm=True, name="classification_head.classification_head"):
    """TemporalClassificationHead attention pooling + classifier (classification.py:804-836, :909-955)."""
    a = torch.tanh(_lin(gf, P, name + ".attention.0"))
    a = F.linear(a, P[name + ".attention.2.weight"])
    w = F.softmax(a, dim=1)
    pooled = (gf * w).sum(1)
    hdn = _lin(pooled, P, name + ".classifier.0")
    if use_layer_norm:
        hdn = _ln(hdn, P, name + ".classifier.1")
        return _lin(F.relu(hdn), P, name + ".classifier.4")
    return _lin(F.relu(hdn), P, name + ".classifier.3")


def bce_loss(predictions, targets):
    """TemporalLossFunction task 'classification' (classification.py:420-456, :583-588)."""
    if predictions.size(-1) == 1:
        if predictions.dim() == 2 and predictions.size(1) == 1 and targets.dim() == 1 \
                and predictions.size(0) == targets.size(0):
            predictions = predictions.squeeze(-1)
        elif predictions.size(0) == 1 and targets.dim() == 1:
            predictions = predictions.squeeze(-1).expand(targets.size(0))
        elif predictions.dim() == 1 and targets.dim() == 2 and predictions.size(0) == targets.size(0):
            targets = targets.squeeze(-1)
        elif predictions.size(0) == 1 and targets.dim() == 2:
            predictions = predictions.expand(targets.size(0), -1)
    if not (predictions.dim() == 2 and predictions.size(1) > 1 and targets.dim() == 1) \
            and predictions.shape != targets.shape:
        raise ValueError("Predictions shape %s does not match targets shape %s" %
                         (tuple(predictions.shape), tuple(targets.shape)))
    return F.binary_cross_entropy_with_logits(predictions, targets, reduction="none").mean()


# ----------------------------------------------------------------------------- model
def _unpack(snapshot):
    if isinstance(snapshot, dict):
        return snapshot["x"], snapshot["edge_index"], snapshot.get("edge_attr"), snapshot["node_ids"]
    return snapshot[0], snapshot[1], snapshot[2], snapshot[3]


def tagan_forward(P: TAGANParams, cfg: dict, seq: List, labels: Optional[torch.Tensor] = None,
                  return_attention_weights=False, mode="sparse", collect=None):
    """TAGAN.forward (model.py:158-473) on CPU; ``cfg`` uses TAGANConfig field names."""
    H = cfg.get("hidden_dim", 64)
    heads = cfg.get("num_heads", 4)
    L = cfg.get("num_layers", 2)
    ln = cfg.get("use_layer_norm", True)
    learnable = cfg.get("learnable_distance", False)
    metric = "scaled_dot_product" if learnable else "euclidean"
    out_dim = cfg.get("output_dim", 2)
    outs = []
    for snap in seq:
        x, ei, _ea, _ids = _unpack(snap)
        h = _lin(x, P, "node_embedding")             # edge_embedding output is dead (model.py:236-239)
        skip = h
        for i in range(L):
            h = graph_attention(h, ei, P, "geometric_attention_layers.%d" % i, heads, metric, ln,
                                learnable, mode=("sparse" if mode == "sparse" else mode))
            if i == 0:
                h = h + (_ln(skip, P, "skip_layer_norm") if ln else skip)
        outs.append(h)
    if collect is not None:
        collect["geo"] = outs
    T = len(outs)
    # TemporalPropagation always raises in the shipped code -> identity (model.py:302-309)
    tkw = dict(cls="asym", causal=cfg.get("causal_attention", False), use_layer_norm=ln,
               relative_position_bias=cfg.get("asymmetric_temporal_bias", True),
               asymmetric_window_size=cfg.get("window_size", 5),
               return_attention_weights=return_attention_weights)
    try:
        res = temporal_attention(outs, P, "temporal_attention", heads,
                                 attention_mask=torch.ones(T, T), **tkw)
    except MaskBroadcastError:
        res = temporal_attention(outs, P, "temporal_attention", heads, attention_mask=None, **tkw)
    xt, tw = res if return_attention_weights else (res, None)
    if collect is not None:
        collect["temporal"] = xt
    B = labels.shape[0] if (labels is not None and labels.dim() > 0) else 1
    gf = torch.zeros(B, T, H, dtype=xt.dtype)
    if xt.shape[0] == T:
        rows = [xt[t].mean(0) for t in range(T)]
    else:
        r = xt.reshape(T, -1, H)
        rows = [r[t].mean(0) for t in range(T)]
    gf = torch.cat([torch.stack(rows, 0).unsqueeze(0), gf[1:]], 0)
    if collect is not None:
        collect["graph_features"] = gf
    logits = classification_head(gf, P, ln)
    loss = None
    if labels is not None:
        lab = labels.long() if labels.dtype == torch.bool else labels
        if out_dim > 1 and lab.dim() == 1:
            loss = F.cross_entropy(logits, lab)
        else:
            loss = bce_loss(logits, lab)
    preds = torch.sigmoid(logits) if out_dim == 1 else F.softmax(logits, dim=1)
    out = dict(logits=logits, predictions=preds, loss=loss)
    if return_attention_weights:
        out["geometric_attention_weights"] = [{"node_attention": None} for _ in range(T)]
        out["temporal_attention_weights"] = tw
    return out
