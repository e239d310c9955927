"""Geometric attention on MI355X (drop-in for src/tagan/layers/geometric_attention.py).

``GeometricAttention`` keeps the reference constructor, parameter names/shapes,
initialisation order and forward signature (geometric_attention.py:228-607), so
reference ``state_dict``s load unchanged and ``torch.manual_seed(s)`` yields the
same initial weights.  The forward runs:

  LN1 fused into the prologue of the QKV projection (hand-written bf16-matrix-core
  GEMM, csrc/stream_gemm.hip; fp32 as three bf16 planes) -> ``tagan_geo_attn_fwd``
  (metric score, edge-softmax, attn-dropout, A·V over the mask's CSR; HIP)
  -> out-projection GEMM with dropout + residual + LN2 in its epilogue (HIP)

(every width BASELINE names, 64 / 128 / 256, has stream-GEMM kernels in both precisions.  The
LayerNorm fusions: all of them at H = 128; at H = 256 in the bf16 activation mode (C5) LN1 in
the QKV prologue and LN2 in the out-projection epilogue, LN2's and LN1's backward standalone;
fp32 at H = 64 / 256 runs the LayerNorms as their own kernels beside the stream GEMMs.  Widths
with no stream-GEMM kernel take hipBLASLt plus the standalone LayerNorm kernels).

Dense masks become CSR (``graph_from_dense_mask``); TAGANGraphAttention hands in
a prebuilt snapshot CSR through ``forward_graph``.  There is no CPU path.
"""
import math
from typing import Callable, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _lib
from ..fused import GeoCore, attention_block, fusable
from ..kernels import (GeoAttnFn, SnapshotGraph, dropout_add_layer_norm, fused_qkv, graph_from_dense_mask,
                       layer_norm, linear, new_seed)


class DistanceMetric:
    """Distance metrics of geometric_attention.py:15-225 (plain torch utilities, any device)."""

    @staticmethod
    def euclidean(x, y):
        return torch.sqrt(torch.sum((x - y) ** 2, dim=-1) + 1e-8)

    @staticmethod
    def squared_euclidean(x, y):
        return torch.sum((x - y) ** 2, dim=-1)

    @staticmethod
    def manhattan(x, y):
        return torch.sum(torch.abs(x - y), dim=-1)

    @staticmethod
    def cosine_similarity(x, y):
        xn = torch.norm(x, p=2, dim=-1, keepdim=True)
        yn = torch.norm(y, p=2, dim=-1, keepdim=True)
        xn = torch.where(xn == 0, torch.ones_like(xn) * 1e-8, xn)
        yn = torch.where(yn == 0, torch.ones_like(yn) * 1e-8, yn)
        return torch.clamp(torch.sum(x * y, dim=-1) / (xn * yn).squeeze(-1), -1.0, 1.0)

    @staticmethod
    def cosine_distance(x, y):
        return 1.0 - DistanceMetric.cosine_similarity(x, y)

    @staticmethod
    def dot_product(x, y):
        return torch.sum(x * y, dim=-1)

    @staticmethod
    def scaled_dot_product(x, y):
        return torch.sum(x * y, dim=-1) / math.sqrt(x.size(-1))

    @staticmethod
    def mahalanobis(x, y, cov_inv):
        diff = x - y
        shape = diff.shape
        d2 = diff.reshape(-1, shape[-1])
        return torch.sqrt(torch.sum(d2 @ cov_inv * d2, dim=-1).view(*shape[:-1]) + 1e-8)

    @staticmethod
    def gaussian_kernel(x, y, sigma=1.0):
        return torch.exp(-DistanceMetric.squared_euclidean(x, y) / (2 * sigma ** 2))

    @staticmethod
    def rbf_kernel(x, y, gamma=1.0):
        return torch.exp(-gamma * DistanceMetric.squared_euclidean(x, y))

    @staticmethod
    def get_metric(metric_name: str) -> Callable:
        # Same accepted names as geometric_attention.py:196-225 ("mahalanobis" is not one of them).
        if metric_name in _lib.METRIC_IDS:
            return getattr(DistanceMetric, metric_name)
        raise ValueError(f"Unknown distance metric: {metric_name}")


class GeometricAttention(nn.Module):
    def __init__(self, hidden_dim: int, num_heads: int = 8, dropout: float = 0.1,
                 distance_metric: str = "scaled_dot_product", use_layer_norm: bool = True,
                 learnable_distance: bool = False):
        super().__init__()
        self.hidden_dim = hidden_dim
        self.num_heads = num_heads
        self.dropout_prob = dropout
        self.distance_metric = distance_metric
        self.use_layer_norm = use_layer_norm
        self.learnable_distance = learnable_distance
        assert hidden_dim % num_heads == 0, "Hidden dimension must be divisible by number of heads"
        self.head_dim = hidden_dim // num_heads
        self.q_linear = nn.Linear(hidden_dim, hidden_dim)
        self.k_linear = nn.Linear(hidden_dim, hidden_dim)
        self.v_linear = nn.Linear(hidden_dim, hidden_dim)
        self.output_proj = nn.Linear(hidden_dim, hidden_dim)
        if use_layer_norm:
            self.layer_norm1 = nn.LayerNorm(hidden_dim)
            self.layer_norm2 = nn.LayerNorm(hidden_dim)
        self.attn_dropout = nn.Dropout(dropout)
        self.output_dropout = nn.Dropout(dropout)
        if learnable_distance:
            if distance_metric in ("gaussian_kernel", "rbf_kernel"):
                self.distance_param = nn.Parameter(torch.ones(num_heads))
            elif distance_metric == "mahalanobis":
                rank = min(16, hidden_dim // 4)
                self.cov_factors = nn.Parameter(torch.zeros(num_heads, rank, self.head_dim))
                nn.init.xavier_uniform_(self.cov_factors)
        self.distance_fn = DistanceMetric.get_metric(distance_metric)
        self.metric_id = _lib.METRIC_IDS[distance_metric]
        self._init_parameters()

    def _init_parameters(self):
        for lin in (self.q_linear, self.k_linear, self.v_linear, self.output_proj):
            nn.init.xavier_uniform_(lin.weight)
        for lin in (self.q_linear, self.k_linear, self.v_linear, self.output_proj):
            nn.init.zeros_(lin.bias)
        if self.learnable_distance and self.distance_metric in ("gaussian_kernel", "rbf_kernel"):
            nn.init.constant_(self.distance_param, 1.0 if self.distance_metric == "gaussian_kernel" else 0.1)

    def _metric_param(self):
        if self.learnable_distance and self.distance_metric in ("gaussian_kernel", "rbf_kernel"):
            return self.distance_param
        return None

    def forward_graph(self, x: torch.Tensor, graph: SnapshotGraph, skip_ln=None) -> torch.Tensor:
        """Hot path: x [N, H] (N = all nodes of a snapshot batch), graph = their CSR/CSC.
        ``skip_ln``: returns layer(x) + skip_ln(x) (model.py:258-262), fused into the last LayerNorm."""
        p = self.attn_dropout.p if self.training else 0.0
        p_out = self.output_dropout.p if self.training else 0.0
        if skip_ln is not None and x.dtype != torch.float32:
            return self.forward_graph(x, graph) + layer_norm(x, skip_ln)
        if fusable(x, self.use_layer_norm):   # one autograd node for the whole layer (fused.py)
            core = GeoCore(graph, self.metric_id, self.num_heads, p, new_seed() if p > 0 else 0)
            return attention_block(x, core, self._metric_param(), None, self.layer_norm1, self.q_linear,
                                   self.k_linear, self.v_linear, self.output_proj, self.layer_norm2, p_out,
                                   new_seed() if p_out > 0 else 0, skip_ln=skip_ln)
        if skip_ln is not None:
            return self.forward_graph(x, graph) + layer_norm(x, skip_ln)
        identity = x
        h = layer_norm(x, self.layer_norm1) if self.use_layer_norm else x
        qkv = fused_qkv(h, self.q_linear, self.k_linear, self.v_linear).contiguous()
        ctx = GeoAttnFn.apply(qkv, self._metric_param(), graph, self.metric_id, self.num_heads, p,
                              new_seed() if p > 0 else 0)
        proj = linear(ctx, self.output_proj.weight, self.output_proj.bias)
        if self.use_layer_norm:
            return dropout_add_layer_norm(proj, identity, self.layer_norm2, p_out)
        return F.dropout(proj, p_out, True) + identity

    def forward(self, x: torch.Tensor, attention_mask: Optional[torch.Tensor] = None,
                geometric_bias: Optional[torch.Tensor] = None) -> torch.Tensor:
        """x [B,S,H]; mask [B,S,S] (0 = masked) or None (dense); see geometric_attention.py:518-598."""
        B, S, H = x.shape
        if geometric_bias is not None:
            return self._forward_dense_bias(x, attention_mask, geometric_bias)
        if attention_mask is None or attention_mask.shape[-2:] != (S, S):
            mask = torch.ones(B, S, S, device=x.device)       # mismatched masks -> full attention (:482-498)
        else:
            mask = attention_mask.expand(B, S, S) if attention_mask.dim() == 3 else attention_mask
        graph = graph_from_dense_mask(mask)
        return self.forward_graph(x.reshape(B * S, H), graph).view(B, S, H)

    def _forward_dense_bias(self, x, attention_mask, geometric_bias):
        """geometric_bias path (geometric_attention.py:564-575): the bias is added to the POST-softmax
        weights of every (i, j) pair and re-normalised over all j, so attention becomes dense.
        Never reached from TAGAN (graph_attention.py passes None); runs as dense device tensor ops."""
        B, S, H = x.shape
        h, d = self.num_heads, self.head_dim
        identity = x
        hx = layer_norm(x, self.layer_norm1) if self.use_layer_norm else x
        qkv = fused_qkv(hx, self.q_linear, self.k_linear, self.v_linear)
        q, k, v = (t.reshape(B, S, h, d).transpose(1, 2) for t in qkv.split(H, dim=-1))
        if self.distance_metric == "scaled_dot_product":
            scores = torch.matmul(q, k.transpose(-2, -1)) / math.sqrt(d)
        else:
            prm = self._metric_param()
            per_head = []
            for hh in range(h):
                fn = self.distance_fn
                if prm is not None:
                    fn = (lambda a, b, s=prm[hh]: DistanceMetric.gaussian_kernel(a, b, s)) \
                        if self.distance_metric == "gaussian_kernel" else \
                        (lambda a, b, g=prm[hh]: DistanceMetric.rbf_kernel(a, b, g))
                sc = fn(q[:, hh, :, None, :], k[:, hh, None, :, :])
                if self.distance_metric in ("euclidean", "squared_euclidean", "manhattan", "cosine_distance"):
                    sc = -sc
                per_head.append(sc)
            scores = torch.stack(per_head, 1)
        if attention_mask is not None:
            em = attention_mask.unsqueeze(1) if attention_mask.shape[-2:] == scores.shape[-2:] else \
                torch.ones(B, 1, S, S, device=x.device)
            scores = scores.masked_fill(em == 0, float("-inf"))
        w = self.attn_dropout(torch.softmax(scores, dim=-1))
        w = self.attn_dropout(torch.softmax(w + geometric_bias.unsqueeze(1), dim=-1))
        ctx = torch.matmul(w, v).transpose(1, 2).reshape(B, S, H)
        proj = linear(ctx, self.output_proj.weight, self.output_proj.bias)
        p_out = self.output_dropout.p if self.training else 0.0
        if self.use_layer_norm:
            return dropout_add_layer_norm(proj, identity, self.layer_norm2, p_out)
        return F.dropout(proj, p_out, True) + identity

    def extra_repr(self) -> str:
        return (f"hidden_dim={self.hidden_dim}, num_heads={self.num_heads}, "
                f"distance_metric={self.distance_metric}, learnable_distance={self.learnable_distance}, "
                f"use_layer_norm={self.use_layer_norm}, dropout={self.dropout_prob}")


GeometricAttentionLayer = GeometricAttention
