"""Temporal attention on MI355X (drop-in for src/tagan/layers/temporal_attention.py).

``TimeEncoding``, ``TemporalAttention`` and ``AsymmetricTemporalAttention`` keep
the reference constructors, parameter names/shapes and initialisation order.
Forward = LN1 + QKV projection (hand-written stream GEMM, csrc/stream_gemm.hip; LN1 in
its prologue at H = 128) -> ``tagan_temporal_attn_fwd`` (QKᵀ/√d + folded
relative-position/asymmetric-kernel bias table [+ time bias] -> masks -> softmax ->
attn-dropout -> A·V per node row, HIP) -> out-projection stream GEMM with dropout +
residual + LN2 in its epilogue at H = 128 (standalone LayerNorm kernels at H = 64 / 256).

Snapshot lists are kept **time-major** ([T, N_max, H], the natural result of
stacking snapshots) — the kernel takes strides, so the reference's
``permute(1, 0, 2)`` (:972) is never materialised on the hot path.

Mask semantics follow the reference exactly, including its quirks
(:1072-1170): an all-ones [T,T] mask becomes causal only when T == num_heads,
otherwise the broadcast fails and attention is unmasked; a shape-mismatched
mask becomes causal; a [B,T,T] all-ones mask becomes causal.
"""
import math
from typing import List, Optional, Tuple, Union

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..fused import TemporalCore, attention_block, fusable
from ..kernels import (BiasTableFn, TemporalAttnFn, TemporalMask, dropout_add_layer_norm, fused_qkv, layer_norm,
                       linear, new_seed)


class MaskBroadcastError(RuntimeError):
    """The reference layer raises here (a mask broadcast enlarges the scores; reshape at :1187 fails)."""


class TimeEncoding(nn.Module):
    """temporal_attention.py:15-306 (basis RBF encoding used by the time-aware branch)."""

    def __init__(self, d_model: int, max_len: int = 5000, learnable: bool = False,
                 encoding_type: str = "sinusoidal", dropout: float = 0.1, num_bases: int = 16, scale: float = 1.0):
        super().__init__()
        self.d_model, self.max_len, self.learnable = d_model, max_len, learnable
        self.encoding_type, self.num_bases, self.scale = encoding_type, num_bases, scale
        self.dropout = nn.Dropout(p=dropout)
        if encoding_type in ("sinusoidal", "linear", "log"):
            pos = torch.arange(0, max_len, dtype=torch.float).unsqueeze(1)
            if encoding_type == "sinusoidal":
                pe = torch.zeros(max_len, d_model)
                div = torch.exp(torch.arange(0, d_model, 2).float() * (-math.log(10000.0) / d_model))
                pe[:, 0::2] = torch.sin(pos * div)
                pe[:, 1::2] = torch.cos(pos * div)
            elif encoding_type == "linear":
                pe = (pos / max_len).repeat(1, d_model)
            else:
                pe = (torch.log(torch.arange(1, max_len + 1, dtype=torch.float).unsqueeze(1))
                      / math.log(max_len)).repeat(1, d_model)
            pe = pe.unsqueeze(0)
            if learnable:
                self.register_parameter("pe", nn.Parameter(pe))
            else:
                self.register_buffer("pe", pe)
        elif encoding_type == "learned":
            self.pe = nn.Parameter(torch.randn(1, max_len, d_model))
        elif encoding_type == "basis":
            self.basis_mu = nn.Parameter(torch.linspace(0, 1, num_bases))
            self.basis_sigma = nn.Parameter(torch.ones(num_bases) * 0.1)
            self.basis_proj = nn.Linear(num_bases, d_model)
        else:
            self.register_buffer("pe", torch.zeros(1, max_len, d_model))

    def _basis(self, tv: torch.Tensor) -> torch.Tensor:
        tv = torch.nan_to_num(tv, nan=0.0)
        tmin, tmax = tv.min(), tv.max()
        rng = tmax - tmin
        ok = (tmax > tmin) & (rng > 1e-7)
        tn = torch.where(ok, (tv - tmin) / torch.where(ok, rng, torch.ones_like(rng)), torch.zeros_like(tv))
        sigma = self.basis_sigma
        sigma = torch.where(sigma.min() < 1e-7, torch.clamp(sigma, min=1e-7), sigma)
        expo = torch.clamp(-(((tn.unsqueeze(-1) - self.basis_mu) ** 2) / (2 * sigma ** 2)), -88.0, 88.0)
        enc = self.basis_proj(torch.nan_to_num(torch.exp(expo), nan=0.0))
        return torch.nan_to_num(enc, nan=0.0)

    def forward(self, time_values: Optional[torch.Tensor] = None, x: Optional[torch.Tensor] = None):
        if self.encoding_type == "basis" and time_values is not None:
            enc = self._basis(time_values)
        else:
            if time_values is not None:
                tmin, tmax = time_values.min(), time_values.max()
                if bool(tmax > tmin):
                    pos = ((time_values - tmin) / (tmax - tmin) * (self.max_len - 1)).long()
                else:
                    pos = torch.zeros_like(time_values, dtype=torch.long)
                pos = torch.clamp(pos, 0, self.max_len - 1)
            elif x is not None:
                pos = torch.arange(0, x.size(1), device=x.device).expand(x.size(0), x.size(1))
            else:
                raise ValueError("Either time_values or x must be provided")
            if not hasattr(self, "pe"):
                return x if x is not None else torch.zeros(*pos.shape, self.d_model, device=pos.device)
            enc = self.pe[:, pos]
        enc = self.dropout(enc * self.scale)
        return x + enc if x is not None else enc


def _stack_time_major(xs: List[torch.Tensor]) -> torch.Tensor:
    """List of [N_t,H] -> zero-padded, time-major [T, N_max, H] (temporal_attention.py:928-968, minus the permute)."""
    xs = [t[0] if isinstance(t, list) and len(t) > 0 else t for t in xs]
    n_max = max(int(t.shape[0]) for t in xs)
    if all(int(t.shape[0]) == n_max for t in xs):
        return torch.stack(xs, 0)
    out = xs[0].new_zeros(len(xs), n_max, xs[0].shape[1])
    for i, t in enumerate(xs):
        out[i, : t.shape[0]] = t
    return out


def _keep_from_em(em: torch.Tensor, B: int, h: int, T: int) -> Tuple[Optional[TemporalMask], bool]:
    """Turn a mask tensor broadcastable to scores [B,h,T,T] into kernel form.

    Returns (mask, explode): (None, False) when masked_fill would raise (the
    reference swallows it: unmasked); (None, True) when the broadcast enlarges
    the score tensor (the reference raises later).
    """
    try:
        shape = torch.broadcast_shapes(tuple(em.shape), (B, h, T, T))
    except RuntimeError:
        return None, False
    if tuple(shape) != (B, h, T, T):
        return None, True
    em4 = em.reshape((1,) * (4 - em.dim()) + tuple(em.shape))
    b_dim = B if (em4.shape[0] == B and B > 1) else 1
    h_dim = h if (em4.shape[1] == h and h > 1) else 1
    keep = (em4 != 0).expand(b_dim, h_dim, T, T).to(torch.uint8).contiguous()
    return TemporalMask(False, keep, h_dim * T * T if b_dim > 1 else 0, T * T if h_dim > 1 else 0), False


class TemporalAttention(nn.Module):
    """temporal_attention.py:309-621."""

    def __init__(self, hidden_dim: int, num_heads: int = 8, dropout: float = 0.1, causal: bool = False,
                 use_layer_norm: bool = True):
        super().__init__()
        self.hidden_dim = hidden_dim
        self.num_heads = num_heads
        self.dropout_prob = dropout
        self.causal = causal
        self.use_layer_norm = use_layer_norm
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
        self._init_parameters()

    def _init_parameters(self):
        for lin in (self.q_linear, self.k_linear, self.v_linear, self.output_proj):
            nn.init.xavier_uniform_(lin.weight)
        for lin in (self.q_linear, self.k_linear, self.v_linear, self.output_proj):
            nn.init.zeros_(lin.bias)

    def _create_causal_mask(self, seq_len: int, device) -> torch.Tensor:
        return torch.tril(torch.ones(seq_len, seq_len, device=device)).unsqueeze(0)

    # ---- hooks for the subclass
    def _bias_table(self, T, device):
        return None

    def _bias_dense_and_mask(self, x_shape, time_stamps, attention_mask, device):
        return None, self._base_mask(attention_mask, x_shape, device), False

    def _base_mask(self, attention_mask, x_shape, device) -> TemporalMask:
        """Mask logic of TemporalAttention.forward (temporal_attention.py:501-588)."""
        B, T, h = x_shape[0], x_shape[1], self.num_heads
        mask = TemporalMask(causal=self.causal)
        if attention_mask is None:
            return mask
        if isinstance(attention_mask, list):
            try:
                attention_mask = torch.stack(attention_mask, dim=0)
            except Exception:
                attention_mask = torch.ones(T, T, device=device)
        ms = tuple(attention_mask.shape)
        em = None
        if len(ms) == 2:
            if ms == (T, T):
                em = attention_mask.unsqueeze(0).unsqueeze(0)
            elif ms[0] == T and self.causal:
                em = None   # ones * tril == the causal flag already set
        elif len(ms) == 3 and ms[0] == B and ms[1] == ms[2]:
            em = attention_mask.unsqueeze(1)
        if em is None:
            return mask
        km, explode = _keep_from_em(em, B, h, T)
        if km is None or explode:
            return mask
        km.causal = self.causal
        return km

    def _run(self, x: torch.Tensor, time_major: bool, time_stamps=None, attention_mask=None,
             want_attn: bool = False, _known_ones_mask: bool = False):
        """x: [B,T,H] (row-major) or [T,B,H] (time_major).  Returns (out same layout, attn or None)."""
        if time_major:
            T, B, H = x.shape
        else:
            B, T, H = x.shape
        if _known_ones_mask:
            bias_dense, mask, explode = None, self._ones_mask_fast(B, T), False
        else:
            bias_dense, mask, explode = self._bias_dense_and_mask((B, T), time_stamps, attention_mask, x.device)
        if explode:
            raise MaskBroadcastError("attention mask broadcast enlarges the score tensor "
                                     "(the reference raises at temporal_attention.py:1187)")
        p = self.attn_dropout.p if self.training else 0.0
        p_out = self.output_dropout.p if self.training else 0.0
        if not want_attn and fusable(x, self.use_layer_norm):   # one autograd node for the layer (fused.py)
            core = TemporalCore(T, B, time_major, self.num_heads, mask, p, new_seed() if p > 0 else 0)
            y = attention_block(x, core, self._bias_table(T, x.device), bias_dense, self.layer_norm1,
                                self.q_linear, self.k_linear, self.v_linear, self.output_proj, self.layer_norm2,
                                p_out, new_seed() if p_out > 0 else 0)
            return y, None
        identity = x
        hx = layer_norm(x, self.layer_norm1) if self.use_layer_norm else x
        qkv = fused_qkv(hx, self.q_linear, self.k_linear, self.v_linear).contiguous()
        ctx, attn = TemporalAttnFn.apply(qkv, self._bias_table(T, x.device), bias_dense, time_major,
                                         self.num_heads, mask, p, new_seed() if p > 0 else 0, want_attn)
        proj = linear(ctx, self.output_proj.weight, self.output_proj.bias)
        if self.use_layer_norm:
            return dropout_add_layer_norm(proj, identity, self.layer_norm2, p_out), attn
        return F.dropout(proj, p_out, True) + identity, attn

    def _ones_mask_fast(self, B, T):
        # an all-ones [T,T] mask expands to every (b, h): nothing is masked beyond the causal flag
        return TemporalMask(causal=self.causal)

    def forward(self, x: Union[torch.Tensor, List[torch.Tensor]], attention_mask=None,
                return_attention_weights: bool = False):
        if isinstance(x, list):
            xt = _stack_time_major(x)
            out, attn = self._run(xt, True, None, attention_mask, return_attention_weights)
            out = out.permute(1, 0, 2).contiguous()
        else:
            out, attn = self._run(x, False, None, attention_mask, return_attention_weights)
        return (out, attn) if return_attention_weights else out


class AsymmetricTemporalAttention(TemporalAttention):
    """temporal_attention.py:624-1217."""

    def __init__(self, hidden_dim: int, num_heads: int = 8, dropout: float = 0.1, causal: bool = False,
                 time_aware: bool = True, use_layer_norm: bool = True, asymmetric_window_size: int = 5,
                 future_discount: float = 0.8, relative_position_bias: bool = True, max_relative_position: int = 32,
                 time_encoding_type: str = "basis", use_time_masks: bool = True):
        super().__init__(hidden_dim, num_heads, dropout, causal, use_layer_norm)
        self.time_aware = time_aware
        self.asymmetric_window_size = asymmetric_window_size
        self.future_discount = future_discount
        self.relative_position_bias = relative_position_bias
        self.max_relative_position = max_relative_position
        self.time_encoding_type = time_encoding_type
        self.use_time_masks = use_time_masks
        if relative_position_bias:
            self.relative_pos_table = nn.Parameter(torch.zeros((2 * max_relative_position + 1, num_heads)))
            nn.init.xavier_uniform_(self.relative_pos_table)
        if time_aware:
            self.time_encoding = TimeEncoding(d_model=hidden_dim, learnable=True, encoding_type=time_encoding_type,
                                              num_bases=hidden_dim // 4)
            self.time_q_proj = nn.Linear(hidden_dim, num_heads)
            self.time_k_proj = nn.Linear(hidden_dim, num_heads)
            nn.init.xavier_uniform_(self.time_q_proj.weight)
            nn.init.xavier_uniform_(self.time_k_proj.weight)
            nn.init.zeros_(self.time_q_proj.bias)
            nn.init.zeros_(self.time_k_proj.bias)
        W = asymmetric_window_size
        kern = torch.ones(2 * W + 1, num_heads)
        for i in range(2 * W + 1):
            dist = abs(i - W)
            if i < W:
                kern[i] = 1.0 - 0.5 * (dist / W)
            elif i > W:
                kern[i] = future_discount * (1.0 - 0.5 * (dist / W))
        self.asymmetric_kernel = nn.Parameter(kern)

    def _get_relative_positions(self, seq_len: int, device) -> torch.Tensor:
        pos = torch.arange(seq_len, device=device)
        rel = pos.unsqueeze(1) - pos.unsqueeze(0) + self.max_relative_position
        return torch.clamp(rel, 0, 2 * self.max_relative_position)

    def _get_asymmetric_kernel_values(self, seq_len: int, device) -> torch.Tensor:
        pos = torch.arange(seq_len, device=device)
        rel = pos.unsqueeze(1) - pos.unsqueeze(0)
        W = self.asymmetric_window_size
        vals = self.asymmetric_kernel[torch.clamp(rel + W, 0, 2 * W)]
        return vals * ((rel >= -W) & (rel <= W)).unsqueeze(-1).float()

    def _selectors(self, T, device, dtype):
        """0/1 matrices that gather the two tables by diagonal: A[t, k] = [k == clamp(t-T+1+W)]·[|t-T+1| <= W],
        Rsel[t, k] = [k == clamp(t-T+1+m)].  A gather as a GEMM: its backward is a GEMM too (deterministic, two
        small launches) instead of the sort-based index_put of advanced-indexing backward.  Cached per (T, device)."""
        key = (T, str(device), dtype)
        cache = self.__dict__.setdefault("_sel_cache", {})
        if key not in cache:
            delta = torch.arange(-(T - 1), T, device=device)
            W = self.asymmetric_window_size
            a = torch.nn.functional.one_hot(torch.clamp(delta + W, 0, 2 * W), 2 * W + 1).to(dtype)
            a = a * ((delta >= -W) & (delta <= W)).unsqueeze(-1).to(dtype)
            r = None
            if self.relative_position_bias:
                m = self.max_relative_position
                r = torch.nn.functional.one_hot(torch.clamp(delta + m, 0, 2 * m), 2 * m + 1).to(dtype)
            cache[key] = (a, r)
        return cache[key]

    def _bias_table(self, T, device):
        """[heads, 2T-1] table, entry [h][i-j+T-1] = R[clamp(i-j+32)] + K[clamp(i-j+W)]·[|i-j|<=W] (:1010-1027)."""
        if (self.asymmetric_kernel.is_cuda and self.asymmetric_kernel.dtype == torch.float32
                and (not self.relative_position_bias or self.relative_pos_table.dtype == torch.float32)):
            return BiasTableFn.apply(self.asymmetric_kernel,
                                     self.relative_pos_table if self.relative_position_bias else None, T,
                                     self.asymmetric_window_size, self.max_relative_position)
        a, r = self._selectors(T, device, self.asymmetric_kernel.dtype)
        tab = a @ self.asymmetric_kernel                   # exact: one nonzero (1.0) term per row
        if r is not None:
            tab = r @ self.relative_pos_table + tab
        return tab.t().contiguous()

    def _time_bias(self, time_stamps: torch.Tensor, B: int, T: int) -> torch.Tensor:
        """_compute_time_based_attention (temporal_attention.py:792-871): [B, heads, T, T]."""
        diffs = (time_stamps.unsqueeze(2) - time_stamps.unsqueeze(1)).reshape(B * T * T, 1)
        enc = self.time_encoding(diffs).view(B, T, T, self.hidden_dim)
        return self.time_q_proj(enc).permute(0, 3, 1, 2)

    def _ones_mask_fast(self, B, T):
        # all-ones [T,T] mask (model.py:335-339): ones.unsqueeze(1)*tril -> [T,T,T]; broadcast vs [B,h,T,T]
        h = self.num_heads
        if T == 1 or T == h:
            return TemporalMask(causal=True)
        if h == 1:
            raise MaskBroadcastError("[T,T] mask with one head (reference raises at :1187)")
        return TemporalMask(causal=self.causal)

    def _bias_dense_and_mask(self, bt_shape, time_stamps, attention_mask, device):
        B, T = bt_shape
        h = self.num_heads
        bias_dense = None
        time_mask = None
        if self.time_aware and time_stamps is not None:
            bias_dense = self._time_bias(time_stamps, B, T)
            if self.use_time_masks:
                time_mask = (torch.abs(time_stamps.unsqueeze(2) - time_stamps.unsqueeze(1)) <= 10.0).float()
        if time_mask is not None:
            if attention_mask is None:
                attention_mask = time_mask
            elif isinstance(attention_mask, torch.Tensor) and attention_mask.shape[-2:] == time_mask.shape[-2:]:
                attention_mask = attention_mask * time_mask
        mask = TemporalMask(causal=self.causal)
        if attention_mask is None:
            return bias_dense, mask, False
        if isinstance(attention_mask, list):
            L = len(attention_mask)
            attention_mask = torch.ones(B, L, L, device=device)
        if attention_mask.shape[-1] != T or attention_mask.shape[-2] != T:
            return bias_dense, TemporalMask(causal=True), False          # resized to tril (:1118-1132)
        em = attention_mask.unsqueeze(1)
        if em.numel() == 0:
            return bias_dense, mask, False
        if bool(torch.all(em == 1.0)):
            em_shape = torch.broadcast_shapes(tuple(em.shape), (T, T))
            try:
                shape = torch.broadcast_shapes(em_shape, (B, h, T, T))
            except RuntimeError:
                return bias_dense, mask, False
            if tuple(shape) != (B, h, T, T):
                return bias_dense, mask, True
            return bias_dense, TemporalMask(causal=True), False
        km, explode = _keep_from_em(em, B, h, T)
        if km is None:
            return bias_dense, mask, explode
        km.causal = self.causal
        return bias_dense, km, False

    def forward(self, x: Union[torch.Tensor, List[torch.Tensor]], time_stamps: Optional[torch.Tensor] = None,
                attention_mask=None, return_attention_weights: bool = False):
        if isinstance(x, list):
            xt = _stack_time_major(x)
            out, attn = self._run(xt, True, time_stamps, attention_mask, return_attention_weights)
            out = out.permute(1, 0, 2).contiguous()
        else:
            out, attn = self._run(x, False, time_stamps, attention_mask, return_attention_weights)
        return (out, attn) if return_attention_weights else out

    def forward_time_major(self, xt: torch.Tensor, ones_mask: bool = True, return_attention_weights=False):
        """TAGAN hot path: xt [T, N_max, H]; ``ones_mask`` = the ones(T,T) mask TAGAN always passes."""
        return self._run(xt, True, None, None if not ones_mask else True, return_attention_weights,
                         _known_ones_mask=ones_mask)

    def extra_repr(self) -> str:
        return (f"hidden_dim={self.hidden_dim}, num_heads={self.num_heads}, time_aware={self.time_aware}, "
                f"causal={self.causal}, asymmetric_window_size={self.asymmetric_window_size}, "
                f"future_discount={self.future_discount}, relative_position_bias={self.relative_position_bias}, "
                f"use_layer_norm={self.use_layer_norm}, dropout={self.dropout_prob}")
