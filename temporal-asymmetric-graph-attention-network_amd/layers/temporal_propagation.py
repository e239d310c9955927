"""TemporalPropagation (drop-in for src/tagan/layers/temporal_propagation.py:402-1522).

Module tree, parameter names/shapes and initialisation order match the
reference (41 tensors at hidden_dim=64), so reference state_dicts load.

Forward keeps the SHIPPED contract (SURVEY.md header fact 4): in the
reference, ``TemporalPropagation.forward`` can never return —
  * node-id lists + no bank   -> UnboundLocalError (temporal_propagation.py:1231)
  * node-id lists + a bank    -> AttributeError 'restrict_temporal_attention' (:1287)
  * any other input           -> TypeError len(NodeMemoryBank) (:1485/:1505)
and TAGAN.forward falls back to identity (model.py:302-309).  This module
raises the same exception types without spending the dead compute; the TAGAN
host path (``tagan_amd.model``) takes the identity branch explicitly instead of
through an exception.  The submodules below are usable on their own.
"""
from typing import Any, List, Optional

import torch
import torch.nn as nn


class TemporalGRUCell(nn.Module):
    """temporal_propagation.py:402-558."""

    def __init__(self, input_dim: int, hidden_dim: int, dropout: float = 0.1, use_layer_norm: bool = True):
        super().__init__()
        self.input_dim, self.hidden_dim, self.dropout, self.use_layer_norm = input_dim, hidden_dim, dropout, use_layer_norm
        self.reset_gate = nn.Linear(input_dim + hidden_dim, hidden_dim)
        self.update_gate = nn.Linear(input_dim + hidden_dim, hidden_dim)
        self.candidate = nn.Linear(input_dim + hidden_dim, hidden_dim)
        if use_layer_norm:
            self.layer_norm_x = nn.LayerNorm(input_dim)
            self.layer_norm_h = nn.LayerNorm(hidden_dim)
            self.layer_norm_out = nn.LayerNorm(hidden_dim)
        self.dropout_layer = nn.Dropout(dropout)
        for lin in (self.reset_gate, self.update_gate, self.candidate):
            nn.init.xavier_uniform_(lin.weight)
            nn.init.zeros_(lin.bias)
        nn.init.constant_(self.reset_gate.bias, 1.0)
        nn.init.constant_(self.update_gate.bias, 1.0)

    def forward(self, x, h=None, time_diff=None):
        if x.dim() == 1:
            x = x.unsqueeze(0)
        if self.use_layer_norm:
            x = self.layer_norm_x(x)
        if h is None:
            h = torch.zeros(x.size(0), self.hidden_dim, device=x.device, dtype=x.dtype)
        elif self.use_layer_norm:
            h = self.layer_norm_h(h)
        if time_diff is not None:
            h = h * torch.exp(-torch.clamp(time_diff, min=0.0, max=10.0)).unsqueeze(1)
        if h.dim() == 1:
            h = h.unsqueeze(0)
        if x.size(0) != h.size(0):
            if x.size(0) == 1:
                x = x.expand(h.size(0), -1)
            elif h.size(0) == 1:
                h = h.expand(x.size(0), -1)
        xh = torch.cat([x, h], dim=-1)
        r = torch.sigmoid(self.reset_gate(xh))
        z = torch.sigmoid(self.update_gate(xh))
        h_tilde = torch.tanh(self.candidate(torch.cat([x, r * h], dim=-1)))
        h_new = self.dropout_layer((1 - z) * h + z * h_tilde)
        return self.layer_norm_out(h_new) if self.use_layer_norm else h_new


class TemporalEvolutionLayer(nn.Module):
    """temporal_propagation.py:561-765."""

    def __init__(self, input_dim: int, hidden_dim: int, dropout: float = 0.1, time_aware: bool = True,
                 bidirectional: bool = False, use_layer_norm: bool = True, residual: bool = True):
        super().__init__()
        self.input_dim, self.hidden_dim, self.dropout = input_dim, hidden_dim, dropout
        self.time_aware, self.bidirectional, self.use_layer_norm, self.residual = \
            time_aware, bidirectional, use_layer_norm, residual
        cell_h = hidden_dim // 2 if bidirectional else hidden_dim
        self.forward_cell = TemporalGRUCell(input_dim, cell_h, dropout, use_layer_norm)
        if bidirectional:
            self.backward_cell = TemporalGRUCell(input_dim, hidden_dim // 2, dropout, use_layer_norm)
        self.output_projection = nn.Linear(hidden_dim if bidirectional else cell_h, hidden_dim)
        if use_layer_norm:
            self.layer_norm = nn.LayerNorm(hidden_dim)
        self.dropout_layer = nn.Dropout(dropout)
        nn.init.xavier_uniform_(self.output_projection.weight)
        nn.init.zeros_(self.output_projection.bias)

    def forward(self, node_features_seq: List[torch.Tensor], time_stamps: Optional[torch.Tensor] = None):
        T = len(node_features_seq)
        has_time = time_stamps is not None and self.time_aware
        fwd, h = [], None
        for t in range(T):
            td = time_stamps[:, t] - time_stamps[:, t - 1] if (has_time and t > 0) else None
            h = self.forward_cell(node_features_seq[t], h, td)
            fwd.append(h)
        if self.bidirectional:
            bwd, hb = [None] * T, None
            for t in range(T - 1, -1, -1):
                td = time_stamps[:, t + 1] - time_stamps[:, t] if (has_time and t < T - 1) else None
                hb = self.backward_cell(node_features_seq[t], hb, td)
                bwd[t] = hb
            states = [torch.cat([fwd[t], bwd[t]], dim=1) for t in range(T)]
        else:
            states = fwd
        out = []
        for t in range(T):
            y = self.dropout_layer(self.output_projection(states[t]))
            if self.residual and self.input_dim == self.hidden_dim:
                y = y + node_features_seq[t]
            out.append(self.layer_norm(y) if self.use_layer_norm else y)
        return out


class TemporalSkipConnection(nn.Module):
    """temporal_propagation.py:768-957."""

    def __init__(self, input_dim: int, hidden_dim: Optional[int] = None, window_size: int = 3,
                 aggregation: str = "mean", dropout: float = 0.1, use_layer_norm: bool = True,
                 apply_activation: bool = True, residual: bool = True):
        super().__init__()
        self.input_dim = input_dim
        self.hidden_dim = hidden_dim if hidden_dim is not None else input_dim
        self.window_size, self.aggregation, self.dropout = window_size, aggregation, dropout
        self.use_layer_norm, self.apply_activation, self.residual = use_layer_norm, apply_activation, residual
        self.input_proj = nn.Linear(input_dim, self.hidden_dim)
        self.output_proj = nn.Linear(self.hidden_dim, input_dim)
        if use_layer_norm:
            self.layer_norm1 = nn.LayerNorm(self.hidden_dim)
            self.layer_norm2 = nn.LayerNorm(input_dim)
        self.dropout_layer = nn.Dropout(dropout)
        self.act_fn = nn.GELU()
        for lin in (self.input_proj, self.output_proj):
            nn.init.xavier_uniform_(lin.weight)
            nn.init.zeros_(lin.bias)

    def forward(self, node_features_seq: List[torch.Tensor], time_weights=None):
        T = len(node_features_seq)
        proj = []
        for f in node_features_seq:
            p = self.input_proj(f)
            if self.apply_activation:
                p = self.act_fn(p)
            if self.use_layer_norm:
                p = self.layer_norm1(p)
            proj.append(self.dropout_layer(p))
        agg = []
        for t in range(T):
            win = torch.stack(proj[max(0, t - self.window_size): min(T, t + self.window_size + 1)], 0)
            if self.aggregation == "mean":
                agg.append(win.mean(0))
            elif self.aggregation == "max":
                agg.append(win.max(0)[0])
            else:
                agg.append(win.sum(0))
        out = [self.dropout_layer(self.output_proj(self.act_fn(a))) for a in agg]
        if self.residual:
            out = [o + x for o, x in zip(out, node_features_seq)]
        if self.use_layer_norm:
            out = [self.layer_norm2(o) for o in out]
        return out


class TemporalGatingUnit(nn.Module):
    """temporal_propagation.py:960-1075."""

    def __init__(self, input_dim: int, hidden_dim: Optional[int] = None, dropout: float = 0.1,
                 use_layer_norm: bool = True, residual: bool = True):
        super().__init__()
        self.input_dim = input_dim
        self.hidden_dim = hidden_dim if hidden_dim is not None else input_dim
        self.dropout, self.use_layer_norm, self.residual = dropout, use_layer_norm, residual
        self.update_gate = nn.Linear(input_dim * 2, input_dim)
        self.reset_gate = nn.Linear(input_dim * 2, input_dim)
        self.output_gate = nn.Linear(input_dim * 2, input_dim)
        if use_layer_norm:
            self.layer_norm_in1 = nn.LayerNorm(input_dim)
            self.layer_norm_in2 = nn.LayerNorm(input_dim)
            self.layer_norm_out = nn.LayerNorm(input_dim)
        self.dropout_layer = nn.Dropout(dropout)
        for lin in (self.update_gate, self.reset_gate, self.output_gate):
            nn.init.xavier_uniform_(lin.weight)
            nn.init.zeros_(lin.bias)

    def forward(self, current_feat, previous_feat):
        if self.use_layer_norm:
            current_feat = self.layer_norm_in1(current_feat)
            previous_feat = self.layer_norm_in2(previous_feat)
        comb = torch.cat([current_feat, previous_feat], dim=1)
        u = torch.sigmoid(self.update_gate(comb))
        r = torch.sigmoid(self.reset_gate(comb))
        cand = torch.tanh(self.output_gate(torch.cat([current_feat, r * previous_feat], dim=1)))
        out = self.dropout_layer((1 - u) * current_feat + u * cand)
        if self.residual:
            out = out + current_feat
        return self.layer_norm_out(out) if self.use_layer_norm else out


class TemporalPropagation(nn.Module):
    """temporal_propagation.py:1078-1522 (shipped contract: forward always raises)."""

    def __init__(self, input_dim: int, hidden_dim: int, dropout: float = 0.1, time_aware: bool = True,
                 bidirectional: bool = False, use_layer_norm: bool = True, use_skip_connection: bool = True,
                 use_gating: bool = True, window_size: int = 3, aggregation: str = "mean", residual: bool = True):
        super().__init__()
        self.input_dim, self.hidden_dim, self.dropout = input_dim, hidden_dim, dropout
        self.time_aware, self.bidirectional, self.use_layer_norm = time_aware, bidirectional, use_layer_norm
        self.use_skip_connection, self.use_gating = use_skip_connection, use_gating
        self.window_size, self.aggregation, self.residual = window_size, aggregation, residual
        self.evolution_layer = TemporalEvolutionLayer(input_dim, hidden_dim, dropout, time_aware, bidirectional,
                                                      use_layer_norm, residual)
        if use_skip_connection:
            self.skip_connection = TemporalSkipConnection(input_dim=hidden_dim, window_size=window_size,
                                                          aggregation=aggregation, dropout=dropout,
                                                          use_layer_norm=use_layer_norm, residual=residual)
        if use_gating:
            self.gating_unit = TemporalGatingUnit(input_dim=hidden_dim, dropout=dropout,
                                                  use_layer_norm=use_layer_norm, residual=residual)
        self.state_tracking = nn.Parameter(torch.ones(1, 3), requires_grad=True)
        self.dropout_layer = nn.Dropout(dropout)
        self.output_proj = nn.Linear(hidden_dim, hidden_dim)
        if use_layer_norm:
            self.layer_norm = nn.LayerNorm(hidden_dim)

    @staticmethod
    def shipped_outcome(node_masks_seq, memory_bank) -> type:
        """Exception type the reference forward raises for these arguments (never returns)."""
        ids = isinstance(node_masks_seq, list) and len(node_masks_seq) > 0 and \
            not isinstance(node_masks_seq[0], torch.Tensor)
        if ids:
            return UnboundLocalError if memory_bank is None else AttributeError
        return TypeError

    def forward(self, node_features_seq: List[torch.Tensor], node_masks_seq=None,
                time_stamps: Optional[torch.Tensor] = None, memory_bank: Optional[Any] = None):
        kind = self.shipped_outcome(node_masks_seq, memory_bank)
        if kind is UnboundLocalError:
            raise UnboundLocalError("local variable 'device' referenced before assignment "
                                    "(temporal_propagation.py:1231)")
        if kind is AttributeError:
            raise AttributeError("'TemporalPropagation' object has no attribute 'restrict_temporal_attention'")
        self.temporal_mask = None
        raise TypeError("object of type 'NodeMemoryBank' has no len()")

    def extra_repr(self) -> str:
        return (f"input_dim={self.input_dim}, hidden_dim={self.hidden_dim}, dropout={self.dropout}, "
                f"time_aware={self.time_aware}, bidirectional={self.bidirectional}, "
                f"use_layer_norm={self.use_layer_norm}, use_skip_connection={self.use_skip_connection}, "
                f"use_gating={self.use_gating}, window_size={self.window_size}, "
                f"aggregation={self.aggregation}, residual={self.residual}")
