"""TemporalPropagation (drop-in for src/tagan/layers/temporal_propagation.py:402-1522).

Module tree, parameter names/shapes and initialisation order match the
reference (41 tensors at hidden_dim=64), so reference state_dicts load.

``forward`` keeps the SHIPPED contract (SURVEY.md header fact 4): in the
reference, ``TemporalPropagation.forward`` can never return —
  * node-id lists + no bank   -> UnboundLocalError (temporal_propagation.py:1231)
  * node-id lists + a bank    -> AttributeError 'restrict_temporal_attention' (:1287)
  * any other input           -> TypeError len(NodeMemoryBank) (:1485/:1505)
and TAGAN.forward falls back to identity (model.py:302-309).  This module
raises the same exception types without spending the dead compute.

``forward_intended`` is the compute the reference was written to do with tensor
masks (pinned by the tprop_* fixtures, G6): GRU evolution
over T -> windowed skip connection -> output_proj -> dropout -> LayerNorm.  It runs
time-major ([T, N, H], node rows independent) on the device: the x-side of all three
GRU gates for all T steps is ONE GEMM, the whole recurrence over T (recurrent products,
gates, both LayerNorms, dropout) is ONE kernel each way (csrc/gru.hip, GRUSeqFn), the
residual tails run on the HIP LayerNorm kernels, the window aggregation is one kernel
pass over T each way (csrc/window.hip, WindowFn).  TAGAN uses it
when constructed with ``temporal_propagation="intended"`` (default "shipped").
The submodules keep their reference list-in/list-out forwards (on the same device
code) for standalone use.
"""
import os
from typing import Any, List, Optional

import torch
import torch.nn as nn

from .._lib import check, lib, ptr, require_hip, stream_of
from ..kernels import dropout_add_layer_norm, layer_norm, linear, new_seed, weight_grad


# TAGAN_GRU_KERNEL=0: step the recurrence from Python (two GEMMs + gate ops per step) instead of csrc/gru.hip
USE_GRU_KERNEL = os.environ.get("TAGAN_GRU_KERNEL", "1") != "0"


def _ln(x, mod):
    return layer_norm(x, mod) if mod is not None else x


class GRUSeqFn(torch.autograd.Function):
    """The whole recurrence over T in one kernel each way (csrc/gru.hip): gx [T, N, 3hc] (x-side gates) ->
    states [T, N, hc]; backward gives d gx, the h-side weight gradients (two split-K GEMMs against the saved
    hn and r⊙hn) and the two LayerNorms' parameter gradients."""

    @staticmethod
    def forward(ctx, gx, w_rz, w_c, lnh_w, lnh_b, lno_w, lno_b, tscale, eps_h: float, eps_o: float, p: float,
                seed: int):
        T, N, H3 = gx.shape
        hc = H3 // 3
        dev = gx.device
        L = lib()
        gx = gx.contiguous()
        states = torch.empty(T, N, hc, device=dev)
        saved = torch.empty(int(L.tagan_gru_saved_floats(N, T, hc)), device=dev)
        prm = [None if t is None else t.detach().contiguous() for t in (w_rz, w_c, lnh_w, lnh_b, lno_w, lno_b)]
        check(L.tagan_gru_fwd(N, T, hc, ptr(gx), ptr(prm[0]), ptr(prm[1]), ptr(prm[2]), ptr(prm[3]), float(eps_h),
                              ptr(prm[4]), ptr(prm[5]), float(eps_o), ptr(tscale), float(p), seed, ptr(states),
                              ptr(saved), stream_of(gx)), "tagan_gru_fwd")
        ctx.save_for_backward(states, saved, tscale, *prm)
        ctx.cfg = (T, N, hc, p, seed)
        return states

    @staticmethod
    def backward(ctx, dstates):
        states, saved, tscale, w_rz, w_c, lnh_w, lnh_b, lno_w, lno_b = ctx.saved_tensors
        T, N, hc, p, seed = ctx.cfg
        dev = states.device
        L = lib()
        dgx = torch.empty(T, N, 3 * hc, device=dev)
        d = [torch.empty(hc, device=dev) if t is not None else None for t in (lnh_w, lnh_b, lno_w, lno_b)]
        wsb = L.tagan_gru_bwd_workspace(N, hc)
        ws = torch.empty(int(wsb), dtype=torch.uint8, device=dev)
        check(L.tagan_gru_bwd(N, T, hc, ptr(w_rz), ptr(w_c), ptr(lnh_w), ptr(lnh_b), ptr(lno_w), ptr(lno_b),
                              ptr(tscale), float(p), seed, ptr(states), ptr(saved), ptr(dstates.contiguous()),
                              ptr(dgx), *[ptr(t) for t in d], ptr(ws), wsb, stream_of(states)), "tagan_gru_bwd")
        S = T * N * hc
        hn = saved[:S].view(T * N, hc)
        rh = saved[S:2 * S].view(T * N, hc)
        g2 = dgx.view(T * N, 3 * hc)
        dw_rz = weight_grad(g2[:, :2 * hc], hn) if ctx.needs_input_grad[1] else None
        dw_c = weight_grad(g2[:, 2 * hc:], rh) if ctx.needs_input_grad[2] else None
        return (dgx, dw_rz, dw_c, *d, None, None, None, None, None)


def gru_sequence(cell: "TemporalGRUCell", gx: torch.Tensor, tscale: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    """All T recurrent steps of ``cell`` on the device kernel (gx [T, N, 3hc] from ``cell.x_gates``), or None when
    the cell's width is not one the kernel takes (the caller then steps in Python)."""
    hc = cell.hidden_dim
    if not (gx.is_cuda and gx.dtype == torch.float32 and lib().tagan_gru_supported(hc)):
        return None
    D = cell.input_dim
    w_rz = torch.cat([cell.reset_gate.weight[:, D:], cell.update_gate.weight[:, D:]], 0)
    w_c = cell.candidate.weight[:, D:]
    ln = cell.use_layer_norm
    p = cell.dropout_layer.p if cell.training else 0.0
    seed = new_seed() if p > 0 else 0
    return GRUSeqFn.apply(gx, w_rz, w_c, cell.layer_norm_h.weight if ln else None,
                          cell.layer_norm_h.bias if ln else None, cell.layer_norm_out.weight if ln else None,
                          cell.layer_norm_out.bias if ln else None, tscale,
                          cell.layer_norm_h.eps if ln else 1e-5, cell.layer_norm_out.eps if ln else 1e-5, p, seed)


_AGG_MODE = {"mean": 0, "max": 1}   # anything else sums (temporal_propagation.py:912-925)


class WindowFn(torch.autograd.Function):
    """±w window aggregation over T of a time-major [T, N, H] tensor in one pass each way (csrc/window.hip)."""

    @staticmethod
    def forward(ctx, x, w: int, mode: int):
        T, N, H = x.shape
        x = x.contiguous()
        out = torch.empty_like(x)
        check(lib().tagan_window_fwd(mode, T, N, H, w, ptr(x), ptr(out), stream_of(x)), "tagan_window_fwd")
        ctx.save_for_backward(x if mode == 1 else None)
        ctx.cfg = (w, mode, T, N, H)
        return out

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        w, mode, T, N, H = ctx.cfg
        dy = dy.contiguous()
        dx = torch.empty_like(dy)
        check(lib().tagan_window_bwd(mode, T, N, H, w, ptr(x), ptr(dy), ptr(dx), stream_of(dy)), "tagan_window_bwd")
        return dx, None, None


def window_aggregate(x: torch.Tensor, w: int, aggregation: str) -> torch.Tensor:
    """TemporalSkipConnection's windowed aggregation (mean over the in-range steps / max / sum) of x [T, N, H]."""
    if w <= 0:
        return x
    if x.shape[-1] % 4 == 0 and x.dtype == torch.float32:
        return WindowFn.apply(x, int(w), _AGG_MODE.get(aggregation, 2))
    # widths the kernel's float4 lanes do not take: the same windows as device pooling along T
    T, N, Hd = x.shape
    seq = x.permute(1, 2, 0).reshape(N * Hd, 1, T)
    k = 2 * w + 1
    if aggregation == "mean":
        agg = torch.nn.functional.avg_pool1d(seq, k, 1, w, count_include_pad=False)
    elif aggregation == "max":
        agg = torch.nn.functional.max_pool1d(seq, k, 1, w)
    else:
        agg = torch.nn.functional.avg_pool1d(seq, k, 1, w, count_include_pad=True) * k
    return agg.reshape(N, Hd, T).permute(2, 0, 1)


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

    def x_gates(self, x: torch.Tensor) -> torch.Tensor:
        """x-side of the three gates for any number of rows: [.., D_in] -> [.., 3*H_c] (LN_x, one GEMM)."""
        D = self.input_dim
        x = _ln(x, self.layer_norm_x if self.use_layer_norm else None)
        w = torch.cat([self.reset_gate.weight[:, :D], self.update_gate.weight[:, :D],
                       self.candidate.weight[:, :D]], 0)
        b = torch.cat([self.reset_gate.bias, self.update_gate.bias, self.candidate.bias], 0)
        return linear(x, w, b)

    def step(self, gx: torch.Tensor, h: Optional[torch.Tensor], time_diff: Optional[torch.Tensor] = None):
        """One recurrent step (temporal_propagation.py:475-551) given the precomputed x-side ``gx``."""
        D, hc = self.input_dim, self.hidden_dim
        if h is None:
            hn = None
        else:
            hn = _ln(h, self.layer_norm_h if self.use_layer_norm else None)
            if time_diff is not None:
                hn = hn * torch.exp(-torch.clamp(time_diff, min=0.0, max=10.0)).unsqueeze(1)
        if hn is None:   # h = 0: the recurrent GEMMs vanish
            rz = torch.sigmoid(gx[:, :2 * hc])
            z = rz[:, hc:]
            h_new = z * torch.tanh(gx[:, 2 * hc:])
        else:
            w_rz = torch.cat([self.reset_gate.weight[:, D:], self.update_gate.weight[:, D:]], 0)
            rz = torch.sigmoid(gx[:, :2 * hc] + linear(hn, w_rz))
            r, z = rz[:, :hc], rz[:, hc:]
            h_tilde = torch.tanh(gx[:, 2 * hc:] + linear(r * hn, self.candidate.weight[:, D:]))
            h_new = (1 - z) * hn + z * h_tilde
        h_new = self.dropout_layer(h_new)
        return _ln(h_new, self.layer_norm_out if self.use_layer_norm else None)

    def forward(self, x, h=None, time_diff=None):
        require_hip(x, h)
        if x.dim() == 1:
            x = x.unsqueeze(0)
        if h is not None and h.dim() == 1:
            h = h.unsqueeze(0)
        if h is not None and x.size(0) != h.size(0):
            if x.size(0) == 1:
                x = x.expand(h.size(0), -1)
            elif h.size(0) == 1:
                h = h.expand(x.size(0), -1)
        return self.step(self.x_gates(x), h, time_diff)


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

    def forward_time_major(self, xt: torch.Tensor, time_stamps: Optional[torch.Tensor] = None) -> torch.Tensor:
        """xt [T, N, D_in] -> [T, N, H] (temporal_propagation.py:648-755)."""
        require_hip(xt)
        T = xt.shape[0]
        has_time = time_stamps is not None and self.time_aware
        gx = self.forward_cell.x_gates(xt)
        # time factors exp(-clamp(Δt, 0, 10)) per step (step 0 has no previous state: unused)
        tsf = tsb = None
        if has_time:
            dt = torch.diff(time_stamps.to(torch.float32), dim=1).t()                    # [T-1, N]: t - (t-1)
            fac = torch.exp(-torch.clamp(dt, min=0.0, max=10.0))
            one = torch.ones_like(fac[:1])
            tsf = torch.cat([one, fac], 0).contiguous()
            tsb = torch.cat([one, fac.flip(0)], 0).contiguous()   # reversed step t' = T-1-t: (t+1) - t
        states = gru_sequence(self.forward_cell, gx, tsf) if USE_GRU_KERNEL else None
        if states is None:
            fwd, h = [], None
            for t in range(T):
                td = time_stamps[:, t] - time_stamps[:, t - 1] if (has_time and t > 0) else None
                h = self.forward_cell.step(gx[t], h, td)
                fwd.append(h)
            states = torch.stack(fwd, 0)
        if self.bidirectional:
            gb = self.backward_cell.x_gates(xt)
            sb = gru_sequence(self.backward_cell, gb.flip(0), tsb) if USE_GRU_KERNEL else None
            if sb is not None:
                sb = sb.flip(0)
            else:
                bwd, hb = [None] * T, None
                for t in range(T - 1, -1, -1):
                    td = time_stamps[:, t + 1] - time_stamps[:, t] if (has_time and t < T - 1) else None
                    hb = self.backward_cell.step(gb[t], hb, td)
                    bwd[t] = hb
                sb = torch.stack(bwd, 0)
            states = torch.cat([states, sb], -1)
        y = linear(states, self.output_projection.weight, self.output_projection.bias)
        res = xt if (self.residual and self.input_dim == self.hidden_dim) else None
        if self.use_layer_norm and res is not None:
            return dropout_add_layer_norm(y, res, self.layer_norm, self.dropout if self.training else 0.0)
        y = self.dropout_layer(y)
        if res is not None:
            y = y + res
        return _ln(y, self.layer_norm if self.use_layer_norm else None)

    def forward(self, node_features_seq: List[torch.Tensor], time_stamps: Optional[torch.Tensor] = None):
        return list(self.forward_time_major(torch.stack(node_features_seq, 0), time_stamps).unbind(0))


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

    def forward_time_major(self, xt: torch.Tensor) -> torch.Tensor:
        """xt [T, N, D] -> [T, N, D] (temporal_propagation.py:846-946); windows of ±window_size over T."""
        require_hip(xt)
        T, N, _ = xt.shape
        p = linear(xt, self.input_proj.weight, self.input_proj.bias)
        if self.apply_activation:
            p = self.act_fn(p)
        p = self.dropout_layer(_ln(p, self.layer_norm1 if self.use_layer_norm else None))
        agg = window_aggregate(p, self.window_size, self.aggregation)
        out = linear(self.act_fn(agg), self.output_proj.weight, self.output_proj.bias)
        if self.residual and self.use_layer_norm:
            return dropout_add_layer_norm(out, xt, self.layer_norm2, self.dropout if self.training else 0.0)
        out = self.dropout_layer(out)
        if self.residual:
            out = out + xt
        return _ln(out, self.layer_norm2 if self.use_layer_norm else None)

    def forward(self, node_features_seq: List[torch.Tensor], time_weights=None):
        return list(self.forward_time_major(torch.stack(node_features_seq, 0)).unbind(0))


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
        """temporal_propagation.py:1022-1067."""
        require_hip(current_feat, previous_feat)
        if self.use_layer_norm:
            current_feat = layer_norm(current_feat, self.layer_norm_in1)
            previous_feat = layer_norm(previous_feat, self.layer_norm_in2)
        comb = torch.cat([current_feat, previous_feat], dim=1)
        ur = torch.sigmoid(linear(comb, torch.cat([self.update_gate.weight, self.reset_gate.weight], 0),
                                  torch.cat([self.update_gate.bias, self.reset_gate.bias], 0)))
        D = self.input_dim
        u, r = ur[:, :D], ur[:, D:]
        cand = torch.tanh(linear(torch.cat([current_feat, r * previous_feat], dim=1), self.output_gate.weight,
                                 self.output_gate.bias))
        out = (1 - u) * current_feat + u * cand
        if self.residual and self.use_layer_norm:
            return dropout_add_layer_norm(out, current_feat, self.layer_norm_out,
                                          self.dropout if self.training else 0.0)
        out = self.dropout_layer(out)
        if self.residual:
            out = out + current_feat
        return layer_norm(out, self.layer_norm_out) if self.use_layer_norm else out


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

    def forward_intended(self, xt: torch.Tensor, time_stamps: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Intended compute, tensor-mask form (temporal_propagation.py:1345-1500): xt [T, N, H] time-major,
        time_stamps [N, T] or None -> [T, N, H]."""
        require_hip(xt)
        x = self.evolution_layer.forward_time_major(xt, time_stamps)
        if self.use_skip_connection:
            x = self.skip_connection.forward_time_major(x)
        x = self.dropout_layer(linear(x, self.output_proj.weight, self.output_proj.bias))
        return layer_norm(x, self.layer_norm) if self.use_layer_norm else x

    def extra_repr(self) -> str:
        return (f"input_dim={self.input_dim}, hidden_dim={self.hidden_dim}, dropout={self.dropout}, "
                f"time_aware={self.time_aware}, bidirectional={self.bidirectional}, "
                f"use_layer_norm={self.use_layer_norm}, use_skip_connection={self.use_skip_connection}, "
                f"use_gating={self.use_gating}, window_size={self.window_size}, "
                f"aggregation={self.aggregation}, residual={self.residual}")
