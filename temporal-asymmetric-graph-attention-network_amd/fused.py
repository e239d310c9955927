"""One autograd node per attention layer: LN1 -> QKV GEMM -> attention core -> out-proj -> add+LN2.

Both attention layers of the hot path share this shape — GeometricAttention.forward
(geometric_attention.py:518-598) around the edge-softmax core and the temporal attention
(temporal_attention.py:1006-1205) around the per-row core.  Composed from per-op autograd
nodes the backward pays for: a separate gradient add where the layer input feeds both LN1 and
the residual, a separate reduction for the out-proj bias, weight concatenations, and ~15
autograd nodes of host overhead per layer.  Here the backward is written out once:

    LN2 bwd (HIP)   -> d(residual), d(out-proj output) and, fused, the out-proj bias gradient
    out-proj        -> dctx = do·W_o (GEMM), dW_o (split-K GEMM)
    core bwd (HIP)  -> dqkv (+ metric parameter / bias-table gradients)
    QKV             -> dh = dqkv·W_qkv (GEMM), dW_qkv (split-K GEMM), db_qkv
    LN1 bwd (HIP)   -> dx = LN1ᵀ(dh) + d(residual), the add fused into the kernel

Cores: ``GeoCore`` (tagan_geo_attn_*) and ``TemporalCore`` (tagan_temporal_attn_*).
"""
import ctypes
import os
from typing import Optional

import torch
import torch.nn.functional as F

from . import _lib
from ._lib import check, lib, ptr, require_hip, stream_of
from . import stream_gemm as sg
from .kernels import TemporalMask, _geo_fwd, _keep_cache, colsum, split_rows, weight_grad


# ----------------------------------------------------------------------------- raw LayerNorm calls
def ln_fwd(a2, b2, p_drop, seed, gamma, beta, eps, keep_s, y=None, y_dtype=torch.float32, a_bias=None):
    """LN(dropout(a2 + a_bias) + b2); ``y`` may be a wider row-strided buffer ([M, ld], first H columns written);
    y is stored in ``y_dtype`` (bf16 when it only feeds a bf16 GEMM)."""
    M, H = a2.shape
    s = torch.empty_like(a2) if keep_s else None
    if y is None:
        y = torch.empty(M, H, device=a2.device, dtype=y_dtype)
    mean = torch.empty(M, device=a2.device)
    rstd = torch.empty(M, device=a2.device)
    check(lib().tagan_add_layernorm_fwd(_lib.dtype_code(y), M, H, ptr(a2), ptr(a_bias), ptr(b2), float(p_drop), seed,
                                        ptr(gamma),
                                        ptr(beta), float(eps), ptr(s), ptr(y), y.stride(0), ptr(mean), ptr(rstd),
                                        stream_of(a2)), "tagan_add_layernorm_fwd")
    return y, s, mean, rstd


def ln_skip_fwd(a2, b2, p_drop, seed, gamma, beta, eps, gamma_s, beta_s, eps_s, a_bias=None):
    """LN(dropout(a2 + a_bias) + b2) + LN_s(b2) (fp32); returns y, s, mean, rstd, (mean_s, rstd_s)."""
    M, H = a2.shape
    dev = a2.device
    s = torch.empty_like(a2)
    y = torch.empty(M, H, device=dev)
    st = torch.empty(4, M, device=dev)
    check(lib().tagan_add_layernorm_skip_fwd(M, H, ptr(a2), ptr(a_bias), ptr(b2), float(p_drop), seed, ptr(gamma),
                                             ptr(beta),
                                             float(eps), ptr(gamma_s), ptr(beta_s), float(eps_s), ptr(s), ptr(y),
                                             ptr(st[0]), ptr(st[1]), ptr(st[2]), ptr(st[3]), stream_of(a2)),
          "tagan_add_layernorm_skip_fwd")
    return y, s, st[0], st[1], (st[2], st[3])


def ln_bwd(s, mean, rstd, gamma, dy2, dres, p_drop, seed, want_ds, want_da, want_sum_a, da_dtype=torch.float32):
    M, H = dy2.shape
    dev = dy2.device
    ds = torch.empty_like(dy2) if want_ds else None
    da = torch.empty(M, H, device=dev, dtype=da_dtype) if want_da else None
    dg = torch.empty(H, device=dev)
    dbt = torch.empty(H, device=dev)
    dsa = torch.empty(H, device=dev) if want_sum_a else None
    L = lib()
    wsb = L.tagan_layernorm_bwd_workspace(M, H)
    ws = torch.empty(int(wsb), dtype=torch.uint8, device=dev)
    check(L.tagan_layernorm_bwd(_lib.dtype_code(da), M, H, ptr(s), ptr(mean), ptr(rstd), ptr(gamma), ptr(dy2), ptr(dres),
                                float(p_drop), seed, ptr(ds), ptr(da), ptr(dg), ptr(dbt), ptr(dsa), ptr(ws), wsb,
                                stream_of(dy2)), "tagan_layernorm_bwd")
    return ds, da, dg, dbt, dsa


def ln_skip_bwd(s, mean, rstd, gamma, b, mean_s, rstd_s, gamma_s, dy2, p_drop, seed, da_dtype=torch.float32):
    """Backward of y = LN(dropout-sum s) + LN_s(b) in one pass: ds (incl. LN_s's input gradient), da, dgamma, dbeta,
    dsum_a, dgamma_s, dbeta_s (the two-call ln_bwd chain's values to fp32 rounding, the same dropout decisions)."""
    M, H = dy2.shape
    dev = dy2.device
    ds = torch.empty_like(dy2)
    da = torch.empty(M, H, device=dev, dtype=da_dtype)
    out = torch.empty(5, H, device=dev)
    L = lib()
    wsb = L.tagan_layernorm_skip_bwd_workspace(M, H)
    ws = torch.empty(int(wsb), dtype=torch.uint8, device=dev)
    check(L.tagan_layernorm_skip_bwd(_lib.dtype_code(da), M, H, ptr(s), ptr(mean), ptr(rstd), ptr(gamma), ptr(b),
                                     ptr(mean_s), ptr(rstd_s), ptr(gamma_s), ptr(dy2), float(p_drop), seed, ptr(ds),
                                     ptr(da), ptr(out[0]), ptr(out[1]), ptr(out[2]), ptr(out[3]), ptr(out[4]), ptr(ws),
                                     wsb, stream_of(dy2)), "tagan_layernorm_skip_bwd")
    return ds, da, out[0], out[1], out[2], out[3], out[4]


def _ln2_bwd(s2, mean2, rstd2, ln2_w, dy2, skip, x2, lns_w, p_out, seed_out, da_dtype):
    """LN2's backward of a block (and, for the skip block, LN_s's): dres, do, dg2, db2, dbo, dgs, dbs."""
    M, H = dy2.shape
    if skip is not None and H in (128, 256):   # one pass for both LayerNorms (150 vs 2 x 118 us at C2)
        return ln_skip_bwd(s2, mean2, rstd2, ln2_w, x2, skip[0], skip[1], lns_w, dy2, p_out, seed_out,
                           da_dtype=da_dtype)
    dres, do, dg2, db2, dbo = ln_bwd(s2, mean2, rstd2, ln2_w, dy2, None, p_out, seed_out, True, True, True,
                                     da_dtype=da_dtype)
    dgs = dbs = None
    if skip is not None:       # skip branch: LN_s backward with the residual gradient added in-kernel
        dres, _, dgs, dbs, _ = ln_bwd(x2, skip[0], skip[1], lns_w, dy2, dres, 0.0, 0, True, False, False)
    return dres, do, dg2, db2, dbo, dgs, dbs


# ----------------------------------------------------------------------------- attention cores
class GeoCore:
    """Edge-softmax attention over a SnapshotGraph (csrc/geo_attn.hip); qkv2 [N, 3H] -> ctx [N, H]."""

    def __init__(self, graph, metric: int, heads: int, p_drop: float, seed: int):
        self.graph, self.metric, self.heads, self.p_drop, self.seed = graph, metric, heads, p_drop, seed

    def fwd(self, qkv2, param, _unused):
        N, H3 = qkv2.shape
        out = torch.empty(N, H3 // 3, device=qkv2.device, dtype=qkv2.dtype)
        lse = torch.empty(N, self.heads, device=qkv2.device)
        prm = param.detach().contiguous() if param is not None else None
        _geo_fwd(qkv2, self.graph, self.metric, self.heads, prm, self.p_drop, self.seed, out, lse, None)
        return out, (lse, prm)

    def bwd(self, qkv2, out, saved, dctx, want_p1, want_p2, want_bias_sum=False):
        lse, prm = saved
        N, H3 = qkv2.shape
        H = H3 // 3
        d = H // self.heads
        dqkv = torch.empty_like(qkv2)
        L = lib()
        gs = self.graph.struct()
        wsb = L.tagan_geo_attn_bwd_workspace(gs, self.heads, d)
        ws = torch.empty(int(wsb), dtype=torch.uint8, device=qkv2.device)
        dprm = torch.empty(self.heads, device=qkv2.device) if (prm is not None and want_p1) else None
        b, db, es = qkv2.data_ptr(), dqkv.data_ptr(), qkv2.element_size()
        check(L.tagan_geo_attn_bwd(_lib.dtype_code(qkv2), self.metric, gs, self.heads, d, b, b + H * es, b + 2 * H * es, H3,
                                   ptr(prm), float(self.p_drop), self.seed, ptr(out), ptr(lse), ptr(dctx), db,
                                   db + H * es, db + 2 * H * es, H3, ptr(dprm), ptr(ws), wsb, stream_of(qkv2)),
              "tagan_geo_attn_bwd")
        return (dqkv, dprm, None, None) if want_bias_sum else (dqkv, dprm, None)


class TemporalCore:
    """Per-row attention over T steps (csrc/temporal_attn.hip) on a [T, R, 3H] (time_major) or [R, T, 3H]
    projection, flattened to rows."""

    def __init__(self, T: int, R: int, time_major: bool, heads: int, mask: TemporalMask, p_drop: float,
                 seed: int):
        self.T, self.R, self.time_major = T, R, time_major
        self.heads, self.mask, self.p_drop, self.seed = heads, mask, p_drop, seed

    def _strides(self, H):
        H3 = 3 * H
        if self.time_major:
            return (H3, self.R * H3), (H, self.R * H)
        return (self.T * H3, H3), (self.T * H, H)

    def fwd(self, qkv2, bias_table, bias_dense):
        T, R, heads = self.T, self.R, self.heads
        H = qkv2.shape[1] // 3
        d = H // heads
        (s_row, s_t), (o_row, o_t) = self._strides(H)
        out = torch.empty(T * R, H, device=qkv2.device, dtype=qkv2.dtype)
        lse = torch.empty(R, heads, T, device=qkv2.device)
        bt = bias_table.detach().contiguous() if bias_table is not None else None
        bd = bias_dense.detach().contiguous() if bias_dense is not None else None
        bd_stride = (0 if bd.shape[0] == 1 else heads * T * T) if bd is not None else 0
        m = self.mask
        b, es = qkv2.data_ptr(), qkv2.element_size()
        keep, kb, written = _keep_cache(R, T, heads, d, m, bd, self.p_drop, qkv2.device)
        check(lib().tagan_temporal_attn_fwd_keep(_lib.dtype_code(qkv2), R, T, heads, d, b, b + H * es,
                                                 b + 2 * H * es, s_row, s_t, ptr(bt), ptr(bd), bd_stride, ptr(m.keep),
                                                 m.bstride, m.hstride, int(m.causal), float(self.p_drop), self.seed,
                                                 ptr(out), o_row, o_t, ptr(lse), None, ptr(keep), kb,
                                                 ctypes.byref(written), stream_of(qkv2)), "tagan_temporal_attn_fwd_keep")
        return out, (lse, bt, bd, bd_stride, keep if written.value else None)

    def bwd(self, qkv2, out, saved, dctx, want_p1, want_p2, want_bias_sum=False):
        """``want_bias_sum``: also return the column sums of dq|dk|dv (the QKV bias gradient) when the
        matrix-core kernel can sum them in place (else None: the caller reduces dqkv itself)."""
        lse, bt, bd, bd_stride, keep = saved
        T, R, heads = self.T, self.R, self.heads
        H = qkv2.shape[1] // 3
        d = H // heads
        (s_row, s_t), (o_row, o_t) = self._strides(H)
        dqkv = torch.empty_like(qkv2)
        dev = qkv2.device
        dbt = torch.empty(heads, 2 * T - 1, device=dev) if (bt is not None and want_p1) else None
        dbd = torch.empty(R, heads, T, T, device=dev) if (bd is not None and want_p2) else None
        L = lib()
        wsb = L.tagan_temporal_attn_bwd_workspace(R, T, heads, d)
        ws = torch.empty(int(wsb), dtype=torch.uint8, device=dev)
        m = self.mask
        dsum = torch.empty(3 * H, device=dev) if want_bias_sum else None
        b, db, es = qkv2.data_ptr(), dqkv.data_ptr(), qkv2.element_size()
        def call(ds):
            return L.tagan_temporal_attn_bwd_keep(_lib.dtype_code(qkv2), R, T, heads, d, b, b + H * es,
                                                  b + 2 * H * es, s_row, s_t, ptr(bt), ptr(bd), bd_stride,
                                                  ptr(m.keep), m.bstride, m.hstride, int(m.causal),
                                                  float(self.p_drop), self.seed, ptr(out), o_row, o_t, ptr(lse),
                                                  ptr(dctx), o_row, o_t, db, db + H * es, db + 2 * H * es, s_row, s_t,
                                                  ptr(dbt), ptr(dbd), ptr(ds), ptr(keep),
                                                  keep.numel() * 4 if keep is not None else 0, ptr(ws), wsb,
                                                  stream_of(qkv2))
        rc = call(dsum)
        if rc == _lib.TAGAN_ERR_UNSUPPORTED and dsum is not None:   # rejected before any launch: not this path
            dsum = None
            rc = call(None)
        check(rc, "tagan_temporal_attn_bwd")
        if dbd is not None and bd.shape[0] == 1:
            dbd = dbd.sum(0, keepdim=True)
        return (dqkv, dbt, dbd, dsum) if want_bias_sum else (dqkv, dbt, dbd)


# ----------------------------------------------------------------------------- precision modes
# "fp32" (default): fp32 storage and math everywhere, the fp32 MFMA GEMMs.
# "bf16-gemm": the projection GEMMs take bf16 operands (fp32 accumulate, fp32 outputs); every
#     other tensor fp32.
# "bf16": activations between kernels in bf16 — h = LN1(x), Q|K|V, the attention output, the
#     projection-input gradients and dQ|dK|dV — with fp32 math inside every kernel, fp32 residual
#     stream, LayerNorm statistics, LSE, parameter gradients and optimizer (the BASELINE's C2 dtype).
# Neither bf16 mode is bit-compatible with the fp32 reference: tests/test_gpu_bf16.py states the
# tolerance they are held to.
_PREC = "fp32"
PRECISIONS = ("fp32", "bf16-gemm", "bf16")


class precision:
    def __init__(self, mode: str):
        if mode not in PRECISIONS:
            raise ValueError("precision must be one of %s" % (PRECISIONS,))
        self.mode = mode

    def __enter__(self):
        global _PREC
        self.prev, _PREC = _PREC, self.mode

    def __exit__(self, *exc):
        global _PREC
        _PREC = self.prev


def _b(t):
    return t if t.dtype == torch.bfloat16 else t.to(torch.bfloat16)


def _addmm(bias, a, w, bf, out_bf16=False):
    """bias + a·wᵀ -> fp32 (or bf16 with ``out_bf16``)."""
    if out_bf16:
        return torch.addmm(_b(bias), _b(a), _b(w).t())
    if bf:
        return torch.addmm(bias, _b(a), _b(w).t(), out_dtype=torch.float32)
    return F.linear(a, w, bias)   # hipBLASLt bias epilogue: 101 vs 88 TF/s for addmm at C2 (tools/gemm_layer.py)


def _mm(a, w, bf, out_bf16=False):
    """a·w -> fp32 (or bf16 with ``out_bf16``)."""
    if out_bf16:
        return _b(a) @ _b(w)
    if bf:
        return torch.mm(_b(a), _b(w), out_dtype=torch.float32)
    return a @ w


def _wgrad(dy, x, bf, rows: int = 2048):
    """dyᵀ·x (split-K) -> fp32."""
    if not bf:
        return weight_grad(dy, x, rows)
    dy, x = _b(dy), _b(x)
    K, M = dy.shape
    N = x.shape[1]
    if K < 4 * rows:
        return torch.mm(dy.t(), x, out_dtype=torch.float32)
    rows = split_rows(K, rows)
    c = K // rows
    main = c * rows
    xs = x.as_strided((c, rows, N), (rows * x.stride(0), x.stride(0), 1))   # x may be a column view
    dw = torch.bmm(dy[:main].view(c, rows, M).transpose(1, 2), xs,
                   out_dtype=torch.float32).sum(0)
    if main < K:
        dw = dw + torch.mm(dy[main:].t(), x[main:], out_dtype=torch.float32)
    return dw


# ----------------------------------------------------------------------------- the fused block
# TAGAN_SGEMM=0: the projection GEMMs through torch (hipBLASLt / rocBLAS) instead of the hand-written
# bf16-matrix-core kernels of csrc/stream_gemm.hip (fp32 mode: three-plane split operands; A/B knob).
SGEMM = os.environ.get("TAGAN_SGEMM", "1") != "0"
_SG_OK = {}


# bf16 operands at H = 256 (C5): since round 5 on the stream GEMMs too -- with LN1 in the QKV projection's prologue, the
# LN2 epilogue on a one-plane N = 256 row-owner kernel and the 768 x 256 weight gradients over three column groups, the
# C5 bf16 step measured 608-610 ms against 618 ms on hipBLASLt (profiles/r5k_c5_bf16_ab.txt; round 4's stream path
# without those lost, 678 vs 643 ms)
SG_BF16_MAX_H = int(os.environ.get("TAGAN_SG_BF16_MAX_H", "256"))   # A/B knob: 128 puts C5 bf16 on hipBLASLt


def _sg_use(H: int, bf: bool, act: bool) -> bool:
    """The block's six projection products all have a stream_gemm kernel at this H / precision, and it is the faster
    path there."""
    if not SGEMM or (bf and H > SG_BF16_MAX_H):
        return False
    key = (H, bf, act)
    ok = _SG_OK.get(key)
    if ok is None:
        P = 1 if bf else 3
        ad = torch.bfloat16 if act else torch.float32
        f32 = torch.float32
        ok = _SG_OK[key] = (sg.supported(3 * H, H, P, ad, ad) and sg.supported(H, H, P, ad, f32) and
                            sg.supported(H, H, P, ad, ad) and sg.supported(H, 3 * H, P, ad, f32) and
                            sg.tn_supported(3 * H, H, P, ad) and sg.tn_supported(H, H, P, ad))
    return ok


# LayerNorm-fused stream-GEMM ops per precision ("in": LN1 in the QKV projection's prologue, h = LN1(x) recomputed
# inside the QKV weight gradient; "out": dropout + residual + LN2 [+ skip LN] in the out-projection's epilogue; "bwd":
# LN1's backward in the QKV input gradient's epilogue).  Same-process interleaved graph-replay A/B on one MI355X
# (tools/ab_step.py, profiles/r3d_ab_step.txt), ms per C2 step:
#   fp32  none 6.99  in 6.82  in+out 6.75  all 6.99   (fp32 "bwd" runs on k_sgemm_nt: its K = 384 three-plane weight
#                                                      fragments do not fit a row-owner kernel's LDS, 288 KB)
#   bf16  none 5.62  in 5.50  in+out 5.41  all 5.26
# "ln2bwd" (round 5): LN2's backward and the out-projection's input / weight / bias gradients in one pass over the
# rows (tagan_ln2_bwd_out: do never reaches HBM).
SG_LN_OPS = {False: frozenset({"in", "out", "ln2bwd"}), True: frozenset({"in", "out", "bwd", "ln2bwd"})}
_SG_LN_OK = {}


def _sg_ln_use(H: int, bf: bool, act: bool, op: str) -> bool:
    if op not in SG_LN_OPS[bf]:
        return False
    key = (H, bf, act, op)
    ok = _SG_LN_OK.get(key)
    if ok is None:
        if op == "ln2bwd":
            ok = _SG_LN_OK[key] = sg.ln2_bwd_out_supported(H, 1 if bf else 3, act)
        else:
            ok = _SG_LN_OK[key] = sg.ln_supported(H, 1 if bf else 3, act, op)
    return ok


# Library-GEMM form of the block (widths without a stream_gemm kernel):
# * fp32: LN1 writes [h | 1 0 0 0] (row stride H + 4) and the QKV bias rides in the GEMM as a weight column -- one
#   GEMM over K = H + 4 without a bias epilogue (tools/runs/qkv_aug.sh: ~1 % of the C2 step on hipBLASLt); the weight
#   gradient over the same augmented operand gives the bias gradient as its column H (+66 us of GEMM against a 491-MB
#   column-sum pass, profiles/r1_wgrad_bias_aug_ab.txt);
# * the out-projection bias is added in the closing LayerNorm (no GEMM epilogue);
# * split-K slice height of the QKV weight gradient (3H outputs): taller than the out-projection's 2048 rows
#   (tools/wgrad_probe.py).
WGRAD_ROWS_QKV = 8192


def _aligned(*ts) -> bool:
    """Every tensor starts on a 16-byte boundary (the stream_gemm C-ABI's row-alignment contract; a parameter that
    is a view into a flat buffer at an odd offset takes the library GEMMs instead)."""
    return all(t is None or t.data_ptr() % 16 == 0 for t in ts)


class AttnBlockFn(torch.autograd.Function):
    """y = LN2(dropout(out_proj(core(QKV(LN1(x))))) + x) with LayerNorm on both sides (use_layer_norm=True)."""

    @staticmethod
    def forward(ctx, x, p1, p2, ln1_w, ln1_b, w_qkv, b_qkv, w_o, b_o, ln2_w, ln2_b, core, eps1: float,
                eps2: float, p_out: float, seed_out: int, lns_w=None, lns_b=None, eps_s: float = 1e-5,
                w_aug_packed=None):
        require_hip(x)
        H = x.shape[-1]
        x2 = x.reshape(-1, H).contiguous()
        bf = _PREC != "fp32"          # bf16 GEMM operands
        act = _PREC == "bf16"         # bf16 activations between kernels
        if _sg_use(H, bf, act) and _aligned(x2, b_qkv, b_o, ln1_w, ln1_b, ln2_w, ln2_b, lns_w, lns_b):
            return AttnBlockFn._fwd_sgemm(ctx, x, x2, H, bf, act, p1, p2, ln1_w, ln1_b, w_qkv, b_qkv, w_o, b_o,
                                          ln2_w, ln2_b, core, eps1, eps2, p_out, seed_out, lns_w, lns_b, eps_s)
        if not bf:
            # fp32: LN1 writes [h | 1 0 0 0] (row stride H + 4) and the QKV bias rides in the GEMM as a weight column
            h_aug = torch.empty(x2.shape[0], H + 4, device=x2.device)
            _, _, mean1, rstd1 = ln_fwd(x2, None, 0.0, 0, ln1_w, ln1_b, eps1, False, y=h_aug)
            w_aug = w_aug_packed   # [W | b | 0 0 0] from PackQKVFn, else concatenated here
            if w_aug is None:
                w_aug = torch.cat([w_qkv, b_qkv[:, None], w_qkv.new_zeros(w_qkv.shape[0], 3)], 1)
            qkv = h_aug @ w_aug.t()
            h = h_aug[:, :H]
        else:
            h_aug = None
            h, _, mean1, rstd1 = ln_fwd(x2, None, 0.0, 0, ln1_w, ln1_b, eps1, False,
                                        y_dtype=torch.bfloat16 if act else torch.float32)
            h = _b(h)
            qkv = _addmm(b_qkv, h, w_qkv, bf, out_bf16=act)
        c, saved = core.fwd(qkv, p1, p2)
        cg = _b(c) if bf else c
        o = _mm(cg, w_o.t(), bf)   # the out-projection bias is added in the closing LayerNorm
        skip = None
        if lns_w is not None:      # y = LN2(drop(o) + x) + LN_s(x) in one pass (model.py:258-262)
            y, s2, mean2, rstd2, skip = ln_skip_fwd(o, x2, p_out, seed_out, ln2_w, ln2_b, eps2, lns_w, lns_b, eps_s,
                                                    a_bias=b_o)
        else:
            y, s2, mean2, rstd2 = ln_fwd(o, x2, p_out, seed_out, ln2_w, ln2_b, eps2, True, a_bias=b_o)
        ctx.save_for_backward(x2, ln1_w, w_qkv, w_o, ln2_w, lns_w)
        ctx.inter = (h, h_aug, mean1, rstd1, qkv, c, cg, saved, s2, mean2, rstd2, skip)
        ctx.cfg = (core, p_out, seed_out, x.shape, bf, act, "library")
        ctx.packed_aug = h_aug is not None and w_aug_packed is not None
        return y.view(x.shape)

    @staticmethod
    def _fwd_sgemm(ctx, x, x2, H, bf, act, p1, p2, ln1_w, ln1_b, w_qkv, b_qkv, w_o, b_o, ln2_w, ln2_b, core, eps1,
                   eps2, p_out, seed_out, lns_w, lns_b, eps_s):
        """The block with its four forward / input-gradient products on k_sgemm_nt / k_rowgemm and its two
        weight-gradient products on k_sgemm_tn (csrc/stream_gemm.hip); LayerNorm fused where SG_LN_OPS says."""
        P = 1 if bf else 3
        adt = torch.bfloat16 if act else torch.float32
        lnf = _sg_ln_use(H, bf, act, "in")
        ln_out = _sg_ln_use(H, bf, act, "out")
        # the block's four weight operands in one launch; the transposed pair waits in ctx for the backward
        wq_nt, wo_nt, wo_km, wq_km = sg.wprep_block(w_qkv, w_o, P)
        if lnf:   # LN1 in the QKV projection's prologue: h is never stored
            h = None
            qkv, mean1, rstd1 = sg.nt_ln_in(x2, ln1_w, ln1_b, eps1, wq_nt, 3 * H, P,
                                            bias=b_qkv.contiguous(), out_dtype=adt)
        else:
            h, _, mean1, rstd1 = ln_fwd(x2, None, 0.0, 0, ln1_w, ln1_b, eps1, False, y_dtype=adt)
            qkv = sg.nt(h, wq_nt, 3 * H, P, bias=b_qkv.contiguous(), out_dtype=adt)
        c, saved = core.fwd(qkv, p1, p2)
        if ln_out:   # dropout + residual + LN2 (+ the skip LayerNorm) in the out-projection's epilogue
            y, s2, mean2, rstd2, skip = sg.nt_ln_out(c, wo_nt, P, b_o.contiguous(), x2, p_out,
                                                     seed_out, ln2_w, ln2_b, eps2, lns_w, lns_b, eps_s)
        else:
            o = sg.nt(c, wo_nt, H, P)          # the bias is added in the closing LayerNorm
            skip = None
            if lns_w is not None:
                y, s2, mean2, rstd2, skip = ln_skip_fwd(o, x2, p_out, seed_out, ln2_w, ln2_b, eps2, lns_w, lns_b,
                                                        eps_s, a_bias=b_o)
            else:
                y, s2, mean2, rstd2 = ln_fwd(o, x2, p_out, seed_out, ln2_w, ln2_b, eps2, True, a_bias=b_o)
        ctx.save_for_backward(x2, ln1_w, w_qkv, w_o, ln2_w, lns_w)
        ctx.inter = (h, ln1_b if lnf else None, mean1, rstd1, qkv, c, c, saved, s2, mean2, rstd2, skip)
        ctx.cfg = (core, p_out, seed_out, x.shape, bf, act, "sgemm")
        ctx.wkm = (wo_km, wq_km)
        ctx.packed_aug = False
        return y.view(x.shape)

    @staticmethod
    def _bwd_sgemm(ctx, dy):
        x2, ln1_w, w_qkv, w_o, ln2_w, lns_w = ctx.saved_tensors
        h, ln1_b, mean1, rstd1, qkv, c, _, saved, s2, mean2, rstd2, skip = ctx.inter
        core, p_out, seed_out, shape, bf, act, _ = ctx.cfg
        lnf = h is None   # the LayerNorm-fused form (h = LN1(x) recomputed where it is needed)
        wo_km, wq_km = ctx.wkm
        ng = ctx.needs_input_grad
        H = shape[-1]
        P = 1 if bf else 3
        adt = torch.bfloat16 if act else torch.float32
        dy2 = dy.reshape(-1, H).contiguous()
        if _sg_ln_use(H, bf, act, "ln2bwd") and dy2.shape[0] > 0 and c.is_contiguous():
            # LN2 backward + dC + dW_o + db_o in one pass (do stays on chip)
            skip_args = (x2, skip[0], skip[1], lns_w) if skip is not None else None
            dres, dc, dw_o, dbo, dg2, db2, dgs, dbs = sg.ln2_bwd_out(dy2, s2, mean2, rstd2, ln2_w, p_out, seed_out, c,
                                                                     wo_km, P, skip=skip_args, want_dw=bool(ng[7]))
        else:
            dres, do, dg2, db2, dbo, dgs, dbs = _ln2_bwd(s2, mean2, rstd2, ln2_w, dy2, skip, x2, lns_w, p_out,
                                                         seed_out, adt)
            dc = sg.nt(do, wo_km, H, P, out_dtype=adt)
            dw_o = sg.tn(do, c, P, want_db=False)[0] if ng[7] else None
            del do
        dqkv, dp1, dp2, db_core = core.bwd(qkv, c, saved, dc, ng[1], ng[2], want_bias_sum=bool(ng[6]))
        del dc
        dw_qkv = db_qkv = None
        if ng[5] or (ng[6] and db_core is None):
            if lnf:
                dw_qkv, db_qkv = sg.tn_ln(dqkv, x2, ln1_w, ln1_b, mean1, rstd1, P, want_dw=bool(ng[5]),
                                          want_db=bool(ng[6]) and db_core is None)
            else:
                dw_qkv, db_qkv = sg.tn(dqkv, h, P, want_dw=bool(ng[5]), want_db=bool(ng[6]) and db_core is None)
        if db_core is not None:
            db_qkv = db_core
        if _sg_ln_use(H, bf, act, "bwd"):   # dh = dqkv·W_qkv and LN1's backward in one kernel
            dx, dg1, db1 = sg.nt_ln_bwd(dqkv, wq_km, P, x2, mean1, rstd1, ln1_w, dres)
            del dqkv
        else:
            dh = sg.nt(dqkv, wq_km, H, P)
            del dqkv
            dx, _, dg1, db1, _ = ln_bwd(x2, mean1, rstd1, ln1_w, dh, dres, 0.0, 0, True, False, False)
        ctx.inter = None
        ctx.wkm = None
        return (dx.view(shape), dp1, dp2, dg1, db1, dw_qkv, db_qkv, dw_o, dbo, dg2, db2,
                None, None, None, None, None, dgs, dbs, None, None)

    @staticmethod
    def backward(ctx, dy):
        if ctx.cfg[-1] == "sgemm":
            return AttnBlockFn._bwd_sgemm(ctx, dy)
        x2, ln1_w, w_qkv, w_o, ln2_w, lns_w = ctx.saved_tensors
        h, h_aug, mean1, rstd1, qkv, c, cg, saved, s2, mean2, rstd2, skip = ctx.inter
        core, p_out, seed_out, shape, bf, act, _ = ctx.cfg
        ng = ctx.needs_input_grad
        dy2 = dy.reshape(-1, shape[-1]).contiguous()
        dres, do, dg2, db2, dbo, dgs, dbs = _ln2_bwd(s2, mean2, rstd2, ln2_w, dy2, skip, x2, lns_w, p_out, seed_out,
                                                     torch.bfloat16 if bf else torch.float32)
        dc = _mm(do, w_o, bf, out_bf16=act)
        dw_o = _wgrad(do, cg, bf) if ng[7] else None
        dqkv, dp1, dp2, db_core = core.bwd(qkv, c, saved, dc, ng[1], ng[2], want_bias_sum=bool(ng[6]))
        del dc, do
        H = shape[-1]
        if db_core is None and ng[5] and ng[6] and h_aug is not None:
            # dqkvᵀ·[h | 1 0 0 0]: column H of the product is the column sum of dqkv (the bias gradient)
            # -- 4 more GEMM columns instead of a 491 MB column-sum pass at C2
            dw_aug = _wgrad(dqkv, h_aug, bf, WGRAD_ROWS_QKV)
            dw_qkv, db_qkv = dw_aug[:, :H], dw_aug[:, H]          # views: PackQKVFn unpacks them in one launch
            if not ctx.packed_aug:
                dw_qkv, db_qkv = dw_qkv.contiguous(), db_qkv.contiguous()
        else:
            db_qkv = (db_core if db_core is not None else colsum(dqkv)) if ng[6] else None
            dw_qkv = None
        if bf:
            dqkv = _b(dqkv)
        dh = _mm(dqkv, w_qkv, bf)
        if dw_qkv is None and ng[5]:
            dw_qkv = _wgrad(dqkv, h, bf, WGRAD_ROWS_QKV)
        del dqkv
        dx, _, dg1, db1, _ = ln_bwd(x2, mean1, rstd1, ln1_w, dh, dres, 0.0, 0, True, False, False)
        ctx.inter = None
        return (dx.view(shape), dp1, dp2, dg1, db1, dw_qkv, db_qkv, dw_o, dbo, dg2, db2,
                None, None, None, None, None, dgs, dbs, None, None)


class PackQKVFn(torch.autograd.Function):
    """[W_q; W_k; W_v] and [b_q; b_k; b_v] in one launch (csrc/params.hip), the parameter gradients unpacked in one
    launch (they arrive as views of the block's augmented weight gradient).  ``aug``: the same launch also writes
    [W | b | 0 0 0] ([3H, H + 4], the fp32 augmented QKV GEMM operand), returned as a third, non-differentiable
    output; W and b stay contiguous so every GEMM keeps the shapes (and leading dimensions) of the tuned table."""

    @staticmethod
    def forward(ctx, wq, wk, wv, bq, bk, bv, aug: bool):
        H = wq.shape[1]
        dev = wq.device
        src = [t.contiguous() for t in (wq, wk, wv, bq, bk, bv)]   # alive until the launches below are issued
        args = [ptr(t) for t in src]
        w = torch.empty(3 * H, H, device=dev)
        b = torch.empty(3 * H, device=dev)
        st = stream_of(wq)
        check(lib().tagan_qkv_pack(H, *args, ptr(w), H, 0, ptr(b), st), "tagan_qkv_pack")
        w_aug = None
        if aug:
            w_aug = torch.empty(3 * H, H + 4, device=dev)
            check(lib().tagan_qkv_pack(H, *args, ptr(w_aug), H + 4, 1, None, st), "tagan_qkv_pack")
            ctx.mark_non_differentiable(w_aug)
        ctx.H = H
        return w, b, w_aug

    @staticmethod
    def backward(ctx, dw, db, _unused):
        H = ctx.H
        ng = ctx.needs_input_grad
        ref = dw if dw is not None else db
        outs = [torch.empty(H, H, device=ref.device) if (ng[i] and dw is not None) else None for i in range(3)] + \
               [torch.empty(H, device=ref.device) if (ng[3 + i] and db is not None) else None for i in range(3)]
        if dw is not None and dw.stride(1) != 1:
            dw = dw.contiguous()
        check(lib().tagan_qkv_unpack(H, ptr(dw), dw.stride(0) if dw is not None else H, ptr(db),
                                     db.stride(0) if db is not None else 1, *[ptr(t) for t in outs],
                                     stream_of(ref)), "tagan_qkv_unpack")
        return (*outs, None)


def attention_block(x, core, p1: Optional[torch.Tensor], p2: Optional[torch.Tensor], ln1, q_lin, k_lin, v_lin,
                    out_lin, ln2, p_out: float, seed_out: int, skip_ln=None):
    """``skip_ln``: a LayerNorm whose output of the block input is added to the block output
    (TAGAN's first geometric layer, model.py:258-262), fused into the closing LayerNorm."""
    H = q_lin.weight.shape[1]
    w_aug = None
    if x.is_cuda and q_lin.weight.dtype == torch.float32:
        # [W_q; W_k; W_v] in one launch; the fp32 library form also takes [W | b | 0 0 0] from the same launch
        aug = _PREC == "fp32" and not (x.shape[-1] == H and _sg_use(H, False, False))
        w_qkv, b_qkv, w_aug = PackQKVFn.apply(q_lin.weight, k_lin.weight, v_lin.weight, q_lin.bias, k_lin.bias,
                                              v_lin.bias, aug)
    else:
        w_qkv = torch.cat([q_lin.weight, k_lin.weight, v_lin.weight], 0)
        b_qkv = torch.cat([q_lin.bias, k_lin.bias, v_lin.bias], 0)
    if skip_ln is not None:
        return AttnBlockFn.apply(x, p1, p2, ln1.weight, ln1.bias, w_qkv, b_qkv, out_lin.weight, out_lin.bias,
                                 ln2.weight, ln2.bias, core, ln1.eps, ln2.eps, float(p_out), seed_out,
                                 skip_ln.weight, skip_ln.bias, skip_ln.eps, w_aug)
    return AttnBlockFn.apply(x, p1, p2, ln1.weight, ln1.bias, w_qkv, b_qkv, out_lin.weight, out_lin.bias,
                             ln2.weight, ln2.bias, core, ln1.eps, ln2.eps, float(p_out), seed_out,
                             None, None, 1e-5, w_aug)


def fusable(x: torch.Tensor, use_layer_norm: bool) -> bool:
    return use_layer_norm and x.is_cuda and bool(lib().tagan_layernorm_supported(x.shape[-1]))
