"""Projection GEMMs on the bf16 matrix cores (csrc/stream_gemm.hip) — thin wrappers of the C-ABI.

The attention blocks' q/k/v and out Linears (geometric_attention.py:541-596, temporal_attention.py:985-1200) and
their backward.  ``planes`` = 3 is the fp32 path (each fp32 operand split into three bf16 planes, six plane
products: fp32-GEMM accuracy), ``planes`` = 1 the bf16 activation mode.  No fallback: a shape the kernels do not
cover is reported by ``supported`` / ``tn_supported`` and the caller picks another GEMM; a failing call raises.
"""
import torch

from ._lib import TAGAN_BF16, check, dtype_code, lib, ptr, stream_of


def supported(N: int, K: int, planes: int, a_dtype=torch.float32, c_dtype=torch.float32) -> bool:
    code = (lambda d: TAGAN_BF16 if d == torch.bfloat16 else 0)
    return bool(lib().tagan_sgemm_supported(N, K, planes, code(a_dtype), code(c_dtype)))


def tn_supported(N: int, K: int, planes: int, dtype=torch.float32) -> bool:
    return bool(lib().tagan_sgemm_tn_supported(N, K, planes, TAGAN_BF16 if dtype == torch.bfloat16 else 0))


def wprep(w: torch.Tensor, kmajor: bool, planes: int) -> torch.Tensor:
    """bf16 fragment planes of B (B = wᵀ if kmajor else w; w fp32 2-D, unit column stride)."""
    assert w.dtype == torch.float32 and w.dim() == 2
    if w.stride(1) != 1:
        w = w.contiguous()
    N, K = (w.shape[1], w.shape[0]) if kmajor else (w.shape[0], w.shape[1])
    wp = torch.empty(N * K * planes, dtype=torch.bfloat16, device=w.device)
    check(lib().tagan_sgemm_wprep(N, K, ptr(w), w.stride(0), int(kmajor), planes, ptr(wp), stream_of(w)),
          "tagan_sgemm_wprep")
    return wp


def wprep_block(w_qkv: torch.Tensor, w_o: torch.Tensor, planes: int):
    """The four operands of an attention block in one launch: (W_qkv, W_o) for the forward products and (W_oᵀ,
    W_qkvᵀ) for the input gradients (= wprep(w_qkv, False), wprep(w_o, False), wprep(w_o, True), wprep(w_qkv, True))."""
    assert w_qkv.dtype == torch.float32 and w_o.dtype == torch.float32
    if w_qkv.stride(1) != 1:
        w_qkv = w_qkv.contiguous()
    if w_o.stride(1) != 1:
        w_o = w_o.contiguous()
    H = w_o.shape[0]
    assert w_qkv.shape == (3 * H, H) and w_o.shape == (H, H)
    buf = torch.empty(8 * H * H * planes, dtype=torch.bfloat16, device=w_o.device)
    wq_nt, wo_nt, wo_km, wq_km = torch.split(buf, [3 * H * H * planes, H * H * planes, H * H * planes,
                                                   3 * H * H * planes])
    check(lib().tagan_sgemm_wprep_block(H, ptr(w_qkv), w_qkv.stride(0), ptr(w_o), w_o.stride(0), planes, ptr(wq_nt),
                                        ptr(wo_nt), ptr(wo_km), ptr(wq_km), stream_of(w_o)), "tagan_sgemm_wprep_block")
    return wq_nt, wo_nt, wo_km, wq_km


def nt(a: torch.Tensor, wp: torch.Tensor, N: int, planes: int, bias=None, out_dtype=torch.float32, out=None):
    """out[M, N] = a[M, K] · Bᵀ (+ bias) with B prepared by ``wprep``."""
    M, K = a.shape
    if a.stride(1) != 1:
        a = a.contiguous()
    if out is None:
        out = torch.empty(M, N, dtype=out_dtype, device=a.device)
    check(lib().tagan_sgemm_nt(dtype_code(a), dtype_code(out), M, N, K, ptr(a), a.stride(0), ptr(wp), planes,
                               ptr(bias), ptr(out), out.stride(0), stream_of(a)), "tagan_sgemm_nt")
    return out


def tn(dy: torch.Tensor, x: torch.Tensor, planes: int, want_dw=True, want_db=True, dw=None, db=None):
    """dw = dyᵀ·x [N, K] and db = Σ_rows dy [N] (fp32; either may be skipped)."""
    M, N = dy.shape
    K = x.shape[1]
    assert x.shape[0] == M and x.dtype == dy.dtype
    if dy.stride(1) != 1:
        dy = dy.contiguous()
    if x.stride(1) != 1:
        x = x.contiguous()
    L = lib()
    if want_dw and dw is None:
        dw = torch.empty(N, K, device=dy.device)
    if want_db and db is None:
        db = torch.empty(N, device=dy.device)
    wsb = int(L.tagan_sgemm_tn_workspace(M, N, K))
    ws = torch.empty(wsb, dtype=torch.uint8, device=dy.device)
    check(L.tagan_sgemm_tn(dtype_code(dy), M, N, K, ptr(dy), dy.stride(0), ptr(x), x.stride(0), planes,
                           ptr(dw) if want_dw else None, dw.stride(0) if want_dw else K,
                           ptr(db) if want_db else None, ptr(ws), wsb, stream_of(dy)), "tagan_sgemm_tn")
    return (dw if want_dw else None), (db if want_db else None)


# ----------------------------------------------------------------------------- LayerNorm-fused forms (H = 128)
LN_OPS = {"in": 1, "out": 2, "bwd": 3}


def ln_supported(H: int, planes: int, act_bf16: bool, op: str = "in") -> bool:
    """The LN-fused kernel(s) of one op exist at this H / precision (tagan_sgemm_ln_supported): "in" = LN1 prologue
    of the QKV projection + its LN-recomputing weight gradient, "out" = out-projection + LN2 epilogue, "bwd" = QKV
    input gradient + LN1-backward epilogue."""
    return bool(lib().tagan_sgemm_ln_supported(H, planes, TAGAN_BF16 if act_bf16 else 0, LN_OPS[op]))


def nt_ln_in(x, ln_w, ln_b, eps, wp, N: int, planes: int, bias=None, out_dtype=torch.float32):
    """out = LN(x)·Bᵀ + bias with LN in the GEMM prologue; returns out [M, N], mean [M], rstd [M]."""
    M, K = x.shape
    assert x.dtype == torch.float32 and x.stride(1) == 1
    out = torch.empty(M, N, dtype=out_dtype, device=x.device)
    st = torch.empty(2, M, device=x.device)
    check(lib().tagan_sgemm_nt_ln_in(dtype_code(out), M, N, K, ptr(x), x.stride(0), ptr(ln_w), ptr(ln_b), float(eps),
                                     ptr(wp), planes, ptr(bias), ptr(out), out.stride(0), ptr(st[0]), ptr(st[1]),
                                     stream_of(x)), "tagan_sgemm_nt_ln_in")
    return out, st[0], st[1]


def tn_ln(dy, x, ln_w, ln_b, mean, rstd, planes: int, want_dw=True, want_db=True):
    """dw = dyᵀ·LN(x), db = Σ_rows dy with LN(x) recomputed from x and the forward's statistics."""
    M, N = dy.shape
    K = x.shape[1]
    assert x.shape[0] == M and x.dtype == torch.float32 and x.stride(1) == 1
    if dy.stride(1) != 1:
        dy = dy.contiguous()
    L = lib()
    dw = torch.empty(N, K, device=dy.device) if want_dw else None
    db = torch.empty(N, device=dy.device) if want_db else None
    wsb = int(L.tagan_sgemm_tn_workspace(M, N, K))
    ws = torch.empty(wsb, dtype=torch.uint8, device=dy.device)
    check(L.tagan_sgemm_tn_ln(dtype_code(dy), M, N, K, ptr(dy), dy.stride(0), ptr(x), x.stride(0), ptr(ln_w),
                              ptr(ln_b), ptr(mean), ptr(rstd), planes, ptr(dw), K, ptr(db), ptr(ws), wsb,
                              stream_of(dy)), "tagan_sgemm_tn_ln")
    return dw, db


def nt_ln_out(a, wp, planes: int, bias, res, p_drop: float, seed: int, ln_w, ln_b, eps, gs=None, bs=None,
              eps_s: float = 1e-5):
    """y = LN(dropout(a·Bᵀ + bias) + res) [+ LN_s(res)]; returns y, s (the LN input), mean, rstd, skip stats."""
    M, H = res.shape
    if a.stride(1) != 1:
        a = a.contiguous()
    dev = res.device
    y = torch.empty(M, H, device=dev)
    s = torch.empty(M, H, device=dev)
    st = torch.empty(4 if gs is not None else 2, M, device=dev)
    skip = (st[2], st[3]) if gs is not None else None
    check(lib().tagan_sgemm_nt_ln_out(dtype_code(a), M, H, ptr(a), a.stride(0), ptr(wp), planes, ptr(bias), ptr(res),
                                      float(p_drop), seed, ptr(ln_w), ptr(ln_b), float(eps), ptr(gs), ptr(bs),
                                      float(eps_s), ptr(s), ptr(y), ptr(st[0]), ptr(st[1]),
                                      ptr(skip[0]) if skip else None, ptr(skip[1]) if skip else None, stream_of(res)),
          "tagan_sgemm_nt_ln_out")
    return y, s, st[0], st[1], skip


def nt_ln_bwd(a, wp, planes: int, x, mean, rstd, gamma, dres=None):
    """dh = a·Bᵀ and the LayerNorm backward of h = LN(x) in the epilogue; returns dx, dgamma, dbeta."""
    M, K = a.shape
    H = x.shape[1]
    dev = x.device
    if M == 0:
        return torch.empty(0, H, device=dev), torch.zeros(H, device=dev), torch.zeros(H, device=dev)
    if a.stride(1) != 1:
        a = a.contiguous()
    dx = torch.empty(M, H, device=dev)
    dgb = torch.empty(2, H, device=dev)
    L = lib()
    wsb = int(L.tagan_sgemm_nt_ln_bwd_workspace(M, H, K))
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    check(L.tagan_sgemm_nt_ln_bwd(dtype_code(a), M, H, K, ptr(a), a.stride(0), ptr(wp), planes, ptr(x), ptr(mean),
                                  ptr(rstd), ptr(gamma), ptr(dres), ptr(dx), ptr(dgb[0]), ptr(dgb[1]), ptr(ws), wsb,
                                  stream_of(a)), "tagan_sgemm_nt_ln_bwd")
    return dx, dgb[0], dgb[1]


def ln2_bwd_out_supported(H: int, planes: int, act_bf16: bool) -> bool:
    """tagan_ln2_bwd_out exists for (H, planes, activation storage)."""
    return bool(lib().tagan_ln2_bwd_out_supported(H, planes, TAGAN_BF16 if act_bf16 else 0))


def ln2_bwd_out(dy, s, mean, rstd, gamma, p_drop: float, seed: int, c, wp_km, planes: int, skip=None,
                want_dw: bool = True):
    """The LN2 backward + out-projection gradients of an attention block in one pass (tagan_ln2_bwd_out):
    returns dres [M, H] fp32, dc [M, H] (c's dtype), dw_o [H, H] (None unless ``want_dw``), db_o, dgamma, dbeta,
    dgamma_s, dbeta_s (the last two None without ``skip`` = (xs, mean_s, rstd_s, gamma_s))."""
    M, H = dy.shape
    dev = dy.device
    for t in (dy, s, c):
        assert t.is_contiguous() and t.shape == (M, H)
    dres = torch.empty(M, H, device=dev)
    dc = torch.empty(M, H, device=dev, dtype=c.dtype)
    out = torch.empty(5 if skip is not None else 3, H, device=dev)   # db_o, dgamma, dbeta [, dgamma_s, dbeta_s]
    dw = torch.empty(H, H, device=dev) if want_dw else None
    xs, ms, rs, gs = skip if skip is not None else (None, None, None, None)
    if xs is not None:
        assert xs.is_contiguous() and xs.shape == (M, H)
    L = lib()
    wsb = int(L.tagan_ln2_bwd_out_workspace(M, H, int(skip is not None)))
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    check(L.tagan_ln2_bwd_out(dtype_code(c), planes, M, H, ptr(dy), ptr(s), ptr(mean), ptr(rstd), ptr(gamma),
                              float(p_drop), seed, ptr(xs), ptr(ms), ptr(rs), ptr(gs), ptr(c), ptr(wp_km), ptr(dres),
                              ptr(dc), ptr(dw), ptr(out[0]), ptr(out[1]), ptr(out[2]),
                              ptr(out[3]) if skip is not None else None, ptr(out[4]) if skip is not None else None,
                              ptr(ws), wsb, stream_of(dy)), "tagan_ln2_bwd_out")
    dgs = out[3] if skip is not None else None
    dbs = out[4] if skip is not None else None
    return dres, dc, dw, out[0], out[1], out[2], dgs, dbs
