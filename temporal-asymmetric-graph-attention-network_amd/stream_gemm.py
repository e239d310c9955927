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
