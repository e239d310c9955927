"""ctypes binding of libtagan_hip.so (C-ABI declared in include/tagan_hip.h).

There is no fallback: if the shared object is missing or a call fails, a
RuntimeError is raised.  The .so is built in-tree by ``__graft_entry__.build()``
(``make -C temporal-asymmetric-graph-attention-network_amd/csrc``).
"""
import ctypes
import os
import re

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TAGAN_LIB") or os.path.join(_HERE, "libtagan_hip.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "tagan_hip.h")

TAGAN_F32 = 0
TAGAN_BF16 = 1
TAGAN_ERR_UNSUPPORTED = -2   # tagan_status (include/tagan_hip.h)


def dtype_code(t) -> int:
    """C-ABI storage code of a tensor: TAGAN_BF16 for bfloat16, else TAGAN_F32."""
    return TAGAN_BF16 if t is not None and t.dtype == torch.bfloat16 else TAGAN_F32
METRIC_IDS = {
    "euclidean": 0, "squared_euclidean": 1, "manhattan": 2, "cosine_similarity": 3,
    "cosine_distance": 4, "dot_product": 5, "scaled_dot_product": 6, "gaussian_kernel": 7,
    "rbf_kernel": 8,
}

_c = ctypes
_p = _c.c_void_p
_i32, _i64, _u64, _f32, _sz = _c.c_int32, _c.c_int64, _c.c_uint64, _c.c_float, _c.c_size_t

_SIGNATURES = {
    "tagan_last_error": (_c.c_char_p, []),
    "tagan_version": (_c.c_int, []),
    "tagan_debug_build": (_c.c_int, []),
    "tagan_device_arch": (_c.c_int, [_c.c_char_p, _c.c_int]),
    "tagan_uniform": (_f32, [_u64, _u64, _c.c_uint32]),
    "tagan_set_seed_counter": (None, [_p]),
    "tagan_seed_counter_step": (_c.c_int, [_p, _p]),
    "tagan_csr_build_workspace": (_sz, [_i64, _i64]),
    "tagan_pool_workspace": (_sz, [_i32, _i32]),
    "tagan_colsum_workspace": (_sz, [_i64, _i32]),
    "tagan_colsum": (_c.c_int, [_c.c_int, _i64, _i32, _p, _i64, _p, _p, _sz, _p]),
    "tagan_temporal_bias_table": (_c.c_int, [_i32, _i32, _p, _i32, _p, _i32, _p, _p]),
    "tagan_temporal_bias_table_bwd": (_c.c_int, [_i32, _i32, _p, _i32, _i32, _p, _p, _p]),
    "tagan_narrow_linear_supported": (_c.c_int, [_i32, _i32]),
    "tagan_narrow_linear_fwd": (_c.c_int, [_i64, _i32, _i32, _p, _i64, _p, _p, _p, _i64, _p]),
    "tagan_narrow_linear_bwd_workspace": (_sz, [_i64, _i32, _i32]),
    "tagan_narrow_linear_bwd": (_c.c_int, [_i64, _i32, _i32, _p, _i64, _p, _i64, _p, _p, _p, _sz, _p]),
    "tagan_pool_fwd": (_c.c_int, [_c.c_int, _i32, _i64, _i32, _p, _i64, _i64, _p, _p, _sz, _p]),
    "tagan_pool_bwd": (_c.c_int, [_c.c_int, _i32, _i64, _i32, _p, _p, _i64, _i64, _p]),
    "tagan_csr_build": (_c.c_int, [_p, _i64, _i64, _p, _p, _i32, _i64, _i64, _p, _p, _p, _p, _p, _p, _p, _p, _p, _sz,
                                   _p]),
    "tagan_chunk_capacity": (_i64, [_i64, _i64, _i32]),
    "tagan_part_capacity": (_i64, [_i64, _i32]),
    "tagan_graph_chunks_workspace": (_sz, [_i64]),
    "tagan_graph_chunks": (_c.c_int, [_p, _i64, _i32, _p, _p, _p, _p, _p, _p, _p, _sz, _p]),
    "tagan_geo_set_bwd_order": (_c.c_int, [_i32]),
    "tagan_qkv_pack": (_c.c_int, [_i64, _p, _p, _p, _p, _p, _p, _p, _i64, _i32, _p, _p]),
    "tagan_qkv_unpack": (_c.c_int, [_i64, _p, _i64, _p, _i64, _p, _p, _p, _p, _p, _p, _p]),
    "tagan_csr_csc_pos": (_c.c_int, [_p, _p, _i64, _p, _p]),
    "tagan_chunk_order": (_c.c_int, [_p, _i64, _p, _p, _p, _i32, _i32, _p, _p]),
    "tagan_geo_attn_fwd_workspace": (_sz, [_p, _i32, _i32]),
    "tagan_geo_attn_fwd": (_c.c_int, [_c.c_int, _c.c_int, _p, _i32, _i32, _p, _p, _p, _i64, _p, _f32,
                                      _u64, _p, _p, _p, _p, _sz, _p]),
    "tagan_geo_attn_bwd_workspace": (_sz, [_p, _i32, _i32]),
    "tagan_geo_attn_bwd": (_c.c_int, [_c.c_int, _c.c_int, _p, _i32, _i32, _p, _p, _p, _i64, _p, _f32, _u64,
                                      _p, _p, _p, _p, _p, _p, _i64, _p, _p, _sz, _p]),
    "tagan_temporal_attn_fwd": (_c.c_int, [_c.c_int, _i64, _i32, _i32, _i32, _p, _p, _p, _i64, _i64, _p, _p,
                                           _i64, _p, _i64, _i64, _c.c_int, _f32, _u64, _p, _i64, _i64, _p, _p,
                                           _p]),
    "tagan_temporal_attn_keep_bytes": (_sz, [_i64, _i32, _i32, _i32, _c.c_int, _c.c_int, _c.c_int, _f32]),
    "tagan_temporal_attn_fwd_keep": (_c.c_int, [_c.c_int, _i64, _i32, _i32, _i32, _p, _p, _p, _i64, _i64, _p, _p,
                                                _i64, _p, _i64, _i64, _c.c_int, _f32, _u64, _p, _i64, _i64, _p, _p,
                                                _p, _sz, _p, _p]),
    "tagan_temporal_attn_bwd_keep": (_c.c_int, [_c.c_int, _i64, _i32, _i32, _i32, _p, _p, _p, _i64, _i64, _p, _p,
                                                _i64, _p, _i64, _i64, _c.c_int, _f32, _u64, _p, _i64, _i64, _p, _p,
                                                _i64, _i64, _p, _p, _p, _i64, _i64, _p, _p, _p, _p, _sz, _p, _sz,
                                                _p]),
    "tagan_temporal_attn_bwd_workspace": (_sz, [_i64, _i32, _i32, _i32]),
    "tagan_temporal_attn_bwd": (_c.c_int, [_c.c_int, _i64, _i32, _i32, _i32, _p, _p, _p, _i64, _i64, _p, _p,
                                           _i64, _p, _i64, _i64, _c.c_int, _f32, _u64, _p, _i64, _i64, _p, _p,
                                           _i64, _i64, _p, _p, _p, _i64, _i64, _p, _p, _p, _p, _sz, _p]),
    "tagan_layernorm_supported": (_c.c_int, [_i32]),
    "tagan_add_layernorm_fwd": (_c.c_int, [_c.c_int, _i64, _i32, _p, _p, _p, _f32, _u64, _p, _p, _f32, _p, _p, _i64,
                                           _p, _p, _p]),
    "tagan_add_layernorm_skip_fwd": (_c.c_int, [_i64, _i32, _p, _p, _p, _f32, _u64, _p, _p, _f32, _p, _p, _f32, _p, _p,
                                                _p, _p, _p, _p, _p]),
    "tagan_layernorm_bwd_workspace": (_sz, [_i64, _i32]),
    "tagan_layernorm_bwd": (_c.c_int, [_c.c_int, _i64, _i32, _p, _p, _p, _p, _p, _p, _f32, _u64, _p, _p, _p, _p,
                                       _p, _p, _sz, _p]),
    "tagan_layernorm_skip_bwd_workspace": (_sz, [_i64, _i32]),
    "tagan_layernorm_skip_bwd": (_c.c_int, [_c.c_int, _i64, _i32] + [_p] * 8 + [_p, _f32, _u64] + [_p] * 8 + [_sz, _p]),
    "tagan_sgemm_supported": (_c.c_int, [_i32, _i32, _i32, _i32, _i32]),
    "tagan_sgemm_tn_supported": (_c.c_int, [_i32, _i32, _i32, _i32]),
    "tagan_sgemm_wprep": (_c.c_int, [_i32, _i32, _p, _i64, _i32, _i32, _p, _p]),
    "tagan_sgemm_wprep_block": (_c.c_int, [_i32, _p, _i64, _p, _i64, _i32, _p, _p, _p, _p, _p]),
    "tagan_sgemm_nt": (_c.c_int, [_i32, _i32, _i64, _i32, _i32, _p, _i64, _p, _i32, _p, _p, _i64, _p]),
    "tagan_sgemm_tn_workspace": (_sz, [_i64, _i32, _i32]),
    "tagan_sgemm_tn": (_c.c_int, [_i32, _i64, _i32, _i32, _p, _i64, _p, _i64, _i32, _p, _i64, _p, _p, _sz, _p]),
    "tagan_sgemm_ln_supported": (_c.c_int, [_i32, _i32, _i32, _i32]),
    "tagan_sgemm_nt_ln_in": (_c.c_int, [_i32, _i64, _i32, _i32, _p, _i64, _p, _p, _f32, _p, _i32, _p, _p, _i64, _p, _p,
                                        _p]),
    "tagan_sgemm_tn_ln": (_c.c_int, [_i32, _i64, _i32, _i32, _p, _i64, _p, _i64, _p, _p, _p, _p, _i32, _p, _i64, _p,
                                     _p, _sz, _p]),
    "tagan_sgemm_nt_ln_out": (_c.c_int, [_i32, _i64, _i32, _p, _i64, _p, _i32, _p, _p, _f32, _u64, _p, _p, _f32, _p,
                                         _p, _f32, _p, _p, _p, _p, _p, _p, _p]),
    "tagan_sgemm_nt_ln_bwd_workspace": (_sz, [_i64, _i32, _i32]),
    "tagan_sgemm_nt_ln_bwd": (_c.c_int, [_i32, _i64, _i32, _i32, _p, _i64, _p, _i32, _p, _p, _p, _p, _p, _p, _p, _p,
                                         _p, _sz, _p]),
    "tagan_ln2_bwd_out_supported": (_c.c_int, [_i32, _i32, _i32]),
    "tagan_ln2_bwd_out_workspace": (_sz, [_i64, _i32, _i32]),
    "tagan_ln2_bwd_out": (_c.c_int, [_i32, _i32, _i64, _i32, _p, _p, _p, _p, _p, _f32, _u64, _p, _p, _p, _p, _p, _p,
                                     _p, _p, _p, _p, _p, _p, _p, _p, _p, _sz, _p]),
    "tagan_head_supported": (_c.c_int, [_i32, _i32, _i32]),
    "tagan_head_saved_floats": (_sz, [_i32, _i32, _i32]),
    "tagan_head_fwd": (_c.c_int, [_i32, _i32, _i32, _i32, _p, _p, _p, _p, _p, _p, _p, _p, _f32, _p, _p, _f32, _u64,
                                  _p, _c.c_int, _p, _p, _p, _p, _p]),
    "tagan_head_bwd": (_c.c_int, [_i32] * 4 + [_p] * 7 + [_f32, _u64, _p, _c.c_int] + [_p] * 6 + [_p] * 10 + [_p]),
    "tagan_gru_supported": (_c.c_int, [_i32]),
    "tagan_gru_saved_floats": (_sz, [_i64, _i32, _i32]),
    "tagan_gru_fwd": (_c.c_int, [_i64, _i32, _i32, _p, _p, _p, _p, _p, _f32, _p, _p, _f32, _p, _f32, _u64, _p, _p, _p]),
    "tagan_gru_bwd_workspace": (_sz, [_i64, _i32]),
    "tagan_gru_bwd": (_c.c_int, [_i64, _i32, _i32, _p, _p, _p, _p, _p, _p, _p, _f32, _u64, _p, _p, _p, _p, _p, _p, _p,
                                 _p, _p, _sz, _p]),
    "tagan_window_fwd": (_c.c_int, [_c.c_int, _i32, _i64, _i32, _i32, _p, _p, _p]),
    "tagan_window_bwd": (_c.c_int, [_c.c_int, _i32, _i64, _i32, _i32, _p, _p, _p, _p]),
    "tagan_membank_init": (_c.c_int, [_p, _p]),
    "tagan_membank_lookup": (_c.c_int, [_p, _p, _i64, _c.c_int, _i32, _p, _p, _p]),
    "tagan_membank_update": (_c.c_int, [_p, _p, _i64, _p, _i64, _i64, _c.c_double, _i32, _i32, _u64, _p, _p, _p]),
    "tagan_membank_gather": (_c.c_int, [_p, _p, _i64, _p, _p]),
    "tagan_membank_scale": (_c.c_int, [_p, _f32, _p]),
    "tagan_membank_rehash": (_c.c_int, [_p, _p, _p]),
}


class TaganMembank(ctypes.Structure):
    """Mirror of ``struct tagan_membank`` (include/tagan_hip.h)."""
    _fields_ = [("cap", _i64), ("tcap", _i64), ("fcap", _i64), ("H", _i32)] + \
        [(n, _p) for n in ("tkeys", "tvals", "slot_id", "slot_tpos", "states", "inact", "last_seen", "born", "touch",
                           "first_occ", "last_ok", "occ_count", "free_list", "fkeys", "fcount", "ctl")]


class TaganGraph(ctypes.Structure):
    """Mirror of ``struct tagan_graph`` (include/tagan_hip.h)."""
    _fields_ = [("n_nodes", _i64), ("rowptr", _p), ("col", _p), ("csc_ptr", _p), ("csc_row", _p),
                ("csc_eid", _p), ("chunk", _i32), ("chunk_cap", _i64), ("part_cap", _i64),
                ("row_chunk_ptr", _p), ("row_chunk_seg", _p), ("row_chunk_beg", _p), ("row_chunk_part", _p),
                ("row_multi", _p), ("row_counts", _p),
                ("col_chunk_ptr", _p), ("col_chunk_seg", _p), ("col_chunk_beg", _p), ("col_chunk_part", _p),
                ("col_multi", _p), ("col_counts", _p), ("row_chunk_order", _p), ("col_chunk_order", _p),
                ("nnz_cap", _i64)]


_lib = None


def header_symbols():
    """Function names declared in include/tagan_hip.h (for the ABI export test)."""
    with open(HEADER_PATH) as f:
        src = f.read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(tagan_[a-z_0-9]+)\s*\(", src, re.M)))


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("libtagan_hip.so is not built (%s); run __graft_entry__.build() or "
                               "make -C temporal-asymmetric-graph-attention-network_amd/csrc" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(L, name, None)
            if fn is None:
                continue
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc, what):
    if rc != 0:
        msg = lib().tagan_last_error().decode(errors="replace")
        raise RuntimeError("%s failed (status %d): %s" % (what, rc, msg))


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_of(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def require_hip(*tensors):
    for t in tensors:
        if t is not None and (not t.is_cuda or torch.version.hip is None):
            raise RuntimeError("tagan_amd runs on a HIP device only (got a tensor on %s); there is no CPU path"
                               % (t.device,))
