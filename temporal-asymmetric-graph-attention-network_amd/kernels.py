"""Device-side building blocks of the hot path, each a thin wrapper of the C-ABI.

* ``SnapshotGraph`` / ``build_graph`` — block-diagonal CSR (+CSC) of a batch of
  snapshots: the sparse equivalent of graph_attention.py:96-105.
* ``GeoAttnFn``      — autograd Function over ``tagan_geo_attn_fwd/bwd``
  (geometric_attention.py:332-516 + :579-583).
* ``TemporalAttnFn`` — autograd Function over ``tagan_temporal_attn_fwd/bwd``
  (temporal_attention.py:1006-1205 minus the projections).

Every output and workspace is allocated here from PyTorch's caching allocator;
kernels are launched on the current HIP stream.
"""
import ctypes
import os
from collections import OrderedDict
from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch

from . import _lib
from ._lib import check, lib, ptr, require_hip, stream_of


def _mix64(x: int) -> int:
    """splitmix64 finaliser (host side)."""
    x = (x + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return x ^ (x >> 31)


def new_seed() -> int:
    """Dropout seed drawn from torch's default CPU generator (reproducible under manual_seed, no device sync).

    Under torch.distributed the rank is mixed in: ranks that seed their generators identically (the usual
    ``manual_seed`` before building the model) still draw independent dropout masks for their shards of
    the global batch instead of the same mask row for row."""
    s = int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())
    dist = torch.distributed
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        s = _mix64(s ^ (_mix64(dist.get_rank() + 1) & 0x3FFFFFFFFFFFFFFF)) & 0x3FFFFFFFFFFFFFFF
    return s


# ----------------------------------------------------------------------------- graph
CHUNK = 64   # max CSR/CSC entries per work chunk (power-law hubs are split)
# Chunks run in windows of 2^ORDER_BITS consecutive rows/columns, longest first inside a window
# (tagan_chunk_order); TAGAN_CHUNK_ORDER=0 keeps the plain row order (A/B measurements).
ORDER_BITS = 12


@dataclass
class SnapshotGraph:
    """CSR by source (query) row + CSC by destination + chunked work lists, int32, device-resident."""
    num_nodes: int
    rowptr: torch.Tensor
    col: torch.Tensor
    csc_ptr: torch.Tensor
    csc_row: torch.Tensor
    csc_eid: torch.Tensor
    nnz: torch.Tensor              # int64[1] on device
    node_counts: Sequence[int]
    row_chunks: Optional[tuple] = None   # (chunk_ptr, seg, beg, part, multi, counts)
    col_chunks: Optional[tuple] = None
    row_order: Optional[torch.Tensor] = None   # chunk processing order (None = identity)
    col_order: Optional[torch.Tensor] = None
    chunk: int = CHUNK
    chunk_cap: int = 0
    part_cap: int = 0
    nnz_cap: int = 0               # capacity of col / csc arrays (sizes the backward's per-edge dS buffer)
    csr_cpos: Optional[torch.Tensor] = None   # CSC position of each CSR entry (only with build(..., cpos=True))
    _struct: object = None
    pending_err: object = None     # (pinned int32 flag, event) of a deferred index validation

    def check_valid(self) -> None:
        """Raise the deferred IndexError of ``build_graph(validate="deferred")`` (waits for the CSR build only)."""
        if self.pending_err is not None:
            host, ev = self.pending_err
            self.pending_err = None
            ev.synchronize()
            if int(host[0]) != 0:
                raise IndexError("edge_index contains an index out of range for its snapshot's node count")

    def nnz_host(self) -> int:
        return int(self.nnz.item())

    def struct(self):
        """ctypes ``tagan_graph`` pointing at this graph's device arrays (kept alive by self)."""
        if self._struct is None:
            r, c = self.row_chunks, self.col_chunks
            p = lambda t: t.data_ptr()  # noqa: E731
            self._struct = _lib.TaganGraph(self.num_nodes, p(self.rowptr), p(self.col), p(self.csc_ptr),
                                           p(self.csc_row), p(self.csc_eid), self.chunk, self.chunk_cap,
                                           self.part_cap, *[p(t) for t in r], *[p(t) for t in c],
                                           *[None if t is None else p(t) for t in (self.row_order, self.col_order)],
                                           self.nnz_cap)
        return ctypes.byref(self._struct)


def _chunk_lists(seg_ptr: torch.Tensor, n: int, nnz_cap: int, chunk: int):
    L = lib()
    dev = seg_ptr.device
    cap = int(L.tagan_chunk_capacity(n, nnz_cap, chunk))
    pcap = int(L.tagan_part_capacity(nnz_cap, chunk))
    buf = torch.empty(n + 1 + 4 * cap + pcap + 4, dtype=torch.int32, device=dev)
    chunk_ptr = buf[:n + 1]
    o = n + 1
    seg, beg, part = buf[o:o + cap], buf[o + cap:o + 2 * cap], buf[o + 2 * cap:o + 3 * cap]
    multi = buf[o + 4 * cap:o + 4 * cap + pcap]
    counts = buf[o + 4 * cap + pcap:]
    wsb = L.tagan_graph_chunks_workspace(n)
    ws = torch.empty(int(wsb), dtype=torch.uint8, device=dev)
    check(L.tagan_graph_chunks(ptr(seg_ptr), n, chunk, ptr(chunk_ptr), ptr(seg), ptr(beg), ptr(part), ptr(multi),
                               ptr(counts), ptr(ws), wsb, stream_of(seg_ptr)), "tagan_graph_chunks")
    order = None
    if os.environ.get("TAGAN_CHUNK_ORDER", "1") != "0":
        order = buf[o + 3 * cap:o + 4 * cap]
        check(L.tagan_chunk_order(ptr(seg_ptr), n, ptr(chunk_ptr), ptr(seg), ptr(beg), chunk, ORDER_BITS,
                                  ptr(order), stream_of(seg_ptr)), "tagan_chunk_order")
    return (chunk_ptr, seg, beg, part, multi, counts), cap, pcap, order


def _finish(g: SnapshotGraph, nnz_cap: int, chunk: int = CHUNK) -> SnapshotGraph:
    g.row_chunks, g.chunk_cap, g.part_cap, g.row_order = _chunk_lists(g.rowptr, g.num_nodes, nnz_cap, chunk)
    g.col_chunks, _, _, g.col_order = _chunk_lists(g.csc_ptr, g.num_nodes, nnz_cap, chunk)
    g.chunk = chunk
    g.nnz_cap = nnz_cap
    return g


_PTR_TABLES = OrderedDict()
_PTR_PINNED = {}     # tables a captured HIP graph reads by address: never evicted


def _ptr_table(dev, values):
    """Device copy of the snapshot edge/node offset table, cached per (device, offsets): a repeated shape (every
    training step of a sequence, a captured HIP graph) issues no host-to-device copy.

    A table looked up while the current stream is capturing is pinned for the life of the process: the graph bakes
    its address into ``tagan_csr_build``, and an LRU eviction (more than 256 other shapes seen between two replays)
    would otherwise free memory the next replay reads.  A table first needed inside a capture is refused (the H2D
    copy from a host temporary would be replayed from a freed host buffer): warm the step up eagerly first."""
    key = (str(dev), tuple(values))
    t = _PTR_PINNED.get(key)
    if t is not None:
        return t
    capturing = torch.device(dev).type == "cuda" and torch.cuda.is_current_stream_capturing()
    t = _PTR_TABLES.get(key)
    if t is None:
        if capturing:
            raise RuntimeError("snapshot offset table first needed inside a HIP-graph capture: run the step "
                               "eagerly once before capturing it")
        t = torch.tensor(values, dtype=torch.int64).to(dev)
        _PTR_TABLES[key] = t
        if len(_PTR_TABLES) > 256:
            _PTR_TABLES.popitem(last=False)
    else:
        _PTR_TABLES.move_to_end(key)
    if capturing:
        _PTR_PINNED[key] = _PTR_TABLES.pop(key)
    return t


def cat_adjacent(ts: Sequence[torch.Tensor], dim: int) -> torch.Tensor:
    """torch.cat(ts, dim) -- as a zero-copy view when the pieces already lie back to back in one buffer along
    ``dim`` (the layout of a batch generated or ingested in one allocation), else a real concatenation."""
    if len(ts) == 1:
        return ts[0]
    if torch.is_grad_enabled() and any(t.requires_grad for t in ts):
        # as_strided's backward is taken with respect to ts[0]'s geometry: the other pieces would get no gradient
        return torch.cat(list(ts), dim)
    t0 = ts[0]
    ok = all(t.dtype == t0.dtype and t.device == t0.device and t.dim() == t0.dim() and t.stride() == t0.stride()
             and t.untyped_storage().data_ptr() == t0.untyped_storage().data_ptr() for t in ts)
    if ok:
        off = t0.storage_offset()
        for t in ts:
            if t.storage_offset() != off or any(t.shape[d] != t0.shape[d] for d in range(t.dim()) if d != dim):
                ok = False
                break
            off += t.shape[dim] * t.stride(dim)
    if not ok:
        return torch.cat(list(ts), dim)
    size = list(t0.shape)
    size[dim] = sum(int(t.shape[dim]) for t in ts)
    return t0.as_strided(size, t0.stride(), t0.storage_offset())


def build_graph(edge_indices: List[torch.Tensor], node_counts: Sequence[int], validate=True,
                chunk: int = CHUNK, cpos: bool = False) -> SnapshotGraph:
    """CSR/CSC of the block-diagonal union of snapshot adjacencies (+ self-loops, de-duplicated).

    ``edge_indices[g]`` is snapshot g's [2, E_g] edge_index with local node ids.
    ``validate``: True raises IndexError for an out-of-range index like the reference's
    ``adj[edge_index[0], edge_index[1]] = 1`` (one device sync, here); "deferred" records the flag and
    ``SnapshotGraph.check_valid()`` raises later (waits only for the CSR build, not the stream); False skips
    it.  An out-of-range edge never enters the CSR either way (tagan_csr_build drops it), so the kernels
    that follow are safe to launch before the check.  ``cpos`` also writes ``csr_cpos`` (the CSC position of
    each CSR entry; a random scatter nothing in the attention path needs).
    """
    require_hip(*edge_indices)
    eis = [e.to(torch.int64) for e in edge_indices]
    ei = cat_adjacent(eis, 1)
    e_ptr = [0]
    for e in eis:
        e_ptr.append(e_ptr[-1] + int(e.shape[1]))
    return build_graph_cat(ei, e_ptr, node_counts, validate, chunk, cpos)


def build_graph_cat(ei: torch.Tensor, e_ptr: Sequence[int], node_counts: Sequence[int], validate=True,
                    chunk: int = CHUNK, cpos: bool = False) -> SnapshotGraph:
    """``build_graph`` on already-concatenated edges: ei [2, ΣE_g] int64 (local ids), snapshot g's edges in
    columns [e_ptr[g], e_ptr[g+1]) (the layout of ``ingest.SnapshotBatch``)."""
    require_hip(ei)
    dev = ei.device
    ei = ei.to(torch.int64)
    if ei.stride(1) != 1 or ei.stride(0) < ei.shape[1]:
        ei = ei.contiguous()
    E = int(ei.shape[1])
    ld = int(ei.stride(0))
    G = len(node_counts)
    assert len(e_ptr) == G + 1 and e_ptr[0] == 0 and e_ptr[-1] == E
    N = int(sum(node_counts))
    n_ptr = [0]
    for n in node_counts:
        n_ptr.append(n_ptr[-1] + int(n))
    meta = _ptr_table(dev, list(e_ptr) + n_ptr)
    edge_ptr, node_ptr = meta[:G + 1], meta[G + 1:]
    cap = E + N
    buf = torch.empty(2 * (N + 1) + (4 if cpos else 3) * cap, dtype=torch.int32, device=dev)
    rowptr, csc_ptr = buf[:N + 1], buf[N + 1:2 * (N + 1)]
    o = 2 * (N + 1)
    col, csc_row, csc_eid = buf[o:o + cap], buf[o + cap:o + 2 * cap], buf[o + 2 * cap:o + 3 * cap]
    cpos_t = buf[o + 3 * cap:o + 4 * cap] if cpos else None
    scal = torch.empty(2, dtype=torch.int64, device=dev)
    nnz = scal[0:1]
    err = scal[1:2].view(torch.int32)[:1]
    L = lib()
    ws_bytes = L.tagan_csr_build_workspace(E, N)
    ws = torch.empty(max(int(ws_bytes), 1), dtype=torch.uint8, device=dev)
    check(L.tagan_csr_build(ptr(ei), ld, E, ptr(edge_ptr), ptr(node_ptr), G, N,
                            max(n_ptr[i + 1] - n_ptr[i] for i in range(G)), ptr(rowptr), ptr(col),
                            ptr(csc_ptr), ptr(csc_row), ptr(csc_eid), ptr(nnz), ptr(err),
                            ptr(cpos_t) if cpos else None, ptr(ws), ws_bytes, stream_of(ei)), "tagan_csr_build")
    g = SnapshotGraph(N, rowptr, col, csc_ptr, csc_row, csc_eid, nnz, list(node_counts))
    g.csr_cpos = cpos_t
    if validate == "deferred":
        host = torch.empty(1, dtype=torch.int32, pin_memory=True)
        host.copy_(err, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev))
        g.pending_err = (host, ev)
    elif validate and int(err.item()) != 0:
        raise IndexError("edge_index contains an index out of range for its snapshot's node count")
    return _finish(g, cap, chunk)


def graph_from_dense_mask(mask: torch.Tensor) -> SnapshotGraph:
    """CSR/CSC of a dense [B,S,S] (or [S,S]) attention mask (nonzero = attend), block-diagonal over B."""
    if mask.dim() == 2:
        mask = mask.unsqueeze(0)
    B, S, _ = mask.shape
    b, i, j = (mask != 0).nonzero(as_tuple=True)
    src = (b * S + i).to(torch.int64)
    dst = (b * S + j).to(torch.int64)
    return _graph_from_pairs(src, dst, B * S, [S] * B)


def _graph_from_pairs(src, dst, N, node_counts):
    """CSR/CSC from already-unique (src,dst) pairs sorted by (src,dst) (torch.nonzero order); no self-loops added."""
    dev = src.device
    nnz = int(src.numel())
    counts = torch.bincount(src, minlength=N)
    rowptr = torch.zeros(N + 1, dtype=torch.int64, device=dev)
    rowptr[1:] = torch.cumsum(counts, 0)
    order = torch.argsort(dst * N + src)
    ccounts = torch.bincount(dst, minlength=N)
    cptr = torch.zeros(N + 1, dtype=torch.int64, device=dev)
    cptr[1:] = torch.cumsum(ccounts, 0)
    i32 = torch.int32
    g = SnapshotGraph(N, rowptr.to(i32), dst.to(i32).contiguous(), cptr.to(i32), src[order].to(i32).contiguous(),
                      order.to(i32).contiguous(), torch.tensor([nnz], dtype=torch.int64, device=dev),
                      list(node_counts))
    return _finish(g, max(nnz, 1))


# ----------------------------------------------------------------------------- geometric attention
class GeoAttnFn(torch.autograd.Function):
    """ctx = edge-softmax attention over ``graph`` for qkv = [N, 3H] (q | k | v)."""

    @staticmethod
    def forward(ctx, qkv, param, graph: SnapshotGraph, metric: int, heads: int, p_drop: float, seed: int):
        require_hip(qkv)
        assert qkv.dim() == 2 and qkv.is_contiguous() and qkv.dtype == torch.float32
        N, H3 = qkv.shape
        H = H3 // 3
        d = H // heads
        out = torch.empty(N, H, device=qkv.device, dtype=torch.float32)
        lse = torch.empty(N, heads, device=qkv.device, dtype=torch.float32)
        prm = param.detach().contiguous() if param is not None else None
        _geo_fwd(qkv, graph, metric, heads, prm, p_drop, seed, out, lse, None)
        ctx.save_for_backward(qkv, out, lse, prm)
        ctx.graph, ctx.metric, ctx.heads, ctx.p_drop, ctx.seed = graph, metric, heads, p_drop, seed
        ctx.has_param = param is not None
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse, prm = ctx.saved_tensors
        g = ctx.graph
        N, H3 = qkv.shape
        H = H3 // 3
        heads = ctx.heads
        d = H // heads
        dout = dout.contiguous()
        dqkv = torch.empty_like(qkv)
        L = lib()
        gs = g.struct()
        ws_bytes = L.tagan_geo_attn_bwd_workspace(gs, heads, d)
        ws = torch.empty(int(ws_bytes), dtype=torch.uint8, device=qkv.device)
        dprm = torch.empty(heads, device=qkv.device, dtype=torch.float32) if ctx.has_param and \
            ctx.needs_input_grad[1] else None
        base, es = qkv.data_ptr(), qkv.element_size()
        dbase = dqkv.data_ptr()
        check(L.tagan_geo_attn_bwd(_lib.TAGAN_F32, ctx.metric, gs, heads, d, base, base + H * es, base + 2 * H * es,
                                   H3, ptr(prm), float(ctx.p_drop), ctx.seed, ptr(out), ptr(lse), ptr(dout), dbase,
                                   dbase + H * es, dbase + 2 * H * es, H3, ptr(dprm), ptr(ws), ws_bytes,
                                   stream_of(qkv)), "tagan_geo_attn_bwd")
        return dqkv, dprm, None, None, None, None, None


def _geo_fwd(qkv, graph, metric, heads, prm, p_drop, seed, out, lse, alpha):
    N, H3 = qkv.shape
    H = H3 // 3
    d = H // heads
    L = lib()
    gs = graph.struct()
    ws_bytes = L.tagan_geo_attn_fwd_workspace(gs, heads, d)
    ws = torch.empty(max(int(ws_bytes), 1), dtype=torch.uint8, device=qkv.device)
    base, es = qkv.data_ptr(), qkv.element_size()
    check(L.tagan_geo_attn_fwd(_lib.dtype_code(qkv), metric, gs, heads, d, base, base + H * es, base + 2 * H * es, H3,
                               ptr(prm), float(p_drop), seed, ptr(out), ptr(lse), ptr(alpha), ptr(ws), ws_bytes,
                               stream_of(qkv)), "tagan_geo_attn_fwd")


def geo_edge_alpha(qkv, graph: SnapshotGraph, metric: int, heads: int, param=None, p_drop=0.0, seed=0):
    """Per-edge post-dropout attention weights [nnz, heads] (no autograd; inspection only)."""
    N, H3 = qkv.shape
    H = H3 // 3
    out = torch.empty(N, H, device=qkv.device)
    lse = torch.empty(N, heads, device=qkv.device)
    alpha = torch.empty(int(graph.col.numel()), heads, device=qkv.device)
    prm = param.detach().contiguous() if param is not None else None
    _geo_fwd(qkv, graph, metric, heads, prm, p_drop, seed, out, lse, alpha)
    return alpha[:graph.nnz_host()]


# ----------------------------------------------------------------------------- temporal attention
@dataclass
class TemporalMask:
    """Effective keep-mask for the temporal kernel (broadcast over rows/heads via zero strides)."""
    causal: bool = False
    keep: Optional[torch.Tensor] = None     # uint8, contiguous, last two dims [T, T]
    bstride: int = 0
    hstride: int = 0


def _keep_cache(R, T, heads, d, mask, bias_dense, p_drop, device):
    """(buffer, bytes, c_int32 flag) for the forward's dropout keep bits (tagan_temporal_attn_keep_bytes: the
    matrix-core path for T in (32, 128] stores them so the backward skips the counter hash); (None, 0, flag) where no
    path uses them.  The flag tells whether the forward wrote the bits: only then does the backward get them."""
    written = ctypes.c_int32(0)
    kb = int(lib().tagan_temporal_attn_keep_bytes(R, T, heads, d, int(mask.causal) if mask is not None else 0,
                                                  int(mask is not None and mask.keep is not None),
                                                  int(bias_dense is not None), float(p_drop)))
    if kb == 0:
        return None, 0, written
    return torch.empty(kb // 4, dtype=torch.int32, device=device), kb, written


class TemporalAttnFn(torch.autograd.Function):
    """Per-row attention over T steps.  ``qkv`` is [R, T, 3H] (row-major) or [T, R, 3H] (time_major)."""

    @staticmethod
    def forward(ctx, qkv, bias_table, bias_dense, time_major: bool, heads: int, mask: TemporalMask,
                p_drop: float, seed: int, want_attn: bool):
        require_hip(qkv)
        assert qkv.dim() == 3 and qkv.is_contiguous() and qkv.dtype == torch.float32
        A0, A1, H3 = qkv.shape
        H = H3 // 3
        d = H // heads
        R, T = (A1, A0) if time_major else (A0, A1)
        s_row, s_t = (H3, R * H3) if time_major else (T * H3, H3)
        o_row, o_t = (H, R * H) if time_major else (T * H, H)
        out = torch.empty(A0, A1, H, device=qkv.device, dtype=torch.float32)
        lse = torch.empty(R, heads, T, device=qkv.device, dtype=torch.float32)
        attn = torch.empty(R, heads, T, T, device=qkv.device, dtype=torch.float32) if want_attn else None
        bt = bias_table.detach().contiguous() if bias_table is not None else None
        bd = bias_dense.detach().contiguous() if bias_dense is not None else None
        bd_stride = (0 if bd.shape[0] == 1 else heads * T * T) if bd is not None else 0
        base, es = qkv.data_ptr(), qkv.element_size()
        keep, kb, written = _keep_cache(R, T, heads, d, mask, bd, p_drop, qkv.device)
        check(lib().tagan_temporal_attn_fwd_keep(_lib.TAGAN_F32, R, T, heads, d, base, base + H * es,
                                                 base + 2 * H * es, s_row, s_t, ptr(bt), ptr(bd), bd_stride,
                                                 ptr(mask.keep), mask.bstride, mask.hstride, int(mask.causal),
                                                 float(p_drop), seed, ptr(out), o_row, o_t, ptr(lse), ptr(attn),
                                                 ptr(keep), kb, ctypes.byref(written), stream_of(qkv)),
              "tagan_temporal_attn_fwd_keep")
        ctx.keep = keep if written.value else None
        ctx.save_for_backward(qkv, out, lse, bt, bd)
        ctx.cfg = (time_major, heads, mask, p_drop, seed, bd_stride)
        ctx.need_bt = bias_table is not None
        ctx.need_bd = bias_dense is not None
        if attn is not None:
            ctx.mark_non_differentiable(attn)
        return out, attn

    @staticmethod
    def backward(ctx, dout, _dattn):
        qkv, out, lse, bt, bd = ctx.saved_tensors
        time_major, heads, mask, p_drop, seed, bd_stride = ctx.cfg
        A0, A1, H3 = qkv.shape
        H = H3 // 3
        d = H // heads
        R, T = (A1, A0) if time_major else (A0, A1)
        s_row, s_t = (H3, R * H3) if time_major else (T * H3, H3)
        o_row, o_t = (H, R * H) if time_major else (T * H, H)
        dout = dout.contiguous()
        dqkv = torch.empty_like(qkv)
        L = lib()
        dbt = torch.empty(heads, 2 * T - 1, device=qkv.device) if (ctx.need_bt and ctx.needs_input_grad[1]) else None
        dbd = torch.empty(R, heads, T, T, device=qkv.device) if (ctx.need_bd and ctx.needs_input_grad[2]) else None
        ws_bytes = L.tagan_temporal_attn_bwd_workspace(R, T, heads, d)
        ws = torch.empty(int(ws_bytes), dtype=torch.uint8, device=qkv.device)
        base, es = qkv.data_ptr(), qkv.element_size()
        dbase = dqkv.data_ptr()
        keep = ctx.keep
        ctx.keep = None
        check(L.tagan_temporal_attn_bwd_keep(_lib.TAGAN_F32, R, T, heads, d, base, base + H * es,
                                             base + 2 * H * es, s_row, s_t, ptr(bt), ptr(bd), bd_stride,
                                             ptr(mask.keep), mask.bstride, mask.hstride, int(mask.causal),
                                             float(p_drop), seed, ptr(out), o_row, o_t, ptr(lse), ptr(dout), o_row,
                                             o_t, dbase, dbase + H * es, dbase + 2 * H * es, s_row, s_t, ptr(dbt),
                                             ptr(dbd), None, ptr(keep), keep.numel() * 4 if keep is not None else 0,
                                             ptr(ws), ws_bytes, stream_of(qkv)),
              "tagan_temporal_attn_bwd_keep")
        if dbd is not None and bd is not None and bd.shape[0] == 1:
            dbd = dbd.sum(0, keepdim=True)
        return dqkv, dbt, dbd, None, None, None, None, None, None




# ----------------------------------------------------------------------------- projections
def split_rows(K: int, rows: int = 2048) -> int:
    """Slice height for a split-K weight gradient: a multiple of 64 in [rows/2, 2·rows] that divides K
    (closest to ``rows`` in ratio), so no remainder GEMM + add is needed (K = 320000 at C2 -> 2560); else ``rows``."""
    best = None
    for r in range(64 * max(1, rows // 128), 2 * rows + 1, 64):
        if K % r == 0 and (best is None or max(r, rows) / min(r, rows) < max(best, rows) / min(best, rows)):
            best = r
    return best or rows


def weight_grad(dy2: torch.Tensor, x2: torch.Tensor, rows: int = 2048) -> torch.Tensor:
    """dW = dyᵀ·x for K = dy.shape[0] >> M, N: split-K batched GEMM (hipBLASLt) + ordered sum.

    A single [M,K]x[K,N] GEMM with K = 320k runs at 15-30 TF/s on gfx950; splitting K
    into 2048-row slices gives hipBLASLt a batched problem it tiles well (≈110 TF/s
    fp32) and sums the slices in a fixed order (profiles/).
    """
    K, M = dy2.shape
    N = x2.shape[1]
    if K < 4 * rows:
        return dy2.t() @ x2
    rows = split_rows(K, rows)
    c = K // rows
    main = c * rows
    xs = x2.as_strided((c, rows, N), (rows * x2.stride(0), x2.stride(0), 1))   # x2 may be a column view
    dw = torch.bmm(dy2[:main].view(c, rows, M).transpose(1, 2), xs).sum(0)
    if main < K:
        dw = dw + dy2[main:].t() @ x2[main:]
    return dw


def colsum(x2):
    """Column sums of a tall [M, N] matrix (bias gradients): HIP two-stage ordered reduction."""
    M, N = x2.shape
    out = torch.empty(N, device=x2.device)
    L = lib()
    wsb = L.tagan_colsum_workspace(M, N)
    ws = torch.empty(max(int(wsb), 1), dtype=torch.uint8, device=x2.device)
    check(L.tagan_colsum(_lib.dtype_code(x2), M, N, ptr(x2), x2.stride(0), ptr(out), ptr(ws), wsb, stream_of(x2)),
          "tagan_colsum")
    return out


class LinearFn(torch.autograd.Function):
    """y = x·Wᵀ + b with the split-K weight gradient above."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        return torch.nn.functional.linear(x, w, b)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = (dy2 @ w).view(x.shape)
        if ctx.needs_input_grad[1]:
            dw = weight_grad(dy2, x.reshape(-1, x.shape[-1]).contiguous())
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = colsum(dy2) if (dy2.is_cuda and dy2.shape[1] % 4 == 0 and dy2.shape[1] <= 1024) else dy2.sum(0)
        return dx, dw, db


def linear(x, w, b=None):
    return LinearFn.apply(x, w, b)


class NarrowLinearFn(torch.autograd.Function):
    """y = x·Wᵀ + b for a narrow fp32 input (K <= 31 features): csrc/narrow.hip's exact-f32 MFMA kernels, the
    weight and bias gradients in one pass over dy (the node embedding, model.py:233)."""

    @staticmethod
    def forward(ctx, x, w, b):
        require_hip(x)
        M, K = x.shape
        N = w.shape[0]
        y = torch.empty(M, N, device=x.device, dtype=torch.float32)
        wc = w.contiguous()
        check(lib().tagan_narrow_linear_fwd(M, K, N, ptr(x), x.stride(0), ptr(wc), ptr(b), ptr(y), N,
                                            stream_of(x)), "tagan_narrow_linear_fwd")
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        M, K = x.shape
        N = w.shape[0]
        dy = dy.float().contiguous()
        if dy.data_ptr() % 16:
            dy = dy.clone()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = dy @ w
        want_w = ctx.needs_input_grad[1]
        want_b = ctx.has_b and ctx.needs_input_grad[2]
        if (want_w or want_b) and M > 0:
            dw = torch.empty(N, K, device=x.device) if want_w else None
            db = torch.empty(N, device=x.device) if want_b else None
            L = lib()
            wsb = L.tagan_narrow_linear_bwd_workspace(M, K, N)
            ws = torch.empty(int(wsb), dtype=torch.uint8, device=x.device)
            check(L.tagan_narrow_linear_bwd(M, K, N, ptr(x), x.stride(0), ptr(dy), N, ptr(dw), ptr(db), ptr(ws), wsb,
                                            stream_of(x)), "tagan_narrow_linear_bwd")
        elif want_w or want_b:
            dw = torch.zeros_like(w) if want_w else None
            db = torch.zeros(N, device=x.device) if want_b else None
        return dx, dw, db


class BiasTableFn(torch.autograd.Function):
    """The temporal layer's [heads, 2T-1] bias table from its asymmetric-kernel and relative-position tables
    (csrc/params.hip: one launch each way; temporal_attention.py:732-790)."""

    @staticmethod
    def forward(ctx, K, R, T: int, W: int, m: int):
        require_hip(K)
        heads = K.shape[1]
        Kc = K.contiguous()
        Rc = R.contiguous() if R is not None else None
        tab = torch.empty(heads, 2 * T - 1, device=K.device, dtype=torch.float32)
        check(lib().tagan_temporal_bias_table(T, heads, ptr(Kc), W, ptr(Rc), m, ptr(tab), stream_of(K)),
              "tagan_temporal_bias_table")
        ctx.cfg = (T, W, m, heads, R is not None)
        return tab

    @staticmethod
    def backward(ctx, g):
        T, W, m, heads, has_r = ctx.cfg
        g = g.float().contiguous()
        dK = torch.empty(2 * W + 1, heads, device=g.device) if ctx.needs_input_grad[0] else None
        dR = torch.empty(2 * m + 1, heads, device=g.device) if (has_r and ctx.needs_input_grad[1]) else None
        if dK is not None or dR is not None:
            check(lib().tagan_temporal_bias_table_bwd(T, heads, ptr(g), W, m, ptr(dK), ptr(dR), stream_of(g)),
                  "tagan_temporal_bias_table_bwd")
        return dK, dR, None, None, None


_NARROW = os.environ.get("TAGAN_NARROW", "1") != "0"


def embed_linear(x, w, b=None):
    """The node embedding: the narrow-input HIP kernels when they apply (fp32 CUDA x with unit column stride,
    K <= 31, N in 64 / 128 / 256, a 16-byte aligned bias), else ``linear``."""
    if (_NARROW and x.is_cuda and x.dim() == 2 and x.dtype == torch.float32 and w.dtype == torch.float32
            and x.stride(1) == 1 and (b is None or (b.is_contiguous() and b.data_ptr() % 16 == 0))
            and lib().tagan_narrow_linear_supported(x.shape[1], w.shape[0])):
        return NarrowLinearFn.apply(x, w, b)
    return linear(x, w, b)


def fused_qkv(x, q_lin, k_lin, v_lin):
    """One GEMM for the three projections (hipBLASLt via torch): [.., H] -> [.., 3H] = q | k | v."""
    w = torch.cat([q_lin.weight, k_lin.weight, v_lin.weight], 0)
    b = torch.cat([q_lin.bias, k_lin.bias, v_lin.bias], 0)
    return linear(x, w, b)


# ----------------------------------------------------------------------------- layer norm
class AddLayerNormFn(torch.autograd.Function):
    """y = LayerNorm(dropout(a) + b) (b optional) on the HIP kernels of csrc/layernorm.hip."""

    @staticmethod
    def forward(ctx, a, b, gamma, beta, eps: float, p_drop: float, seed: int):
        require_hip(a)
        H = a.shape[-1]
        a2 = a.reshape(-1, H).contiguous()
        M = a2.shape[0]
        b2 = b.reshape(-1, H).contiguous() if b is not None else None
        keep_s = b is not None or p_drop > 0
        s = torch.empty_like(a2) if keep_s else None
        y = torch.empty_like(a2)
        mean = torch.empty(M, device=a.device)
        rstd = torch.empty(M, device=a.device)
        check(lib().tagan_add_layernorm_fwd(_lib.TAGAN_F32, M, H, ptr(a2), None, ptr(b2), float(p_drop), seed,
                                            ptr(gamma), ptr(beta), float(eps), ptr(s), ptr(y), 0, ptr(mean),
                                            ptr(rstd), stream_of(a2)), "tagan_add_layernorm_fwd")
        ctx.save_for_backward(s if keep_s else a2, mean, rstd, gamma)
        ctx.cfg = (p_drop, seed, b is not None, a.shape)
        return y.view(a.shape)

    @staticmethod
    def backward(ctx, dy):
        s, mean, rstd, gamma = ctx.saved_tensors
        p_drop, seed, has_b, shape = ctx.cfg
        H = shape[-1]
        dy2 = dy.reshape(-1, H).contiguous()
        M = dy2.shape[0]
        need_a, need_b = ctx.needs_input_grad[0], has_b and ctx.needs_input_grad[1]
        da = torch.empty_like(dy2) if need_a else None
        ds = torch.empty_like(dy2) if need_b else None
        dg = torch.empty(H, device=dy.device) if ctx.needs_input_grad[2] else None
        dbt = torch.empty(H, device=dy.device) if ctx.needs_input_grad[3] else None
        L = lib()
        wsb = L.tagan_layernorm_bwd_workspace(M, H)
        ws = torch.empty(int(wsb), dtype=torch.uint8, device=dy.device)
        check(L.tagan_layernorm_bwd(_lib.TAGAN_F32, M, H, ptr(s), ptr(mean), ptr(rstd), ptr(gamma), ptr(dy2), None,
                                    float(p_drop), seed, ptr(ds), ptr(da), ptr(dg), ptr(dbt), None, ptr(ws), wsb,
                                    stream_of(dy2)), "tagan_layernorm_bwd")
        return (da.view(shape) if da is not None else None, ds.view(shape) if ds is not None else None,
                dg, dbt, None, None, None)


def layer_norm(x, ln: torch.nn.LayerNorm):
    """LayerNorm on the HIP kernel when the width is supported (else ATen's, same math)."""
    if x.is_cuda and lib().tagan_layernorm_supported(x.shape[-1]):
        return AddLayerNormFn.apply(x, None, ln.weight, ln.bias, ln.eps, 0.0, 0)
    return ln(x)


def dropout_add_layer_norm(a, b, ln: torch.nn.LayerNorm, p: float):
    """LayerNorm(dropout(a) + b) fused (the residual tail of every attention layer)."""
    if a.is_cuda and lib().tagan_layernorm_supported(a.shape[-1]):
        return AddLayerNormFn.apply(a, b, ln.weight, ln.bias, ln.eps, float(p), new_seed() if p > 0 else 0)
    return ln(torch.nn.functional.dropout(a, p, True) + b)


# ----------------------------------------------------------------------------- pooling
class PoolFn(torch.autograd.Function):
    """gf [T, H] of model.py:377-427 from the time-major temporal output [T, N, H] (csrc/pool.hip)."""

    @staticmethod
    def forward(ctx, x_tm):
        require_hip(x_tm)
        T, N, H = x_tm.shape
        assert x_tm.stride(2) == 1 and x_tm.dtype == torch.float32
        out = torch.empty(T, H, device=x_tm.device, dtype=torch.float32)
        L = lib()
        wsb = L.tagan_pool_workspace(T, H)
        ws = torch.empty(int(wsb), dtype=torch.uint8, device=x_tm.device)
        check(L.tagan_pool_fwd(_lib.TAGAN_F32, T, N, H, ptr(x_tm), x_tm.stride(1), x_tm.stride(0), ptr(out), ptr(ws),
                               wsb, stream_of(x_tm)), "tagan_pool_fwd")
        ctx.shape = (T, N, H)
        return out

    @staticmethod
    def backward(ctx, g):
        T, N, H = ctx.shape
        g = g.contiguous()
        dx = torch.empty(T, N, H, device=g.device, dtype=torch.float32)
        check(lib().tagan_pool_bwd(_lib.TAGAN_F32, T, N, H, ptr(g), ptr(dx), H, N * H, stream_of(g)),
              "tagan_pool_bwd")
        return dx


def pool_time_major(x_tm: torch.Tensor) -> torch.Tensor:
    return PoolFn.apply(x_tm)

