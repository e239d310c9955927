// Snapshot CSR/CSC builder: the sparse form of graph_attention.py:96-105
//   adj = zeros(N,N); adj[edge_index[0], edge_index[1]] = 1; adj += eye(N)
// for a block-diagonal batch of snapshots.  Integer/byte work: HBM-bound,
// no MFMA.  Keys global_src * NL + local_dst (NL = the largest snapshot) are
// radix-sorted with rocPRIM over only the bits of N * NL -- 32-bit keys when that
// fits (32 bits at C2 instead of a 33-bit key in 64), de-duplicated, scattered into CSR.  The CSC (with CSR edge
// ids) is a STABLE 32-bit key-value sort of the CSR entries by dst alone: the CSR
// order is by src, so stability keeps src ascending within each column.
#include <cstring>

#include <rocprim/rocprim.hpp>

#include "common.cuh"

namespace tagan {
namespace {

constexpr int BLK = 256;

// Graph of edge e: binary search in edge_ptr[0..G] (G small; edge_ptr in L2/scalar cache).
__device__ __forceinline__ int find_graph(const int64_t* __restrict__ edge_ptr, int G, int64_t e) {
    int lo = 0, hi = G - 1;
    while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if (edge_ptr[mid] <= e) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// Graph of global node n (n < N): binary search in node_ptr[0..G].
__device__ __forceinline__ int64_t node_base(const int64_t* __restrict__ node_ptr, int G, int64_t n) {
    return node_ptr[find_graph(node_ptr, G, n)];
}

// Sort key of the pair (global src s, local dst d): s * NL + d with NL = the largest snapshot's node
// count, so ascending keys are the CSR order (src-major, dst-minor); the key N * NL marks a dropped
// (out-of-range) edge.  K = uint32_t whenever N * NL < 2^32 (C1, C2: 320k x 10k = 3.2e9): half the key
// bytes of the 64-bit form and one radix pass fewer.
template <typename K>
__global__ void __launch_bounds__(BLK) k_make_keys(const int64_t* __restrict__ ei, int64_t ld_ei, int64_t E,
                                                   const int64_t* __restrict__ edge_ptr,
                                                   const int64_t* __restrict__ node_ptr, int G,
                                                   int64_t N, int64_t NL, K* __restrict__ keys,
                                                   int32_t* __restrict__ err) {
    const K sentinel = (K)N * (K)NL;
    for (int64_t p = blockIdx.x * (int64_t)BLK + threadIdx.x; p < E + N; p += (int64_t)gridDim.x * BLK) {
        K key;
        if (p < E) {
            const int g = find_graph(edge_ptr, G, p);
            const int64_t base = node_ptr[g];
            const int64_t n = node_ptr[g + 1] - base;
            int64_t s = ei[p], d = ei[ld_ei + p];
            s += (s < 0) ? n : 0;                 // torch advanced indexing wraps negatives
            d += (d < 0) ? n : 0;
            if (s < 0 || s >= n || d < 0 || d >= n) {
                atomicOr(err, 1);
                key = sentinel;
            } else {
                key = (K)(base + s) * (K)NL + (K)d;
            }
        } else {
            const int64_t i = p - E;                // self-loop of global node i (the "+ eye")
            key = (K)i * (K)NL + (K)(i - node_base(node_ptr, G, i));
        }
        keys[p] = key;
    }
}

template <typename K>
__global__ void __launch_bounds__(BLK) k_unique_flags(const K* __restrict__ keys, int64_t M, int64_t N, int64_t NL,
                                                      int32_t* __restrict__ flags) {
    const K sentinel = (K)N * (K)NL;
    for (int64_t p = blockIdx.x * (int64_t)BLK + threadIdx.x; p < M; p += (int64_t)gridDim.x * BLK) {
        const K k = keys[p];
        flags[p] = (k < sentinel && (p == 0 || keys[p - 1] != k)) ? 1 : 0;
    }
}

// Scatter unique keys into CSR; emit CSC keys (global dst) with value = CSR position and the
// row of every CSR position (srcq) for the CSC scatter.
template <typename K>
__global__ void __launch_bounds__(BLK) k_scatter_csr(const K* __restrict__ keys, const int32_t* __restrict__ flags,
                                                     const int32_t* __restrict__ pos, int64_t M, int64_t N,
                                                     int64_t NL, const int64_t* __restrict__ node_ptr, int G,
                                                     int32_t* __restrict__ rowptr, int32_t* __restrict__ col,
                                                     uint32_t* __restrict__ ckeys, int32_t* __restrict__ cvals,
                                                     int32_t* __restrict__ srcq, int64_t* __restrict__ nnz_out) {
    const K nl = (K)NL;
    for (int64_t p = blockIdx.x * (int64_t)BLK + threadIdx.x; p < M; p += (int64_t)gridDim.x * BLK) {
        if (p == M - 1) {
            const int64_t nnz = (int64_t)pos[p] + flags[p];
            *nnz_out = nnz;
            rowptr[N] = (int32_t)nnz;
        }
        if (!flags[p]) continue;
        const K k = keys[p];
        const K rk = k / nl;
        const int64_t r = (int64_t)rk;
        const int32_t c = (int32_t)(node_base(node_ptr, G, r) + (int64_t)(k - rk * nl));
        const int32_t q = pos[p];
        col[q] = c;
        if (p == 0 || keys[p - 1] / nl != rk) rowptr[r] = q;   // every row has its self-loop
        ckeys[q] = (uint32_t)c;
        cvals[q] = q;
        srcq[q] = (int32_t)r;
    }
}

__global__ void __launch_bounds__(BLK) k_fill_tail(uint32_t* __restrict__ ckeys, int32_t* __restrict__ cvals,
                                                   const int64_t* __restrict__ nnz_p, int64_t M, int64_t N) {
    const int64_t nnz = *nnz_p;
    for (int64_t p = nnz + blockIdx.x * (int64_t)BLK + threadIdx.x; p < M; p += (int64_t)gridDim.x * BLK) {
        ckeys[p] = (uint32_t)N;    // sentinel: sorts after every column
        cvals[p] = -1;
    }
}

__global__ void __launch_bounds__(BLK) k_scatter_csc(const uint32_t* __restrict__ ckeys,
                                                     const int32_t* __restrict__ cvals,
                                                     const int32_t* __restrict__ srcq,
                                                     const int64_t* __restrict__ nnz_p, int64_t N,
                                                     int32_t* __restrict__ csc_ptr, int32_t* __restrict__ csc_row,
                                                     int32_t* __restrict__ csc_eid) {
    const int64_t nnz = *nnz_p;
    for (int64_t p = blockIdx.x * (int64_t)BLK + threadIdx.x; p < nnz; p += (int64_t)gridDim.x * BLK) {
        const uint32_t c = ckeys[p];
        const int32_t q = cvals[p];
        csc_row[p] = srcq[q];
        csc_eid[p] = q;
        if (p == 0 || ckeys[p - 1] != c) csc_ptr[c] = (int32_t)p;
        if (p == nnz - 1) csc_ptr[N] = (int32_t)nnz;
    }
}

// inverse of csc_eid: the CSC position of each CSR entry (the column-first edge backward reads dS through it)
__global__ void __launch_bounds__(BLK) k_csc_pos(const int32_t* __restrict__ csc_eid, const int64_t* __restrict__ nnz_p,
                                                 int32_t* __restrict__ cpos) {
    const int64_t nnz = *nnz_p;
    for (int64_t p = blockIdx.x * (int64_t)BLK + threadIdx.x; p < nnz; p += (int64_t)gridDim.x * BLK)
        cpos[csc_eid[p]] = (int32_t)p;
}

// CSC sort (32-bit dst keys over key_bits(N) bits, int32 values): 10-bit digits instead of rocPRIM's default 8 --
// two onesweep passes instead of three at N < 2^20.  3.2M pairs / 19 bits (C2): 129 -> 105 us; the CSR key sort
// stays on the default (11-bit digits measured slower there: 142 vs 180 us; tools/probes/sort_probe.hip).
using CscSortCfg = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 32>, rocprim::kernel_config<1024, 12>, 10,
                                        rocprim::block_radix_rank_algorithm::match>,
    0>;

int key_bits(int64_t N) {
    int b = 1;
    while (b < 32 && ((int64_t)1 << b) <= N) ++b;   // values 0..N inclusive (sentinel = N)
    return b;
}

struct CsrWs {
    size_t keys_a, keys_b, ckeys_b, cvals_b, srcq, flags, pos, temp, total;
    size_t temp_bytes;
};

CsrWs plan(int64_t E, int64_t N) {
    const int64_t M = E + N;
    CsrWs w{};
    size_t off = 0;
    auto take = [&](size_t bytes) { size_t o = off; off = align_up(off + bytes, 256); return o; };
    w.keys_a = take(M * 8);
    w.keys_b = take(M * 8);
    w.ckeys_b = take(M * 4);
    w.cvals_b = take(M * 4);
    w.srcq = take(M * 4);
    w.flags = take(M * 4);
    w.pos = take(M * 4);
    const int bits = key_bits(N);
    size_t t1 = 0, t2 = 0, t3 = 0;
    size_t t1b = 0;
    (void)rocprim::radix_sort_keys(nullptr, t1, (uint64_t*)nullptr, (uint64_t*)nullptr, (size_t)M, 0, 64);
    (void)rocprim::radix_sort_keys(nullptr, t1b, (uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)M, 0, 32);
    t1 = std::max(t1, t1b);
    (void)rocprim::radix_sort_pairs<CscSortCfg>(nullptr, t2, (uint32_t*)nullptr, (uint32_t*)nullptr, (int32_t*)nullptr,
                                                (int32_t*)nullptr, (size_t)M, 0, bits);
    (void)rocprim::exclusive_scan(nullptr, t3, (int32_t*)nullptr, (int32_t*)nullptr, 0, (size_t)M,
                            rocprim::plus<int32_t>());
    w.temp_bytes = std::max(t1, std::max(t2, t3));
    w.temp = take(w.temp_bytes);
    w.total = off;
    return w;
}

int grid_for(int64_t n) {
    int64_t g = (n + BLK - 1) / BLK;
    if (g > 256 * 16) g = 256 * 16;
    return (int)(g < 1 ? 1 : g);
}

// Key build, key sort, de-duplication and CSR scatter with K-wide keys; writes the unsorted CSC
// keys/values (ckeys_a aliases the unsorted key buffer, free once the key sort is done).
template <typename K>
int csr_keys(const int64_t* edge_index, int64_t ld_ei, int64_t n_edges, const int64_t* edge_ptr,
             const int64_t* node_ptr, int32_t n_graphs, int64_t n_nodes, int64_t NL, int sort_bits, char* ws,
             const CsrWs& w, int32_t* rowptr, int32_t* col, uint32_t* ckeys_a, int32_t* cvals_a, int32_t* srcq,
             int32_t* flags, int32_t* pos, int64_t* nnz_out, int32_t* err_out, hipStream_t s) {
    const int64_t M = n_edges + n_nodes;
    K* keys_a = (K*)(ws + w.keys_a);
    K* keys_b = (K*)(ws + w.keys_b);
    void* temp = ws + w.temp;
    k_make_keys<K><<<grid_for(M), BLK, 0, s>>>(edge_index, ld_ei, n_edges, edge_ptr, node_ptr, n_graphs, n_nodes, NL,
                                               keys_a, err_out);
    TAGAN_CHECK_LAUNCH("csr_build.make_keys");
    size_t tb = w.temp_bytes;
    TAGAN_CHECK_HIP(rocprim::radix_sort_keys(temp, tb, keys_a, keys_b, (size_t)M, 0, sort_bits, s),
                    "csr_build radix_sort_keys");
    k_unique_flags<K><<<grid_for(M), BLK, 0, s>>>(keys_b, M, n_nodes, NL, flags);
    TAGAN_CHECK_LAUNCH("csr_build.unique_flags");
    tb = w.temp_bytes;
    TAGAN_CHECK_HIP(rocprim::exclusive_scan(temp, tb, flags, pos, 0, (size_t)M, rocprim::plus<int32_t>(), s),
                    "csr_build exclusive_scan");
    k_scatter_csr<K><<<grid_for(M), BLK, 0, s>>>(keys_b, flags, pos, M, n_nodes, NL, node_ptr, n_graphs, rowptr, col,
                                                 ckeys_a, cvals_a, srcq, nnz_out);
    TAGAN_CHECK_LAUNCH("csr_build.scatter_csr");
    return TAGAN_OK;
}

}  // namespace
}  // namespace tagan

extern "C" {

size_t tagan_csr_build_workspace(int64_t n_edges, int64_t n_nodes) {
    if (n_edges < 0 || n_nodes <= 0) return 0;
    return tagan::plan(n_edges, n_nodes).total;
}

int tagan_csr_build(const int64_t* edge_index, int64_t ld_ei, int64_t n_edges, const int64_t* edge_ptr,
                    const int64_t* node_ptr, int32_t n_graphs, int64_t n_nodes, int64_t max_graph_nodes,
                    int32_t* rowptr, int32_t* col,
                    int32_t* csc_ptr, int32_t* csc_row, int32_t* csc_eid, int64_t* nnz_out, int32_t* err_out,
                    void* workspace, size_t workspace_bytes, void* stream) {
    using namespace tagan;
    TAGAN_REQUIRE(n_nodes > 0 && n_nodes < (int64_t)INT32_MAX - 1, TAGAN_ERR_ARG,
                  "tagan_csr_build: n_nodes=%lld out of range", (long long)n_nodes);
    TAGAN_REQUIRE(n_edges >= 0 && (n_edges == 0 || (edge_index && ld_ei >= n_edges)), TAGAN_ERR_ARG,
                  "tagan_csr_build: bad edge_index (E=%lld ld=%lld)", (long long)n_edges, (long long)ld_ei);
    TAGAN_REQUIRE(n_edges + n_nodes < (int64_t)INT32_MAX, TAGAN_ERR_ARG, "tagan_csr_build: too many edges");
    TAGAN_REQUIRE(n_graphs >= 1 && edge_ptr && node_ptr, TAGAN_ERR_ARG, "tagan_csr_build: bad graph pointers");
    TAGAN_REQUIRE(rowptr && col && csc_ptr && csc_row && csc_eid && nnz_out && err_out, TAGAN_ERR_ARG,
                  "tagan_csr_build: null output");
    const CsrWs w = plan(n_edges, n_nodes);
    TAGAN_REQUIRE(workspace && workspace_bytes >= w.total, TAGAN_ERR_WORKSPACE,
                  "tagan_csr_build: workspace %zu < %zu", workspace_bytes, w.total);
    hipStream_t s = as_stream(stream);
    char* ws = (char*)workspace;
    uint32_t* ckeys_b = (uint32_t*)(ws + w.ckeys_b);
    int32_t* cvals_b = (int32_t*)(ws + w.cvals_b);
    int32_t* srcq = (int32_t*)(ws + w.srcq);
    int32_t* flags = (int32_t*)(ws + w.flags);
    int32_t* pos = (int32_t*)(ws + w.pos);
    void* temp = ws + w.temp;
    const int64_t M = n_edges + n_nodes;
    const int bits = key_bits(n_nodes);
    TAGAN_REQUIRE(max_graph_nodes <= n_nodes, TAGAN_ERR_ARG, "tagan_csr_build: max_graph_nodes > n_nodes");
    const int64_t NL = max_graph_nodes > 0 ? max_graph_nodes : n_nodes;   // local ids 0..NL-1
    const uint64_t sentinel = (uint64_t)n_nodes * (uint64_t)NL;
    int sort_bits = 0;
    while (sort_bits < 64 && (sentinel >> sort_bits) != 0) ++sort_bits;   // keys 0..sentinel

    TAGAN_CHECK_HIP(hipMemsetAsync(err_out, 0, sizeof(int32_t), s), "csr_build memset");
    uint32_t* ckeys_a = (uint32_t*)(ws + w.keys_a);   // unsorted CSC keys (the key buffer is free by then)
    int32_t* cvals_a = csc_row;   // staging only; overwritten by the final CSC scatter
    const int rc = sentinel <= 0xFFFFFFFFull
                       ? csr_keys<uint32_t>(edge_index, ld_ei, n_edges, edge_ptr, node_ptr, n_graphs, n_nodes, NL,
                                            sort_bits, ws, w, rowptr, col, ckeys_a, cvals_a, srcq, flags, pos,
                                            nnz_out, err_out, s)
                       : csr_keys<uint64_t>(edge_index, ld_ei, n_edges, edge_ptr, node_ptr, n_graphs, n_nodes, NL,
                                            sort_bits, ws, w, rowptr, col, ckeys_a, cvals_a, srcq, flags, pos,
                                            nnz_out, err_out, s);
    if (rc) return rc;
    size_t tb = 0;
    k_fill_tail<<<grid_for(M), BLK, 0, s>>>(ckeys_a, cvals_a, nnz_out, M, n_nodes);
    TAGAN_CHECK_LAUNCH("csr_build.fill_tail");
    tb = w.temp_bytes;
    TAGAN_CHECK_HIP(rocprim::radix_sort_pairs<CscSortCfg>(temp, tb, ckeys_a, ckeys_b, cvals_a, cvals_b, (size_t)M, 0,
                                                          bits, s),
                    "csr_build radix_sort_pairs");
    k_scatter_csc<<<grid_for(M), BLK, 0, s>>>(ckeys_b, cvals_b, srcq, nnz_out, n_nodes, csc_ptr, csc_row,
                                              csc_eid);
    TAGAN_CHECK_LAUNCH("csr_build.scatter_csc");
    return TAGAN_OK;
}

int tagan_csr_csc_pos(const int32_t* csc_eid, const int64_t* nnz, int64_t nnz_cap, int32_t* csr_cpos, void* stream) {
    using namespace tagan;
    TAGAN_REQUIRE(csc_eid && nnz && csr_cpos && nnz_cap > 0, TAGAN_ERR_ARG, "csr_csc_pos: bad argument");
    k_csc_pos<<<grid_for(nnz_cap), BLK, 0, as_stream(stream)>>>(csc_eid, nnz, csr_cpos);
    TAGAN_CHECK_LAUNCH("csr_csc_pos");
    return TAGAN_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------- chunked work lists
namespace tagan {
namespace {

// Per segment: {chunks, is_multi, partial slots}; ONE exclusive scan over the triple gives each
// segment's first chunk, its index among multi segments and its first partial slot.
struct Tri {
    int32_t a, b, c;
};
struct TriPlus {
    __host__ __device__ Tri operator()(const Tri& x, const Tri& y) const { return Tri{x.a + y.a, x.b + y.b, x.c + y.c}; }
};

__global__ void __launch_bounds__(BLK) k_chunk_count(const int32_t* __restrict__ ptr, int64_t n, int chunk,
                                                     Tri* __restrict__ cnt) {
    for (int64_t s = blockIdx.x * (int64_t)BLK + threadIdx.x; s < n; s += (int64_t)gridDim.x * BLK) {
        const int deg = ptr[s + 1] - ptr[s];
        const int c = deg <= chunk ? 1 : (deg + chunk - 1) / chunk;
        cnt[s] = Tri{c, c > 1 ? 1 : 0, c > 1 ? c : 0};
    }
}

__global__ void __launch_bounds__(BLK) k_chunk_fill(const int32_t* __restrict__ ptr, int64_t n, int chunk,
                                                    const Tri* __restrict__ cnt, const Tri* __restrict__ off,
                                                    int32_t* __restrict__ chunk_ptr, int32_t* __restrict__ seg,
                                                    int32_t* __restrict__ beg, int32_t* __restrict__ part,
                                                    int32_t* __restrict__ multi, int32_t* __restrict__ counts) {
    for (int64_t s = blockIdx.x * (int64_t)BLK + threadIdx.x; s < n; s += (int64_t)gridDim.x * BLK) {
        const int c = cnt[s].a, e0 = ptr[s];
        const Tri o = off[s];
        chunk_ptr[s] = o.a;
        for (int k = 0; k < c; ++k) {
            seg[o.a + k] = (int32_t)s;
            beg[o.a + k] = e0 + k * chunk;
            part[o.a + k] = c > 1 ? o.c + k : -1;
        }
        if (c > 1) multi[o.b] = (int32_t)s;
        if (s == n - 1) {
            chunk_ptr[n] = o.a + c;
            counts[0] = o.a + c;
            counts[1] = o.b + (c > 1);
            counts[2] = o.c + (c > 1 ? c : 0);
        }
    }
}

// One workgroup per window of 2^wbits consecutive segments (a contiguous chunk range): counting
// sort of the window's chunks by entry count, longest first, in LDS.  Positions inside a count
// bucket come from LDS atomics, so ties may run in any order; no result depends on the order.
constexpr int ORDER_BINS = 256;

__global__ void __launch_bounds__(BLK) k_chunk_order_window(const int32_t* __restrict__ ptr, int64_t n,
                                                            const int32_t* __restrict__ chunk_ptr,
                                                            const int32_t* __restrict__ seg,
                                                            const int32_t* __restrict__ beg, int chunk, int wbits,
                                                            int32_t* __restrict__ order) {
    __shared__ int hist[ORDER_BINS];
    __shared__ int base[ORDER_BINS];
    const int64_t s0 = (int64_t)blockIdx.x << wbits;
    const int64_t s1 = min(n, s0 + ((int64_t)1 << wbits));
    const int c0 = chunk_ptr[s0], c1 = chunk_ptr[s1];
    for (int i = threadIdx.x; i < ORDER_BINS; i += BLK) hist[i] = 0;
    __syncthreads();
    for (int c = c0 + threadIdx.x; c < c1; c += BLK) {
        const int cnt = min(chunk, ptr[seg[c] + 1] - beg[c]);
        atomicAdd(&hist[ORDER_BINS - 1 - cnt], 1);
    }
    __syncthreads();
    if (threadIdx.x < WAVE) {      // exclusive scan of the bins by one wave, 4 bins per lane
        const int l = threadIdx.x;
        int v[4], t = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) { v[k] = hist[4 * l + k]; t += v[k]; }
        int incl = t;
#pragma unroll
        for (int o = 1; o < WAVE; o <<= 1) {
            const int y = __shfl_up(incl, o, WAVE);
            if (l >= o) incl += y;
        }
        int run = incl - t;
#pragma unroll
        for (int k = 0; k < 4; ++k) { base[4 * l + k] = run; run += v[k]; }
    }
    __syncthreads();
    for (int c = c0 + threadIdx.x; c < c1; c += BLK) {
        const int cnt = min(chunk, ptr[seg[c] + 1] - beg[c]);
        order[c0 + atomicAdd(&base[ORDER_BINS - 1 - cnt], 1)] = c;
    }
}

}  // namespace
}  // namespace tagan

extern "C" {

int tagan_chunk_order(const int32_t* seg_ptr, int64_t n_segments, const int32_t* chunk_ptr,
                      const int32_t* chunk_seg, const int32_t* chunk_beg, int32_t chunk, int32_t window_bits,
                      int32_t* order, void* stream) {
    using namespace tagan;
    TAGAN_REQUIRE(n_segments > 0 && chunk > 0 && chunk < ORDER_BINS && window_bits >= 0 && window_bits < 31,
                  TAGAN_ERR_ARG, "tagan_chunk_order: n=%lld chunk=%d window_bits=%d", (long long)n_segments,
                  chunk, window_bits);
    TAGAN_REQUIRE(seg_ptr && chunk_ptr && chunk_seg && chunk_beg && order, TAGAN_ERR_ARG,
                  "tagan_chunk_order: null pointer");
    const int64_t windows = ((n_segments - 1) >> window_bits) + 1;
    TAGAN_REQUIRE(windows <= 0x7fffffff, TAGAN_ERR_ARG, "tagan_chunk_order: too many windows");
    hipStream_t s = as_stream(stream);
    k_chunk_order_window<<<(unsigned)windows, BLK, 0, s>>>(seg_ptr, n_segments, chunk_ptr, chunk_seg, chunk_beg,
                                                           chunk, window_bits, order);
    TAGAN_CHECK_LAUNCH("chunk_order");
    return TAGAN_OK;
}

int64_t tagan_chunk_capacity(int64_t n_segments, int64_t nnz_cap, int32_t chunk) {
    return chunk > 0 ? n_segments + nnz_cap / chunk + 1 : 0;
}

int64_t tagan_part_capacity(int64_t nnz_cap, int32_t chunk) {
    return chunk > 0 ? 2 * (nnz_cap / chunk) + 2 : 0;   // a multi segment with deg > chunk has <= 2*deg/chunk chunks
}

size_t tagan_graph_chunks_workspace(int64_t n) {
    using namespace tagan;
    if (n <= 0) return 0;
    size_t t = 0;
    (void)rocprim::exclusive_scan(nullptr, t, (Tri*)nullptr, (Tri*)nullptr, Tri{0, 0, 0}, (size_t)n, TriPlus());
    return 2 * align_up((size_t)n * sizeof(Tri), 256) + align_up(t, 256);
}

int tagan_graph_chunks(const int32_t* seg_ptr, int64_t n, int32_t chunk, int32_t* chunk_ptr, int32_t* chunk_seg,
                       int32_t* chunk_beg, int32_t* chunk_part, int32_t* multi_seg, int32_t* counts,
                       void* workspace, size_t workspace_bytes, void* stream) {
    using namespace tagan;
    TAGAN_REQUIRE(n > 0 && chunk > 0, TAGAN_ERR_ARG, "tagan_graph_chunks: n=%lld chunk=%d", (long long)n, chunk);
    TAGAN_REQUIRE(seg_ptr && chunk_ptr && chunk_seg && chunk_beg && chunk_part && multi_seg && counts,
                  TAGAN_ERR_ARG, "tagan_graph_chunks: null pointer");
    const size_t need = tagan_graph_chunks_workspace(n);
    TAGAN_REQUIRE(workspace && workspace_bytes >= need, TAGAN_ERR_WORKSPACE, "tagan_graph_chunks: workspace");
    hipStream_t s = as_stream(stream);
    char* ws = (char*)workspace;
    const size_t a = align_up((size_t)n * sizeof(Tri), 256);
    Tri* cnt = (Tri*)ws;
    Tri* off = (Tri*)(ws + a);
    void* temp = ws + 2 * a;
    size_t tb = need - 2 * a;
    k_chunk_count<<<grid_for(n), BLK, 0, s>>>(seg_ptr, n, chunk, cnt);
    TAGAN_CHECK_LAUNCH("graph_chunks.count");
    TAGAN_CHECK_HIP(rocprim::exclusive_scan(temp, tb, cnt, off, Tri{0, 0, 0}, (size_t)n, TriPlus(), s), "scan");
    k_chunk_fill<<<grid_for(n), BLK, 0, s>>>(seg_ptr, n, chunk, cnt, off, chunk_ptr, chunk_seg, chunk_beg,
                                             chunk_part, multi_seg, counts);
    TAGAN_CHECK_LAUNCH("graph_chunks.fill");
    return TAGAN_OK;
}

}  // extern "C"
