/*
 * tagan_hip.h — C-ABI of libtagan_hip.so, the MI355X (gfx950) hot path of TAGAN.
 *
 * The reference (MaLoskins/Temporal-Asymmetric-Graph-Attention-Network @ 2025-04-18)
 * is pure PyTorch; it has no FFI.  Each entry point below replaces the ATen op
 * sequence of one reference function (cited per function).  The Python host
 * package binds these with ctypes (INTEGRATION.md shows the stub).
 *
 * Conventions
 *   - Plain pointers + sizes, no torch/HIP types.  `stream` is a hipStream_t
 *     passed as void* (NULL = default stream).  All launches are asynchronous.
 *   - The library never allocates or frees device memory.  Callers pass outputs
 *     and workspaces (sized by the *_workspace() queries).
 *   - Return 0 (TAGAN_OK) or a negative tagan_status; tagan_last_error() gives a
 *     thread-local message for the last failure on the calling thread.
 *   - Device arrays are row-major.  "ld" arguments are row strides in elements.
 *   - dtype: TAGAN_F32 (fp32 storage, fp32 math) everywhere; TAGAN_BF16 (bf16 storage of the
 *     activation tensors, fp32 math) where an entry point says so.  LSE, partials, LayerNorm
 *     statistics and parameter gradients are fp32 in both.  Other values -> TAGAN_ERR_UNSUPPORTED.
 *   - Dropout masks are counter-based: keep(u) with u = tagan_uniform(seed, stream, counter)
 *     (stream/counter layouts documented per kernel), so tests can regenerate them.
 */
#ifndef TAGAN_HIP_H
#define TAGAN_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum tagan_status {
    TAGAN_OK = 0,
    TAGAN_ERR_ARG = -1,          /* bad pointer / size / stride */
    TAGAN_ERR_UNSUPPORTED = -2,  /* dtype / metric / shape not implemented */
    TAGAN_ERR_LAUNCH = -3,       /* hipGetLastError after launch */
    TAGAN_ERR_WORKSPACE = -4     /* workspace too small */
};

enum tagan_dtype { TAGAN_F32 = 0, TAGAN_BF16 = 1 };

/* Distance metrics of DistanceMetric.get_metric (geometric_attention.py:196-225).
 * Scores are similarities: distance metrics are negated as in
 * _get_attention_weights (geometric_attention.py:378-401). */
enum tagan_metric {
    TAGAN_METRIC_EUCLIDEAN = 0,
    TAGAN_METRIC_SQUARED_EUCLIDEAN = 1,
    TAGAN_METRIC_MANHATTAN = 2,
    TAGAN_METRIC_COSINE_SIMILARITY = 3,
    TAGAN_METRIC_COSINE_DISTANCE = 4,
    TAGAN_METRIC_DOT_PRODUCT = 5,
    TAGAN_METRIC_SCALED_DOT_PRODUCT = 6,
    TAGAN_METRIC_GAUSSIAN_KERNEL = 7,   /* sigma = metric_param[h] or 1.0 if NULL */
    TAGAN_METRIC_RBF_KERNEL = 8         /* gamma = metric_param[h] or 1.0 if NULL */
};

const char* tagan_last_error(void);
/* 1 when the library is the bounds-check build (`make debug`: device checks on gather indices, chunk ranges and
 * partial slots; a failing check skips its access and the next launch check returns TAGAN_ERR_LAUNCH with the
 * source line in tagan_last_error(); eager launches only), 0 for the shipped build. */
int tagan_debug_build(void);
int tagan_version(void);
int tagan_device_arch(char* buf, int len);   /* e.g. "gfx950"; needs a device */

/* Counter-based uniform in [0,1) used by every dropout mask: a 32-bit key mixed from
 * (seed, stream) by four lowbias32 rounds, then u = lowbias32(counter ^ key) >> 8 / 2^24. */
float tagan_uniform(uint64_t seed, uint64_t stream, uint32_t counter);

/* HIP-graph replay of a training step.  tagan_set_seed_counter registers a device uint64 counter (NULL to
 * clear; process-wide, read by the launches that follow): every kernel that draws a dropout mask then uses
 * seed ^ (counter · 0x9E3779B97F4A7C15) with the counter's value AT RUN TIME, so the seeds baked into a captured
 * graph still give fresh masks per replay once the graph advances the counter with tagan_seed_counter_step
 * (one tiny launch, capturable).  With no counter registered every seed is used as passed. */
void tagan_set_seed_counter(const uint64_t* counter);
int tagan_seed_counter_step(uint64_t* counter, void* stream);

/* ---------------------------------------------------------------------------
 * Snapshot CSR builder.  Replaces graph_attention.py:96-105
 *   adj = zeros(N,N); adj[edge_index[0], edge_index[1]] = 1; adj += eye(N)
 * for a BATCH of G snapshots laid out block-diagonally: snapshot g owns global
 * nodes [node_ptr[g], node_ptr[g+1]) and edges [edge_ptr[g], edge_ptr[g+1]) of
 * edge_index ([2, ld_ei] int64, local indices; negative indices wrap like torch
 * indexing).  Output = the set {(src,dst)} ∪ {(i,i)} (duplicates collapsed):
 *   CSR by src (query row):  rowptr[n_nodes+1], col[nnz]
 *   CSC by dst:               csc_ptr[n_nodes+1], csc_row[nnz], csc_eid[nnz]
 *                             (csc_eid = CSR position of the same pair)
 * Capacity of col/csc_* must be >= n_edges + n_nodes.  *nnz_out and *err_out
 * are device int64/int32 scalars; *err_out != 0 if any index was out of range
 * (those edges are dropped; the reference raises IndexError).
 * max_graph_nodes = the largest snapshot's node count (<= 0: n_nodes); it sets
 * the width of the local-id field of the sort keys.  n_nodes < 2^31.
 * csr_cpos (nullable, capacity as col): the CSC position of each CSR entry (the
 * inverse of csc_eid), written by the same pass when asked for (a random scatter:
 * the attention backward does not need it).  Kernel launches only (no library
 * sort, no memset nodes): safe to capture in a HIP graph and to replay with other
 * work in between.
 * ------------------------------------------------------------------------- */
size_t tagan_csr_build_workspace(int64_t n_edges, int64_t n_nodes);
int tagan_csr_build(const int64_t* edge_index, int64_t ld_ei, int64_t n_edges,
                    const int64_t* edge_ptr, const int64_t* node_ptr, int32_t n_graphs,
                    int64_t n_nodes, int64_t max_graph_nodes,
                    int32_t* rowptr, int32_t* col,
                    int32_t* csc_ptr, int32_t* csc_row, int32_t* csc_eid,
                    int64_t* nnz_out, int32_t* err_out, int32_t* csr_cpos,
                    void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Work decomposition for skewed (power-law) graphs: every CSR row / CSC column
 * ("segment") is split into chunks of at most `chunk` entries.  A segment
 * with more than one chunk is "multi"; its chunks write partial results to a
 * workspace slot chunk_part[c] (>= 0; -1 for single-chunk segments) and a merge
 * pass combines them in chunk order (deterministic).
 *   chunk_ptr[n+1]: chunks of segment s are [chunk_ptr[s], chunk_ptr[s+1])
 *   chunk_seg[c], chunk_beg[c]: segment and first entry of chunk c
 *   multi_seg[k]: k-th multi segment;  counts = {n_chunks, n_multi, n_parts} (device int32[3])
 * Capacities: chunk arrays >= tagan_chunk_capacity(n, nnz_cap, chunk),
 * multi_seg / parts >= tagan_part_capacity(nnz_cap, chunk).
 * ------------------------------------------------------------------------- */
int64_t tagan_chunk_capacity(int64_t n_segments, int64_t nnz_cap, int32_t chunk);
int64_t tagan_part_capacity(int64_t nnz_cap, int32_t chunk);
size_t tagan_graph_chunks_workspace(int64_t n_segments);
int tagan_graph_chunks(const int32_t* seg_ptr, int64_t n_segments, int32_t chunk,
                       int32_t* chunk_ptr, int32_t* chunk_seg, int32_t* chunk_beg, int32_t* chunk_part,
                       int32_t* multi_seg, int32_t* counts,
                       void* workspace, size_t workspace_bytes, void* stream);

/* Processing order of the chunks (a permutation of [0, n_chunks)): chunks stay
 * grouped by window of 2^window_bits consecutive segments (keeps the gathers of
 * one window of rows / snapshots together in the caches) and, inside a window,
 * run longest first (counting sort, one workgroup per window).  The edge
 * kernels run up to 64/lanes-per-chunk chunks side by side in one wave and
 * loop to the longest of them: on a power-law graph consecutive chunks differ
 * wildly in length (C2: 47 % of the lane slots busy in row order, 92 % in this
 * order).  Ties run in any order and no result depends on the order (each
 * chunk's output and partial slot are fixed by its index), so every kernel
 * stays bitwise deterministic.  order[] needs n_chunks (<= chunk capacity)
 * entries; chunk < 256.  No workspace. */
int tagan_chunk_order(const int32_t* seg_ptr, int64_t n_segments, const int32_t* chunk_ptr,
                      const int32_t* chunk_seg, const int32_t* chunk_beg, int32_t chunk, int32_t window_bits,
                      int32_t* order, void* stream);

/* A built snapshot-batch graph (all device pointers).  Filled by the host from
 * tagan_csr_build + two tagan_graph_chunks calls (rows over the CSR, columns
 * over the CSC). */
typedef struct tagan_graph {
    int64_t n_nodes;
    const int32_t* rowptr;      /* [n+1] */
    const int32_t* col;         /* [nnz] */
    const int32_t* csc_ptr;     /* [n+1] */
    const int32_t* csc_row;     /* [nnz] */
    const int32_t* csc_eid;     /* [nnz] CSR position of each CSC entry */
    int32_t chunk;              /* max entries per chunk */
    int64_t chunk_cap;          /* capacity of the chunk arrays (launch bound) */
    int64_t part_cap;           /* capacity of partial slots / multi segments */
    const int32_t* row_chunk_ptr;
    const int32_t* row_chunk_seg;
    const int32_t* row_chunk_beg;
    const int32_t* row_chunk_part;
    const int32_t* row_multi;
    const int32_t* row_counts;  /* {n_chunks, n_multi, n_parts} */
    const int32_t* col_chunk_ptr;
    const int32_t* col_chunk_seg;
    const int32_t* col_chunk_beg;
    const int32_t* col_chunk_part;
    const int32_t* col_multi;
    const int32_t* col_counts;
    const int32_t* row_chunk_order;  /* [chunk_cap] processing order (tagan_chunk_order); NULL = identity */
    const int32_t* col_chunk_order;
    int64_t nnz_cap;            /* capacity of col / csc_row / csc_eid (>= nnz).  With nnz_cap > 0 the backward
                                   may run column-first (see tagan_geo_attn_bwd); otherwise row-first */
} tagan_graph;

/* csr_cpos[csc_eid[p]] = p for p < *nnz: the inverse of csc_eid (the CSC position of each CSR entry). */
int tagan_csr_csc_pos(const int32_t* csc_eid, const int64_t* nnz, int64_t nnz_cap, int32_t* csr_cpos, void* stream);

/* ---------------------------------------------------------------------------
 * Geometric (edge-softmax) attention.  Replaces geometric_attention.py:332-516
 * (_get_attention_weights: metric scores -> masked_fill(-inf) -> softmax ->
 * attn_dropout) and :579-583 (context = A·V) for query rows = CSR rows.
 *   q,k,v: [n_nodes, heads*head_dim] with row stride ld_qkv (may alias one
 *          fused [n,3H] buffer).  out: [n_nodes, H] (ld = H).
 *   lse:   [n_nodes, heads] log-sum-exp of the row's scores (saved for bwd).
 *   edge_alpha (optional): [nnz, heads] post-dropout attention weights.
 * Dropout layout: stream = head h, counter = edge e (CSR position).
 * A row with no entries yields NaN (softmax over all -inf, as the reference).
 * ------------------------------------------------------------------------- */
size_t tagan_geo_attn_fwd_workspace(const tagan_graph* g, int32_t heads, int32_t head_dim);
int tagan_geo_attn_fwd(int dtype, int metric, const tagan_graph* g, int32_t heads, int32_t head_dim,
                       const void* q, const void* k, const void* v, int64_t ld_qkv,
                       const float* metric_param, float p_drop, uint64_t seed,
                       void* out, float* lse, float* edge_alpha,
                       void* workspace, size_t workspace_bytes, void* stream);

/* Backward of tagan_geo_attn_fwd.  Atomic-free and deterministic.  With g->nnz_cap > 0
 * (fast-path shapes) on graphs whose K|V rows exceed the caches (n_nodes·H·8 > 512 MB): node pass (delta = rowsum(dO∘O) per head) -> column pass over CSC (dk, dv; dS per edge
 * into the workspace at its CSR position csc_eid) -> row pass over CSR (dq from dS[e], gathering K only).  Otherwise
 * (or with TAGAN_GEO_BWD_ORDER=row): row pass over CSR (dq, delta) then column pass over CSC (dk, dv).  Both
 * orders give the same bits.
 * dq/dk/dv: [n_nodes, H] with row stride ld_dqkv (may alias one [n,3H] buffer).
 * dmetric_param: [heads] (gaussian/rbf learnable parameter) or NULL. */
size_t tagan_geo_attn_bwd_workspace(const tagan_graph* g, int32_t heads, int32_t head_dim);
/* Process-wide backward order: 0 row-first, 1 column-first (where the graph allows it), 2 by graph size (the
 * default; env TAGAN_GEO_BWD_ORDER=row|col sets 0|1 at load).  Returns the previous mode, or TAGAN_ERR_ARG.
 * Change it only between a workspace query and the matching call's completion on no stream. */
int tagan_geo_set_bwd_order(int32_t mode);
int tagan_geo_attn_bwd(int dtype, int metric, const tagan_graph* g, int32_t heads, int32_t head_dim,
                       const void* q, const void* k, const void* v, int64_t ld_qkv,
                       const float* metric_param, float p_drop, uint64_t seed,
                       const void* out, const float* lse, const void* dout,
                       void* dq, void* dk, void* dv, int64_t ld_dqkv,
                       float* dmetric_param, void* workspace, size_t workspace_bytes,
                       void* stream);

/* ---------------------------------------------------------------------------
 * Per-row temporal attention.  Replaces temporal_attention.py:1006-1183
 * (QKᵀ/√d + relative-position bias + asymmetric-kernel bias [+ dense bias]
 * -> masks -> softmax -> attn_dropout -> A·V) for `rows` independent rows
 * (nodes) of T snapshots each.
 *   q,k,v: element (row r, time t, feature f) at ptr[r*s_row + t*s_t + f]
 *   bias_table (optional): [heads, 2T-1]; entry [h][i-j+T-1] added to score(i,j).
 *   bias_dense (optional): [*, heads, T, T] fp32, row stride bias_bstride (0 = shared).
 *   mask (optional): uint8 keep-mask, element (r,h,i,j) at
 *        mask[r*mask_bstride + h*mask_hstride + i*T + j]; causal != 0 adds j<=i.
 *   out: element (r,t,f) at out[r*o_row + t*o_t + f];  lse: [rows, heads, T].
 *   attn (optional): [rows, heads, T, T] post-dropout weights.
 * Dropout layout: key = the mixed (seed, stream = r*heads + h), counter c = i*T + j; one
 * lowbias32((c >> 1) ^ key) decides the pair {c & ~1, c | 1}: bits 0-15 the even counter, bits 16-31
 * the odd one, kept iff that half >= ceil(p * 65536) (drop probability within 2^-16 of p), kept
 * weights scaled by 1 / (1 - p).
 * ------------------------------------------------------------------------- */
int tagan_temporal_attn_fwd(int dtype, int64_t rows, int32_t T, int32_t heads, int32_t head_dim,
                            const void* q, const void* k, const void* v, int64_t s_row, int64_t s_t,
                            const float* bias_table, const float* bias_dense, int64_t bias_bstride,
                            const uint8_t* mask, int64_t mask_bstride, int64_t mask_hstride, int causal,
                            float p_drop, uint64_t seed,
                            void* out, int64_t o_row, int64_t o_t,
                            float* lse, float* attn, void* stream);

/* Dropout keep-bit cache (the matrix-core path at T = 128, head_dim 16/32, no mask, causal or dense bias,
 * p_drop > 0; at smaller T it measured no gain): the forward can store every element's keep decision as one bit, and the
 * backward reads them instead of re-evaluating the counter hash (the same bits: the hash decides them once).
 * tagan_temporal_attn_keep_bytes returns the bytes such a forward writes, 0 where no path uses the cache.
 * tagan_temporal_attn_fwd_keep = tagan_temporal_attn_fwd + keep (device, keep_bytes) and *keep_written (host,
 * may be NULL): 1 iff this call wrote the bits.  Pass keep to tagan_temporal_attn_bwd_keep ONLY when the
 * matching forward reported keep_written = 1 (same shapes, strides, seed and kernel-selection environment);
 * otherwise pass NULL, which is tagan_temporal_attn_bwd. */
size_t tagan_temporal_attn_keep_bytes(int64_t rows, int32_t T, int32_t heads, int32_t head_dim, int causal,
                                      int has_mask, int has_bias_dense, float p_drop);
int tagan_temporal_attn_fwd_keep(int dtype, int64_t rows, int32_t T, int32_t heads, int32_t head_dim,
                                 const void* q, const void* k, const void* v, int64_t s_row, int64_t s_t,
                                 const float* bias_table, const float* bias_dense, int64_t bias_bstride,
                                 const uint8_t* mask, int64_t mask_bstride, int64_t mask_hstride, int causal,
                                 float p_drop, uint64_t seed,
                                 void* out, int64_t o_row, int64_t o_t,
                                 float* lse, float* attn, uint32_t* keep, size_t keep_bytes, int32_t* keep_written,
                                 void* stream);

/* Backward.  dbias_table: [heads, 2T-1] (reduced over rows, deterministic) or NULL.
 * dbias_dense: [rows, heads, T, T] per-row score gradients (caller reduces a
 * shared bias) or NULL.  dq/dk/dv element (r,t,f) at d*[r*d_row + t*d_t + f].
 * dsum_qkv (optional): [3 * heads * head_dim] = column sums of dq | dk | dv over all rows and
 * steps (the QKV projection's bias gradient), summed inside the matrix-core kernel in a fixed
 * order; only that path (T <= 32, head_dim 16 or 32, 16-B aligned strides) provides it — otherwise
 * the call returns TAGAN_ERR_UNSUPPORTED before launching anything. */
size_t tagan_temporal_attn_bwd_workspace(int64_t rows, int32_t T, int32_t heads, int32_t head_dim);
int tagan_temporal_attn_bwd(int dtype, int64_t rows, int32_t T, int32_t heads, int32_t head_dim,
                            const void* q, const void* k, const void* v, int64_t s_row, int64_t s_t,
                            const float* bias_table, const float* bias_dense, int64_t bias_bstride,
                            const uint8_t* mask, int64_t mask_bstride, int64_t mask_hstride, int causal,
                            float p_drop, uint64_t seed,
                            const void* out, int64_t o_row, int64_t o_t, const float* lse,
                            const void* dout, int64_t do_row, int64_t do_t,
                            void* dq, void* dk, void* dv, int64_t d_row, int64_t d_t,
                            float* dbias_table, float* dbias_dense, float* dsum_qkv,
                            void* workspace, size_t workspace_bytes, void* stream);
int tagan_temporal_attn_bwd_keep(int dtype, int64_t rows, int32_t T, int32_t heads, int32_t head_dim,
                                 const void* q, const void* k, const void* v, int64_t s_row, int64_t s_t,
                                 const float* bias_table, const float* bias_dense, int64_t bias_bstride,
                                 const uint8_t* mask, int64_t mask_bstride, int64_t mask_hstride, int causal,
                                 float p_drop, uint64_t seed,
                                 const void* out, int64_t o_row, int64_t o_t, const float* lse,
                                 const void* dout, int64_t do_row, int64_t do_t,
                                 void* dq, void* dk, void* dv, int64_t d_row, int64_t d_t,
                                 float* dbias_table, float* dbias_dense, float* dsum_qkv,
                                 const uint32_t* keep, size_t keep_bytes,
                                 void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Row LayerNorm with fused residual + dropout.  Replaces the ATen chain
 * output_dropout(proj) + identity -> layer_norm2 (geometric_attention.py:586-596,
 * temporal_attention.py:1190-1200) and plain layer_norm1 (b = NULL, p_drop = 0).
 *   s = dropout(a + a_bias; p_drop, seed) + b     (element (r,c): stream r, counter c)
 * a_bias (optional, [H]) is the producing projection's bias, added here instead of in the GEMM
 * epilogue (its gradient is dsum_a of the backward).
 *   y = (s - mean) / sqrt(var + eps) * gamma + beta       (biased var, as torch)
 * dtype = storage of y (TAGAN_BF16: y feeds a bf16 GEMM); a, b, s, statistics fp32.
 * s_out (optional) keeps s for the backward pass; mean/rstd: [M].  y has row stride
 * ldy (0 = H).  With ldy >= H + 4, columns H..H+3 of every y row are written as
 * (1, 0, 0, 0): the next projection then takes its bias as an extra weight column
 * (one GEMM over K = H + 4 without a bias epilogue).
 * Supported H: tagan_layernorm_supported(H) (32, 64, 128, 256, 512).
 * ------------------------------------------------------------------------- */
int tagan_layernorm_supported(int32_t H);
int tagan_add_layernorm_fwd(int dtype, int64_t M, int32_t H, const float* a, const float* a_bias,
                            const float* b, float p_drop, uint64_t seed, const float* gamma, const float* beta,
                            float eps, float* s_out, float* y, int64_t ldy, float* mean, float* rstd,
                            void* stream);
/* Layer 0 of the geometric stack with the skip branch of model.py:258-262 fused
 * into its closing LayerNorm: y = LN(dropout(a) + b) + LN_s(b) (b = the layer
 * input), one pass instead of LN, LN_s and an add.  fp32 only.  mean_s/rstd_s
 * [M] are LN_s's statistics, for its backward (tagan_layernorm_bwd with s = b,
 * dres = the LN's own ds, so both gradients of b arrive summed). */
int tagan_add_layernorm_skip_fwd(int64_t M, int32_t H, const float* a, const float* a_bias, const float* b,
                                 float p_drop,
                                 uint64_t seed, const float* gamma, const float* beta, float eps,
                                 const float* gamma_s, const float* beta_s, float eps_s, float* s_out,
                                 float* y, float* mean, float* rstd, float* mean_s, float* rstd_s,
                                 void* stream);
/* Backward: ds = dL/ds (+ dres when given: the gradient of the LN input's other
 * consumer, fused instead of a separate add), da = dL/ds masked/scaled by the same
 * dropout (the projection branch's gradient), dgamma/dbeta [H], dsum_a [H] = column
 * sums of da (the projection's bias gradient); block partials summed in block order.
 * dtype = storage of da (TAGAN_BF16: da feeds a bf16 GEMM); everything else fp32.
 * Any of dres/ds/da/dgamma/dbeta/dsum_a may be NULL. */
size_t tagan_layernorm_bwd_workspace(int64_t M, int32_t H);
int tagan_layernorm_bwd(int dtype, int64_t M, int32_t H, const float* s, const float* mean,
                        const float* rstd, const float* gamma, const float* dy, const float* dres,
                        float p_drop, uint64_t seed, float* ds, float* da, float* dgamma, float* dbeta,
                        float* dsum_a, void* workspace, size_t workspace_bytes, void* stream);
/* The backward of the skip form y = LN(s) + LN_s(b) (model.py:258-262) in one pass (H = 128 or 256): ds = dL/ds of LN plus
 * LN_s's input gradient (the residual gradient of the block input b), da = dL/ds of LN masked / scaled by the
 * dropout, dgamma/dbeta/dsum_a as tagan_layernorm_bwd, dgamma_s/dbeta_s of LN_s; equal, to fp32 rounding (the same
 * dropout decisions), to tagan_layernorm_bwd on (s, LN) followed by tagan_layernorm_bwd on (b, LN_s) with that ds
 * as dres. */
size_t tagan_layernorm_skip_bwd_workspace(int64_t M, int32_t H);
int tagan_layernorm_skip_bwd(int dtype, int64_t M, int32_t H, const float* s, const float* mean, const float* rstd,
                             const float* gamma, const float* b, const float* mean_s, const float* rstd_s,
                             const float* gamma_s, const float* dy, float p_drop, uint64_t seed, float* ds, float* da,
                             float* dgamma, float* dbeta, float* dsum_a, float* dgamma_s, float* dbeta_s,
                             void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Streaming projection GEMMs on the bf16 matrix cores (csrc/stream_gemm.hip).  Replace the q/k/v and out Linears
 * of every attention block and their backward (geometric_attention.py:541-596, temporal_attention.py:985-1200:
 * the nn.Linear forwards, input gradients and weight / bias gradients autograd derives for them).
 * planes = 3: fp32 operands, each split into three bf16 planes (x = x0 + x1 + x2, RN), six plane products kept
 *             (terms >= 2^-16 relative), fp32 accumulate: fp32-GEMM accuracy;  planes = 1: bf16 operands.
 * tagan_sgemm_wprep: B[n][k] = kmajor ? w[k*ldw + n] : w[n*ldw + k] (fp32, N % 16 == 0, K % 32 == 0) ->
 *   wp, N*K*planes bf16 in MFMA fragment order (the weight operand of tagan_sgemm_nt).
 * tagan_sgemm_nt:  c[M, N] = a[M, K] · Bᵀ (+ bias[N], fp32, may be NULL); a / c storage TAGAN_F32 or TAGAN_BF16
 *   (bf16 a needs planes = 1); rows 16-byte aligned.  Shapes: tagan_sgemm_supported.
 * tagan_sgemm_tn:  dw[n*lddw + k] = Σ_m dy[m][n]·x[m][k] and db[n] = Σ_m dy[m][n] (either output may be NULL),
 *   dy [M, N], x [M, K] of one storage dtype; workspace tagan_sgemm_tn_workspace bytes; fixed-order reduction
 *   (bitwise reproducible).  Shapes: tagan_sgemm_tn_supported.
 * ------------------------------------------------------------------------- */
int tagan_sgemm_supported(int32_t N, int32_t K, int32_t planes, int32_t a_dtype, int32_t c_dtype);
int tagan_sgemm_tn_supported(int32_t N, int32_t K, int32_t planes, int32_t dtype);
int tagan_sgemm_wprep(int32_t N, int32_t K, const float* w, int64_t ldw, int32_t kmajor, int32_t planes, void* wp,
                      void* stream);
/* tagan_sgemm_wprep_block: an attention block's four weight preparations in one launch -- wq_nt = wprep(w_qkv [3H, H],
 * kmajor 0), wo_nt = wprep(w_o [H, H], 0), wo_km = wprep(w_o, 1), wq_km = wprep(w_qkv, 1) -- each bitwise equal to
 * the tagan_sgemm_wprep call it stands for. */
int tagan_sgemm_wprep_block(int32_t H, const float* w_qkv, int64_t ld_qkv, const float* w_o, int64_t ld_o,
                            int32_t planes, void* wq_nt, void* wo_nt, void* wo_km, void* wq_km, void* stream);
int tagan_sgemm_nt(int32_t a_dtype, int32_t c_dtype, int64_t M, int32_t N, int32_t K, const void* a, int64_t lda,
                   const void* wp, int32_t planes, const float* bias, void* c, int64_t ldc, void* stream);
size_t tagan_sgemm_tn_workspace(int64_t M, int32_t N, int32_t K);
int tagan_sgemm_tn(int32_t dtype, int64_t M, int32_t N, int32_t K, const void* dy, int64_t ldy, const void* x,
                   int64_t ldx, int32_t planes, float* dw, int64_t lddw, float* db, void* workspace,
                   size_t workspace_bytes, void* stream);

/* LayerNorm-fused forms of the same kernels (H = 128; each replaces one standalone k_ln_fwd / k_ln_bwd pass of an
 * attention block: geometric_attention.py:541-542 / 586-596, temporal_attention.py:985-986 / 1190-1200).
 * tagan_sgemm_ln_supported: op 1 = tagan_sgemm_nt_ln_in + tagan_sgemm_tn_ln, 2 = tagan_sgemm_nt_ln_out,
 *   3 = tagan_sgemm_nt_ln_bwd exist for (H, planes, activation storage act_dtype).
 * tagan_sgemm_nt_ln_in:  c = LN(x)·Bᵀ + bias, LN(x) = (x - mean) rstd ln_g + ln_b computed in the GEMM's prologue
 *   (x fp32 [M, K = H]); the row statistics go to mean / rstd [M]; LN(x) itself is not stored.
 * tagan_sgemm_tn_ln:     the weight gradient dyᵀ·LN(x) (+ Σ dy) with LN(x) recomputed from x and the forward's
 *   statistics, bitwise as the prologue made it (x fp32; dy in dtype).
 * tagan_sgemm_nt_ln_out: s = dropout(a·Bᵀ + bias) + res -> s_out; y = LN(s) (ln_g, ln_b, eps) [+ LN_s(res) when
 *   gs / bs are given] -> y; statistics -> mean / rstd [/ mean_s / rstd_s] (res, s_out, y fp32 [M, H]).
 *   The dropout mask is tagan_add_layernorm_fwd's (stream = row, counter = column).
 * tagan_sgemm_nt_ln_bwd: dh = a·Bᵀ [M, H] (a = dqkv [M, K]) and the LayerNorm backward in the epilogue:
 *   dx = rstd (g dh - mean(g dh x̂) x̂ - mean(g dh)) + dres (dres may be NULL), dgamma = Σ dh x̂, dbeta = Σ dh
 *   (fixed-order partial sums: bitwise reproducible); workspace tagan_sgemm_nt_ln_bwd_workspace bytes; M > 0. */
int tagan_sgemm_ln_supported(int32_t H, int32_t planes, int32_t act_dtype, int32_t op);
int tagan_sgemm_nt_ln_in(int32_t c_dtype, int64_t M, int32_t N, int32_t K, const float* x, int64_t ldx,
                         const float* ln_g, const float* ln_b, float eps, const void* wp, int32_t planes,
                         const float* bias, void* c, int64_t ldc, float* mean, float* rstd, void* stream);
int tagan_sgemm_tn_ln(int32_t dtype, int64_t M, int32_t N, int32_t K, const void* dy, int64_t ldy, const float* x,
                      int64_t ldx, const float* ln_g, const float* ln_b, const float* mean, const float* rstd,
                      int32_t planes, float* dw, int64_t lddw, float* db, void* workspace, size_t workspace_bytes,
                      void* stream);
int tagan_sgemm_nt_ln_out(int32_t a_dtype, int64_t M, int32_t H, const void* a, int64_t lda, const void* wp,
                          int32_t planes, const float* bias, const float* res, float p_drop, uint64_t seed,
                          const float* ln_g, const float* ln_b, float eps, const float* gs, const float* bs,
                          float eps_s, float* s_out, float* y, float* mean, float* rstd, float* mean_s,
                          float* rstd_s, void* stream);
size_t tagan_sgemm_nt_ln_bwd_workspace(int64_t M, int32_t H, int32_t K);
int tagan_sgemm_nt_ln_bwd(int32_t a_dtype, int64_t M, int32_t H, int32_t K, const void* a, int64_t lda,
                          const void* wp, int32_t planes, const float* x, const float* mean, const float* rstd,
                          const float* gamma, const float* dres, float* dx, float* dgamma, float* dbeta,
                          void* workspace, size_t workspace_bytes, void* stream);

/* tagan_ln2_bwd_out: the start of an attention block's backward in one pass over the rows (H = 128; H = 256 with
 * planes = 1, as two column groups over the same rows):
 *   LN2 backward of y = LN(s) [+ LN_s(xs)]:  ds = rstd (g dy - mean(g dy x̂) x̂ - mean(g dy)) [+ LN_s's input gradient]
 *     -> dres [M, H] fp32; do = dropout(ds) with the forward's mask (p_drop, seed; stream = row, counter = column);
 *     dgamma, dbeta [, dgamma_s, dbeta_s] = column sums;
 *   the out projection's gradients from do without storing it: dc = do·W_o [M, H] (c's storage dtype), dw_o = doᵀ·c
 *     [H, H] and db_o = Σ do [H] (fp32);
 *   wp_km = tagan_sgemm_wprep(w_o, kmajor = 1, planes); act_dtype = storage of c and dc (TAGAN_BF16 needs planes = 1);
 *   xs == NULL: no skip LayerNorm.  Fixed-order partial sums (bitwise reproducible); workspace
 *   tagan_ln2_bwd_out_workspace bytes; M > 0.  Replaces tagan_layernorm_bwd + tagan_sgemm_nt + tagan_sgemm_tn of
 *   geometric_attention.py:586-596 / temporal_attention.py:1190-1200 (backward). */
int tagan_ln2_bwd_out_supported(int32_t H, int32_t planes, int32_t act_dtype);
size_t tagan_ln2_bwd_out_workspace(int64_t M, int32_t H, int32_t skip);
int tagan_ln2_bwd_out(int32_t act_dtype, int32_t planes, int64_t M, int32_t H, const float* dy, const float* s,
                      const float* mean, const float* rstd, const float* gamma, float p_drop, uint64_t seed,
                      const float* xs, const float* mean_s, const float* rstd_s, const float* gamma_s, const void* c,
                      const void* wp_km, float* dres, void* dc, float* dw_o, float* db_o, float* dgamma, float* dbeta,
                      float* dgamma_s, float* dbeta_s, void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Fused classification head + loss (csrc/head.hip).  Replaces model.py:377-459 after the pooling:
 * graph_features [B, T, H] (row 0 = x0 [T, H], rows 1..B-1 zero, model.py:382-394) ->
 * attention pooling over T (classification.py:912-925: s_t = w2·tanh(W1 x_t + b1), softmax over T,
 * Σ_t a_t x_t) -> Linear(Wc1, bc1) -> LayerNorm(ln_w, ln_b, eps) -> ReLU -> Dropout(p_drop; stream =
 * batch row, counter = feature) -> Linear(Wc2, bc2) = logits [B, C]; preds = sigmoid (C = 1) or
 * softmax; loss_kind 1 = BCE-with-logits mean over B·C (labels [B·C]), 2 = cross entropy mean over B
 * (labels [B] class indices stored as float), 0 = none.  saved: tagan_head_saved_floats(B, T, H) floats
 * kept for the backward.  One workgroup per call.  Backward: any of g_loss [1] / g_logits [B, C] /
 * g_preds [B, C] (the incoming gradients) may be NULL; writes dx0 [T, H] and every parameter gradient.
 * Supported: tagan_head_supported(T, H, C) (H <= 256, H % 4 == 0, T <= 128, C <= 16, T·H <= 8192).
 * x0, W1 and Wc1 must be 16-byte aligned (read as float4 runs; TAGAN_ERR_ARG before any launch otherwise).
 * ------------------------------------------------------------------------- */
int tagan_head_supported(int32_t T, int32_t H, int32_t C);
size_t tagan_head_saved_floats(int32_t B, int32_t T, int32_t H);
int tagan_head_fwd(int32_t B, int32_t T, int32_t H, int32_t C, const float* x0, const float* W1, const float* b1,
                   const float* w2, const float* Wc1, const float* bc1, const float* ln_w, const float* ln_b,
                   float eps, const float* Wc2, const float* bc2, float p_drop, uint64_t seed, const float* labels,
                   int loss_kind, float* logits, float* preds, float* loss, float* saved, void* stream);
int tagan_head_bwd(int32_t B, int32_t T, int32_t H, int32_t C, const float* x0, const float* W1, const float* w2,
                   const float* Wc1, const float* ln_w, const float* ln_b, const float* Wc2, float p_drop,
                   uint64_t seed, const float* labels, int loss_kind, const float* logits, const float* preds,
                   const float* saved, const float* g_loss, const float* g_logits, const float* g_preds,
                   float* dx0, float* dW1, float* db1, float* dw2, float* dWc1, float* dbc1, float* dln_w,
                   float* dln_b, float* dWc2, float* dbc2, void* stream);

/* ---------------------------------------------------------------------------
 * GRU recurrence of TemporalEvolutionLayer over T (csrc/gru.hip; TemporalPropagation's intended compute,
 * temporal_propagation.py:402-558 inside :648-755), one launch per direction over all T steps.
 * gx [T, N, 3hc] = the x-side of the reset | update | candidate gates (LN_x(x)·W_xᵀ + b, one GEMM by the
 * caller); Wrz [2hc, hc] = the h-side columns of W_reset | W_update; Wc [hc, hc] = the h-side columns of
 * W_candidate (nn.Linear layout).  Per step: hn = LN_h(h_{t-1})·tscale[t] (h_{-1} = 0, no LayerNorm),
 * r, z = σ(gx + W·hn), h~ = tanh(gx_c + Wc·(r⊙hn)), u = dropout((1-z)⊙hn + z⊙h~) (stream row·T + t,
 * counter unit), states[t] = LN_out(u).  LayerNorm pointers NULL = use_layer_norm False; tscale [T, N]
 * (row t = exp(-clamp(Δt, 0, 10)) of step t) or NULL.  saved: tagan_gru_saved_floats(N, T, hc) floats.
 * Backward: dstates [T, N, hc] -> dgx [T, N, 3hc] (gate pre-activation gradients; the W_h gradients are
 * dgxᵀ·hn and dgx_cᵀ·(r⊙hn), hn and r⊙hn being the first two [T, N, hc] blocks of saved) and the four
 * LayerNorm parameter gradients.  hc in {16, 32, 64, 128, 256} (tagan_gru_supported).
 * ------------------------------------------------------------------------- */
int tagan_gru_supported(int32_t hc);
size_t tagan_gru_saved_floats(int64_t N, int32_t T, int32_t hc);
int tagan_gru_fwd(int64_t N, int32_t T, int32_t hc, const float* gx, const float* Wrz, const float* Wc,
                  const float* ln_h_w, const float* ln_h_b, float eps_h, const float* ln_o_w, const float* ln_o_b,
                  float eps_o, const float* tscale, float p_drop, uint64_t seed, float* states, float* saved,
                  void* stream);
size_t tagan_gru_bwd_workspace(int64_t N, int32_t hc);
int tagan_gru_bwd(int64_t N, int32_t T, int32_t hc, const float* Wrz, const float* Wc, const float* ln_h_w,
                  const float* ln_h_b, const float* ln_o_w, const float* ln_o_b, const float* tscale, float p_drop,
                  uint64_t seed, const float* states, const float* saved, const float* dstates, float* dgx,
                  float* dln_h_w, float* dln_h_b, float* dln_o_w, float* dln_o_b, void* workspace,
                  size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Window aggregation of TemporalSkipConnection over T (csrc/window.hip; temporal_propagation.py:846-946),
 * time-major: out[t, n, :] = agg over t' in [t-w, t+w] ∩ [0, T) of x[t', n, :].  mode 0 = mean over the
 * in-range steps (avg_pool1d, count_include_pad False), 1 = max (first maximum in window order, as
 * max_pool1d), 2 = sum.  x/out/dy/dx [T, N, H] contiguous fp32, H % 4 == 0.  Backward needs x only for max.
 * ------------------------------------------------------------------------- */
int tagan_window_fwd(int mode, int32_t T, int64_t N, int32_t H, int32_t w, const float* x, float* out, void* stream);
int tagan_window_bwd(int mode, int32_t T, int64_t N, int32_t H, int32_t w, const float* x, const float* dy, float* dx,
                     void* stream);

/* ---------------------------------------------------------------------------
 * NodeMemoryBank on the device.  Replaces src/tagan/utils/memory_bank.py:14-360
 * (a dict of per-node CPU tensors):  update (:65-173), get_state(s) (:175-211),
 * update_state (:235-244), decay_all (:222-225).  All arrays are caller-owned
 * device memory; tagan_membank_init formats them.
 *   tkeys/tvals [tcap]   id -> slot hash (tcap a power of two, load <= 1/2)
 *   slot arrays [cap]    slot_id (INT64_MIN = free), slot_tpos, inact,
 *                        last_seen (INT64_MIN = unset), born, touch, and the
 *                        per-call scratch first_occ/last_ok/occ_count
 *   states [cap, H]      fp32 node states
 *   free_list [cap]      freed slots
 *   fkeys/fcount [fcap]  per-id appearance counts (never pruned, :97, :165)
 *   ctl int64[8]         {slots used (high-water), free_top, stored, tombstones,
 *                         distinct ids, error flags, -, -}
 * `epoch` is a caller counter, unique per call; `timestep` as in the reference.
 * ------------------------------------------------------------------------- */
typedef struct tagan_membank {
    int64_t cap, tcap, fcap;
    int32_t H;
    int64_t* tkeys;
    int32_t* tvals;
    int64_t* slot_id;
    int32_t* slot_tpos;
    float* states;
    int32_t* inact;
    int64_t* last_seen;
    int32_t* born;
    int32_t* touch;
    int32_t* first_occ;
    int32_t* last_ok;
    int32_t* occ_count;
    int32_t* free_list;
    int64_t* fkeys;
    int64_t* fcount;
    int64_t* ctl;
} tagan_membank;

int tagan_membank_init(const tagan_membank* bank, void* stream);
/* ids[n] -> slots[n] (-1 if absent).  insert != 0 inserts absent ids as zero
 * states with inactivity 0 (get_states semantics).  scratch: int32[2n]. */
int tagan_membank_lookup(const tagan_membank* bank, const int64_t* ids, int64_t n, int insert, int32_t epoch,
                         int32_t* slots, int32_t* scratch, void* stream);
/* One NodeMemoryBank.update(ids, states, timestep) (states [n, H], row stride ld). */
int tagan_membank_update(const tagan_membank* bank, const int64_t* ids, int64_t n, const float* states,
                         int64_t ld, int64_t timestep, double decay, int32_t max_inactivity, int32_t epoch,
                         uint64_t seed, int32_t* slots, int32_t* scratch, void* stream);
/* out[n, H] = states[slots] (zeros where slot < 0). */
int tagan_membank_gather(const tagan_membank* bank, const int32_t* slots, int64_t n, float* out, void* stream);
/* states *= factor for every stored slot (decay_all). */
int tagan_membank_scale(const tagan_membank* bank, float factor, void* stream);
/* Copy every stored node of src into a freshly formatted dst (growth / tombstone purge). */
int tagan_membank_rehash(const tagan_membank* src, const tagan_membank* dst, void* stream);

/* ---------------------------------------------------------------------------
 * Graph-feature pooling.  Replaces model.py:377-427: the reference pools the
 * node-major temporal output [N, T, H] as gf[t] = mean(out.view(T, -1, H)[t]),
 * i.e. the mean of node-major flat rows [t*N, (t+1)*N) (flat row f = n*T + t').
 * Input here is time-major x[T][N][H] with row strides ld_row (node) and
 * ld_t (step), in elements; out = gf [T, H].  Deterministic (ordered partials).
 * Backward: dx[t'][n] = g[(n*T + t') / N] / N.
 * ------------------------------------------------------------------------- */
size_t tagan_pool_workspace(int32_t T, int32_t H);
int tagan_pool_fwd(int dtype, int32_t T, int64_t N, int32_t H, const float* x, int64_t ld_row, int64_t ld_t,
                   float* out, void* workspace, size_t workspace_bytes, void* stream);
int tagan_pool_bwd(int dtype, int32_t T, int64_t N, int32_t H, const float* g, float* dx, int64_t ld_row,
                   int64_t ld_t, void* stream);

/* Column sums of a tall row-major [M, N] matrix (row stride ld; dtype = its storage, fp32 or
 * bf16): the bias gradients of the projections (sum of dY over rows), fp32 out.  Two-stage,
 * ordered, deterministic.  N % 4 == 0. */
size_t tagan_colsum_workspace(int64_t M, int32_t N);
int tagan_colsum(int dtype, int64_t M, int32_t N, const void* x, int64_t ld, float* out, void* workspace,
                 size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Projection-parameter packing.  Replaces the per-step torch.cat of q_linear / k_linear / v_linear
 * (geometric_attention.py:263-266, temporal_attention.py:356-359 -- the reference calls the three Linears
 * separately; the fused block multiplies by their concatenation).
 * pack:   w[r, c] (row stride ld_w) = [Wq; Wk; Wv][r, c] for c < H; with bias_col: w[r, H] = [bq; bk; bv][r] and
 *         w[r, H+1 .. ld_w-1] = 0 (the augmented QKV GEMM operand); b (optional) = [bq; bk; bv].
 * unpack: dwq | dwk | dwv [H, H] = row blocks of dw (row stride ld_dw), dbq | dbk | dbv [H] = db[r * db_stride];
 *         any output (or dw / db) may be NULL.
 * ------------------------------------------------------------------------- */
int tagan_qkv_pack(int64_t H, const float* wq, const float* wk, const float* wv, const float* bq, const float* bk,
                   const float* bv, float* w, int64_t ld_w, int32_t bias_col, float* b, void* stream);
int tagan_qkv_unpack(int64_t H, const float* dw, int64_t ld_dw, const float* db, int64_t db_stride, float* dwq,
                     float* dwk, float* dwv, float* dbq, float* dbk, float* dbv, void* stream);

/* Temporal bias table (temporal_attention.py:732-790; the additive terms of :1010-1027): tab[h][d] (row length
 * 2T-1, d = i - j + T - 1, delta = d - (T-1)) = R[clamp(delta + m, 0, 2m)][h] + K[delta + W][h]*[|delta| <= W];
 * K = asymmetric_kernel [2W+1][heads], R = relative_pos_table [2m+1][heads] (NULL: no relative term).
 * Backward: dK, dR (either may be NULL) from g [heads][2T-1]; ordered sums, deterministic. */
int tagan_temporal_bias_table(int32_t T, int32_t heads, const float* K, int32_t W, const float* R, int32_t m,
                              float* tab, void* stream);
int tagan_temporal_bias_table_bwd(int32_t T, int32_t heads, const float* g, int32_t W, int32_t m, float* dK,
                                  float* dR, void* stream);

/* ---------------------------------------------------------------------------
 * Narrow-input projection (the node embedding, model.py:233: nn.Linear(node_feature_dim, hidden_dim) on
 * every snapshot's x).  y[M, N] = x[M, K] Wᵀ + b, W row-major [N, K], fp32, K <= 31, N in {64, 128, 256};
 * x row stride ldx (>= K, any alignment), y / dY 16-byte aligned with row strides ldy / lddy % 4 == 0, b 16-byte
 * aligned.  Backward: dW [N, K] = dYᵀ x and db [N] = Σ dY
 * (either may be NULL) in one pass over dY, exact-f32 MFMA, ordered per-workgroup partials: deterministic.
 * The input gradient is not produced (the caller's x is data).
 * ------------------------------------------------------------------------- */
int tagan_narrow_linear_supported(int32_t K, int32_t N);
int tagan_narrow_linear_fwd(int64_t M, int32_t K, int32_t N, const float* x, int64_t ldx, const float* w,
                            const float* b, float* y, int64_t ldy, void* stream);
size_t tagan_narrow_linear_bwd_workspace(int64_t M, int32_t K, int32_t N);
int tagan_narrow_linear_bwd(int64_t M, int32_t K, int32_t N, const float* x, int64_t ldx, const float* dy,
                            int64_t lddy, float* dw, float* db, void* workspace, size_t workspace_bytes,
                            void* stream);

#ifdef __cplusplus
}
#endif
#endif /* TAGAN_HIP_H */
