// Geometric (edge-softmax) attention for TAGAN on gfx950.
//
// Replaces geometric_attention.py:332-516 (_get_attention_weights: metric scores,
// masked_fill(-inf) with the dense adjacency of graph_attention.py:96-105,
// softmax, attn_dropout) and :579-583 (A·V), for rows = CSR rows = src = query.
//
// Work decomposition (fast path): rows are split into chunks of <= `chunk`
// CSR entries (tagan_graph_chunks) so power-law hubs do not serialise on one
// wave; multi-chunk rows merge their partial (max, sum, acc) states in chunk
// order (deterministic).  A group of LPR = H/4 lanes owns one chunk: lane l of
// the group holds features [4l, 4l+4) (float4 gathers of whole K/V rows), a
// head is an aligned sub-group of LPH = d/4 lanes (per-head reductions are XOR
// butterflies), and a wave runs 64/LPR chunks side by side (more independent
// gathers in flight).  Softmax is online (running max / sum per head), so
// scores are never stored; the row's log-sum-exp is saved for the backward
// pass.  HBM-bound: algorithmic bytes per (layer, snapshot) in DESIGN.md §4.
// Shapes outside the fast path (H not in {32..256}, d % 4 != 0) use the
// one-wave-per-row and one-thread-per-(row, head) fallbacks below.
//
// Backward (atomic-free, bitwise deterministic):
//   row pass (CSR):    delta_i = Σ_f dO_i·O_i per head, dq_i = Σ_j ds_ij ∂s/∂q_i
//   column pass (CSC): dk_j = Σ_i ds_ij ∂s/∂k_j,  dv_j = Σ_i α'_ij dO_i
// with ds_ij = α_ij (dα'_ij·v_j·mask/(1-p) − delta_i), α recomputed from LSE.
// {lse_i, delta_i} per (node, head) are one packed 8-B record, so the column pass's per-edge gather of both
// touches one line instead of two (C4: -2 GB of fetch per backward).  Column-first order: see below.
#include "common.cuh"

namespace tagan {
namespace {

constexpr int BLK = 256;

enum Family { FAM_DOT, FAM_SQ, FAM_ABS, FAM_COS };

template <int METRIC>
struct MetricTraits {
    static constexpr int fam = (METRIC == TAGAN_METRIC_DOT_PRODUCT || METRIC == TAGAN_METRIC_SCALED_DOT_PRODUCT)
                                   ? FAM_DOT
                               : (METRIC == TAGAN_METRIC_MANHATTAN) ? FAM_ABS
                               : (METRIC == TAGAN_METRIC_COSINE_SIMILARITY || METRIC == TAGAN_METRIC_COSINE_DISTANCE)
                                   ? FAM_COS
                                   : FAM_SQ;
};

template <int CTRL>
__device__ __forceinline__ float dpp(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}

// Sum over aligned groups of lph lanes (lph = d/4, wave-uniform).  DPP quad_perm xor1 / xor2,
// row_half_mirror, row_mirror instead of ds_bpermute shuffles: every lane of a group ends with
// the same value, bitwise equal to the xor-butterfly (each step adds two equal partial sums).
__device__ __forceinline__ float grp_sum(float x, int lph) {
    if (lph > 1) x += dpp<0xB1>(x);
    if (lph > 2) x += dpp<0x4E>(x);
    if (lph > 4) x += dpp<0x141>(x);
    if (lph > 8) x += dpp<0x140>(x);
    if (lph > 16) {   // across rows: v_permlane16_swap / v_permlane32_swap (common.cuh)
        float a, b;
        swap16(x, a, b);
        x = a + b;
    }
    if (lph > 32) {
        float a, b;
        swap32(x, a, b);
        x = a + b;
    }
    return x;
}

// Per-lane partial of the pair function over this lane's VEC features.
template <int METRIC, int VEC>
__device__ __forceinline__ void pair_partial(const float (&q)[VEC], const float (&k)[VEC], float& a, float& b) {
    a = 0.f;
    b = 0.f;
#pragma unroll
    for (int c = 0; c < VEC; ++c) {
        if constexpr (MetricTraits<METRIC>::fam == FAM_DOT) {
            a = fmaf(q[c], k[c], a);
        } else if constexpr (MetricTraits<METRIC>::fam == FAM_SQ) {
            const float t = q[c] - k[c];
            a = fmaf(t, t, a);
        } else if constexpr (MetricTraits<METRIC>::fam == FAM_ABS) {
            a += fabsf(q[c] - k[c]);
        } else {
            a = fmaf(q[c], k[c], a);
            b = fmaf(k[c], k[c], b);
        }
    }
}

// Score from the reduced partials (DistanceMetric, geometric_attention.py:24-193;
// negation of distances :398, scaled_dot_product :354).  qq = |q|^2 (cosine only).
template <int METRIC>
__device__ __forceinline__ float finalize(float a, float b, float qq, float inv_sqrt_d, float prm) {
    if constexpr (METRIC == TAGAN_METRIC_SCALED_DOT_PRODUCT) return a * inv_sqrt_d;
    if constexpr (METRIC == TAGAN_METRIC_DOT_PRODUCT) return a;
    if constexpr (METRIC == TAGAN_METRIC_EUCLIDEAN) return -__builtin_amdgcn_sqrtf(a + 1e-8f);   // v_sqrt_f32 (1 ulp)
    if constexpr (METRIC == TAGAN_METRIC_SQUARED_EUCLIDEAN) return -a;
    if constexpr (METRIC == TAGAN_METRIC_MANHATTAN) return -a;
    if constexpr (METRIC == TAGAN_METRIC_GAUSSIAN_KERNEL) return __expf(-a / (2.f * prm * prm));
    if constexpr (METRIC == TAGAN_METRIC_RBF_KERNEL) return __expf(-prm * a);
    if constexpr (MetricTraits<METRIC>::fam == FAM_COS) {
        float qn = sqrtf(qq), kn = sqrtf(b);
        qn = (qn == 0.f) ? 1e-8f : qn;
        kn = (kn == 0.f) ? 1e-8f : kn;
        const float c = fminf(fmaxf(a / (qn * kn), -1.f), 1.f);
        return (METRIC == TAGAN_METRIC_COSINE_SIMILARITY) ? c : -(1.f - c);
    }
    return 0.f;
}

// Gradient of the score w.r.t. q and k:  ∂s/∂q_c = cq_q*q_c + cq_k*k_c + sg*sign(q_c-k_c)
//                                        ∂s/∂k_c = ck_q*q_c + ck_k*k_c - sg*sign(q_c-k_c)
// and ∂s/∂param.  s is the finalized score.
struct Grad {
    float cq_q, cq_k, ck_q, ck_k, sg, dprm;
};

template <int METRIC>
__device__ __forceinline__ Grad score_grad(float a, float b, float qq, float s, float inv_sqrt_d, float prm) {
    Grad g{0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if constexpr (METRIC == TAGAN_METRIC_SCALED_DOT_PRODUCT) {
        g.cq_k = inv_sqrt_d;
        g.ck_q = inv_sqrt_d;
    } else if constexpr (METRIC == TAGAN_METRIC_DOT_PRODUCT) {
        g.cq_k = 1.f;
        g.ck_q = 1.f;
    } else if constexpr (MetricTraits<METRIC>::fam == FAM_SQ) {
        float c;  // ∂s/∂(q-k) = c·(q-k)
        if constexpr (METRIC == TAGAN_METRIC_EUCLIDEAN) c = __builtin_amdgcn_rcpf(s);   // s = -r  ->  -(q-k)/r
        else if constexpr (METRIC == TAGAN_METRIC_SQUARED_EUCLIDEAN) c = -2.f;
        else if constexpr (METRIC == TAGAN_METRIC_GAUSSIAN_KERNEL) {
            c = -s / (prm * prm);
            g.dprm = s * a / (prm * prm * prm);
        } else {
            c = -2.f * prm * s;
            g.dprm = -s * a;
        }
        g.cq_q = c;
        g.cq_k = -c;
        g.ck_q = -c;
        g.ck_k = c;
    } else if constexpr (MetricTraits<METRIC>::fam == FAM_ABS) {
        g.sg = -1.f;
    } else {
        const float qn0 = sqrtf(qq), kn0 = sqrtf(b);
        const float qn = (qn0 == 0.f) ? 1e-8f : qn0, kn = (kn0 == 0.f) ? 1e-8f : kn0;
        const float raw = a / (qn * kn);
        const float pass = (raw >= -1.f && raw <= 1.f) ? 1.f : 0.f;      // clamp backward mask
        const float inv = pass / (qn * kn);
        g.cq_k = inv;
        g.ck_q = inv;
        g.cq_q = (qn0 == 0.f) ? 0.f : -pass * raw / (qn * qn);
        g.ck_k = (kn0 == 0.f) ? 0.f : -pass * raw / (kn * kn);
    }
    return g;
}

template <int VEC>
__device__ __forceinline__ void load_vec(const float* __restrict__ p, float (&r)[VEC]) {
    if constexpr (VEC == 4) {
        const float4 t = *reinterpret_cast<const float4*>(p);
        r[0] = t.x; r[1] = t.y; r[2] = t.z; r[3] = t.w;
    } else if constexpr (VEC == 2) {
        const float2 t = *reinterpret_cast<const float2*>(p);
        r[0] = t.x; r[1] = t.y;
    } else {
#pragma unroll
        for (int c = 0; c < VEC; ++c) r[c] = p[c];
    }
}

template <int VEC>
__device__ __forceinline__ void store_vec(float* __restrict__ p, const float (&r)[VEC]) {
    if constexpr (VEC == 4) {
        *reinterpret_cast<float4*>(p) = make_float4(r[0], r[1], r[2], r[3]);
    } else if constexpr (VEC == 2) {
        *reinterpret_cast<float2*>(p) = make_float2(r[0], r[1]);
    } else {
#pragma unroll
        for (int c = 0; c < VEC; ++c) p[c] = r[c];
    }
}

struct GeoArgs {
    tagan_graph g;
    int64_t N;
    int heads, d, lph, H;
    const float* q;
    const float* k;
    const float* v;
    int64_t ld;
    const float* mparam;
    float p_drop, inv_keep;
    uint64_t seed;
    const uint64_t* seed_ctr;   // graph-replay seed source (tagan_set_seed_counter) or null
    const float* o;
    const float* lse_in;
    const float* dout;
    float* out;
    float* lse;
    float* dq;
    float* dk;
    float* dv;
    int64_t ldd;
    float* delta;
    float* ds_edge;     // [nnz_cap, heads] dS per edge in CSR order (column-first backward) or null
    float* prm_partial;
    float* part_m;      // [part_cap, heads]
    float* part_l;      // [part_cap, heads]
    float* part_v;      // [part_cap, H]  (fwd acc / bwd dq)
    float* part_v2;     // [part_cap, 2H] (bwd col: dk | dv)
    float inv_sqrt_d;
    int bf16;           // activation storage: 0 fp32, 1 bf16 (fast path only)
    int xcd;            // chunk-kernel block order (geo_xcd_mode): 0 launch order, 1 XCD-contiguous over the grid,
                        // 2 XCD-contiguous over the blocks that hold valid chunks
};

#ifndef TAGAN_GEO_UNROLL
#define TAGAN_GEO_UNROLL 2
#endif
#ifndef TAGAN_GEO_UNROLL8
#define TAGAN_GEO_UNROLL8 2
#endif
template <int FPL>
struct Unroll { static constexpr int v = FPL == 8 ? TAGAN_GEO_UNROLL8 : TAGAN_GEO_UNROLL; };

__device__ __forceinline__ float sgnf(float x) { return (x > 0.f) ? 1.f : (x < 0.f ? -1.f : 0.f); }

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ float f4(const float4& v, int c) { return c == 0 ? v.x : c == 1 ? v.y : c == 2 ? v.z : v.w; }

template <int METRIC>
__device__ __forceinline__ void partial4(const float4& q, const float4& k, float& a, float& b) {
    float qa[4] = {q.x, q.y, q.z, q.w}, ka[4] = {k.x, k.y, k.z, k.w};
    pair_partial<METRIC, 4>(qa, ka, a, b);
}

// =================================================================== fast path: chunked kernels
// Lane geometry shared by the chunk kernels.
// The grid is sized for the chunk CAPACITY (rows + entries / chunk: a static shape for graph capture), and the
// valid chunks (a device-side count) fill only its front -- 75 % of it for the uniform C3 / C4 / C5 graphs.  Mode 1
// (the round-2..4 map) gives each XCD a contiguous eighth of the whole grid, so the XCDs whose eighths lie past the
// valid count had nothing to do; mode 2 spreads the VALID blocks over the XCDs the same way; mode 0 keeps the launch
// order (consecutive blocks round-robin over the XCDs: every XCD works on the same region of the graph at a time).
template <int LPR>
struct Lanes {
    static constexpr int RPW = WAVE / LPR;   // chunks per wave
    int lane, sub, sl, base;                  // base = first lane of this chunk's group
    int64_t chunk;                            // global chunk id of this group
    __device__ __forceinline__ Lanes(int64_t nvalid, int mode) {
        lane = threadIdx.x & (WAVE - 1);
        sub = lane / LPR;
        sl = lane % LPR;
        base = sub * LPR;
        int64_t b = blockIdx.x;
        if (mode == 1) {
            b = xcd_remap(b, gridDim.x);
        } else if (mode == 2) {
            const int64_t nv = (nvalid + RPW * (BLK / WAVE) - 1) / (RPW * (BLK / WAVE));
            if (b < nv) b = xcd_remap(b, nv);
        }
        const int64_t wave = b * (BLK / WAVE) + (threadIdx.x >> 6);
        chunk = wave * RPW + sub;
    }
};

// ------------------------------------------------------------------ lane vectors
// A lane owns FPL consecutive features (FPL = 4 or 8).  FPL = 8 halves the lanes per row, so a
// wave runs twice as many chunks side by side with twice the bytes per gather instruction: the
// edge kernels are bound by gathers in flight, not by bytes (bf16 storage alone hardly helps).
template <typename S>
struct IsBf16 { static constexpr bool v = false; };
template <>
struct IsBf16<bf16s> { static constexpr bool v = true; };

template <typename S, int F>
__device__ __forceinline__ void ldf(const void* p, int64_t i, float (&r)[F]) {
    if constexpr (IsBf16<S>::v && F == 8) {
        const uint4 u = *(const uint4*)((const uint16_t*)p + i);
        const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            r[2 * c] = __uint_as_float(w[c] << 16);
            r[2 * c + 1] = __uint_as_float(w[c] & 0xffff0000u);
        }
    } else {
#pragma unroll
        for (int c = 0; c < F; c += 4) {
            const float4 t = Io<S>::ld(p, i + c);
            r[c] = t.x; r[c + 1] = t.y; r[c + 2] = t.z; r[c + 3] = t.w;
        }
    }
}

template <typename S, int F>
__device__ __forceinline__ void stf(void* p, int64_t i, const float (&r)[F]) {
    if constexpr (IsBf16<S>::v && F == 8) {
        uint4 u;
        u.x = f2bf2(r[0], r[1]);
        u.y = f2bf2(r[2], r[3]);
        u.z = f2bf2(r[4], r[5]);
        u.w = f2bf2(r[6], r[7]);
        *(uint4*)((uint16_t*)p + i) = u;
    } else {
#pragma unroll
        for (int c = 0; c < F; c += 4) Io<S>::st(p, i + c, make_float4(r[c], r[c + 1], r[c + 2], r[c + 3]));
    }
}

template <int F>
__device__ __forceinline__ float dotf(const float (&a)[F], const float (&b)[F]) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < F; ++c) s = fmaf(a[c], b[c], s);
    return s;
}

// ------------------------------------------------------------------ forward
template <int METRIC, int LPR, int FPL, typename S>
__global__ void __launch_bounds__(BLK) k_geo_fwd_chunk(GeoArgs A) {
    TAGAN_LIVE_SEED(A);
    constexpr int UN = Unroll<FPL>::v;
    const int nchunks = A.g.row_counts[0];
    Lanes<LPR> L(nchunks, A.xcd);
    const bool valid = L.chunk < nchunks;
    if (valid && A.g.row_chunk_order) L.chunk = A.g.row_chunk_order[L.chunk];   // length-sorted order
    int row = 0, e0 = 0, cnt = 0;
    if (valid) {
        row = A.g.row_chunk_seg[L.chunk];
        e0 = A.g.row_chunk_beg[L.chunk];
        if (TAGAN_DBAD(row >= 0 && row < A.g.n_nodes && e0 >= A.g.rowptr[row] && e0 <= A.g.rowptr[row + 1], row, e0))
            row = e0 = 0;
        cnt = min(A.g.chunk, A.g.rowptr[row + 1] - e0);
    }
    if (!__any(valid)) return;
    const int lph = A.d / FPL;                   // lanes per head
    const int f0 = L.sl * FPL;
    const int h = f0 / A.d;
    const uint32_t dkey = drop_key(A.seed, (uint64_t)h);
    float qv[FPL];
    ldf<S>(A.q, (int64_t)row * A.ld + f0, qv);
    float qq = 0.f;
    if constexpr (MetricTraits<METRIC>::fam == FAM_COS) qq = grp_sum(dotf(qv, qv), lph);
    const float prm = A.mparam ? A.mparam[h] : 1.f;
    float m = -INFINITY, l = 0.f;
    float acc[FPL];
#pragma unroll
    for (int c = 0; c < FPL; ++c) acc[c] = 0.f;
    int mycol = 0;
    for (int jj = 0; __any(jj < cnt); jj += UN) {
        if ((jj % LPR) == 0) mycol = (jj + L.sl < cnt) ? A.g.col[e0 + jj + L.sl] : 0;
        if (TAGAN_DBAD(mycol >= 0 && mycol < A.g.n_nodes, mycol, row)) mycol = 0;   // gather index
        float kv[UN][FPL], vv[UN][FPL];
#pragma unroll
        for (int u = 0; u < UN; ++u) {
            const int j = __shfl(mycol, L.base + ((jj + u) % LPR), WAVE);
            ldf<S>(A.k, (int64_t)j * A.ld + f0, kv[u]);
            ldf<S>(A.v, (int64_t)j * A.ld + f0, vv[u]);
        }
#pragma unroll
        for (int u = 0; u < UN; ++u) {
            const bool live = jj + u < cnt;
            float a, b;
            pair_partial<METRIC, FPL>(qv, kv[u], a, b);
            a = grp_sum(a, lph);
            if constexpr (MetricTraits<METRIC>::fam == FAM_COS) b = grp_sum(b, lph);
            if (!live) continue;
            const float s = finalize<METRIC>(a, b, qq, A.inv_sqrt_d, prm);
            const float mn = fmaxf(m, s);
            const float corr = __expf(m - mn);
            const float p = __expf(s - mn);
            l = fmaf(l, corr, p);
            float pw = p;
            if (A.p_drop > 0.f) pw = (drop_u(dkey, (uint32_t)(e0 + jj + u)) >= A.p_drop) ? p * A.inv_keep : 0.f;
#pragma unroll
            for (int c = 0; c < FPL; ++c) acc[c] = fmaf(acc[c], corr, pw * vv[u][c]);
            m = mn;
        }
    }
    if (!valid) return;
    const int part = A.g.row_chunk_part[L.chunk];
    if (TAGAN_DBAD(part < A.g.part_cap, part, A.g.part_cap)) return;   // partial slot
    if (part < 0) {
        const float inv = (l > 0.f) ? 1.f / l : NAN;
#pragma unroll
        for (int c = 0; c < FPL; ++c) acc[c] *= inv;
        stf<S>(A.out, (int64_t)row * A.H + f0, acc);
        if ((L.sl % lph) == 0) A.lse[(int64_t)row * A.heads + h] = m + __logf(l);
    } else {
        stf<float>(A.part_v, (int64_t)part * A.H + f0, acc);
        if ((L.sl % lph) == 0) {
            A.part_m[(int64_t)part * A.heads + h] = m;
            A.part_l[(int64_t)part * A.heads + h] = l;
        }
    }
}

// Merge of multi-chunk segments (hub rows / columns).  A wave per segment, persistent over segments (the grid is
// bounded: the partial capacity is a worst case, most of it unused).  A lane owns 4 features; the wave's
// 64 / (width / 4) lane groups ("phases") take interleaved chunks, and each lane keeps G independent partial states
// over its chunks, so G·phases partial loads are in flight instead of one dependent chain per chunk (a C2 hub row
// spans ~100 chunks).  The states combine in a fixed order (accumulators, then phases by xor-shuffle): the result
// is deterministic (bitwise reproducible), in another summation order than a chunk-serial loop.
// Round 6: the accumulator count G is a template parameter (env TAGAN_GEO_MG = 4 / 8 / 16, see geo_mg()), and the
// G chunk loads of an iteration are branch-free (index clamped into the segment, dead slots dropped by a select):
// with a guarded load per accumulator each one sat in its own basic block behind a wait, so the G loads of an
// iteration ran as a dependent chain (a C2 hub: k_geo_sum_parts 25 us, k_geo_fwd_merge 20 us per call).
// fixed-order pairwise tree over the G accumulators (bitwise reproducible)
template <int G, typename T, typename F>
__device__ __forceinline__ T tree_combine(T (&v)[G], F f) {
    static_assert(G == 1 || G == 2 || G == 4 || G == 8 || G == 16, "G: a power of two <= 16");
#pragma unroll
    for (int w = 1; w < G; w <<= 1)
#pragma unroll
        for (int u = 0; u + w < G; u += 2 * w) v[u] = f(v[u], v[u + w]);
    return v[0];
}
struct SoftState {
    float m, l;
    float4 a;
};

__device__ __forceinline__ SoftState soft_merge(const SoftState& x, const SoftState& y) {
    const float mn = fmaxf(x.m, y.m);
    const float cx = (x.m == -INFINITY) ? 0.f : __expf(x.m - mn);
    const float cy = (y.m == -INFINITY) ? 0.f : __expf(y.m - mn);
    SoftState r;
    r.m = mn;
    r.l = x.l * cx + y.l * cy;
    r.a = make_float4(x.a.x * cx + y.a.x * cy, x.a.y * cx + y.a.y * cy, x.a.z * cx + y.a.z * cy,
                      x.a.w * cx + y.a.w * cy);
    return r;
}

__device__ __forceinline__ SoftState soft_shfl_xor(const SoftState& x, int mask) {
    SoftState r;
    r.m = __shfl_xor(x.m, mask, WAVE);
    r.l = __shfl_xor(x.l, mask, WAVE);
    r.a = make_float4(__shfl_xor(x.a.x, mask, WAVE), __shfl_xor(x.a.y, mask, WAVE), __shfl_xor(x.a.z, mask, WAVE),
                      __shfl_xor(x.a.w, mask, WAVE));
    return r;
}

__device__ __forceinline__ float4 f4add(const float4& x, const float4& y) {
    return make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w);
}

// component-wise select (a float4 ternary lowers to a select of stack addresses through scratch)
__device__ __forceinline__ float4 f4live(bool live, const float4& x) {
    return make_float4(live ? x.x : 0.f, live ? x.y : 0.f, live ? x.z : 0.f, live ? x.w : 0.f);
}

__device__ __forceinline__ float4 f4shfl_xor(const float4& x, int mask) {
    return make_float4(__shfl_xor(x.x, mask, WAVE), __shfl_xor(x.y, mask, WAVE), __shfl_xor(x.z, mask, WAVE),
                       __shfl_xor(x.w, mask, WAVE));
}

// accumulators per lane of the merge kernels, read once: TAGAN_GEO_MG for k_geo_sum_parts (default 16),
// TAGAN_GEO_MG_FWD for k_geo_fwd_merge (default 8: its 6-float states take 243 VGPRs at 16); 4, 8 or 16.
// C2 per call (profiles/r6q_*, r6r_*): sum_parts 25.0 -> 10.4 us, fwd_merge 19.5 -> 11.2 us at G = 8 (branch-free
// loads); G = 16 takes the C2 backward another ~8 us lower and the forward ~5 us higher.
int geo_mg_env(const char* name, int dflt) {
    const char* e = std::getenv(name);
    const int x = e ? std::atoi(e) : dflt;
    return (x == 4 || x == 8 || x == 16) ? x : dflt;
}
int geo_mg(bool fwd) {
    static const int vs = geo_mg_env("TAGAN_GEO_MG", 16), vf = geo_mg_env("TAGAN_GEO_MG_FWD", 8);
    return fwd ? vf : vs;
}
template <typename F>
void geo_mg_dispatch(bool fwd, F&& f) {
    switch (geo_mg(fwd)) {
        case 4: f(std::integral_constant<int, 4>{}); break;
        case 16: f(std::integral_constant<int, 16>{}); break;
        default: f(std::integral_constant<int, 8>{}); break;
    }
}

unsigned merge_grid(int64_t part_cap) {
    const int64_t b = (part_cap + (BLK / WAVE) - 1) / (BLK / WAVE);
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>(b, 1024));
}

// Merge the partial softmax states {m, l, acc} of multi-chunk rows (H <= 256).
template <int G, typename S>
__global__ void __launch_bounds__(BLK) k_geo_fwd_merge(GeoArgs A) {
    TAGAN_LIVE_SEED(A);
    using IO = Io<S>;
    const int lane = threadIdx.x & (WAVE - 1);
    const int lanes = A.H / 4;                              // lanes per phase (<= 64)
    const int nph = WAVE / lanes;                           // phases
    const int ph = lane / lanes;
    const int f0 = (lane % lanes) * 4;
    const int h = f0 / A.d;
    const int64_t nmulti = A.g.row_counts[1];
    const int64_t stride = (int64_t)gridDim.x * (BLK / WAVE);
    for (int64_t k = blockIdx.x * (int64_t)(BLK / WAVE) + (threadIdx.x >> 6); k < nmulti; k += stride) {
        const int row = A.g.row_multi[k];
        const int c0 = A.g.row_chunk_ptr[row], c1 = A.g.row_chunk_ptr[row + 1];
        SoftState st[G];
#pragma unroll
        for (int u = 0; u < G; ++u) st[u] = SoftState{-INFINITY, 0.f, make_float4(0.f, 0.f, 0.f, 0.f)};
        for (int c = c0 + ph; c < c1; c += nph * G) {
            int part[G];
            bool live[G];
#pragma unroll
            for (int u = 0; u < G; ++u) {
                const int cc = c + u * nph;
                part[u] = A.g.row_chunk_part[min(cc, c1 - 1)];
                live[u] = cc < c1;
                if (TAGAN_DBAD(part[u] >= 0 && part[u] < A.g.part_cap, part[u], A.g.part_cap)) live[u] = false, part[u] = 0;
            }
            SoftState y[G];
#pragma unroll
            for (int u = 0; u < G; ++u) {
                y[u].m = A.part_m[(int64_t)part[u] * A.heads + h];
                y[u].l = A.part_l[(int64_t)part[u] * A.heads + h];
                y[u].a = ld4(A.part_v + (int64_t)part[u] * A.H + f0);
            }
#pragma unroll
            for (int u = 0; u < G; ++u) {
                y[u].m = live[u] ? y[u].m : -INFINITY;              // a dead slot merges as the empty state
                y[u].l = live[u] ? y[u].l : 0.f;
                y[u].a = f4live(live[u], y[u].a);
                st[u] = soft_merge(st[u], y[u]);
            }
        }
        SoftState r = tree_combine<G>(st, [](const SoftState& x, const SoftState& y) { return soft_merge(x, y); });
        for (int m = lanes; m < WAVE; m <<= 1) r = soft_merge(r, soft_shfl_xor(r, m));   // phases, fixed order
        if (ph == 0) {
            const float inv = (r.l > 0.f) ? 1.f / r.l : NAN;
            IO::st(A.out, (int64_t)row * A.H + f0, make_float4(r.a.x * inv, r.a.y * inv, r.a.z * inv, r.a.w * inv));
            if ((f0 / 4) % A.lph == 0) A.lse[(int64_t)row * A.heads + h] = r.m + __logf(r.l);
        }
    }
}

// ------------------------------------------------------------------ backward, row pass (CSR chunks)
template <int METRIC, int LPR, int FPL, typename S>
__global__ void __launch_bounds__(BLK) k_geo_bwd_row_chunk(GeoArgs A) {
    TAGAN_LIVE_SEED(A);
    constexpr int UN = Unroll<FPL>::v;
    __shared__ float red[BLK];
    const int nchunks = A.g.row_counts[0];
    Lanes<LPR> L(nchunks, A.xcd);
    const bool valid = L.chunk < nchunks;
    if (valid && A.g.row_chunk_order) L.chunk = A.g.row_chunk_order[L.chunk];   // length-sorted order
    int row = 0, e0 = 0, cnt = 0;
    if (valid) {
        row = A.g.row_chunk_seg[L.chunk];
        e0 = A.g.row_chunk_beg[L.chunk];
        if (TAGAN_DBAD(row >= 0 && row < A.g.n_nodes && e0 >= A.g.rowptr[row] && e0 <= A.g.rowptr[row + 1], row, e0))
            row = e0 = 0;
        cnt = min(A.g.chunk, A.g.rowptr[row + 1] - e0);
    }
    const int lph = A.d / FPL;
    const int f0 = L.sl * FPL;
    const int h = f0 / A.d;
    const uint32_t dkey = drop_key(A.seed, (uint64_t)h);
    float prm_acc = 0.f;
    if (__any(valid)) {
        float qv[FPL], ov[FPL], dov[FPL];
        ldf<S>(A.q, (int64_t)row * A.ld + f0, qv);
        ldf<S>(A.o, (int64_t)row * A.H + f0, ov);
        ldf<S>(A.dout, (int64_t)row * A.H + f0, dov);
        const float D = grp_sum(dotf(dov, ov), lph);
        float qq = 0.f;
        if constexpr (MetricTraits<METRIC>::fam == FAM_COS) qq = grp_sum(dotf(qv, qv), lph);
        const float lse = A.lse_in[(int64_t)row * A.heads + h];
        const float prm = A.mparam ? A.mparam[h] : 1.f;
        float dq[FPL];
#pragma unroll
        for (int c = 0; c < FPL; ++c) dq[c] = 0.f;
        int mycol = 0;
        for (int jj = 0; __any(jj < cnt); jj += UN) {
            if ((jj % LPR) == 0) mycol = (jj + L.sl < cnt) ? A.g.col[e0 + jj + L.sl] : 0;
            if (TAGAN_DBAD(mycol >= 0 && mycol < A.g.n_nodes, mycol, row)) mycol = 0;   // gather index
            float kv[UN][FPL], vv[UN][FPL];
#pragma unroll
            for (int u = 0; u < UN; ++u) {
                const int j = __shfl(mycol, L.base + ((jj + u) % LPR), WAVE);
                ldf<S>(A.k, (int64_t)j * A.ld + f0, kv[u]);
                ldf<S>(A.v, (int64_t)j * A.ld + f0, vv[u]);
            }
#pragma unroll
            for (int u = 0; u < UN; ++u) {
                const bool live = jj + u < cnt;
                float a, b;
                pair_partial<METRIC, FPL>(qv, kv[u], a, b);
                float dp = dotf(dov, vv[u]);
                a = grp_sum(a, lph);
                dp = grp_sum(dp, lph);
                if constexpr (MetricTraits<METRIC>::fam == FAM_COS) b = grp_sum(b, lph);
                if (!live) continue;
                const float s = finalize<METRIC>(a, b, qq, A.inv_sqrt_d, prm);
                const float p = __expf(s - lse);
                if (A.p_drop > 0.f) dp = (drop_u(dkey, (uint32_t)(e0 + jj + u)) >= A.p_drop) ? dp * A.inv_keep : 0.f;
                const float ds = p * (dp - D);
                const Grad g = score_grad<METRIC>(a, b, qq, s, A.inv_sqrt_d, prm);
#pragma unroll
                for (int c = 0; c < FPL; ++c) {
                    const float qc = qv[c], kc = kv[u][c];
                    float t = fmaf(g.cq_q, qc, g.cq_k * kc);
                    if constexpr (MetricTraits<METRIC>::fam == FAM_ABS) t = g.sg * sgnf(qc - kc);
                    dq[c] += ds * t;
                }
                prm_acc = fmaf(ds, g.dprm, prm_acc);
            }
        }
        if (valid) {
            const int part = A.g.row_chunk_part[L.chunk];
            if (TAGAN_DBAD(part < A.g.part_cap, part, A.g.part_cap)) {   // partial slot (no return: a barrier follows)
            } else if (part < 0) stf<S>(A.dq, (int64_t)row * A.ldd + f0, dq);
            else stf<float>(A.part_v, (int64_t)part * A.H + f0, dq);
            if ((L.sl % lph) == 0 && A.g.row_chunk_ptr[row] == L.chunk)   // packed {lse, delta} per (row, head)
                *(float2*)(A.delta + ((int64_t)row * A.heads + h) * 2) = make_float2(lse, D);
        }
    }
    if (A.prm_partial) {
        red[threadIdx.x] = (valid && (L.sl % lph) == 0) ? prm_acc : 0.f;
        __syncthreads();
        if (threadIdx.x < A.heads) {
            float sacc = 0.f;
            const int off = threadIdx.x * lph;              // lane of head threadIdx.x inside a group
            for (int w = 0; w < BLK / WAVE; ++w)
                for (int sg = 0; sg < Lanes<LPR>::RPW; ++sg) sacc += red[w * WAVE + sg * LPR + off];
            A.prm_partial[(int64_t)blockIdx.x * A.heads + threadIdx.x] = sacc;
        }
    }
}

// Sum partial rows (bwd row: dq; bwd col: dk|dv) of multi-chunk segments; same lane / phase / G-accumulator
// scheme and bounded persistent grid as k_geo_fwd_merge, fixed combination order.
template <int G, typename S>
__global__ void __launch_bounds__(BLK) k_geo_sum_parts(const int32_t* __restrict__ counts,
                                                       const int32_t* __restrict__ multi,
                                                       const int32_t* __restrict__ chunk_ptr,
                                                       const int32_t* __restrict__ chunk_part,
                                                       const float* __restrict__ part, int width,
                                                       void* __restrict__ dst0, void* __restrict__ dst1,
                                                       int64_t ldd, int H) {
    const int lane = threadIdx.x & (WAVE - 1);
    const int lanes = min(width / 4, WAVE);                 // lanes per phase
    const int nph = WAVE / lanes;
    const int ph = lane / lanes;
    const int64_t nmulti = counts[1];
    const int64_t stride = (int64_t)gridDim.x * (BLK / WAVE);
    for (int64_t k = blockIdx.x * (int64_t)(BLK / WAVE) + (threadIdx.x >> 6); k < nmulti; k += stride) {
        const int seg = multi[k];
        const int c0 = chunk_ptr[seg], c1 = chunk_ptr[seg + 1];
        for (int fb = 0; fb < width; fb += lanes * 4) {
            const int f0 = fb + (lane % lanes) * 4;
            float4 acc[G];
#pragma unroll
            for (int u = 0; u < G; ++u) acc[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int c = c0 + ph; c < c1; c += nph * G) {
                int pidx[G];
                bool live[G];
#pragma unroll
                for (int u = 0; u < G; ++u) {
                    const int cc = c + u * nph;
                    pidx[u] = chunk_part[min(cc, c1 - 1)];
                    live[u] = cc < c1;
                    if (TAGAN_DBAD(pidx[u] >= 0, pidx[u], cc)) live[u] = false, pidx[u] = 0;   // partial slot
                }
                float4 v[G];
#pragma unroll
                for (int u = 0; u < G; ++u) v[u] = ld4(part + (int64_t)pidx[u] * width + f0);
#pragma unroll
                for (int u = 0; u < G; ++u) acc[u] = f4add(acc[u], f4live(live[u], v[u]));
            }
            float4 sum = tree_combine<G>(acc, [](const float4& x, const float4& y) { return f4add(x, y); });
            for (int m = lanes; m < WAVE; m <<= 1) sum = f4add(sum, f4shfl_xor(sum, m));
            if (ph == 0) {
                if (f0 < H) Io<S>::st(dst0, (int64_t)seg * ldd + f0, sum);
                else Io<S>::st(dst1, (int64_t)seg * ldd + (f0 - H), sum);
            }
        }
    }
}

// ------------------------------------------------------------------ backward, column pass (CSC chunks)
template <int METRIC, int LPR, int FPL, typename S>
__global__ void __launch_bounds__(BLK) k_geo_bwd_col_chunk(GeoArgs A) {
    TAGAN_LIVE_SEED(A);
    constexpr int UN = Unroll<FPL>::v;
    const int nchunks = A.g.col_counts[0];
    Lanes<LPR> L(nchunks, A.xcd);
    const bool valid = L.chunk < nchunks;
    if (valid && A.g.col_chunk_order) L.chunk = A.g.col_chunk_order[L.chunk];   // length-sorted order
    int colj = 0, e0 = 0, cnt = 0;
    if (valid) {
        colj = A.g.col_chunk_seg[L.chunk];
        e0 = A.g.col_chunk_beg[L.chunk];
        if (TAGAN_DBAD(colj >= 0 && colj < A.g.n_nodes && e0 >= A.g.csc_ptr[colj] && e0 <= A.g.csc_ptr[colj + 1], colj,
                       e0))
            colj = e0 = 0;
        cnt = min(A.g.chunk, A.g.csc_ptr[colj + 1] - e0);
    }
    if (!__any(valid)) return;
    const int lph = A.d / FPL;
    const int f0 = L.sl * FPL;
    const int h = f0 / A.d;
    const uint32_t dkey = drop_key(A.seed, (uint64_t)h);
    float kv[FPL], vv[FPL];
    ldf<S>(A.k, (int64_t)colj * A.ld + f0, kv);
    ldf<S>(A.v, (int64_t)colj * A.ld + f0, vv);
    const float prm = A.mparam ? A.mparam[h] : 1.f;
    float dk[FPL], dv[FPL];
#pragma unroll
    for (int c = 0; c < FPL; ++c) { dk[c] = 0.f; dv[c] = 0.f; }
    int myrow = 0, myeid = 0;
    for (int jj = 0; __any(jj < cnt); jj += UN) {
        if ((jj % LPR) == 0) {
            const bool in = jj + L.sl < cnt;
            myrow = in ? A.g.csc_row[e0 + jj + L.sl] : 0;
            myeid = in ? A.g.csc_eid[e0 + jj + L.sl] : 0;
            if (TAGAN_DBAD(myrow >= 0 && myrow < A.g.n_nodes, myrow, colj)) myrow = 0;   // gather index
            if (TAGAN_DBAD(myeid >= 0 && (A.g.nnz_cap <= 0 || myeid < A.g.nnz_cap), myeid, A.g.nnz_cap)) myeid = 0;
        }
        float qv[UN][FPL], dov[UN][FPL];
        float lse[UN], D[UN];
        int eid[UN];
#pragma unroll
        for (int u = 0; u < UN; ++u) {
            const int src = L.base + ((jj + u) % LPR);
            const int i = __shfl(myrow, src, WAVE);
            eid[u] = __shfl(myeid, src, WAVE);
            ldf<S>(A.q, (int64_t)i * A.ld + f0, qv[u]);
            ldf<S>(A.dout, (int64_t)i * A.H + f0, dov[u]);
            const float2 ld = *(const float2*)(A.delta + ((int64_t)i * A.heads + h) * 2);   // one 8-B read
            lse[u] = ld.x;
            D[u] = ld.y;
        }
#pragma unroll
        for (int u = 0; u < UN; ++u) {
            const bool live = jj + u < cnt;
            float a, b, qq = 0.f;
            pair_partial<METRIC, FPL>(qv[u], kv, a, b);
            float dp = dotf(dov[u], vv);
            a = grp_sum(a, lph);
            dp = grp_sum(dp, lph);
            if constexpr (MetricTraits<METRIC>::fam == FAM_COS) {
                b = grp_sum(b, lph);
                qq = grp_sum(dotf(qv[u], qv[u]), lph);
            }
            if (!live) continue;
            const float s = finalize<METRIC>(a, b, qq, A.inv_sqrt_d, prm);
            const float p = __expf(s - lse[u]);
            float pw = p;
            if (A.p_drop > 0.f) {
                const bool keep = drop_u(dkey, (uint32_t)eid[u]) >= A.p_drop;
                dp = keep ? dp * A.inv_keep : 0.f;
                pw = keep ? p * A.inv_keep : 0.f;
            }
            const float ds = p * (dp - D[u]);
            if (A.ds_edge && (L.sl % lph) == 0) A.ds_edge[(int64_t)eid[u] * A.heads + h] = ds;   // CSR order
            const Grad g = score_grad<METRIC>(a, b, qq, s, A.inv_sqrt_d, prm);
#pragma unroll
            for (int c = 0; c < FPL; ++c) {
                const float qc = qv[u][c], kc = kv[c];
                float t = fmaf(g.ck_q, qc, g.ck_k * kc);
                if constexpr (MetricTraits<METRIC>::fam == FAM_ABS) t = -g.sg * sgnf(qc - kc);
                dk[c] += ds * t;
                dv[c] += pw * dov[u][c];
            }
        }
    }
    if (!valid) return;
    const int part = A.g.col_chunk_part[L.chunk];
    if (TAGAN_DBAD(part < A.g.part_cap, part, A.g.part_cap)) return;   // partial slot
    if (part < 0) {
        stf<S>(A.dk, (int64_t)colj * A.ldd + f0, dk);
        stf<S>(A.dv, (int64_t)colj * A.ldd + f0, dv);
    } else {
        stf<float>(A.part_v2, (int64_t)part * 2 * A.H + f0, dk);
        stf<float>(A.part_v2, (int64_t)part * 2 * A.H + A.H + f0, dv);
    }
}

// ------------------------------------------------------------------ backward, column-first order
// With a per-edge dS buffer the backward runs: node pass (delta_i) -> column pass (dk, dv, and dS_ij stored
// per CSR edge) -> row pass (dq from the stored dS).  The row pass then gathers only K_j (not K_j and V_j) and
// reads no O / dO / LSE: 1.5 KB instead of 2 KB of gathers per edge at H = 128 fp32.  dS and delta are the
// same bits the row-first order computes (same lane layout, same reductions), so dq, dk, dv do not change.

// delta_i = Σ_f dO_i·O_i per head, written with lse_i as the packed {lse, delta} record; rows as "chunks".
template <int LPR, int FPL, typename S>
__global__ void __launch_bounds__(BLK) k_geo_bwd_delta(GeoArgs A) {
    TAGAN_LIVE_SEED(A);
    Lanes<LPR> L(A.N, A.xcd != 0 ? 1 : 0);   // grid sized by N: every block valid (modes 1 and 2 agree)
    const bool valid = L.chunk < A.N;
    if (!__any(valid)) return;
    const int64_t row = valid ? L.chunk : 0;
    const int lph = A.d / FPL;
    const int f0 = L.sl * FPL;
    const int h = f0 / A.d;
    float ov[FPL], dov[FPL];
    ldf<S>(A.o, row * A.H + f0, ov);
    ldf<S>(A.dout, row * A.H + f0, dov);
    const float D = grp_sum(dotf(dov, ov), lph);
    if (valid && (L.sl % lph) == 0)
        *(float2*)(A.delta + (row * A.heads + h) * 2) = make_float2(A.lse_in[row * A.heads + h], D);
}

// Row pass from the stored dS: dq_i = Σ_j dS_ij ∂s/∂q_i, gathering K_j only; dS is read in CSR order (the column
// pass stores each edge's dS at its CSR position, csc_eid, so no CSR -> CSC position map is needed).
template <int METRIC, int LPR, int FPL, typename S>
__global__ void __launch_bounds__(BLK) k_geo_bwd_row_ds(GeoArgs A) {
    TAGAN_LIVE_SEED(A);
    constexpr int UN = Unroll<FPL>::v;
    __shared__ float red[BLK];
    const int nchunks = A.g.row_counts[0];
    Lanes<LPR> L(nchunks, A.xcd);
    const bool valid = L.chunk < nchunks;
    if (valid && A.g.row_chunk_order) L.chunk = A.g.row_chunk_order[L.chunk];   // length-sorted order
    int row = 0, e0 = 0, cnt = 0;
    if (valid) {
        row = A.g.row_chunk_seg[L.chunk];
        e0 = A.g.row_chunk_beg[L.chunk];
        if (TAGAN_DBAD(row >= 0 && row < A.g.n_nodes && e0 >= A.g.rowptr[row] && e0 <= A.g.rowptr[row + 1], row, e0))
            row = e0 = 0;
        cnt = min(A.g.chunk, A.g.rowptr[row + 1] - e0);
    }
    const int lph = A.d / FPL;
    const int f0 = L.sl * FPL;
    const int h = f0 / A.d;
    float prm_acc = 0.f;
    if (__any(valid)) {
        float qv[FPL];
        ldf<S>(A.q, (int64_t)row * A.ld + f0, qv);
        float qq = 0.f;
        if constexpr (MetricTraits<METRIC>::fam == FAM_COS) qq = grp_sum(dotf(qv, qv), lph);
        const float prm = A.mparam ? A.mparam[h] : 1.f;
        float dq[FPL];
#pragma unroll
        for (int c = 0; c < FPL; ++c) dq[c] = 0.f;
        int mycol = 0;
        for (int jj = 0; __any(jj < cnt); jj += UN) {
            if ((jj % LPR) == 0) {
                const bool in = jj + L.sl < cnt;
                mycol = in ? A.g.col[e0 + jj + L.sl] : 0;
                if (TAGAN_DBAD(mycol >= 0 && mycol < A.g.n_nodes, mycol, row)) mycol = 0;   // gather index
            }
            float kv[UN][FPL], dsv[UN];
#pragma unroll
            for (int u = 0; u < UN; ++u) {
                const int src = L.base + ((jj + u) % LPR);
                const int j = __shfl(mycol, src, WAVE);
                ldf<S>(A.k, (int64_t)j * A.ld + f0, kv[u]);
                dsv[u] = (jj + u < cnt) ? A.ds_edge[(int64_t)(e0 + jj + u) * A.heads + h] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < UN; ++u) {
                const bool live = jj + u < cnt;
                float a, b;
                pair_partial<METRIC, FPL>(qv, kv[u], a, b);
                a = grp_sum(a, lph);
                if constexpr (MetricTraits<METRIC>::fam == FAM_COS) b = grp_sum(b, lph);
                if (!live) continue;
                const float s = finalize<METRIC>(a, b, qq, A.inv_sqrt_d, prm);
                const float ds = dsv[u];
                const Grad g = score_grad<METRIC>(a, b, qq, s, A.inv_sqrt_d, prm);
#pragma unroll
                for (int c = 0; c < FPL; ++c) {
                    const float qc = qv[c], kc = kv[u][c];
                    float t = fmaf(g.cq_q, qc, g.cq_k * kc);
                    if constexpr (MetricTraits<METRIC>::fam == FAM_ABS) t = g.sg * sgnf(qc - kc);
                    dq[c] += ds * t;
                }
                prm_acc = fmaf(ds, g.dprm, prm_acc);
            }
        }
        if (valid) {
            const int part = A.g.row_chunk_part[L.chunk];
            if (TAGAN_DBAD(part < A.g.part_cap, part, A.g.part_cap)) {   // partial slot (no return: a barrier follows)
            } else if (part < 0) stf<S>(A.dq, (int64_t)row * A.ldd + f0, dq);
            else stf<float>(A.part_v, (int64_t)part * A.H + f0, dq);
        }
    }
    if (A.prm_partial) {
        red[threadIdx.x] = (valid && (L.sl % lph) == 0) ? prm_acc : 0.f;
        __syncthreads();
        if (threadIdx.x < A.heads) {
            float sacc = 0.f;
            const int off = threadIdx.x * lph;              // lane of head threadIdx.x inside a group
            for (int w = 0; w < BLK / WAVE; ++w)
                for (int sg = 0; sg < Lanes<LPR>::RPW; ++sg) sacc += red[w * WAVE + sg * LPR + off];
            A.prm_partial[(int64_t)blockIdx.x * A.heads + threadIdx.x] = sacc;
        }
    }
}

// Deterministic reduction of per-block parameter-gradient partials.
__global__ void __launch_bounds__(BLK) k_reduce_partials(const float* __restrict__ part, int64_t nblk, int heads,
                                                         float* __restrict__ out) {
    __shared__ float red[BLK];
    const int h = blockIdx.x;
    float s = 0.f;
    for (int64_t b = threadIdx.x; b < nblk; b += BLK) s += part[b * heads + h];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = BLK / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[h] = red[0];
}

// =================================================================== fallback path (any H, d)
// One thread per (row, head), whole rows, no chunking.  Correct for every shape;
// used only when the fast path's lane geometry does not fit.
template <int METRIC>
__global__ void __launch_bounds__(BLK) k_geo_alpha(GeoArgs A, float* __restrict__ alpha) {
    TAGAN_LIVE_SEED(A);
    const int64_t t = blockIdx.x * (int64_t)BLK + threadIdx.x;
    if (t >= A.N * A.heads) return;
    const int64_t row = t / A.heads;
    const int h = (int)(t % A.heads);
    const float* qr = A.q + row * A.ld + h * A.d;
    float qq = 0.f;
    for (int c = 0; c < A.d; ++c) qq = fmaf(qr[c], qr[c], qq);
    const float prm = A.mparam ? A.mparam[h] : 1.f;
    const float lse = A.lse[row * A.heads + h];
    for (int e = A.g.rowptr[row]; e < A.g.rowptr[row + 1]; ++e) {
        const float* kr = A.k + (int64_t)A.g.col[e] * A.ld + h * A.d;
        float a = 0.f, b = 0.f;
        for (int c = 0; c < A.d; ++c) {
            float qa[1] = {qr[c]}, ka[1] = {kr[c]}, pa, pb;
            pair_partial<METRIC, 1>(qa, ka, pa, pb);
            a += pa;
            b += pb;
        }
        float p = __expf(finalize<METRIC>(a, b, qq, A.inv_sqrt_d, prm) - lse);
        if (A.p_drop > 0.f)
            p = (drop_u(drop_key(A.seed, (uint64_t)h), (uint32_t)e) >= A.p_drop) ? p * A.inv_keep : 0.f;
        alpha[(int64_t)e * A.heads + h] = p;
    }
}

template <int METRIC>
__global__ void __launch_bounds__(BLK) k_geo_fwd_generic(GeoArgs A) {
    TAGAN_LIVE_SEED(A);
    const int64_t t = blockIdx.x * (int64_t)BLK + threadIdx.x;
    if (t >= A.N * A.heads) return;
    const int64_t row = t / A.heads;
    const int h = (int)(t % A.heads);
    const int d = A.d;
    const float* qr = A.q + row * A.ld + h * d;
    float qq = 0.f;
    for (int c = 0; c < d; ++c) qq = fmaf(qr[c], qr[c], qq);
    const float prm = A.mparam ? A.mparam[h] : 1.f;
    float m = -INFINITY, l = 0.f;
    float* orow = A.out + row * (int64_t)A.H + h * d;
    for (int c = 0; c < d; ++c) orow[c] = 0.f;
    for (int e = A.g.rowptr[row]; e < A.g.rowptr[row + 1]; ++e) {
        const int64_t j = A.g.col[e];
        const float* kr = A.k + j * A.ld + h * d;
        const float* vr = A.v + j * A.ld + h * d;
        float a = 0.f, b = 0.f;
        for (int c = 0; c < d; ++c) {
            float qa[1] = {qr[c]}, ka[1] = {kr[c]}, pa, pb;
            pair_partial<METRIC, 1>(qa, ka, pa, pb);
            a += pa;
            b += pb;
        }
        const float s = finalize<METRIC>(a, b, qq, A.inv_sqrt_d, prm);
        const float mn = fmaxf(m, s), corr = __expf(m - mn), p = __expf(s - mn);
        l = fmaf(l, corr, p);
        float pw = p;
        if (A.p_drop > 0.f)
            pw = (drop_u(drop_key(A.seed, (uint64_t)h), (uint32_t)e) >= A.p_drop) ? p * A.inv_keep : 0.f;
        for (int c = 0; c < d; ++c) orow[c] = fmaf(orow[c], corr, pw * vr[c]);
        m = mn;
    }
    for (int c = 0; c < d; ++c) orow[c] = (l > 0.f) ? orow[c] / l : NAN;
    A.lse[row * A.heads + h] = m + __logf(l);
}

template <int METRIC>
__global__ void __launch_bounds__(BLK) k_geo_bwd_row_generic(GeoArgs A) {
    TAGAN_LIVE_SEED(A);
    const int64_t t = blockIdx.x * (int64_t)BLK + threadIdx.x;
    if (t >= A.N * A.heads) return;
    const int64_t row = t / A.heads;
    const int h = (int)(t % A.heads);
    const int d = A.d;
    const float* qr = A.q + row * A.ld + h * d;
    const float* orow = A.o + row * (int64_t)A.H + h * d;
    const float* dor = A.dout + row * (int64_t)A.H + h * d;
    float* dqr = A.dq + row * A.ldd + h * d;
    float D = 0.f, qq = 0.f;
    for (int c = 0; c < d; ++c) {
        D = fmaf(dor[c], orow[c], D);
        qq = fmaf(qr[c], qr[c], qq);
        dqr[c] = 0.f;
    }
    const float prm = A.mparam ? A.mparam[h] : 1.f;
    const float lse = A.lse_in[row * A.heads + h];
    float prm_acc = 0.f;
    for (int e = A.g.rowptr[row]; e < A.g.rowptr[row + 1]; ++e) {
        const int64_t j = A.g.col[e];
        const float* kr = A.k + j * A.ld + h * d;
        const float* vr = A.v + j * A.ld + h * d;
        float a = 0.f, b = 0.f, dp = 0.f;
        for (int c = 0; c < d; ++c) {
            float qa[1] = {qr[c]}, ka[1] = {kr[c]}, pa, pb;
            pair_partial<METRIC, 1>(qa, ka, pa, pb);
            a += pa;
            b += pb;
            dp = fmaf(dor[c], vr[c], dp);
        }
        const float s = finalize<METRIC>(a, b, qq, A.inv_sqrt_d, prm);
        const float p = __expf(s - lse);
        if (A.p_drop > 0.f)
            dp = (drop_u(drop_key(A.seed, (uint64_t)h), (uint32_t)e) >= A.p_drop) ? dp * A.inv_keep : 0.f;
        const float ds = p * (dp - D);
        const Grad g = score_grad<METRIC>(a, b, qq, s, A.inv_sqrt_d, prm);
        for (int c = 0; c < d; ++c) {
            float tt = fmaf(g.cq_q, qr[c], g.cq_k * kr[c]);
            if constexpr (MetricTraits<METRIC>::fam == FAM_ABS) tt = g.sg * sgnf(qr[c] - kr[c]);
            dqr[c] = fmaf(ds, tt, dqr[c]);
        }
        prm_acc = fmaf(ds, g.dprm, prm_acc);
    }
    A.delta[(row * A.heads + h) * 2] = lse;
    A.delta[(row * A.heads + h) * 2 + 1] = D;
    if (A.prm_partial) A.prm_partial[t] = prm_acc;   // [N*heads] partials, reduced per head
}

template <int METRIC>
__global__ void __launch_bounds__(BLK) k_geo_bwd_col_generic(GeoArgs A) {
    TAGAN_LIVE_SEED(A);
    const int64_t t = blockIdx.x * (int64_t)BLK + threadIdx.x;
    if (t >= A.N * A.heads) return;
    const int64_t colj = t / A.heads;
    const int h = (int)(t % A.heads);
    const int d = A.d;
    const float* kr = A.k + colj * A.ld + h * d;
    const float* vr = A.v + colj * A.ld + h * d;
    float* dkr = A.dk + colj * A.ldd + h * d;
    float* dvr = A.dv + colj * A.ldd + h * d;
    for (int c = 0; c < d; ++c) { dkr[c] = 0.f; dvr[c] = 0.f; }
    const float prm = A.mparam ? A.mparam[h] : 1.f;
    for (int e = A.g.csc_ptr[colj]; e < A.g.csc_ptr[colj + 1]; ++e) {
        const int64_t i = A.g.csc_row[e];
        const int eid = A.g.csc_eid[e];
        const float* qr = A.q + i * A.ld + h * d;
        const float* dor = A.dout + i * (int64_t)A.H + h * d;
        float a = 0.f, b = 0.f, dp = 0.f, qq = 0.f;
        for (int c = 0; c < d; ++c) {
            float qa[1] = {qr[c]}, ka[1] = {kr[c]}, pa, pb;
            pair_partial<METRIC, 1>(qa, ka, pa, pb);
            a += pa;
            b += pb;
            dp = fmaf(dor[c], vr[c], dp);
            qq = fmaf(qr[c], qr[c], qq);
        }
        const float s = finalize<METRIC>(a, b, qq, A.inv_sqrt_d, prm);
        const float p = __expf(s - A.lse_in[i * A.heads + h]);
        float pw = p;
        if (A.p_drop > 0.f) {
            const bool keep = drop_u(drop_key(A.seed, (uint64_t)h), (uint32_t)eid) >= A.p_drop;
            dp = keep ? dp * A.inv_keep : 0.f;
            pw = keep ? p * A.inv_keep : 0.f;
        }
        const float ds = p * (dp - A.delta[(i * A.heads + h) * 2 + 1]);
        const Grad g = score_grad<METRIC>(a, b, qq, s, A.inv_sqrt_d, prm);
        for (int c = 0; c < d; ++c) {
            float tt = fmaf(g.ck_q, qr[c], g.ck_k * kr[c]);
            if constexpr (MetricTraits<METRIC>::fam == FAM_ABS) tt = -g.sg * sgnf(qr[c] - kr[c]);
            dkr[c] = fmaf(ds, tt, dkr[c]);
            dvr[c] = fmaf(pw, dor[c], dvr[c]);
        }
    }
}

// =================================================================== dispatch
// Fast path: H in {32, 64, 128, 256}, d = 4*LPH with LPH a power of two.  A lane owns FPL
// features: FPL = 8 (LPR = H/8 lanes per chunk group) where d % 8 == 0 and H >= 64 for the
// passes TAGAN_GEO_FPL_* select, else 4.  Measured at C2/C4 (tools/geo_kernels.py):
// the forward gains from 8 (more chunks per wave in flight); the fp32 backward passes, whose
// register footprint at FPL = 8 halves the occupancy, do not (C2 0.74 vs 0.755 ms); in bf16 storage
// they do: 16-B instead of 8-B loads per lane, C2 bwd 0.63 -> 0.53 ms, C4 83.5 -> 76.1 ms
// (profiles/r4g8_geo_fpl_bwd_ab.txt).
#ifndef TAGAN_GEO_FPL_FWD
#define TAGAN_GEO_FPL_FWD 8
#endif
#ifndef TAGAN_GEO_FPL_BWD
#define TAGAN_GEO_FPL_BWD 4
#endif
#ifndef TAGAN_GEO_FPL_BWD_BF16
#define TAGAN_GEO_FPL_BWD_BF16 8
#endif

enum Pass { P_FWD, P_BWD_ROW, P_BWD_COL, P_ALPHA, P_BWD_DELTA, P_BWD_ROW_DS };

int pick_lpr(int H, int d) {   // nonzero = fast path
    if (d % 4 != 0) return 0;
    const int lph = d / 4;
    if (lph & (lph - 1)) return 0;
    if (H == 32 || H == 64 || H == 128 || H == 256) return H / 4;
    return 0;
}

// A batch is cache-cold when its K and V node rows exceed 512 MB (kv_cold, also geo_xcd_mode's default rule).  The
// forward then takes 4 features per lane: twice the lanes per chunk keep more gathers in flight against HBM (fp32
// C4 3.65-3.69 -> 3.51 ms, neutral at C2: profiles/r5zp_geo_fpl_ab.txt; bf16 C5 38.6 -> 38.1 ms,
// profiles/r6h_cold_fpl.txt).  Keyed on the batch, not on the block order, so forcing an order (TAGAN_GEO_XCD) never
// changes the lane reduction.  TAGAN_GEO_FPL_FWD_COLD=4|8 overrides the cold choice (read per call: A/B runs);
// TAGAN_GEO_COLD=0|1 forces the classification (tests: the cold forward on small graphs).
bool kv_cold(int64_t n, int H, bool bf16) {
    const char* e = getenv("TAGAN_GEO_COLD");
    if (e && (e[0] == '0' || e[0] == '1') && !e[1]) return e[0] == '1';
    return 2 * n * (int64_t)H * (bf16 ? 2 : 4) > ((int64_t)512 << 20);
}

int pick_fpl(int H, int d, Pass pass, bool bf16, bool cold = false) {
    int want = pass == P_FWD ? TAGAN_GEO_FPL_FWD : bf16 ? TAGAN_GEO_FPL_BWD_BF16 : TAGAN_GEO_FPL_BWD;
    if (pass == P_FWD && cold) {
        const char* e = getenv("TAGAN_GEO_FPL_FWD_COLD");
        want = (e && (e[0] == '4' || e[0] == '8') && !e[1]) ? e[0] - '0' : 4;
    }
    if (want == 8 && d % 8 == 0 && ((d / 8) & (d / 8 - 1)) == 0 && (H == 64 || H == 128 || H == 256)) return 8;
    return 4;
}

int64_t chunk_blocks(const GeoArgs& A, int lpr) {
    const int64_t rpw = WAVE / lpr;
    const int64_t waves = (A.g.chunk_cap + rpw - 1) / rpw;
    return std::max<int64_t>(1, (waves + (BLK / WAVE) - 1) / (BLK / WAVE));
}

template <int METRIC, int LPR, int FPL, typename S>
void launch_fast_s(Pass pass, const GeoArgs& A, hipStream_t s) {
    const dim3 g((unsigned)chunk_blocks(A, LPR));
    if (pass == P_FWD) k_geo_fwd_chunk<METRIC, LPR, FPL, S><<<g, BLK, 0, s>>>(A);
    else if (pass == P_BWD_ROW) k_geo_bwd_row_chunk<METRIC, LPR, FPL, S><<<g, BLK, 0, s>>>(A);
    else if (pass == P_BWD_ROW_DS) k_geo_bwd_row_ds<METRIC, LPR, FPL, S><<<g, BLK, 0, s>>>(A);
    else if (pass == P_BWD_DELTA) {
        const int64_t waves = (A.N + (WAVE / LPR) - 1) / (WAVE / LPR);
        k_geo_bwd_delta<LPR, FPL, S><<<(unsigned)((waves + (BLK / WAVE) - 1) / (BLK / WAVE)), BLK, 0, s>>>(A);
    } else k_geo_bwd_col_chunk<METRIC, LPR, FPL, S><<<g, BLK, 0, s>>>(A);
}

template <int METRIC, int LPR, int FPL>
void launch_fast(Pass pass, const GeoArgs& A, hipStream_t s) {
    if (A.bf16) launch_fast_s<METRIC, LPR, FPL, bf16s>(pass, A, s);
    else launch_fast_s<METRIC, LPR, FPL, float>(pass, A, s);
}

template <int METRIC>
int launch_metric(Pass pass, int lpr, const GeoArgs& A, hipStream_t s, float* alpha) {
    const dim3 gg((unsigned)((A.N * A.heads + BLK - 1) / BLK));
    if (pass == P_ALPHA) {
        k_geo_alpha<METRIC><<<gg, BLK, 0, s>>>(A, alpha);
        return TAGAN_OK;
    }
    const int fpl = lpr ? pick_fpl(A.H, A.d, pass, A.bf16 != 0, kv_cold(A.N, A.H, A.bf16 != 0)) : 0;
    lpr = lpr ? A.H / fpl : 0;
    if (fpl == 8) {
        switch (lpr) {
            case 8: launch_fast<METRIC, 8, 8>(pass, A, s); return TAGAN_OK;
            case 16: launch_fast<METRIC, 16, 8>(pass, A, s); return TAGAN_OK;
            case 32: launch_fast<METRIC, 32, 8>(pass, A, s); return TAGAN_OK;
            default: break;
        }
    } else {
        switch (lpr) {
            case 8: launch_fast<METRIC, 8, 4>(pass, A, s); return TAGAN_OK;
            case 16: launch_fast<METRIC, 16, 4>(pass, A, s); return TAGAN_OK;
            case 32: launch_fast<METRIC, 32, 4>(pass, A, s); return TAGAN_OK;
            case 64: launch_fast<METRIC, 64, 4>(pass, A, s); return TAGAN_OK;
            default: break;
        }
    }
    if (pass == P_FWD) k_geo_fwd_generic<METRIC><<<gg, BLK, 0, s>>>(A);
    else if (pass == P_BWD_ROW) k_geo_bwd_row_generic<METRIC><<<gg, BLK, 0, s>>>(A);
    else k_geo_bwd_col_generic<METRIC><<<gg, BLK, 0, s>>>(A);
    return TAGAN_OK;
}

int launch(int metric, Pass pass, int lpr, const GeoArgs& A, hipStream_t s, float* alpha = nullptr) {
    switch (metric) {
        case TAGAN_METRIC_EUCLIDEAN: return launch_metric<TAGAN_METRIC_EUCLIDEAN>(pass, lpr, A, s, alpha);
        case TAGAN_METRIC_SQUARED_EUCLIDEAN:
            return launch_metric<TAGAN_METRIC_SQUARED_EUCLIDEAN>(pass, lpr, A, s, alpha);
        case TAGAN_METRIC_MANHATTAN: return launch_metric<TAGAN_METRIC_MANHATTAN>(pass, lpr, A, s, alpha);
        case TAGAN_METRIC_COSINE_SIMILARITY:
            return launch_metric<TAGAN_METRIC_COSINE_SIMILARITY>(pass, lpr, A, s, alpha);
        case TAGAN_METRIC_COSINE_DISTANCE:
            return launch_metric<TAGAN_METRIC_COSINE_DISTANCE>(pass, lpr, A, s, alpha);
        case TAGAN_METRIC_DOT_PRODUCT: return launch_metric<TAGAN_METRIC_DOT_PRODUCT>(pass, lpr, A, s, alpha);
        case TAGAN_METRIC_SCALED_DOT_PRODUCT:
            return launch_metric<TAGAN_METRIC_SCALED_DOT_PRODUCT>(pass, lpr, A, s, alpha);
        case TAGAN_METRIC_GAUSSIAN_KERNEL:
            return launch_metric<TAGAN_METRIC_GAUSSIAN_KERNEL>(pass, lpr, A, s, alpha);
        case TAGAN_METRIC_RBF_KERNEL: return launch_metric<TAGAN_METRIC_RBF_KERNEL>(pass, lpr, A, s, alpha);
        default:
            set_error("geo_attn: unsupported metric %d", metric);
            return TAGAN_ERR_UNSUPPORTED;
    }
}

int check_common(int dtype, int metric, const tagan_graph* g, int heads, int d, int64_t ld, float p_drop) {
    TAGAN_REQUIRE(dtype == TAGAN_F32 || (dtype == TAGAN_BF16 && pick_lpr(heads * d, d) != 0),
                  TAGAN_ERR_UNSUPPORTED, "geo_attn: dtype %d unsupported for H=%d d=%d", dtype, heads * d, d);
    TAGAN_REQUIRE(metric >= 0 && metric <= TAGAN_METRIC_RBF_KERNEL, TAGAN_ERR_UNSUPPORTED,
                  "geo_attn: unsupported metric %d", metric);
    TAGAN_REQUIRE(g != nullptr && g->n_nodes > 0 && g->rowptr && g->col, TAGAN_ERR_ARG, "geo_attn: bad graph");
    TAGAN_REQUIRE(heads > 0 && d > 0, TAGAN_ERR_ARG, "geo_attn: bad sizes heads=%d d=%d", heads, d);
    TAGAN_REQUIRE(ld >= (int64_t)heads * d, TAGAN_ERR_ARG, "geo_attn: ld %lld < H", (long long)ld);
    TAGAN_REQUIRE(p_drop >= 0.f && p_drop < 1.f, TAGAN_ERR_ARG, "geo_attn: p_drop %f", (double)p_drop);
    const int lpr = pick_lpr(heads * d, d);
    if (lpr) {
        TAGAN_REQUIRE(g->chunk > 0 && g->chunk_cap > 0 && g->row_chunk_ptr && g->row_chunk_seg &&
                          g->row_chunk_beg && g->row_chunk_part && g->row_multi && g->row_counts,
                      TAGAN_ERR_ARG, "geo_attn: graph lacks row chunk lists");
        TAGAN_REQUIRE(((uintptr_t)0 == (ld % 4)), TAGAN_ERR_ARG, "geo_attn: ld must be a multiple of 4");
    }
    return TAGAN_OK;
}

// Block order of the chunk kernels (Lanes).  Launch order (0) when the gathered K | V rows of the whole batch exceed
// what the 256 MB Infinity Cache can hold: every XCD then works on the same stretch of rows -- one snapshot's
// neighbourhoods at a time -- and the gathers share that cache; with XCD-contiguous eighths each XCD streams its own
// region and the eight regions' K | V evict one another.  XCD-contiguous over the valid blocks (2) when the whole
// batch fits (C2).  Edge kernels alone, fwd / bwd ms, shipped map (1) -> chosen order (profiles/r5u_geo_xcd_ab.txt):
// C2 0.296 / 0.745 -> 0.281 / 0.706, C3 50.1 / 86.8 -> 38.7 / 66.5, C4 68.2 / 128.4 -> 57.3 / 105.9, C5 bf16
// 48.3 / 97.4 -> 38.0 / 75.4.  TAGAN_GEO_XCD=0|1|2 forces one (read per call: A/B runs, tests).
// The test is on the batch's K and V NODE rows (2·N·H·bytes, the distinct rows the gathers can touch), not on the
// gathered bytes, against 512 MB (twice the cache): a separator between the measured cases, not the cache size.  C2's
// node rows are 328 MB -- more than the cache -- yet XCD-contiguous order wins there, because each XCD's eighth of
// the blocks touches only its own ~41 MB of K | V, which its share of the cache holds; C3-C5 (6.5-13 GB) gain from
// launch order.  A batch between 256 and 512 MB has not been measured.
int geo_xcd_mode(int64_t n, int H, bool bf16) {
    const char* e = getenv("TAGAN_GEO_XCD");
    if (e && e[0] >= '0' && e[0] <= '2' && !e[1]) return e[0] - '0';
    return kv_cold(n, H, bf16) ? 0 : 2;
}

GeoArgs make_args(const tagan_graph* g, int heads, int d, const void* q, const void* k, const void* v, int64_t ld,
                  const float* mparam, float p_drop, uint64_t seed) {
    GeoArgs A{};
    A.g = *g;
    A.N = g->n_nodes;
    A.heads = heads;
    A.d = d;
    A.H = heads * d;
    const int lpr = pick_lpr(A.H, d);
    A.lph = lpr ? d / 4 : 1;
    A.q = (const float*)q;
    A.k = (const float*)k;
    A.v = (const float*)v;
    A.ld = ld;
    A.mparam = mparam;
    A.p_drop = p_drop;
    A.inv_keep = 1.f / (1.f - p_drop);
    A.seed = seed; A.seed_ctr = seed_counter();
    A.inv_sqrt_d = 1.f / sqrtf((float)d);
    return A;
}

size_t fwd_ws(const tagan_graph* g, int heads, int d) {
    if (!pick_lpr(heads * d, d)) return 0;
    return align_up((size_t)g->part_cap * (2 * heads + heads * d) * 4, 256);
}

struct BwdWs {
    size_t delta, prm, pv, pv2, ds, total;
    bool col_first;
};

// Backward order.  Column-first (node pass -> column pass storing dS -> row pass from dS) saves the row pass's V_j
// gathers at the price of a node pass over O and dO and a dS round trip; it pays where the gathers miss the caches:
// C4 backward 8.8 -> 7.7 ms, while at C2 (its K|V rows mostly served by L2 / Infinity Cache) it measured 0.04 ms per
// layer slower (profiles/r2_geo_bwd_order_ab.txt).  Default: column-first when the graph's K|V rows at fp32
// (N·H·8 bytes) exceed 512 MB, twice the 256-MB Infinity Cache.  tagan_geo_set_bwd_order() forces an order (A/B
// runs and the order-equivalence test).  The choice depends on the graph and H only,
// so the workspace query agrees with the call.
int g_bwd_order = 2;

bool col_first_wanted(int64_t N, int H) {
    const int mode = __atomic_load_n(&g_bwd_order, __ATOMIC_RELAXED);
    return mode == 2 ? (double)N * H * 8.0 > 512.0 * 1024 * 1024 : mode == 1;
}

BwdWs bwd_ws(const tagan_graph* g, int heads, int d) {
    BwdWs w{};
    const int H = heads * d;
    const int lpr = pick_lpr(H, d);
    size_t off = 0;
    auto take = [&](size_t b) { size_t o = off; off = align_up(off + b, 256); return o; };
    w.delta = take((size_t)g->n_nodes * heads * 8);   // packed {lse, delta} per (node, head)
    int64_t nprm = g->n_nodes;
    if (lpr) {
        GeoArgs tmp{};
        tmp.g = *g;
        // the row pass's partial rows under either storage type (the workspace query does not know it)
        nprm = std::max<int64_t>(nprm, chunk_blocks(tmp, H / pick_fpl(H, d, P_BWD_ROW, false)));
        nprm = std::max<int64_t>(nprm, chunk_blocks(tmp, H / pick_fpl(H, d, P_BWD_ROW, true)));
    }
    w.prm = take((size_t)nprm * heads * 4);
    w.pv = take(lpr ? (size_t)g->part_cap * H * 4 : 0);
    w.pv2 = take(lpr ? (size_t)g->part_cap * 2 * H * 4 : 0);
    w.col_first = lpr && g->nnz_cap > 0 && col_first_wanted(g->n_nodes, H);
    w.ds = take(w.col_first ? (size_t)g->nnz_cap * heads * 4 : 0);
    w.total = off;
    return w;
}

}  // namespace
}  // namespace tagan

extern "C" {

size_t tagan_geo_attn_fwd_workspace(const tagan_graph* g, int32_t heads, int32_t head_dim) {
    if (!g || heads <= 0 || head_dim <= 0) return 0;
    return tagan::fwd_ws(g, heads, head_dim);
}

int tagan_geo_attn_fwd(int dtype, int metric, const tagan_graph* g, int32_t heads, int32_t head_dim, const void* q,
                       const void* k, const void* v, int64_t ld_qkv, const float* metric_param, float p_drop,
                       uint64_t seed, void* out, float* lse, float* edge_alpha, void* workspace,
                       size_t workspace_bytes, void* stream) {
    using namespace tagan;
    int rc = check_common(dtype, metric, g, heads, head_dim, ld_qkv, p_drop);
    if (rc) return rc;
    TAGAN_REQUIRE(q && k && v && out && lse, TAGAN_ERR_ARG, "geo_attn_fwd: null pointer");
    const size_t need = fwd_ws(g, heads, head_dim);
    TAGAN_REQUIRE(need == 0 || (workspace && workspace_bytes >= need), TAGAN_ERR_WORKSPACE,
                  "geo_attn_fwd: workspace %zu < %zu", workspace_bytes, need);
    TAGAN_REQUIRE(!(dtype == TAGAN_BF16 && edge_alpha), TAGAN_ERR_UNSUPPORTED, "geo_attn_fwd: edge_alpha needs fp32");
    GeoArgs A = make_args(g, heads, head_dim, q, k, v, ld_qkv, metric_param, p_drop, seed);
    A.bf16 = dtype == TAGAN_BF16;
    A.xcd = geo_xcd_mode(A.N, A.H, A.bf16 != 0);
    A.out = (float*)out;
    A.lse = lse;
    if (need) {
        A.part_m = (float*)workspace;
        A.part_l = A.part_m + g->part_cap * heads;
        A.part_v = A.part_l + g->part_cap * heads;
    }
    hipStream_t s = as_stream(stream);
    const int lpr = pick_lpr(A.H, head_dim);
    rc = launch(metric, P_FWD, lpr, A, s);
    if (rc) return rc;
    TAGAN_CHECK_LAUNCH("geo_attn_fwd");
    if (lpr) {
        const unsigned gm = merge_grid(g->part_cap);
        geo_mg_dispatch(true, [&](auto g) {
            constexpr int G = decltype(g)::value;
            if (A.bf16) k_geo_fwd_merge<G, bf16s><<<gm, BLK, 0, s>>>(A);
            else k_geo_fwd_merge<G, float><<<gm, BLK, 0, s>>>(A);
        });
        TAGAN_CHECK_LAUNCH("geo_attn_fwd_merge");
    }
    if (edge_alpha) {
        rc = launch(metric, P_ALPHA, lpr, A, s, edge_alpha);
        if (rc) return rc;
        TAGAN_CHECK_LAUNCH("geo_attn_alpha");
    }
    return TAGAN_OK;
}

int tagan_geo_set_bwd_order(int32_t mode) {
    TAGAN_REQUIRE(mode >= 0 && mode <= 2, TAGAN_ERR_ARG, "geo_set_bwd_order: mode %d", mode);
    return __atomic_exchange_n(&tagan::g_bwd_order, mode, __ATOMIC_RELAXED);
}

size_t tagan_geo_attn_bwd_workspace(const tagan_graph* g, int32_t heads, int32_t head_dim) {
    if (!g || g->n_nodes <= 0 || heads <= 0 || head_dim <= 0) return 0;
    return tagan::bwd_ws(g, heads, head_dim).total;
}

int tagan_geo_attn_bwd(int dtype, int metric, const tagan_graph* g, int32_t heads, int32_t head_dim, const void* q,
                       const void* k, const void* v, int64_t ld_qkv, const float* metric_param, float p_drop,
                       uint64_t seed, const void* out, const float* lse, const void* dout, void* dq, void* dk,
                       void* dv, int64_t ld_dqkv, float* dmetric_param, void* workspace, size_t workspace_bytes,
                       void* stream) {
    using namespace tagan;
    int rc = check_common(dtype, metric, g, heads, head_dim, ld_qkv, p_drop);
    if (rc) return rc;
    TAGAN_REQUIRE(g->csc_ptr && g->csc_row && g->csc_eid && q && k && v && out && lse && dout && dq && dk && dv,
                  TAGAN_ERR_ARG, "geo_attn_bwd: null pointer");
    TAGAN_REQUIRE(ld_dqkv >= (int64_t)heads * head_dim && ld_dqkv % 4 == 0, TAGAN_ERR_ARG, "geo_attn_bwd: ld_dqkv");
    const BwdWs w = bwd_ws(g, heads, head_dim);
    TAGAN_REQUIRE(workspace && workspace_bytes >= w.total, TAGAN_ERR_WORKSPACE, "geo_attn_bwd: workspace %zu < %zu",
                  workspace_bytes, w.total);
    const int H = heads * head_dim;
    const int lpr = pick_lpr(H, head_dim);
    if (lpr) {
        TAGAN_REQUIRE(g->col_chunk_ptr && g->col_chunk_seg && g->col_chunk_beg && g->col_chunk_part &&
                          g->col_multi && g->col_counts,
                      TAGAN_ERR_ARG, "geo_attn_bwd: graph lacks column chunk lists");
    }
    GeoArgs A = make_args(g, heads, head_dim, q, k, v, ld_qkv, metric_param, p_drop, seed);
    A.bf16 = dtype == TAGAN_BF16;
    A.xcd = geo_xcd_mode(A.N, A.H, A.bf16 != 0);
    A.o = (const float*)out;
    A.lse_in = lse;
    A.dout = (const float*)dout;
    A.dq = (float*)dq;
    A.dk = (float*)dk;
    A.dv = (float*)dv;
    A.ldd = ld_dqkv;
    char* ws = (char*)workspace;
    A.delta = (float*)(ws + w.delta);
    const bool want_prm = dmetric_param != nullptr && metric_param != nullptr &&
                          (metric == TAGAN_METRIC_GAUSSIAN_KERNEL || metric == TAGAN_METRIC_RBF_KERNEL);
    A.prm_partial = want_prm ? (float*)(ws + w.prm) : nullptr;
    A.part_v = (float*)(ws + w.pv);
    A.part_v2 = (float*)(ws + w.pv2);
    hipStream_t s = as_stream(stream);
    const unsigned gm = merge_grid(g->part_cap);
    auto sum_cols = [&]() {
        geo_mg_dispatch(false, [&](auto gg) {
            constexpr int G = decltype(gg)::value;
            if (A.bf16)
                k_geo_sum_parts<G, bf16s><<<gm, BLK, 0, s>>>(g->col_counts, g->col_multi, g->col_chunk_ptr,
                                                             g->col_chunk_part, A.part_v2, 2 * H, A.dk, A.dv, A.ldd, H);
            else
                k_geo_sum_parts<G, float><<<gm, BLK, 0, s>>>(g->col_counts, g->col_multi, g->col_chunk_ptr,
                                                             g->col_chunk_part, A.part_v2, 2 * H, A.dk, A.dv, A.ldd, H);
        });
        return hipGetLastError();
    };
    auto sum_rows = [&]() {
        geo_mg_dispatch(false, [&](auto gg) {
            constexpr int G = decltype(gg)::value;
            if (A.bf16)
                k_geo_sum_parts<G, bf16s><<<gm, BLK, 0, s>>>(g->row_counts, g->row_multi, g->row_chunk_ptr,
                                                             g->row_chunk_part, A.part_v, H, A.dq, A.dq, A.ldd, H);
            else
                k_geo_sum_parts<G, float><<<gm, BLK, 0, s>>>(g->row_counts, g->row_multi, g->row_chunk_ptr,
                                                             g->row_chunk_part, A.part_v, H, A.dq, A.dq, A.ldd, H);
        });
        return hipGetLastError();
    };
    if (w.col_first) {
        A.ds_edge = (float*)(ws + w.ds);
        rc = launch(metric, P_BWD_DELTA, lpr, A, s);
        if (rc) return rc;
        TAGAN_CHECK_LAUNCH("geo_attn_bwd_delta");
        rc = launch(metric, P_BWD_COL, lpr, A, s);
        if (rc) return rc;
        TAGAN_CHECK_LAUNCH("geo_attn_bwd_col");
        TAGAN_CHECK_HIP(sum_cols(), "geo_attn_bwd_col_merge");
        rc = launch(metric, P_BWD_ROW_DS, lpr, A, s);
        if (rc) return rc;
        TAGAN_CHECK_LAUNCH("geo_attn_bwd_row_ds");
        TAGAN_CHECK_HIP(sum_rows(), "geo_attn_bwd_row_merge");
    } else {   // row pass (dq, delta) -> column pass (dk, dv)
        rc = launch(metric, P_BWD_ROW, lpr, A, s);
        if (rc) return rc;
        TAGAN_CHECK_LAUNCH("geo_attn_bwd_row");
        if (lpr) TAGAN_CHECK_HIP(sum_rows(), "geo_attn_bwd_row_merge");
        rc = launch(metric, P_BWD_COL, lpr, A, s);
        if (rc) return rc;
        TAGAN_CHECK_LAUNCH("geo_attn_bwd_col");
        if (lpr) TAGAN_CHECK_HIP(sum_cols(), "geo_attn_bwd_col_merge");
    }
    if (dmetric_param) {
        if (want_prm) {
            const int64_t nparts = lpr ? chunk_blocks(A, H / pick_fpl(H, head_dim, P_BWD_ROW, A.bf16 != 0)) : g->n_nodes;
            k_reduce_partials<<<heads, BLK, 0, s>>>(A.prm_partial, nparts, heads, dmetric_param);
            TAGAN_CHECK_LAUNCH("geo_attn_bwd_reduce");
        } else {
            TAGAN_CHECK_HIP(hipMemsetAsync(dmetric_param, 0, sizeof(float) * heads, s), "memset dparam");
        }
    }
    return TAGAN_OK;
}

}  // extern "C"
