// Geometric (edge-softmax) attention for TAGAN on gfx950.
//
// Replaces geometric_attention.py:332-516 (_get_attention_weights: metric scores,
// masked_fill(-inf) with the dense adjacency of graph_attention.py:96-105,
// softmax, attn_dropout) and :579-583 (A·V), for rows = CSR rows = src = query.
//
// Layout: one wave64 per query row, all heads at once.  Lane l owns features
// [l*VEC, l*VEC+VEC) of the H = heads*d row, so a head is an aligned group of
// LPH = d/VEC lanes and per-head reductions are XOR butterflies inside the
// group.  K/V rows of neighbours are gathered as whole coalesced rows
// (64 lanes x VEC floats); the neighbour index is read once per 64 edges with a
// coalesced load and broadcast with v_readlane (scalar base address).  Softmax
// is online (running max / sum per head), so scores are never stored; the row's
// log-sum-exp is saved for the backward pass.  HBM-bound: algorithmic bytes per
// (layer, snapshot) in DESIGN.md §4.
//
// Backward (atomic-free, bitwise deterministic):
//   row pass (CSR):    delta_i = Σ_f dO_i·O_i per head, dq_i = Σ_j ds_ij ∂s/∂q_i
//   column pass (CSC): dk_j = Σ_i ds_ij ∂s/∂k_j,  dv_j = Σ_i α'_ij dO_i
// with ds_ij = α_ij (dα'_ij·v_j·mask/(1-p) − delta_i), α recomputed from LSE.
#include "common.cuh"

namespace tagan {
namespace {

constexpr int BLK = 256;
constexpr int ROWS_PER_BLK = BLK / WAVE;

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

__device__ __forceinline__ float grp_sum(float x, int lph) {
    for (int o = 1; o < lph; o <<= 1) x += __shfl_xor(x, o, 64);
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
    if constexpr (METRIC == TAGAN_METRIC_EUCLIDEAN) return -sqrtf(a + 1e-8f);
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
        if constexpr (METRIC == TAGAN_METRIC_EUCLIDEAN) c = 1.f / s;           // s = -r  ->  -(q-k)/r
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
    int64_t N;
    int heads, d, lph, H;
    const int32_t* rowptr;
    const int32_t* col;
    const int32_t* csc_ptr;
    const int32_t* csc_row;
    const int32_t* csc_eid;
    const float* q;
    const float* k;
    const float* v;
    int64_t ld;
    const float* mparam;
    float p_drop, inv_keep;
    uint64_t seed;
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
    float* prm_partial;
    float inv_sqrt_d;
};

constexpr int UNROLL = 4;

// ------------------------------------------------------------------ forward
template <int METRIC, int VEC>
__global__ void __launch_bounds__(BLK) k_geo_fwd(GeoArgs A) {
    const int lane = threadIdx.x & (WAVE - 1);
    const int64_t row = xcd_remap(blockIdx.x, gridDim.x) * ROWS_PER_BLK + (threadIdx.x >> 6);
    if (row >= A.N) return;
    const int f0 = lane * VEC;
    const bool active = f0 < A.H;
    const int fo = active ? f0 : 0;
    const int h = fo / A.d;
    float qv[VEC];
    load_vec<VEC>(A.q + row * A.ld + fo, qv);
    float qq = 0.f;
    if constexpr (MetricTraits<METRIC>::fam == FAM_COS) {
#pragma unroll
        for (int c = 0; c < VEC; ++c) qq = fmaf(qv[c], qv[c], qq);
        qq = grp_sum(active ? qq : 0.f, A.lph);
    }
    const float prm = A.mparam ? A.mparam[h] : 1.f;
    float m = -INFINITY, l = 0.f, acc[VEC];
#pragma unroll
    for (int c = 0; c < VEC; ++c) acc[c] = 0.f;
    const int e0 = A.rowptr[row], e1 = A.rowptr[row + 1];
    for (int base = e0; base < e1; base += WAVE) {
        const int cnt = min(WAVE, e1 - base);
        const int mycol = (lane < cnt) ? A.col[base + lane] : 0;
        for (int jj = 0; jj < cnt; jj += UNROLL) {
            float kv[UNROLL][VEC], vv[UNROLL][VEC];
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) {
                const int src_lane = min(jj + u, cnt - 1);
                const int j = __builtin_amdgcn_readlane(mycol, src_lane);
                load_vec<VEC>(A.k + (int64_t)j * A.ld + fo, kv[u]);
                load_vec<VEC>(A.v + (int64_t)j * A.ld + fo, vv[u]);
            }
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) {
                if (jj + u >= cnt) break;
                float a, b;
                pair_partial<METRIC, VEC>(qv, kv[u], a, b);
                a = grp_sum(a, A.lph);
                if constexpr (MetricTraits<METRIC>::fam == FAM_COS) b = grp_sum(b, A.lph);
                const float s = finalize<METRIC>(a, b, qq, A.inv_sqrt_d, prm);
                const float mn = fmaxf(m, s);
                const float corr = __expf(m - mn);
                const float p = __expf(s - mn);
                l = fmaf(l, corr, p);
                float pw = p;
                if (A.p_drop > 0.f) {
                    const uint64_t idx = (uint64_t)(base + jj + u) * (uint64_t)A.heads + (uint64_t)h;
                    pw = (uniform01(A.seed, idx) >= A.p_drop) ? p * A.inv_keep : 0.f;
                }
#pragma unroll
                for (int c = 0; c < VEC; ++c) acc[c] = fmaf(acc[c], corr, pw * vv[u][c]);
                m = mn;
            }
        }
    }
    if (!active) return;
    const float inv_l = 1.f / l;   // l == 0 (no entries) -> NaN output, as softmax over all -inf
    float r[VEC];
#pragma unroll
    for (int c = 0; c < VEC; ++c) r[c] = (l > 0.f) ? acc[c] * inv_l : NAN;
    store_vec<VEC>(A.out + row * (int64_t)A.H + f0, r);
    if ((lane % A.lph) == 0) A.lse[row * A.heads + h] = m + __logf(l);
}

// ------------------------------------------------------------------ backward, row pass
template <int METRIC, int VEC>
__global__ void __launch_bounds__(BLK) k_geo_bwd_row(GeoArgs A) {
    __shared__ float red[ROWS_PER_BLK][64];
    const int lane = threadIdx.x & (WAVE - 1);
    const int wid = threadIdx.x >> 6;
    const int64_t blk = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t row = blk * ROWS_PER_BLK + wid;
    const int f0 = lane * VEC;
    const bool active = f0 < A.H;
    const int fo = active ? f0 : 0;
    const int h = fo / A.d;
    float prm_acc = 0.f;
    if (row < A.N) {
        float qv[VEC], ov[VEC], dov[VEC];
        load_vec<VEC>(A.q + row * A.ld + fo, qv);
        load_vec<VEC>(A.o + row * (int64_t)A.H + fo, ov);
        load_vec<VEC>(A.dout + row * (int64_t)A.H + fo, dov);
        float D = 0.f;
#pragma unroll
        for (int c = 0; c < VEC; ++c) D = fmaf(dov[c], ov[c], D);
        D = grp_sum(active ? D : 0.f, A.lph);
        float qq = 0.f;
        if constexpr (MetricTraits<METRIC>::fam == FAM_COS) {
#pragma unroll
            for (int c = 0; c < VEC; ++c) qq = fmaf(qv[c], qv[c], qq);
            qq = grp_sum(active ? qq : 0.f, A.lph);
        }
        const float lse = A.lse_in[row * A.heads + h];
        const float prm = A.mparam ? A.mparam[h] : 1.f;
        float dqa[VEC];
#pragma unroll
        for (int c = 0; c < VEC; ++c) dqa[c] = 0.f;
        const int e0 = A.rowptr[row], e1 = A.rowptr[row + 1];
        for (int base = e0; base < e1; base += WAVE) {
            const int cnt = min(WAVE, e1 - base);
            const int mycol = (lane < cnt) ? A.col[base + lane] : 0;
            for (int jj = 0; jj < cnt; jj += UNROLL) {
                float kv[UNROLL][VEC], vv[UNROLL][VEC];
#pragma unroll
                for (int u = 0; u < UNROLL; ++u) {
                    const int j = __builtin_amdgcn_readlane(mycol, min(jj + u, cnt - 1));
                    load_vec<VEC>(A.k + (int64_t)j * A.ld + fo, kv[u]);
                    load_vec<VEC>(A.v + (int64_t)j * A.ld + fo, vv[u]);
                }
#pragma unroll
                for (int u = 0; u < UNROLL; ++u) {
                    if (jj + u >= cnt) break;
                    float a, b, dp = 0.f;
                    pair_partial<METRIC, VEC>(qv, kv[u], a, b);
#pragma unroll
                    for (int c = 0; c < VEC; ++c) dp = fmaf(dov[c], vv[u][c], dp);
                    a = grp_sum(a, A.lph);
                    dp = grp_sum(dp, A.lph);
                    if constexpr (MetricTraits<METRIC>::fam == FAM_COS) b = grp_sum(b, A.lph);
                    const float s = finalize<METRIC>(a, b, qq, A.inv_sqrt_d, prm);
                    const float p = __expf(s - lse);
                    if (A.p_drop > 0.f) {
                        const uint64_t idx = (uint64_t)(base + jj + u) * (uint64_t)A.heads + (uint64_t)h;
                        dp = (uniform01(A.seed, idx) >= A.p_drop) ? dp * A.inv_keep : 0.f;
                    }
                    const float ds = p * (dp - D);
                    const Grad g = score_grad<METRIC>(a, b, qq, s, A.inv_sqrt_d, prm);
#pragma unroll
                    for (int c = 0; c < VEC; ++c) {
                        float t = fmaf(g.cq_q, qv[c], g.cq_k * kv[u][c]);
                        if constexpr (MetricTraits<METRIC>::fam == FAM_ABS) {
                            const float dfc = qv[c] - kv[u][c];
                            t = g.sg * ((dfc > 0.f) ? 1.f : (dfc < 0.f ? -1.f : 0.f));
                        }
                        dqa[c] = fmaf(ds, t, dqa[c]);
                    }
                    prm_acc = fmaf(ds, g.dprm, prm_acc);
                }
            }
        }
        if (active) {
            store_vec<VEC>(A.dq + row * A.ldd + f0, dqa);
            if ((lane % A.lph) == 0) A.delta[row * A.heads + h] = D;
        }
    }
    if (A.prm_partial) {
        // one value per (wave, head): lanes with lane % lph == 0 own a head
        red[wid][lane] = (row < A.N && active && (lane % A.lph) == 0) ? prm_acc : 0.f;
        __syncthreads();
        if (threadIdx.x < A.heads) {
            float s = 0.f;
            const int lane0 = threadIdx.x * A.lph;   // first lane of head threadIdx.x (VEC*lph = d)
            for (int w = 0; w < ROWS_PER_BLK; ++w) s += red[w][lane0];
            A.prm_partial[blk * A.heads + threadIdx.x] = s;
        }
    }
}

// ------------------------------------------------------------------ backward, column pass
template <int METRIC, int VEC>
__global__ void __launch_bounds__(BLK) k_geo_bwd_col(GeoArgs A) {
    const int lane = threadIdx.x & (WAVE - 1);
    const int64_t colj = xcd_remap(blockIdx.x, gridDim.x) * ROWS_PER_BLK + (threadIdx.x >> 6);
    if (colj >= A.N) return;
    const int f0 = lane * VEC;
    const bool active = f0 < A.H;
    const int fo = active ? f0 : 0;
    const int h = fo / A.d;
    float kv[VEC], vv[VEC];
    load_vec<VEC>(A.k + colj * A.ld + fo, kv);
    load_vec<VEC>(A.v + colj * A.ld + fo, vv);
    const float prm = A.mparam ? A.mparam[h] : 1.f;
    float dka[VEC], dva[VEC];
#pragma unroll
    for (int c = 0; c < VEC; ++c) { dka[c] = 0.f; dva[c] = 0.f; }
    const int e0 = A.csc_ptr[colj], e1 = A.csc_ptr[colj + 1];
    for (int base = e0; base < e1; base += WAVE) {
        const int cnt = min(WAVE, e1 - base);
        const int myrow = (lane < cnt) ? A.csc_row[base + lane] : 0;
        const int myeid = (lane < cnt) ? A.csc_eid[base + lane] : 0;
        for (int jj = 0; jj < cnt; jj += UNROLL) {
            float qv[UNROLL][VEC], dov[UNROLL][VEC], lse[UNROLL], D[UNROLL];
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) {
                const int i = __builtin_amdgcn_readlane(myrow, min(jj + u, cnt - 1));
                load_vec<VEC>(A.q + (int64_t)i * A.ld + fo, qv[u]);
                load_vec<VEC>(A.dout + (int64_t)i * A.H + fo, dov[u]);
                lse[u] = A.lse_in[(int64_t)i * A.heads + h];
                D[u] = A.delta[(int64_t)i * A.heads + h];
            }
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) {
                if (jj + u >= cnt) break;
                float a, b, dp = 0.f, qq = 0.f;
                pair_partial<METRIC, VEC>(qv[u], kv, a, b);
#pragma unroll
                for (int c = 0; c < VEC; ++c) dp = fmaf(dov[u][c], vv[c], dp);
                a = grp_sum(a, A.lph);
                dp = grp_sum(dp, A.lph);
                if constexpr (MetricTraits<METRIC>::fam == FAM_COS) {
                    b = grp_sum(b, A.lph);
#pragma unroll
                    for (int c = 0; c < VEC; ++c) qq = fmaf(qv[u][c], qv[u][c], qq);
                    qq = grp_sum(active ? qq : 0.f, A.lph);
                }
                const float s = finalize<METRIC>(a, b, qq, A.inv_sqrt_d, prm);
                const float p = __expf(s - lse[u]);
                float pw = p;
                if (A.p_drop > 0.f) {
                    const int eid = __builtin_amdgcn_readlane(myeid, jj + u);
                    const uint64_t idx = (uint64_t)eid * (uint64_t)A.heads + (uint64_t)h;
                    const bool keep = uniform01(A.seed, idx) >= A.p_drop;
                    dp = keep ? dp * A.inv_keep : 0.f;
                    pw = keep ? p * A.inv_keep : 0.f;
                }
                const float ds = p * (dp - D[u]);
                const Grad g = score_grad<METRIC>(a, b, qq, s, A.inv_sqrt_d, prm);
#pragma unroll
                for (int c = 0; c < VEC; ++c) {
                    float t = fmaf(g.ck_q, qv[u][c], g.ck_k * kv[c]);
                    if constexpr (MetricTraits<METRIC>::fam == FAM_ABS) {
                        const float dfc = qv[u][c] - kv[c];
                        t = -g.sg * ((dfc > 0.f) ? 1.f : (dfc < 0.f ? -1.f : 0.f));
                    }
                    dka[c] = fmaf(ds, t, dka[c]);
                    dva[c] = fmaf(pw, dov[u][c], dva[c]);
                }
            }
        }
    }
    if (!active) return;
    store_vec<VEC>(A.dk + colj * A.ldd + f0, dka);
    store_vec<VEC>(A.dv + colj * A.ldd + f0, dva);
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

// Optional per-edge attention weights (post-dropout), [nnz, heads].  Generic
// one-thread-per-(row, head) walker: only used for return_attention_weights and
// the geometric_bias path of the standalone GeometricAttention API.
template <int METRIC>
__global__ void __launch_bounds__(BLK) k_geo_alpha(GeoArgs A, float* __restrict__ alpha) {
    const int64_t t = blockIdx.x * (int64_t)BLK + threadIdx.x;
    if (t >= A.N * A.heads) return;
    const int64_t row = t / A.heads;
    const int h = (int)(t % A.heads);
    const float* qr = A.q + row * A.ld + h * A.d;
    float qq = 0.f;
    for (int c = 0; c < A.d; ++c) qq = fmaf(qr[c], qr[c], qq);
    const float prm = A.mparam ? A.mparam[h] : 1.f;
    const float lse = A.lse[row * A.heads + h];
    for (int e = A.rowptr[row]; e < A.rowptr[row + 1]; ++e) {
        const float* kr = A.k + (int64_t)A.col[e] * A.ld + h * A.d;
        float a = 0.f, b = 0.f;
        for (int c = 0; c < A.d; ++c) {
            float qa[1] = {qr[c]}, ka[1] = {kr[c]}, pa, pb;
            pair_partial<METRIC, 1>(qa, ka, pa, pb);
            a += pa;
            b += pb;
        }
        float p = __expf(finalize<METRIC>(a, b, qq, A.inv_sqrt_d, prm) - lse);
        if (A.p_drop > 0.f)
            p = (uniform01(A.seed, (uint64_t)e * A.heads + h) >= A.p_drop) ? p * A.inv_keep : 0.f;
        alpha[(int64_t)e * A.heads + h] = p;
    }
}

// ------------------------------------------------------------------ generic fallback
// One thread per (row, head); any H, d (used when H is not a power of two <= 256).
template <int METRIC>
__global__ void __launch_bounds__(BLK) k_geo_fwd_generic(GeoArgs A) {
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
    for (int e = A.rowptr[row]; e < A.rowptr[row + 1]; ++e) {
        const int64_t j = A.col[e];
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
            pw = (uniform01(A.seed, (uint64_t)e * A.heads + h) >= A.p_drop) ? p * A.inv_keep : 0.f;
        for (int c = 0; c < d; ++c) orow[c] = fmaf(orow[c], corr, pw * vr[c]);
        m = mn;
    }
    for (int c = 0; c < d; ++c) orow[c] = (l > 0.f) ? orow[c] / l : NAN;
    A.lse[row * A.heads + h] = m + __logf(l);
}

template <int METRIC>
__global__ void __launch_bounds__(BLK) k_geo_bwd_row_generic(GeoArgs A) {
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
    for (int e = A.rowptr[row]; e < A.rowptr[row + 1]; ++e) {
        const int64_t j = A.col[e];
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
            dp = (uniform01(A.seed, (uint64_t)e * A.heads + h) >= A.p_drop) ? dp * A.inv_keep : 0.f;
        const float ds = p * (dp - D);
        const Grad g = score_grad<METRIC>(a, b, qq, s, A.inv_sqrt_d, prm);
        for (int c = 0; c < d; ++c) {
            float tt = fmaf(g.cq_q, qr[c], g.cq_k * kr[c]);
            if constexpr (MetricTraits<METRIC>::fam == FAM_ABS) {
                const float dfc = qr[c] - kr[c];
                tt = g.sg * ((dfc > 0.f) ? 1.f : (dfc < 0.f ? -1.f : 0.f));
            }
            dqr[c] = fmaf(ds, tt, dqr[c]);
        }
        prm_acc = fmaf(ds, g.dprm, prm_acc);
    }
    A.delta[row * A.heads + h] = D;
    if (A.prm_partial) A.prm_partial[t] = prm_acc;   // [N*heads] partials: reduced per head below
}

template <int METRIC>
__global__ void __launch_bounds__(BLK) k_geo_bwd_col_generic(GeoArgs A) {
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
    for (int e = A.csc_ptr[colj]; e < A.csc_ptr[colj + 1]; ++e) {
        const int64_t i = A.csc_row[e];
        const int eid = A.csc_eid[e];
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
            const bool keep = uniform01(A.seed, (uint64_t)eid * A.heads + h) >= A.p_drop;
            dp = keep ? dp * A.inv_keep : 0.f;
            pw = keep ? p * A.inv_keep : 0.f;
        }
        const float ds = p * (dp - A.delta[i * A.heads + h]);
        const Grad g = score_grad<METRIC>(a, b, qq, s, A.inv_sqrt_d, prm);
        for (int c = 0; c < d; ++c) {
            float tt = fmaf(g.ck_q, qr[c], g.ck_k * kr[c]);
            if constexpr (MetricTraits<METRIC>::fam == FAM_ABS) {
                const float dfc = qr[c] - kr[c];
                tt = -g.sg * ((dfc > 0.f) ? 1.f : (dfc < 0.f ? -1.f : 0.f));
            }
            dkr[c] = fmaf(ds, tt, dkr[c]);
            dvr[c] = fmaf(pw, dor[c], dvr[c]);
        }
    }
}

// ------------------------------------------------------------------ dispatch
// Fast path: H a power of two in [1, 256] (VEC = max(1, H/64) floats per lane)
// and d a multiple of VEC with d/VEC a power of two.
int pick_vec(int H, int d) {
    if (H <= 0 || H > 256 || (H & (H - 1))) return 0;
    const int vec = H <= 64 ? 1 : H / 64;
    if (d % vec) return 0;
    const int lph = d / vec;
    if (lph < 1 || (lph & (lph - 1)) || lph > 64) return 0;
    return vec;
}

enum Pass { P_FWD, P_BWD_ROW, P_BWD_COL, P_ALPHA };

template <int METRIC>
int launch_metric(Pass pass, int vec, const GeoArgs& A, hipStream_t s, float* alpha) {
    const int64_t nblk_fast = (A.N + ROWS_PER_BLK - 1) / ROWS_PER_BLK;
    const int64_t nblk_gen = (A.N * A.heads + BLK - 1) / BLK;
    dim3 gf((unsigned)nblk_fast), gg((unsigned)nblk_gen);
    if (pass == P_ALPHA) {
        k_geo_alpha<METRIC><<<gg, BLK, 0, s>>>(A, alpha);
        return TAGAN_OK;
    }
#define TAGAN_GEO_CASE(V)                                                                     \
    case V:                                                                                   \
        if (pass == P_FWD) k_geo_fwd<METRIC, V><<<gf, BLK, 0, s>>>(A);                         \
        else if (pass == P_BWD_ROW) k_geo_bwd_row<METRIC, V><<<gf, BLK, 0, s>>>(A);            \
        else k_geo_bwd_col<METRIC, V><<<gf, BLK, 0, s>>>(A);                                   \
        return TAGAN_OK;
    switch (vec) {
        TAGAN_GEO_CASE(1)
        TAGAN_GEO_CASE(2)
        TAGAN_GEO_CASE(4)
        default:
            break;
    }
#undef TAGAN_GEO_CASE
    if (pass == P_FWD) k_geo_fwd_generic<METRIC><<<gg, BLK, 0, s>>>(A);
    else if (pass == P_BWD_ROW) k_geo_bwd_row_generic<METRIC><<<gg, BLK, 0, s>>>(A);
    else k_geo_bwd_col_generic<METRIC><<<gg, BLK, 0, s>>>(A);
    return TAGAN_OK;
}

int launch(int metric, Pass pass, int vec, const GeoArgs& A, hipStream_t s, float* alpha = nullptr) {
    switch (metric) {
        case TAGAN_METRIC_EUCLIDEAN: return launch_metric<TAGAN_METRIC_EUCLIDEAN>(pass, vec, A, s, alpha);
        case TAGAN_METRIC_SQUARED_EUCLIDEAN:
            return launch_metric<TAGAN_METRIC_SQUARED_EUCLIDEAN>(pass, vec, A, s, alpha);
        case TAGAN_METRIC_MANHATTAN: return launch_metric<TAGAN_METRIC_MANHATTAN>(pass, vec, A, s, alpha);
        case TAGAN_METRIC_COSINE_SIMILARITY:
            return launch_metric<TAGAN_METRIC_COSINE_SIMILARITY>(pass, vec, A, s, alpha);
        case TAGAN_METRIC_COSINE_DISTANCE:
            return launch_metric<TAGAN_METRIC_COSINE_DISTANCE>(pass, vec, A, s, alpha);
        case TAGAN_METRIC_DOT_PRODUCT: return launch_metric<TAGAN_METRIC_DOT_PRODUCT>(pass, vec, A, s, alpha);
        case TAGAN_METRIC_SCALED_DOT_PRODUCT:
            return launch_metric<TAGAN_METRIC_SCALED_DOT_PRODUCT>(pass, vec, A, s, alpha);
        case TAGAN_METRIC_GAUSSIAN_KERNEL:
            return launch_metric<TAGAN_METRIC_GAUSSIAN_KERNEL>(pass, vec, A, s, alpha);
        case TAGAN_METRIC_RBF_KERNEL: return launch_metric<TAGAN_METRIC_RBF_KERNEL>(pass, vec, A, s, alpha);
        default:
            set_error("geo_attn: unsupported metric %d", metric);
            return TAGAN_ERR_UNSUPPORTED;
    }
}

int check_common(int dtype, int metric, int64_t N, int heads, int d, int64_t ld, float p_drop) {
    TAGAN_REQUIRE(dtype == TAGAN_F32, TAGAN_ERR_UNSUPPORTED, "geo_attn: dtype %d unsupported", dtype);
    TAGAN_REQUIRE(metric >= 0 && metric <= TAGAN_METRIC_RBF_KERNEL, TAGAN_ERR_UNSUPPORTED,
                  "geo_attn: unsupported metric %d", metric);
    TAGAN_REQUIRE(N > 0 && heads > 0 && d > 0, TAGAN_ERR_ARG, "geo_attn: bad sizes N=%lld heads=%d d=%d",
                  (long long)N, heads, d);
    TAGAN_REQUIRE(ld >= (int64_t)heads * d, TAGAN_ERR_ARG, "geo_attn: ld %lld < H", (long long)ld);
    TAGAN_REQUIRE(p_drop >= 0.f && p_drop < 1.f, TAGAN_ERR_ARG, "geo_attn: p_drop %f", (double)p_drop);
    return TAGAN_OK;
}

GeoArgs make_args(int64_t N, int heads, int d, const int32_t* rowptr, const int32_t* col, const void* q,
                  const void* k, const void* v, int64_t ld, const float* mparam, float p_drop, uint64_t seed) {
    GeoArgs A{};
    A.N = N;
    A.heads = heads;
    A.d = d;
    A.H = heads * d;
    const int vec = pick_vec(A.H, d);
    A.lph = vec ? d / vec : 1;
    A.rowptr = rowptr;
    A.col = col;
    A.q = (const float*)q;
    A.k = (const float*)k;
    A.v = (const float*)v;
    A.ld = ld;
    A.mparam = mparam;
    A.p_drop = p_drop;
    A.inv_keep = 1.f / (1.f - p_drop);
    A.seed = seed;
    A.inv_sqrt_d = 1.f / sqrtf((float)d);
    return A;
}

}  // namespace
}  // namespace tagan

extern "C" {

int tagan_geo_attn_fwd(int dtype, int metric, int64_t n_nodes, int32_t heads, int32_t head_dim,
                       const int32_t* rowptr, const int32_t* col, const void* q, const void* k, const void* v,
                       int64_t ld_qkv, const float* metric_param, float p_drop, uint64_t seed, void* out,
                       float* lse, float* edge_alpha, void* stream) {
    using namespace tagan;
    int rc = check_common(dtype, metric, n_nodes, heads, head_dim, ld_qkv, p_drop);
    if (rc) return rc;
    TAGAN_REQUIRE(rowptr && col && q && k && v && out && lse, TAGAN_ERR_ARG, "geo_attn_fwd: null pointer");
    GeoArgs A = make_args(n_nodes, heads, head_dim, rowptr, col, q, k, v, ld_qkv, metric_param, p_drop, seed);
    A.out = (float*)out;
    A.lse = lse;
    hipStream_t s = as_stream(stream);
    const int vec = pick_vec(A.H, head_dim);
    rc = launch(metric, P_FWD, vec, A, s);
    if (rc) return rc;
    TAGAN_CHECK_LAUNCH("geo_attn_fwd");
    if (edge_alpha) {
        rc = launch(metric, P_ALPHA, vec, A, s, edge_alpha);
        if (rc) return rc;
        TAGAN_CHECK_LAUNCH("geo_attn_alpha");
    }
    return TAGAN_OK;
}

size_t tagan_geo_attn_bwd_workspace(int64_t n_nodes, int32_t heads) {
    using namespace tagan;
    if (n_nodes <= 0 || heads <= 0) return 0;
    const int64_t nblk = (n_nodes + ROWS_PER_BLK - 1) / ROWS_PER_BLK;
    const size_t delta = align_up((size_t)n_nodes * heads * 4, 256);
    const size_t part = align_up((size_t)std::max<int64_t>(nblk, n_nodes) * heads * 4, 256);
    return delta + part;
}

int tagan_geo_attn_bwd(int dtype, int metric, int64_t n_nodes, int32_t heads, int32_t head_dim,
                       const int32_t* rowptr, const int32_t* col, const int32_t* csc_ptr, const int32_t* csc_row,
                       const int32_t* csc_eid, const void* q, const void* k, const void* v, int64_t ld_qkv,
                       const float* metric_param, float p_drop, uint64_t seed, const void* out, const float* lse,
                       const void* dout, void* dq, void* dk, void* dv, int64_t ld_dqkv, float* dmetric_param,
                       void* workspace, size_t workspace_bytes, void* stream) {
    using namespace tagan;
    int rc = check_common(dtype, metric, n_nodes, heads, head_dim, ld_qkv, p_drop);
    if (rc) return rc;
    TAGAN_REQUIRE(rowptr && col && csc_ptr && csc_row && csc_eid && q && k && v && out && lse && dout && dq &&
                      dk && dv,
                  TAGAN_ERR_ARG, "geo_attn_bwd: null pointer");
    TAGAN_REQUIRE(ld_dqkv >= (int64_t)heads * head_dim, TAGAN_ERR_ARG, "geo_attn_bwd: ld_dqkv < H");
    const size_t need = tagan_geo_attn_bwd_workspace(n_nodes, heads);
    TAGAN_REQUIRE(workspace && workspace_bytes >= need, TAGAN_ERR_WORKSPACE, "geo_attn_bwd: workspace %zu < %zu",
                  workspace_bytes, need);
    GeoArgs A = make_args(n_nodes, heads, head_dim, rowptr, col, q, k, v, ld_qkv, metric_param, p_drop, seed);
    A.csc_ptr = csc_ptr;
    A.csc_row = csc_row;
    A.csc_eid = csc_eid;
    A.o = (const float*)out;
    A.lse_in = lse;
    A.dout = (const float*)dout;
    A.dq = (float*)dq;
    A.dk = (float*)dk;
    A.dv = (float*)dv;
    A.ldd = ld_dqkv;
    A.delta = (float*)workspace;
    const bool want_prm = dmetric_param != nullptr && metric_param != nullptr &&
                          (metric == TAGAN_METRIC_GAUSSIAN_KERNEL || metric == TAGAN_METRIC_RBF_KERNEL);
    A.prm_partial = want_prm ? (float*)((char*)workspace + align_up((size_t)n_nodes * heads * 4, 256)) : nullptr;
    hipStream_t s = as_stream(stream);
    const int vec = pick_vec(A.H, head_dim);
    rc = launch(metric, P_BWD_ROW, vec, A, s);
    if (rc) return rc;
    TAGAN_CHECK_LAUNCH("geo_attn_bwd_row");
    rc = launch(metric, P_BWD_COL, vec, A, s);
    if (rc) return rc;
    TAGAN_CHECK_LAUNCH("geo_attn_bwd_col");
    if (dmetric_param) {
        if (want_prm) {
            // fast path: one partial per (block, head); generic path: one per (row, head)
            const int64_t nparts = vec ? (n_nodes + ROWS_PER_BLK - 1) / ROWS_PER_BLK : n_nodes;
            k_reduce_partials<<<heads, BLK, 0, s>>>(A.prm_partial, nparts, heads, dmetric_param);
            TAGAN_CHECK_LAUNCH("geo_attn_bwd_reduce");
        } else {
            TAGAN_CHECK_HIP(hipMemsetAsync(dmetric_param, 0, sizeof(float) * heads, s), "memset dparam");
        }
    }
    return TAGAN_OK;
}

}  // extern "C"
