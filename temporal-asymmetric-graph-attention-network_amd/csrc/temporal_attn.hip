// Per-row temporal attention for TAGAN on gfx950.
//
// Replaces temporal_attention.py:1006-1205 after the Q/K/V projections:
//   S = Q·Kᵀ/√d + R[h, clamp(i-j+32)] + K[h, clamp(i-j+W)]·[|i-j|<=W] (+ time bias)
//   masks (causal / T==heads rule / explicit) -> softmax -> attn_dropout -> A·V
// for every node row independently (the [N_max, T, H] tensor of :928-976).
// The relative-position and asymmetric-kernel tables are folded host-side into
// one per-head table bias[h][i-j+T-1] (a [heads, 2T-1] tensor), so the kernel
// never materialises [rows, heads, T, T] (105 GB at C5).
//
// Mapping: one workgroup (4 waves) per node row, wave w takes heads w, w+4, ...
// so all heads of a row (whole 512-B feature rows) are produced by one CU close
// in time.  Lane = query step i (chunks of 64 when T > 64).  K/V rows of step j
// are wave-uniform addresses (scalar-cache broadcast), Q/acc stay in VGPRs,
// softmax is online; LSE per (row, head, i) is saved for the backward pass.
//
// Backward: phase A (lane = i) recomputes P, dP, delta and dq; phase B
// (lane = j) recomputes them again from (q_i, dO_i, lse_i, delta_i) broadcast
// loads and accumulates dk, dv and the bias-table gradient.  In phase B every
// lane of one instruction owns a distinct diagonal i-j, so the per-block LDS
// accumulation of dbias is conflict-free and deterministic; block partials are
// then summed in block order by a second kernel.
#include "common.cuh"

#include <mutex>
#include <type_traits>
#include <unordered_set>

namespace tagan {
namespace {

constexpr int BLK = 256;
constexpr int NW = BLK / WAVE;

struct TArgs {
    int64_t rows;
    int T, heads, d, H;
    int64_t s_row, s_t;
    const float* bias_table;
    const float* bias_dense;
    int64_t bias_bstride;
    const uint8_t* mask;
    int64_t mask_bstride, mask_hstride;
    int causal;
    float p_drop, inv_keep, inv_sqrt_d;
    uint64_t seed;
    const uint64_t* seed_ctr;   // graph-replay seed source (tagan_set_seed_counter) or null
    float* out;
    int64_t o_row, o_t;
    float* lse;
    float* attn;
    // backward
    const float* o_in;
    const float* lse_in;
    const float* dout;
    int64_t do_row, do_t;
    float* dq;
    float* dk;
    float* dv;
    int64_t d_row, d_t;
    float* dbias_dense;
    float* part;   // [gridDim.x, heads, 2T-1] block partials of dbias_table
    float* qkv_part;   // v4: [row groups, 3H] partial column sums of dq | dk | dv (QKV bias gradient)
    uint32_t* keep;    // v5 MODE 3: the dropout keep bits, one word per (row, head, wave, lane); fwd writes, bwd reads
};

__device__ __forceinline__ bool keep_ij(const TArgs& A, int64_t r, int h, int i, int j) {
    if (A.causal && j > i) return false;
    if (A.mask && !A.mask[r * A.mask_bstride + (int64_t)h * A.mask_hstride + (int64_t)i * A.T + j]) return false;
    return true;
}

__device__ __forceinline__ float bias_ij(const TArgs& A, int64_t r, int h, int i, int j) {
    float b = 0.f;
    if (A.bias_table) b += A.bias_table[h * (2 * A.T - 1) + (i - j + A.T - 1)];
    if (A.bias_dense) b += A.bias_dense[r * A.bias_bstride + (((int64_t)h * A.T + i) * A.T + j)];
    return b;
}

__device__ __forceinline__ uint32_t tkey(const TArgs& A, int64_t r, int h) {
    return A.p_drop > 0.f ? drop_key(A.seed, (uint64_t)r * A.heads + h) : 0u;
}

// Attention dropout: stream = r*heads + h (the key), counter c = i*T + j.  One lowbias32 of (c >> 1) ^ key decides
// the counter pair {2m, 2m + 1}: its low 16 bits the even counter, its high 16 bits the odd one; kept iff that half
// >= tthr(p) = ceil(p 2^16) -- drop probability tthr / 2^16, within 2^-16 of p.  (A matrix-core lane's four
// elements j = 16 jt + 4g + e are two such pairs: two hashes per four elements.)
__host__ __device__ __forceinline__ uint32_t tthr(float p) { return (uint32_t)ceilf(p * 65536.f); }
template <int E>   // half E & 1 of the pair word
__device__ __forceinline__ uint32_t thalf(uint32_t w) { return (E & 1) ? (w >> 16) : (w & 0xFFFFu); }
__device__ __forceinline__ bool tkeep(uint32_t key, uint32_t c, uint32_t thr) {
    const uint32_t w = lowbias32((c >> 1) ^ key);
    return ((c & 1u) ? (w >> 16) : (w & 0xFFFFu)) >= thr;
}
__device__ __forceinline__ float drop_scale(const TArgs& A, uint32_t key, int i, int j) {
    if (A.p_drop <= 0.f) return 1.f;
    return tkeep(key, (uint32_t)(i * A.T + j), tthr(A.p_drop)) ? A.inv_keep : 0.f;
}

template <int D>
__device__ __forceinline__ void load_row(const float* __restrict__ p, int d, float (&r)[D]) {
#pragma unroll
    for (int c = 0; c < D; ++c) r[c] = (c < d) ? p[c] : 0.f;
}

template <int D>
__global__ void __launch_bounds__(BLK) k_tattn_fwd(TArgs A, const float* __restrict__ q,
                                                   const float* __restrict__ k, const float* __restrict__ v) {
    TAGAN_LIVE_SEED(A);
    const int lane = threadIdx.x & (WAVE - 1);
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int T = A.T, d = A.d;
    for (int64_t r = blockIdx.x; r < A.rows; r += gridDim.x) {
        for (int h = wid; h < A.heads; h += NW) {
            const uint32_t drk = tkey(A, r, h);
            const float* kb = k + r * A.s_row + h * d;
            const float* vb = v + r * A.s_row + h * d;
            for (int i0 = 0; i0 < T; i0 += WAVE) {
                const int i = i0 + lane;
                const bool live = i < T;
                const int ii = live ? i : T - 1;
                float qv[D], acc[D];
                load_row<D>(q + r * A.s_row + (int64_t)ii * A.s_t + h * d, d, qv);
#pragma unroll
                for (int c = 0; c < D; ++c) acc[c] = 0.f;
                float m = -INFINITY, l = 0.f;
                for (int j = 0; j < T; ++j) {
                    const float* kr = kb + (int64_t)j * A.s_t;
                    const float* vr = vb + (int64_t)j * A.s_t;
                    float s = 0.f;
#pragma unroll
                    for (int c = 0; c < D; ++c)
                        if (c < d) s = fmaf(qv[c], kr[c], s);
                    if (!keep_ij(A, r, h, ii, j)) continue;
                    s = fmaf(s, A.inv_sqrt_d, bias_ij(A, r, h, ii, j));
                    const float mn = fmaxf(m, s);
                    const float corr = __expf(m - mn);
                    const float p = __expf(s - mn);
                    l = fmaf(l, corr, p);
                    const float pw = p * drop_scale(A, drk, ii, j);
#pragma unroll
                    for (int c = 0; c < D; ++c)
                        if (c < d) acc[c] = fmaf(acc[c], corr, pw * vr[c]);
                    m = mn;
                }
                if (live) {
                    float* orow = A.out + r * A.o_row + (int64_t)i * A.o_t + h * d;
                    const float inv_l = 1.f / l;
#pragma unroll
                    for (int c = 0; c < D; ++c)
                        if (c < d) orow[c] = (l > 0.f) ? acc[c] * inv_l : NAN;
                    const float ls = m + __logf(l);
                    A.lse[(r * A.heads + h) * T + i] = ls;
                    if (A.attn) {
                        float* ar = A.attn + ((r * A.heads + h) * T + i) * (int64_t)T;
                        for (int j = 0; j < T; ++j) {
                            const float* kr = kb + (int64_t)j * A.s_t;
                            float s = 0.f;
#pragma unroll
                            for (int c = 0; c < D; ++c)
                                if (c < d) s = fmaf(qv[c], kr[c], s);
                            float a = 0.f;
                            if (keep_ij(A, r, h, i, j)) {
                                s = fmaf(s, A.inv_sqrt_d, bias_ij(A, r, h, i, j));
                                a = __expf(s - ls) * drop_scale(A, drk, i, j);
                            }
                            ar[j] = (l > 0.f) ? a : NAN;
                        }
                    }
                }
            }
        }
    }
}

template <int D>
__global__ void __launch_bounds__(BLK) k_tattn_bwd(TArgs A, const float* __restrict__ q,
                                                   const float* __restrict__ k, const float* __restrict__ v,
                                                   const float* __restrict__ dout, const float* __restrict__ lse) {
    TAGAN_LIVE_SEED(A);
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int lane = threadIdx.x & (WAVE - 1);
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int T = A.T, d = A.d, NB = 2 * T - 1;
    float* dbias = smem;                       // [heads][2T-1] block accumulator
    float* delta = smem + A.heads * NB + wid * T;   // [NW][T]
    if (A.part) {
        for (int x = threadIdx.x; x < A.heads * NB; x += BLK) dbias[x] = 0.f;
    }
    __syncthreads();
    for (int64_t r = blockIdx.x; r < A.rows; r += gridDim.x) {
        for (int h = wid; h < A.heads; h += NW) {
            const uint32_t drk = tkey(A, r, h);
            const float* qb = q + r * A.s_row + h * d;
            const float* kb = k + r * A.s_row + h * d;
            const float* vb = v + r * A.s_row + h * d;
            const float* dob = dout + r * A.do_row + h * d;
            const float* lsb = lse + (r * A.heads + h) * T;
            // ---- phase A: lane = i
            for (int i0 = 0; i0 < T; i0 += WAVE) {
                const int i = i0 + lane;
                const bool live = i < T;
                const int ii = live ? i : T - 1;
                float qv[D], dov[D], ov[D], dqa[D];
                load_row<D>(qb + (int64_t)ii * A.s_t, d, qv);
                load_row<D>(dob + (int64_t)ii * A.do_t, d, dov);
                load_row<D>(A.o_in + r * A.o_row + (int64_t)ii * A.o_t + h * d, d, ov);
                float Di = 0.f;
#pragma unroll
                for (int c = 0; c < D; ++c) {
                    Di = fmaf(dov[c], ov[c], Di);
                    dqa[c] = 0.f;
                }
                const float li = lsb[ii];
                for (int j = 0; j < T; ++j) {
                    const float* kr = kb + (int64_t)j * A.s_t;
                    const float* vr = vb + (int64_t)j * A.s_t;
                    float s = 0.f, dp = 0.f;
#pragma unroll
                    for (int c = 0; c < D; ++c)
                        if (c < d) {
                            s = fmaf(qv[c], kr[c], s);
                            dp = fmaf(dov[c], vr[c], dp);
                        }
                    float ds = 0.f;
                    if (keep_ij(A, r, h, ii, j)) {
                        s = fmaf(s, A.inv_sqrt_d, bias_ij(A, r, h, ii, j));
                        const float p = __expf(s - li);
                        ds = p * (dp * drop_scale(A, drk, ii, j) - Di);
                    }
#pragma unroll
                    for (int c = 0; c < D; ++c)
                        if (c < d) dqa[c] = fmaf(ds, kr[c], dqa[c]);
                    if (A.dbias_dense && live)
                        A.dbias_dense[((r * A.heads + h) * T + i) * (int64_t)T + j] = ds;
                }
                if (live) {
                    float* dqr = A.dq + r * A.d_row + (int64_t)i * A.d_t + h * d;
#pragma unroll
                    for (int c = 0; c < D; ++c)
                        if (c < d) dqr[c] = dqa[c] * A.inv_sqrt_d;
                    delta[i] = Di;
                }
            }
            // delta[] is private to this wave; LDS ops of one wave complete in order.
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            // ---- phase B: lane = j
            for (int j0 = 0; j0 < T; j0 += WAVE) {
                const int j = j0 + lane;
                const bool live = j < T;
                const int jj = live ? j : T - 1;
                float kv[D], vv[D], dka[D], dva[D];
                load_row<D>(kb + (int64_t)jj * A.s_t, d, kv);
                load_row<D>(vb + (int64_t)jj * A.s_t, d, vv);
#pragma unroll
                for (int c = 0; c < D; ++c) {
                    dka[c] = 0.f;
                    dva[c] = 0.f;
                }
                for (int i = 0; i < T; ++i) {
                    const float* qr = qb + (int64_t)i * A.s_t;
                    const float* dor = dob + (int64_t)i * A.do_t;
                    float s = 0.f, dp = 0.f;
#pragma unroll
                    for (int c = 0; c < D; ++c)
                        if (c < d) {
                            s = fmaf(qr[c], kv[c], s);
                            dp = fmaf(dor[c], vv[c], dp);
                        }
                    float ds = 0.f, pw = 0.f;
                    if (keep_ij(A, r, h, i, jj)) {
                        s = fmaf(s, A.inv_sqrt_d, bias_ij(A, r, h, i, jj));
                        const float p = __expf(s - lsb[i]);
                        const float sc = drop_scale(A, drk, i, jj);
                        pw = p * sc;
                        ds = p * (dp * sc - delta[i]);
                    }
#pragma unroll
                    for (int c = 0; c < D; ++c)
                        if (c < d) {
                            dka[c] = fmaf(ds, qr[c], dka[c]);
                            dva[c] = fmaf(pw, dor[c], dva[c]);
                        }
                    if (A.part && live) dbias[h * NB + (i - j + T - 1)] += ds;   // distinct diagonal per lane
                }
                if (live) {
                    float* dkr = A.dk + r * A.d_row + (int64_t)j * A.d_t + h * d;
                    float* dvr = A.dv + r * A.d_row + (int64_t)j * A.d_t + h * d;
#pragma unroll
                    for (int c = 0; c < D; ++c)
                        if (c < d) {
                            dkr[c] = dka[c] * A.inv_sqrt_d;
                            dvr[c] = dva[c];
                        }
                }
            }
        }
    }
    if (A.part) {
        __syncthreads();
        for (int x = threadIdx.x; x < A.heads * NB; x += BLK) A.part[(int64_t)blockIdx.x * A.heads * NB + x] = dbias[x];
    }
}


// =================================================================== v2: LDS-staged fast path
// One workgroup per node row; the row's Q/K/V (and dO) of a group of G heads are
// staged into LDS with coalesced float4 loads, then one thread per (head, step)
// runs the online softmax over LDS rows (threads of one head read the same K/V
// row: LDS broadcast).  Gate: d in {4,8,16,32,64,128} and at least one head per
// LDS budget; otherwise the v1 kernels above run.
constexpr size_t FWD_LDS_BUDGET = 64 * 1024;
constexpr size_t BWD_LDS_BUDGET = 96 * 1024;

size_t v2_fwd_lds(int G, int T, int d) { return ((size_t)3 * G * T * d + (size_t)G * (2 * T - 1)) * sizeof(float); }
size_t v2_bwd_lds(int G, int T, int d, int heads) {
    return ((size_t)4 * G * T * d + (size_t)2 * G * T + (size_t)G * (2 * T - 1) + (size_t)heads * (2 * T - 1)) *
           sizeof(float);
}

int v2_groups(bool bwd, int T, int d, int heads) {
    if (!(d == 4 || d == 8 || d == 16 || d == 32 || d == 64 || d == 128)) return 0;
    int G = heads;
    while (G > 0 && (bwd ? v2_bwd_lds(G, T, d, heads) > BWD_LDS_BUDGET : v2_fwd_lds(G, T, d) > FWD_LDS_BUDGET)) --G;
    return G;
}

template <int D>
__device__ __forceinline__ float dotD(const float* __restrict__ a, const float* __restrict__ b) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < D; c += 4) {
        const float4 x = *(const float4*)(a + c), y = *(const float4*)(b + c);
        s = fmaf(x.x, y.x, s);
        s = fmaf(x.y, y.y, s);
        s = fmaf(x.z, y.z, s);
        s = fmaf(x.w, y.w, s);
    }
    return s;
}

template <int D>
__device__ __forceinline__ void stage_rows(float* __restrict__ dst, const float* __restrict__ src, int64_t row_off,
                                           int64_t s_t, int h0, int gc, int T) {
    constexpr int D4 = D / 4;
    const int per = T * D4;
    for (int x = threadIdx.x; x < gc * per; x += BLK) {
        const int hl = x / per, rem = x - hl * per, t = rem / D4, c = rem - t * D4;
        *(float4*)(dst + (hl * T + t) * D + c * 4) =
            *(const float4*)(src + row_off + (int64_t)t * s_t + (h0 + hl) * D + c * 4);
    }
}

template <int D>
__global__ void __launch_bounds__(BLK) k_tattn_fwd_v2(TArgs A, const float* __restrict__ q,
                                                      const float* __restrict__ k, const float* __restrict__ v,
                                                      int G) {
    TAGAN_LIVE_SEED(A);
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int T = A.T, NB = 2 * T - 1;
    float* Qs = sm;
    float* Ks = Qs + G * T * D;
    float* Vs = Ks + G * T * D;
    float* Bs = Vs + G * T * D;
    for (int64_t r = blockIdx.x; r < A.rows; r += gridDim.x) {
        for (int h0 = 0; h0 < A.heads; h0 += G) {
            const int gc = min(G, A.heads - h0);
            stage_rows<D>(Qs, q, r * A.s_row, A.s_t, h0, gc, T);
            stage_rows<D>(Ks, k, r * A.s_row, A.s_t, h0, gc, T);
            stage_rows<D>(Vs, v, r * A.s_row, A.s_t, h0, gc, T);
            for (int x = threadIdx.x; x < gc * NB; x += BLK) Bs[x] = A.bias_table ? A.bias_table[h0 * NB + x] : 0.f;
            __syncthreads();
            for (int it = threadIdx.x; it < gc * T; it += BLK) {
                const int hl = it / T, i = it - hl * T, h = h0 + hl;
                const uint32_t drk = tkey(A, r, h);
                const float* qi = Qs + (hl * T + i) * D;
                const float* kb = Ks + hl * T * D;
                const float* vb = Vs + hl * T * D;
                const float* bb = Bs + hl * NB + i + T - 1;     // bb[-j] = bias of (i, j)
                float acc[D];
#pragma unroll
                for (int c = 0; c < D; ++c) acc[c] = 0.f;
                float m = -INFINITY, l = 0.f;
                for (int j = 0; j < T; ++j) {
                    if (!keep_ij(A, r, h, i, j)) continue;
                    float bias = bb[-j];
                    if (A.bias_dense) bias += A.bias_dense[r * A.bias_bstride + (((int64_t)h * T + i) * T + j)];
                    const float s = fmaf(dotD<D>(qi, kb + j * D), A.inv_sqrt_d, bias);
                    const float mn = fmaxf(m, s);
                    const float corr = __expf(m - mn);
                    const float p = __expf(s - mn);
                    l = fmaf(l, corr, p);
                    const float pw = p * drop_scale(A, drk, i, j);
                    const float* vj = vb + j * D;
#pragma unroll
                    for (int c = 0; c < D; c += 4) {
                        const float4 vv = *(const float4*)(vj + c);
                        acc[c] = fmaf(acc[c], corr, pw * vv.x);
                        acc[c + 1] = fmaf(acc[c + 1], corr, pw * vv.y);
                        acc[c + 2] = fmaf(acc[c + 2], corr, pw * vv.z);
                        acc[c + 3] = fmaf(acc[c + 3], corr, pw * vv.w);
                    }
                    m = mn;
                }
                float* orow = A.out + r * A.o_row + (int64_t)i * A.o_t + h * D;
                const float inv_l = (l > 0.f) ? 1.f / l : NAN;
#pragma unroll
                for (int c = 0; c < D; c += 4)
                    *(float4*)(orow + c) = make_float4(acc[c] * inv_l, acc[c + 1] * inv_l, acc[c + 2] * inv_l,
                                                       acc[c + 3] * inv_l);
                const float ls = m + __logf(l);
                A.lse[(r * A.heads + h) * T + i] = ls;
                if (A.attn) {
                    float* ar = A.attn + ((r * A.heads + h) * T + i) * (int64_t)T;
                    for (int j = 0; j < T; ++j) {
                        float a = 0.f;
                        if (keep_ij(A, r, h, i, j)) {
                            float bias = bb[-j];
                            if (A.bias_dense) bias += A.bias_dense[r * A.bias_bstride + (((int64_t)h * T + i) * T + j)];
                            const float s = fmaf(dotD<D>(qi, kb + j * D), A.inv_sqrt_d, bias);
                            a = __expf(s - ls) * drop_scale(A, drk, i, j);
                        }
                        ar[j] = (l > 0.f) ? a : NAN;
                    }
                }
            }
            __syncthreads();
        }
    }
}

template <int D>
__global__ void __launch_bounds__(BLK) k_tattn_bwd_v2(TArgs A, const float* __restrict__ q,
                                                      const float* __restrict__ k, const float* __restrict__ v,
                                                      const float* __restrict__ dout, const float* __restrict__ lse,
                                                      int G) {
    TAGAN_LIVE_SEED(A);
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int T = A.T, NB = 2 * T - 1;
    float* Qs = sm;
    float* Ks = Qs + G * T * D;
    float* Vs = Ks + G * T * D;
    float* Os = Vs + G * T * D;          // dO
    float* Ls = Os + G * T * D;          // lse   [G][T]
    float* Del = Ls + G * T;             // delta [G][T]
    float* Bs = Del + G * T;             // bias  [G][NB]
    float* Acc = Bs + G * NB;            // dbias [heads][NB], persistent over rows
    for (int x = threadIdx.x; x < A.heads * NB; x += BLK) Acc[x] = 0.f;
    for (int64_t r = blockIdx.x; r < A.rows; r += gridDim.x) {
        for (int h0 = 0; h0 < A.heads; h0 += G) {
            const int gc = min(G, A.heads - h0);
            __syncthreads();
            stage_rows<D>(Qs, q, r * A.s_row, A.s_t, h0, gc, T);
            stage_rows<D>(Ks, k, r * A.s_row, A.s_t, h0, gc, T);
            stage_rows<D>(Vs, v, r * A.s_row, A.s_t, h0, gc, T);
            stage_rows<D>(Os, dout, r * A.do_row, A.do_t, h0, gc, T);
            for (int x = threadIdx.x; x < gc * T; x += BLK) Ls[x] = lse[(r * A.heads + h0) * T + x];
            for (int x = threadIdx.x; x < gc * NB; x += BLK) Bs[x] = A.bias_table ? A.bias_table[h0 * NB + x] : 0.f;
            __syncthreads();
            // ---- phase A: (head, i): delta_i, dq_i, optional per-pair ds
            for (int it = threadIdx.x; it < gc * T; it += BLK) {
                const int hl = it / T, i = it - hl * T, h = h0 + hl;
                const uint32_t drk = tkey(A, r, h);
                const float* qi = Qs + (hl * T + i) * D;
                const float* doi = Os + (hl * T + i) * D;
                const float* kb = Ks + hl * T * D;
                const float* vb = Vs + hl * T * D;
                const float* bb = Bs + hl * NB + i + T - 1;
                const float* orow = A.o_in + r * A.o_row + (int64_t)i * A.o_t + h * D;
                float Di = 0.f;
#pragma unroll
                for (int c = 0; c < D; c += 4) {
                    const float4 o4 = *(const float4*)(orow + c), d4 = *(const float4*)(doi + c);
                    Di = fmaf(d4.x, o4.x, Di);
                    Di = fmaf(d4.y, o4.y, Di);
                    Di = fmaf(d4.z, o4.z, Di);
                    Di = fmaf(d4.w, o4.w, Di);
                }
                Del[hl * T + i] = Di;
                const float li = Ls[hl * T + i];
                float dq[D];
#pragma unroll
                for (int c = 0; c < D; ++c) dq[c] = 0.f;
                for (int j = 0; j < T; ++j) {
                    float ds = 0.f;
                    if (keep_ij(A, r, h, i, j)) {
                        float bias = bb[-j];
                        if (A.bias_dense) bias += A.bias_dense[r * A.bias_bstride + (((int64_t)h * T + i) * T + j)];
                        const float s = fmaf(dotD<D>(qi, kb + j * D), A.inv_sqrt_d, bias);
                        const float p = __expf(s - li);
                        ds = p * (dotD<D>(doi, vb + j * D) * drop_scale(A, drk, i, j) - Di);
                        const float* kj = kb + j * D;
#pragma unroll
                        for (int c = 0; c < D; c += 4) {
                            const float4 k4 = *(const float4*)(kj + c);
                            dq[c] = fmaf(ds, k4.x, dq[c]);
                            dq[c + 1] = fmaf(ds, k4.y, dq[c + 1]);
                            dq[c + 2] = fmaf(ds, k4.z, dq[c + 2]);
                            dq[c + 3] = fmaf(ds, k4.w, dq[c + 3]);
                        }
                    }
                    if (A.dbias_dense) A.dbias_dense[((r * A.heads + h) * T + i) * (int64_t)T + j] = ds;
                }
                float* dqr = A.dq + r * A.d_row + (int64_t)i * A.d_t + h * D;
#pragma unroll
                for (int c = 0; c < D; c += 4)
                    *(float4*)(dqr + c) = make_float4(dq[c] * A.inv_sqrt_d, dq[c + 1] * A.inv_sqrt_d,
                                                      dq[c + 2] * A.inv_sqrt_d, dq[c + 3] * A.inv_sqrt_d);
            }
            __syncthreads();
            // ---- phase B: (head, j): dk_j, dv_j
            for (int it = threadIdx.x; it < gc * T; it += BLK) {
                const int hl = it / T, j = it - hl * T, h = h0 + hl;
                const uint32_t drk = tkey(A, r, h);
                const float* kj = Ks + (hl * T + j) * D;
                const float* vj = Vs + (hl * T + j) * D;
                const float* bb = Bs + hl * NB - j + T - 1;     // bb[i] = bias of (i, j)
                float dk[D], dv[D];
#pragma unroll
                for (int c = 0; c < D; ++c) {
                    dk[c] = 0.f;
                    dv[c] = 0.f;
                }
                for (int i = 0; i < T; ++i) {
                    if (!keep_ij(A, r, h, i, j)) continue;
                    const float* qi = Qs + (hl * T + i) * D;
                    const float* doi = Os + (hl * T + i) * D;
                    float bias = bb[i];
                    if (A.bias_dense) bias += A.bias_dense[r * A.bias_bstride + (((int64_t)h * T + i) * T + j)];
                    const float s = fmaf(dotD<D>(qi, kj), A.inv_sqrt_d, bias);
                    const float p = __expf(s - Ls[hl * T + i]);
                    const float sc = drop_scale(A, drk, i, j);
                    const float ds = p * (dotD<D>(doi, vj) * sc - Del[hl * T + i]);
                    const float pw = p * sc;
#pragma unroll
                    for (int c = 0; c < D; c += 4) {
                        const float4 q4 = *(const float4*)(qi + c), d4 = *(const float4*)(doi + c);
                        dk[c] = fmaf(ds, q4.x, dk[c]);
                        dk[c + 1] = fmaf(ds, q4.y, dk[c + 1]);
                        dk[c + 2] = fmaf(ds, q4.z, dk[c + 2]);
                        dk[c + 3] = fmaf(ds, q4.w, dk[c + 3]);
                        dv[c] = fmaf(pw, d4.x, dv[c]);
                        dv[c + 1] = fmaf(pw, d4.y, dv[c + 1]);
                        dv[c + 2] = fmaf(pw, d4.z, dv[c + 2]);
                        dv[c + 3] = fmaf(pw, d4.w, dv[c + 3]);
                    }
                }
                float* dkr = A.dk + r * A.d_row + (int64_t)j * A.d_t + h * D;
                float* dvr = A.dv + r * A.d_row + (int64_t)j * A.d_t + h * D;
#pragma unroll
                for (int c = 0; c < D; c += 4) {
                    *(float4*)(dkr + c) = make_float4(dk[c] * A.inv_sqrt_d, dk[c + 1] * A.inv_sqrt_d,
                                                      dk[c + 2] * A.inv_sqrt_d, dk[c + 3] * A.inv_sqrt_d);
                    *(float4*)(dvr + c) = make_float4(dv[c], dv[c + 1], dv[c + 2], dv[c + 3]);
                }
            }
            // ---- phase C: (head, diagonal i-j) sums of ds for the bias table (fixed order)
            if (A.part) {
                for (int it = threadIdx.x; it < gc * NB; it += BLK) {
                    const int hl = it / NB, dl = it - hl * NB, h = h0 + hl;
                    const uint32_t drk = tkey(A, r, h);
                    const int delta = dl - (T - 1);            // i - j
                    const float bias = Bs[hl * NB + dl];
                    float sum = 0.f;
                    for (int i = max(0, delta); i < min(T, T + delta); ++i) {
                        const int j = i - delta;
                        if (!keep_ij(A, r, h, i, j)) continue;
                        const float* qi = Qs + (hl * T + i) * D;
                        const float* doi = Os + (hl * T + i) * D;
                        float b = bias;
                        if (A.bias_dense) b += A.bias_dense[r * A.bias_bstride + (((int64_t)h * T + i) * T + j)];
                        const float s = fmaf(dotD<D>(qi, Ks + (hl * T + j) * D), A.inv_sqrt_d, b);
                        const float p = __expf(s - Ls[hl * T + i]);
                        sum += p * (dotD<D>(doi, Vs + (hl * T + j) * D) * drop_scale(A, drk, i, j) -
                                    Del[hl * T + i]);
                    }
                    Acc[h * NB + dl] += sum;
                }
            }
        }
    }
    if (A.part) {
        __syncthreads();
        for (int x = threadIdx.x; x < A.heads * NB; x += BLK) A.part[(int64_t)blockIdx.x * A.heads * NB + x] = Acc[x];
    }
}

// =================================================================== v3: one wave per (row, head group)
// The fast path for T <= 128 and head_dim in {8,16,32,64} without attention-weight output.
// A wave owns HPW = 64/LG heads of one node row (LG = lanes per head >= T; lane = step),
// so its K/V (fwd) or K/V then Q/dO (bwd) live in a private LDS slice written and read by
// the same wave — no workgroup barriers, 64-thread workgroups, many waves per CU to hide
// the strided time-major loads.  Waves are persistent over units (row, head group); a
// wave always keeps the same head group, so the backward's bias-table gradient is a
// per-wave LDS table updated conflict-free (at a fixed query step i, the lanes j of a head
// hit distinct diagonals i-j) in a fixed order — deterministic — and written once as a
// partial row for the ordered column sum.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int D>
__device__ __forceinline__ void ld_row(const float* __restrict__ p, float (&r)[D]) {
#pragma unroll
    for (int c = 0; c < D; c += 4) {
        const float4 t = *(const float4*)(p + c);
        r[c] = t.x; r[c + 1] = t.y; r[c + 2] = t.z; r[c + 3] = t.w;
    }
}

template <int D>
__device__ __forceinline__ void st_row(float* __restrict__ p, const float (&r)[D], float scale) {
#pragma unroll
    for (int c = 0; c < D; c += 4)
        *(float4*)(p + c) = make_float4(r[c] * scale, r[c + 1] * scale, r[c + 2] * scale, r[c + 3] * scale);
}

// Global row I/O in the activation storage type S (fp32 or bf16), element index i.
template <int D, typename S>
__device__ __forceinline__ void gld_row(const void* __restrict__ p, int64_t i, float (&r)[D]) {
#pragma unroll
    for (int c = 0; c < D; c += 4) {
        const float4 t = Io<S>::ld(p, i + c);
        r[c] = t.x; r[c + 1] = t.y; r[c + 2] = t.z; r[c + 3] = t.w;
    }
}

template <int D, typename S>
__device__ __forceinline__ void gst_row(void* __restrict__ p, int64_t i, const float (&r)[D], float scale) {
#pragma unroll
    for (int c = 0; c < D; c += 4)
        Io<S>::st(p, i + c, make_float4(r[c] * scale, r[c + 1] * scale, r[c + 2] * scale, r[c + 3] * scale));
}

template <int D>
__device__ __forceinline__ float dot_rl(const float (&a)[D], const float* __restrict__ b) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < D; c += 4) {
        const float4 y = *(const float4*)(b + c);
        s = fmaf(a[c], y.x, s);
        s = fmaf(a[c + 1], y.y, s);
        s = fmaf(a[c + 2], y.z, s);
        s = fmaf(a[c + 3], y.w, s);
    }
    return s;
}

template <int D>
__device__ __forceinline__ float dot_rr(const float (&a)[D], const float (&b)[D]) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < D; ++c) s = fmaf(a[c], b[c], s);
    return s;
}

// axpy with an LDS row: acc = acc*corr + w*row
template <int D>
__device__ __forceinline__ void axpy_l(float (&acc)[D], float corr, float w, const float* __restrict__ row) {
#pragma unroll
    for (int c = 0; c < D; c += 4) {
        const float4 y = *(const float4*)(row + c);
        acc[c] = fmaf(acc[c], corr, w * y.x);
        acc[c + 1] = fmaf(acc[c + 1], corr, w * y.y);
        acc[c + 2] = fmaf(acc[c + 2], corr, w * y.z);
        acc[c + 3] = fmaf(acc[c + 3], corr, w * y.w);
    }
}

template <int D>
__device__ __forceinline__ void fma_l(float (&acc)[D], float w, const float* __restrict__ row) {
#pragma unroll
    for (int c = 0; c < D; c += 4) {
        const float4 y = *(const float4*)(row + c);
        acc[c] = fmaf(w, y.x, acc[c]);
        acc[c + 1] = fmaf(w, y.y, acc[c + 1]);
        acc[c + 2] = fmaf(w, y.z, acc[c + 2]);
        acc[c + 3] = fmaf(w, y.w, acc[c + 3]);
    }
}

template <int D>
__device__ __forceinline__ void to_lds(float* __restrict__ p, const float (&r)[D]) {
#pragma unroll
    for (int c = 0; c < D; c += 4) *(float4*)(p + c) = make_float4(r[c], r[c + 1], r[c + 2], r[c + 3]);
}

constexpr int V3_BLK = WAVE;

// T in (64, 128]: WPH = 2 waves share one head (wave w owns steps 64w .. 64w+63), the LDS slice is
// the block's and the syncs are block barriers; each wave keeps its own bias-gradient table.
template <int WPH>
__device__ __forceinline__ void v3_sync() {
    if constexpr (WPH == 1) wave_sync();
    else __syncthreads();
}

size_t v3_fwd_lds(int T, int D, int HPW) { return (size_t)HPW * (2 * T * D + align_up(2 * T - 1, 4)) * 4; }
size_t v3_bwd_lds(int T, int D, int HPW, int WPH) {
    return (size_t)HPW * (2 * T * D + 2 * T + (1 + WPH) * align_up(2 * T - 1, 4)) * 4;
}

template <int D, int LG, typename S, int WPH>
__global__ void __launch_bounds__(V3_BLK * WPH) k_tattn_fwd_v3(TArgs A, const float* __restrict__ q,
                                                               const float* __restrict__ k,
                                                               const float* __restrict__ v, int n_hg) {
    TAGAN_LIVE_SEED(A);
    constexpr int HPW = WAVE / LG;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int T = A.T, NB = 2 * T - 1, NBp = (NB + 3) & ~3;
    const int lane = threadIdx.x & (WAVE - 1), hl = lane / LG, li = lane % LG + (threadIdx.x >> 6) * WAVE;
    float* Ks = sm;                  // [HPW][T][D]
    float* Vs = Ks + HPW * T * D;    // [HPW][T][D]
    float* Bs = Vs + HPW * T * D;    // [HPW][NBp]
    const int64_t units = A.rows * n_hg;
    const bool live = li < T;
    const int i = live ? li : T - 1;
    for (int64_t u = blockIdx.x; u < units; u += gridDim.x) {
        const int64_t r = u / n_hg;
        const int h0 = (int)(u - r * n_hg) * HPW, h = h0 + hl;
        const bool hok = h < A.heads;
        const int hc = hok ? h : A.heads - 1;
        const int64_t base = r * A.s_row + (int64_t)i * A.s_t + hc * D;
        float qv[D], kv[D], vv[D];
        gld_row<D, S>(q, base, qv);
        gld_row<D, S>(k, base, kv);
        gld_row<D, S>(v, base, vv);
        v3_sync<WPH>();   // previous unit's LDS reads are done before the slice is rewritten
        to_lds<D>(Ks + (hl * T + i) * D, kv);
        to_lds<D>(Vs + (hl * T + i) * D, vv);
        for (int x = li; x < NB; x += LG * WPH) Bs[hl * NBp + x] = A.bias_table ? A.bias_table[hc * NB + x] : 0.f;
        v3_sync<WPH>();
        const uint32_t drk = tkey(A, r, hc);
        const float* kb = Ks + hl * T * D;
        const float* vb = Vs + hl * T * D;
        const float* bb = Bs + hl * NBp + i + T - 1;   // bb[-j] = bias of (i, j)
        float acc[D];
#pragma unroll
        for (int c = 0; c < D; ++c) acc[c] = 0.f;
        float m = -INFINITY, l = 0.f;
#pragma unroll 1
        for (int j = 0; j < T; ++j) {
            if (!keep_ij(A, r, hc, i, j)) continue;
            float bias = bb[-j];
            if (A.bias_dense) bias += A.bias_dense[r * A.bias_bstride + (((int64_t)hc * T + i) * T + j)];
            const float s = fmaf(dot_rl<D>(qv, kb + j * D), A.inv_sqrt_d, bias);
            const float mn = fmaxf(m, s);
            const float corr = __expf(m - mn);
            const float p = __expf(s - mn);
            l = fmaf(l, corr, p);
            axpy_l<D>(acc, corr, p * drop_scale(A, drk, i, j), vb + j * D);
            m = mn;
        }
        if (live && hok) {
            const float inv_l = (l > 0.f) ? 1.f / l : NAN;
            gst_row<D, S>(A.out, r * A.o_row + (int64_t)i * A.o_t + h * D, acc, inv_l);
            A.lse[(r * A.heads + h) * T + i] = m + __logf(l);
        }
    }
}

template <int D, int LG, typename S, int WPH>
__global__ void __launch_bounds__(V3_BLK * WPH) k_tattn_bwd_v3(TArgs A, const float* __restrict__ q,
                                                               const float* __restrict__ k,
                                                               const float* __restrict__ v,
                                                               const float* __restrict__ dout,
                                                               const float* __restrict__ lse, int n_hg) {
    TAGAN_LIVE_SEED(A);
    constexpr int HPW = WAVE / LG;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int T = A.T, NB = 2 * T - 1, NBp = (NB + 3) & ~3;
    const int lane = threadIdx.x & (WAVE - 1), hl = lane / LG, wv = threadIdx.x >> 6;
    const int li = lane % LG + wv * WAVE;
    float* X1 = sm;                   // [HPW][T][D]  K in phase A, Q in phase B
    float* X2 = X1 + HPW * T * D;     // [HPW][T][D]  V in phase A, dO in phase B
    float* Ls = X2 + HPW * T * D;     // [HPW][T]
    float* Dl = Ls + HPW * T;         // [HPW][T]
    float* Bs = Dl + HPW * T;         // [HPW][NBp]
    float* Acc = Bs + HPW * NBp;      // [WPH][HPW][NBp] bias-table gradient, one table per wave
    for (int x = threadIdx.x; x < WPH * HPW * NBp; x += WAVE * WPH) Acc[x] = 0.f;
    const int64_t units = A.rows * n_hg;
    const bool live = li < T;
    const int i = live ? li : T - 1;   // this lane's step: query i in phase A, key j in phase B
    const int hg = (int)(blockIdx.x % n_hg);
    for (int64_t u = blockIdx.x; u < units; u += gridDim.x) {
        const int64_t r = u / n_hg;
        const int h = hg * HPW + hl;
        const bool hok = h < A.heads;
        const int hc = hok ? h : A.heads - 1;
        const int64_t base = r * A.s_row + (int64_t)i * A.s_t + hc * D;
        float qv[D], kv[D], vv[D], dov[D];
        gld_row<D, S>(q, base, qv);
        gld_row<D, S>(k, base, kv);
        gld_row<D, S>(v, base, vv);
        gld_row<D, S>(dout, r * A.do_row + (int64_t)i * A.do_t + hc * D, dov);   // kv/vv die after staging
        float Di;
        {
            float ov[D];
            gld_row<D, S>(A.o_in, r * A.o_row + (int64_t)i * A.o_t + hc * D, ov);
            Di = dot_rr<D>(dov, ov);
        }
        const float li_lse = lse[(r * A.heads + hc) * T + i];
        v3_sync<WPH>();
        to_lds<D>(X1 + (hl * T + i) * D, kv);
        to_lds<D>(X2 + (hl * T + i) * D, vv);
        Ls[hl * T + i] = li_lse;
        Dl[hl * T + i] = Di;
        for (int x = li; x < NB; x += LG * WPH) Bs[hl * NBp + x] = A.bias_table ? A.bias_table[hc * NB + x] : 0.f;
        v3_sync<WPH>();
        const uint32_t drk = tkey(A, r, hc);
        // ---- phase A (lane = query i): dq_i
        {
            const float* kb = X1 + hl * T * D;
            const float* vb = X2 + hl * T * D;
            const float* bb = Bs + hl * NBp + i + T - 1;
            float dq[D];
#pragma unroll
            for (int c = 0; c < D; ++c) dq[c] = 0.f;
    #pragma unroll 1
        for (int j = 0; j < T; ++j) {
                if (!keep_ij(A, r, hc, i, j)) continue;
                float bias = bb[-j];
                if (A.bias_dense) bias += A.bias_dense[r * A.bias_bstride + (((int64_t)hc * T + i) * T + j)];
                const float s = fmaf(dot_rl<D>(qv, kb + j * D), A.inv_sqrt_d, bias);
                const float p = __expf(s - li_lse);
                const float ds = p * (dot_rl<D>(dov, vb + j * D) * drop_scale(A, drk, i, j) - Di);
                fma_l<D>(dq, ds, kb + j * D);
            }
            if (live && hok) gst_row<D, S>(A.dq, r * A.d_row + (int64_t)i * A.d_t + h * D, dq, A.inv_sqrt_d);
        }
        v3_sync<WPH>();
        // swap: each lane takes its own K/V row back from LDS and leaves its Q/dO row in its place
        // (same lane, same address: no cross-lane hazard once phase A's reads are done)
        float* x1 = X1 + (hl * T + i) * D;
        float* x2 = X2 + (hl * T + i) * D;
        ld_row<D>(x1, kv);
        ld_row<D>(x2, vv);
        to_lds<D>(x1, qv);
        to_lds<D>(x2, dov);
        v3_sync<WPH>();
        // ---- phase B (lane = key j): dk_j, dv_j, bias-table / dense-bias gradient
        {
            const int j = i;
            const float* qb = X1 + hl * T * D;
            const float* ob = X2 + hl * T * D;
            const float* bb = Bs + hl * NBp - j + T - 1;   // bb[i'] = bias of (i', j)
            float* ab = Acc + (wv * HPW + hl) * NBp - j + T - 1;   // ab[i'] accumulates diagonal i'-j
            float dk[D], dv[D];
#pragma unroll
            for (int c = 0; c < D; ++c) {
                dk[c] = 0.f;
                dv[c] = 0.f;
            }
            const bool acc_ok = live && hok && A.part;
#pragma unroll 1
            for (int ii = 0; ii < T; ++ii) {
                float ds = 0.f;
                if (keep_ij(A, r, hc, ii, j)) {
                    float bias = bb[ii];
                    if (A.bias_dense) bias += A.bias_dense[r * A.bias_bstride + (((int64_t)hc * T + ii) * T + j)];
                    const float s = fmaf(dot_rl<D>(kv, qb + ii * D), A.inv_sqrt_d, bias);
                    const float p = __expf(s - Ls[hl * T + ii]);
                    const float sc = drop_scale(A, drk, ii, j);
                    ds = p * (dot_rl<D>(vv, ob + ii * D) * sc - Dl[hl * T + ii]);
                    fma_l<D>(dk, ds, qb + ii * D);
                    fma_l<D>(dv, p * sc, ob + ii * D);
                    if (acc_ok) ab[ii] += ds;
                }
                if (A.dbias_dense && live && hok)
                    A.dbias_dense[((r * A.heads + h) * T + ii) * (int64_t)T + j] = ds;
            }
            if (live && hok) {
                gst_row<D, S>(A.dk, r * A.d_row + (int64_t)j * A.d_t + h * D, dk, A.inv_sqrt_d);
                gst_row<D, S>(A.dv, r * A.d_row + (int64_t)j * A.d_t + h * D, dv, 1.f);
            }
        }
    }
    if (A.part) {
        v3_sync<WPH>();
        // partial row blockIdx / n_hg holds this block's head group's columns (waves summed in order)
        float* prow = A.part + (int64_t)(blockIdx.x / n_hg) * A.heads * NB;
        for (int x = threadIdx.x; x < HPW * NB; x += WAVE * WPH) {
            const int hh = x / NB, c = x - hh * NB, h = hg * HPW + hh;
            float a = 0.f;
#pragma unroll
            for (int ww = 0; ww < WPH; ++ww) a += Acc[(ww * HPW + hh) * NBp + c];
            if (h < A.heads) prow[h * NB + c] = a;
        }
    }
}

// =================================================================== v4: matrix-core kernels (T <= 64)
// One wave per (node row, head) unit; every product of the layer runs on v_mfma_f32_16x16x4_f32
// (fp32 in, fp32 accumulate: the same numbers as the fp32 VALU dots, in another summation order),
// with 16x16 tiles over steps (T padded to TP = 16*TT) and head features (d = 16*DT):
//   Sᵀ = K·Qᵀ       A = K rows (lane = key j), B = Q rows (lane = query i)
//   Oᵀ = Vᵀ·Pᵀ      B = Pᵀ straight from Sᵀ's accumulator registers (the sum runs over the
//                   accumulator's row index j), A = V read transposed (one element per lane)
// so the softmax over j is in-lane over the registers plus two cross-lane steps (xor 16, 32),
// and the output tile holds 4 consecutive features of one step per lane (one 16-B store).
// Backward: Sᵀ and dPᵀ = V·dOᵀ the same way, dQᵀ = Kᵀ·dSᵀ from the accumulators, and dKᵀ = Qᵀ·dS,
// dVᵀ = dOᵀ·P' with dS / P' transposed through a per-wave LDS tile (row stride TP+4); the
// bias-table gradient is a fixed-order diagonal sum over that tile (bitwise deterministic).
// Each wave keeps one head (wave stride = a multiple of heads), so its bias-table slice is staged
// in LDS once.  MFMA work per unit: 8·TT²·DT instructions forward, 20·TT²·DT backward.
typedef float f4v __attribute__((ext_vector_type(4)));

// Build-time knobs (A/B builds: make variant, tools/runs/r4tv.sh / r4tv2.sh).  Register prefetch of the next
// row (PREFETCH=1): the C2 backward 0.337 -> 0.308 ms in bf16 storage and 0.352 -> 0.344 ms in fp32
// (profiles/r4tv_c2_tattn_v4_knobs.txt; round 2 had measured the fp32 kernels within noise), so it is the
// default; 2 or 4 waves / EU instead of 3 (WPE_B) are within noise.  NOHOIST re-derives the lane indices per
// row (no hoisted per-element constants); SPLIT prefetches only Q, K, LSE in the backward.
#ifndef TAGAN_V4_PREFETCH
#define TAGAN_V4_PREFETCH 1
#endif
#ifndef TAGAN_V4_WPE_F
#define TAGAN_V4_WPE_F 1
#endif
#ifndef TAGAN_V4_NOHOIST
#define TAGAN_V4_NOHOIST 1
#endif
#ifndef TAGAN_V4_SPLIT
#define TAGAN_V4_SPLIT 0
#endif
#ifndef TAGAN_V4_WPE_B
#define TAGAN_V4_WPE_B 3
#endif

__device__ __forceinline__ f4v mfma4(float a, float b, f4v c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// bf16 storage: the score products Sᵀ = K·Qᵀ and dPᵀ = V·dOᵀ multiply STORED bf16 values only, so one
// v_mfma_f32_16x16x16_bf16 per 16 features gives the same products (a bf16 x bf16 product is exact in fp32) and
// fp32 accumulation in another summation order -- against four v_mfma_f32_16x16x4_f32 (32 cycles each).  Its operand
// layout is the f32 instruction's with the k index widened to 4 per lane: lane (c, g) holds row c, k = 4g + [0, 4)
// -- exactly the f4v a lane already holds (features 16dt + 4g + e).  The products with the softmax-derived
// operands (P', dS) stay on the f32 instruction.  TAGAN_TATTN_BFMM=0 keeps every product f32 (A/B builds).
#ifndef TAGAN_TATTN_BFMM
#define TAGAN_TATTN_BFMM 1
#endif
typedef short s16x4 __attribute__((ext_vector_type(4)));
// four fp32 registers holding exact bf16 values -> the packed bf16 operand (the high halves; no rounding)
__device__ __forceinline__ s16x4 pk4bf(const f4v& x) {
    const uint32_t lo = __builtin_amdgcn_perm(__float_as_uint(x[1]), __float_as_uint(x[0]), 0x07060302u);
    const uint32_t hi = __builtin_amdgcn_perm(__float_as_uint(x[3]), __float_as_uint(x[2]), 0x07060302u);
    return __builtin_bit_cast(s16x4, make_uint2(lo, hi));
}
__device__ __forceinline__ f4v mfma16bf(const s16x4& a, const s16x4& b, f4v c) {
    return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}
template <typename S>
constexpr bool bf_scores() { return TAGAN_TATTN_BFMM && std::is_same<S, bf16s>::value; }

template <typename S>
__device__ __forceinline__ f4v ld4v(const void* p, int64_t i, bool ok) {
    if (!ok) return f4v{0.f, 0.f, 0.f, 0.f};
    const float4 t = Io<S>::ld(p, i);
    return f4v{t.x, t.y, t.z, t.w};
}

// A prefetched 4-element chunk kept in its STORED form until use: in bf16 storage a conversion right at the load
// would make the prefetch wait for its data there (the v5 / v6 backwards spent twice the fp32 kernels' cycles in
// s_waitcnt: profiles/r5q_tattn_bf16_pmc.txt); f() converts where the values are consumed, pk() hands the four bf16
// straight to the bf16 matrix instruction.
template <typename S>
struct Raw4 {
    f4v v;
    __device__ __forceinline__ f4v f() const { return v; }
};
template <>
struct Raw4<bf16s> {
    uint2 u;
    __device__ __forceinline__ f4v f() const {
        return f4v{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                   __uint_as_float(u.y & 0xffff0000u)};
    }
};
template <typename S>
__device__ __forceinline__ Raw4<S> ldr4(const void* p, int64_t i, bool ok) {
    if constexpr (std::is_same<S, bf16s>::value) {
        Raw4<bf16s> r{make_uint2(0u, 0u)};
        if (ok) r.u = *(const uint2*)((const uint16_t*)p + i);
        return r;
    } else {
        return Raw4<S>{ld4v<S>(p, i, ok)};
    }
}
template <typename S>
__device__ __forceinline__ s16x4 pk4(const Raw4<S>& r) {
    if constexpr (std::is_same<S, bf16s>::value) return __builtin_bit_cast(s16x4, r.u);
    else return pk4bf(r.v);
}

template <typename S>
__device__ __forceinline__ float ld1v(const void* p, int64_t i, bool ok) {
    return ok ? Io<S>::ld1(p, i) : 0.f;
}

template <typename S>
__device__ __forceinline__ void st4v(void* p, int64_t i, f4v v, float scale) {
    Io<S>::st(p, i, make_float4(v[0] * scale, v[1] * scale, v[2] * scale, v[3] * scale));
}

constexpr int v4_nbp(int TP) { return (2 * TP - 1 + 3) & ~3; }
// Row stride of the transposed LDS tiles.  A 16-B read at Xt[row c][4g] (lane = 16g + c) is served in
// ds_read_b128's 16-lane groups {c 0-3,12-15 of g} + {c 4-11 of g+1}; with stride 4m dwords those
// lanes start on 4-dword bank slots c*m + g (mod 16), all distinct iff m = 2 (mod 4): TP + 8
// (m = 6 at TP = 16, 10 at TP = 32).  TP + 4 (m = 5, 9) gives 2-way conflicts.
constexpr int v4_ld(int TP) { return TP + 8; }
// per-wave LDS: fwd Vt [D][LD]; bwd X [TP][LD] | Kt, Qt, dOt [D][LD]
size_t v4_fwd_lds(int TT, int DT) { return (size_t)(16 * DT * v4_ld(16 * TT)) * 4; }
size_t v4_bwd_lds(int TT, int DT) { return (size_t)(16 * TT * v4_ld(16 * TT) + 3 * 16 * DT * v4_ld(16 * TT)) * 4; }

// Fast path (MODE 1: no dropout, 2: dropout, 3: dropout with the keep-bit cache of v5) for the common shape:
// T = TP, no causal flag, no keep-mask, no dense bias (or dense-bias gradient).  Every element is then valid, so the
// per-element range / mask tests go; the scores are kept in log2 units (log2 e folded into the 1/sqrt(d) scale and
// the staged bias table: one v_exp_f32 per element, no separate multiply); the dropout test is one integer compare
// of the element's pair-word half against tthr(p) (two hashes per four elements) -- the same decision as
// drop_scale, bit for bit; the backward carries the keep bit in the sign of the stored probability.  MODE 0 is the
// general path.
constexpr float LOG2E_F = 1.4426950408889634f;
constexpr float LN2_F = 0.6931471805599453f;

bool v5_fast_shape(int T, int TT, int causal, const void* mask, const void* bias_dense, const void* dbias_dense,
                   float p_drop) {
    return T == 16 * TT && !causal && !mask && !bias_dense && !dbias_dense && (p_drop <= 0.f || tthr(p_drop) < 65536u);
}

// the keep decisions of the lane's four elements of key tile jt (counters cb + 16 jt + e, cb even): two pair words
__device__ __forceinline__ void tpair(uint32_t key, uint32_t cb, int jt, uint32_t (&w)[2]) {
    const uint32_t m = (cb + (uint32_t)(jt * 16)) >> 1;
    w[0] = lowbias32(m ^ key);
    w[1] = lowbias32((m + 1u) ^ key);
}
// all ones iff element e of the pair words is kept (half >= thr, thr1 = thr - 1 >= 0), else 0: arithmetic (no
// lane-mask compares, whose masks the compiler otherwise keeps live in SGPRs and spills)
template <int E>
__device__ __forceinline__ uint32_t tkeepmask(const uint32_t (&w)[2], uint32_t thr1) {
    const uint32_t half = (E & 1) ? (w[E >> 1] >> 16) : (w[E >> 1] & 0xFFFFu);
    uint32_t m = (uint32_t)((int32_t)(thr1 - half) >> 31);
    asm("" : "+v"(m));   // see tbitmask
    return m;
}
// the keep-bit cache: all ones iff bit b of the word is set (opaque VGPR value: otherwise the compiler turns the
// masking into lane-mask compares + selects, whose masks it keeps in SGPRs and spills)
__device__ __forceinline__ uint32_t tbitmask(uint32_t kw, int b) {
    uint32_t m = (uint32_t)((int32_t)(kw << (31 - b)) >> 31);
    asm("" : "+v"(m));
    return m;
}
__device__ __forceinline__ float fand(float x, uint32_t m) { return __uint_as_float(__float_as_uint(x) & m); }
// +p where kept, -p where dropped (the backward's keep bit in the sign of P)
__device__ __forceinline__ float fsignkeep(float p, uint32_t m) {
    return __uint_as_float(__float_as_uint(p) ^ (~m & 0x80000000u));
}

// The unit-invariant part of the score of the lane's elements (i = it*16 + c, j = jt*16 + 4g + e):
// the head's bias-table value, or -inf outside [0, T)² and above the diagonal when causal.  A wave
// keeps one head, so this lives in registers for the whole kernel (no per-element table lookup).
template <int TT>
__device__ __forceinline__ void v4_static_bias(const TArgs& A, int h, int c, int g, float (&bst)[TT][TT][4]) {
    const int T = A.T, NB = 2 * T - 1;
#pragma unroll
    for (int jt = 0; jt < TT; ++jt)
#pragma unroll
        for (int it = 0; it < TT; ++it)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int i = it * 16 + c, j = jt * 16 + 4 * g + e;
                const bool ok = i < T && j < T && !(A.causal && j > i);
                bst[jt][it][e] = ok ? (A.bias_table ? A.bias_table[h * NB + i - j + T - 1] : 0.f) : -INFINITY;
            }
}

// fast path (v5_fast_shape): the log2-scaled table values, every element valid
template <int TT>
__device__ __forceinline__ void v4_fast_bias(const TArgs& A, int h, int c, int g, float (&bst)[TT][TT][4]) {
    const int T = A.T, NB = 2 * T - 1;
#pragma unroll
    for (int jt = 0; jt < TT; ++jt)
#pragma unroll
        for (int it = 0; it < TT; ++it)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int i = it * 16 + c, j = jt * 16 + 4 * g + e;
                bst[jt][it][e] = A.bias_table ? A.bias_table[h * NB + i - j + T - 1] * LOG2E_F : 0.f;
            }
}

// score of (i, j) from the raw dot product and the static part; -inf where masked
__device__ __forceinline__ float v4_score(const TArgs& A, float bst, int64_t r, int h, int i, int j, float dot) {
    if (bst == -INFINITY) return -INFINITY;
    if (A.mask && !A.mask[r * A.mask_bstride + (int64_t)h * A.mask_hstride + (int64_t)i * A.T + j]) return -INFINITY;
    float s = fmaf(dot, A.inv_sqrt_d, bst);
    if (A.bias_dense) s += A.bias_dense[r * A.bias_bstride + (((int64_t)h * A.T + i) * A.T + j)];
    return s;
}

// Transposed staging of a row tile held as lane (c, g): X[row = t*16 + c][dt*16 + 4g .. +3]
// into Xt[feature][row] (row stride LT), so a lane can read Xt[dt*16 + c][t*16 + 4g .. +3] -- the
// A operand of a product that sums over rows -- as one 16-B LDS read.
template <int TT, int DT, int LT, typename S>
__device__ __forceinline__ void v4_stage_t(float* Xt, const Raw4<S> (&x)[TT][DT], int c, int g) {
#pragma unroll
    for (int t = 0; t < TT; ++t)
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
            const f4v xf = x[t][dt].f();
#pragma unroll
            for (int e = 0; e < 4; ++e) Xt[(dt * 16 + 4 * g + e) * LT + t * 16 + c] = xf[e];
        }
}

__device__ __forceinline__ f4v lds4(const float* p) { return *(const f4v*)p; }

// Wave -> (row group rg, head h); the wave runs rows rg, rg + G, ... (G = gridDim.x / heads) of head h.
// Consecutive workgroups go to different XCDs (b % 8), so the heads of one node row go to
// workgroups b, b+8, b+16, ... -- ONE XCD -- and a row's Q|K|V|dO lines (a 128-B line holds the
// 64-B slices of two heads at d = 16) are fetched into one L2 once instead of into several.
// Needs gridDim.x % (8 * heads) == 0 (the host grid guarantees it when rows >= 8), else the plain map.
__device__ __forceinline__ void v4_wave_map(int heads, int& h, int64_t& rg) {
    const int b = blockIdx.x, nb = gridDim.x;
    if (nb % (8 * heads) == 0) {
        const int y = b >> 3;
        h = y % heads;
        rg = (int64_t)(y / heads) * 8 + (b & 7);
    } else {
        h = b % heads;
        rg = b / heads;
    }
}

// Sᵀ[jt][it] += A[jt]·B[it]ᵀ over the head's features, the row tiles of both operands in registers (lane (c, g):
// row 16t + c, features 16dt + 4g + e): Sᵀ = K·Qᵀ and dPᵀ = V·dOᵀ; BF: stored bf16 operands on the bf16 instruction
template <int TT, int DT, bool BF, typename S>
__device__ __forceinline__ void v4_scores(const Raw4<S> (&a)[TT][DT], const Raw4<S> (&b)[TT][DT], f4v (&acc)[TT][TT]) {
    if constexpr (BF) {
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
            s16x4 pa[TT], pb[TT];
#pragma unroll
            for (int t = 0; t < TT; ++t) {
                pa[t] = pk4(a[t][dt]);
                pb[t] = pk4(b[t][dt]);
            }
#pragma unroll
            for (int jt = 0; jt < TT; ++jt)
#pragma unroll
                for (int it = 0; it < TT; ++it) acc[jt][it] = mfma16bf(pa[jt], pb[it], acc[jt][it]);
        }
    } else {
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
            f4v af[TT], bf[TT];
#pragma unroll
            for (int t = 0; t < TT; ++t) {
                af[t] = a[t][dt].f();
                bf[t] = b[t][dt].f();
            }
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int jt = 0; jt < TT; ++jt)
#pragma unroll
                    for (int it = 0; it < TT; ++it) acc[jt][it] = mfma4(af[jt][e], bf[it][e], acc[jt][it]);
        }
    }
}

template <int TT, int DT, typename S>
__global__ void __launch_bounds__(WAVE, TAGAN_V4_WPE_F) k_tattn_fwd_v4(TArgs A, const float* __restrict__ q,
                                                       const float* __restrict__ k,
                                                       const float* __restrict__ v) {
    TAGAN_LIVE_SEED(A);
    constexpr int TP = 16 * TT, LT = v4_ld(TP);
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int T = A.T, d = A.d;
    const int lane = threadIdx.x, c0 = lane & 15, g0 = lane >> 4;
    int h;
    int64_t rg;
    v4_wave_map(A.heads, h, rg);
    const int64_t G = gridDim.x / A.heads;
    float* Vt = sm;    // [16*DT][LT]
    float bst[TT][TT][4];
    v4_static_bias<TT>(A, h, c0, g0, bst);
    Raw4<S> qv[TT][DT], kv[TT][DT], vv[TT][DT];
    auto load = [&](int64_t rr, int c, int g) {
        const int64_t hb = rr * A.s_row + (int64_t)h * d;
#pragma unroll
        for (int t = 0; t < TT; ++t) {
            const int i = t * 16 + c;
#pragma unroll
            for (int dt = 0; dt < DT; ++dt) {
                const int64_t off = hb + (int64_t)i * A.s_t + dt * 16 + 4 * g;
                qv[t][dt] = ldr4<S>(q, off, i < T);
                kv[t][dt] = ldr4<S>(k, off, i < T);
                vv[t][dt] = ldr4<S>(v, off, i < T);
            }
        }
    };
    if (TAGAN_V4_PREFETCH && rg < A.rows) load(rg, c0, g0);
    for (int64_t r = rg; r < A.rows; r += G) {
        // The lane indices are re-derived per row behind an empty asm: otherwise the compiler hoists
        // every per-element constant built from them (mask / dropout counters, store offsets) out of
        // the row loop into dozens of live registers, and occupancy drops.
        int c = c0, g = g0;
        if (TAGAN_V4_NOHOIST) asm volatile("" : "+v"(c), "+v"(g));
        if (!TAGAN_V4_PREFETCH) load(r, c, g);
        f4v s[TT][TT];   // [jt][it]: Sᵀ tiles
#pragma unroll
        for (int jt = 0; jt < TT; ++jt)
#pragma unroll
            for (int it = 0; it < TT; ++it) s[jt][it] = f4v{0.f, 0.f, 0.f, 0.f};
        v4_scores<TT, DT, bf_scores<S>(), S>(kv, qv, s);
        wave_sync();   // the previous unit's reads of Vt are done
        v4_stage_t<TT, DT, LT>(Vt, vv, c, g);
        if (TAGAN_V4_PREFETCH && r + G < A.rows) load(r + G, c, g);   // next unit's rows in flight during this one
        wave_sync();
        const uint32_t drk = tkey(A, r, h);
        float inv_l[TT];
#pragma unroll
        for (int it = 0; it < TT; ++it) {
            const int i = it * 16 + c;
            float mx = -INFINITY;
#pragma unroll
            for (int jt = 0; jt < TT; ++jt)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float sc = v4_score(A, bst[jt][it][e], r, h, i, jt * 16 + 4 * g + e, s[jt][it][e]);
                    s[jt][it][e] = sc;
                    mx = fmaxf(mx, sc);
                }
            mx = rows_max(mx);
            float l = 0.f;
#pragma unroll
            for (int jt = 0; jt < TT; ++jt)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float sc = s[jt][it][e];
                    const float p = (sc == -INFINITY) ? 0.f : __expf(sc - mx);
                    l += p;
                    s[jt][it][e] = p * drop_scale(A, drk, i, jt * 16 + 4 * g + e);
                }
            l = rows_sum(l);
            inv_l[it] = (l > 0.f) ? 1.f / l : NAN;
            if (g == 0 && i < T) A.lse[(r * A.heads + h) * T + i] = mx + __logf(l);
        }
        f4v o[DT][TT];
#pragma unroll
        for (int dt = 0; dt < DT; ++dt)
#pragma unroll
            for (int it = 0; it < TT; ++it) o[dt][it] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int jt = 0; jt < TT; ++jt)
#pragma unroll
            for (int dt = 0; dt < DT; ++dt) {
                const f4v va = lds4(Vt + (dt * 16 + c) * LT + jt * 16 + 4 * g);   // V[jt*16+4g+e][dt*16+c]
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int it = 0; it < TT; ++it) o[dt][it] = mfma4(va[e], s[jt][it][e], o[dt][it]);
            }
#pragma unroll
        for (int it = 0; it < TT; ++it) {
            const int i = it * 16 + c;
            if (i >= T) continue;
#pragma unroll
            for (int dt = 0; dt < DT; ++dt)
                st4v<S>(A.out, r * A.o_row + (int64_t)i * A.o_t + h * d + dt * 16 + 4 * g, o[dt][it], inv_l[it]);
        }
    }
}

template <int TT, int DT, typename S, int MODE>
__global__ void __launch_bounds__(WAVE, TAGAN_V4_WPE_B) k_tattn_bwd_v4(TArgs A, const float* __restrict__ q,
                                                       const float* __restrict__ k,
                                                       const float* __restrict__ v,
                                                       const float* __restrict__ dout,
                                                       const float* __restrict__ lse) {
    TAGAN_LIVE_SEED(A);
    constexpr int TP = 16 * TT, LD = v4_ld(TP), DP = 16 * DT;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int T = A.T, NB = 2 * T - 1, d = A.d;
    const int lane = threadIdx.x, c0 = lane & 15, g0 = lane >> 4;
    int h;
    int64_t rg;
    v4_wave_map(A.heads, h, rg);
    const int64_t G = gridDim.x / A.heads;
    float* X = sm;               // [TP][LD] transpose tile X[j][i] (dS, then P')
    float* Kt = X + TP * LD;     // [DP][LD] K transposed
    float* Qt = Kt + DP * LD;    // [DP][LD] Q transposed
    float* Ot = Qt + DP * LD;    // [DP][LD] dO transposed
    float bst[TT][TT][4];
    if constexpr (MODE != 0) v4_fast_bias<TT>(A, h, c0, g0, bst);
    else v4_static_bias<TT>(A, h, c0, g0, bst);
    const float msc = A.p_drop > 0.f ? A.inv_keep : 1.f;   // drop_scale of a kept element
    const uint32_t thr = MODE == 2 ? tthr(A.p_drop) : 0u;
    // Σ of dSᵀ over this wave's units, in unit order: the bias-table gradient before its diagonal
    // sums, which run once at the end (fixed order: bitwise reproducible)
    f4v gsum[TT][TT];
#pragma unroll
    for (int jt = 0; jt < TT; ++jt)
#pragma unroll
        for (int it = 0; it < TT; ++it) gsum[jt][it] = f4v{0.f, 0.f, 0.f, 0.f};
    // Σ over this wave's rows and steps of the stored dq | dk | dv (lane: features 16dt + 4g + e), reduced over
    // the step lanes at the end: the QKV projection's bias gradient without a pass over dqkv
    f4v bsum[3][DT];
#pragma unroll
    for (int t3 = 0; t3 < 3; ++t3)
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) bsum[t3][dt] = f4v{0.f, 0.f, 0.f, 0.f};
    Raw4<S> qv[TT][DT], kv[TT][DT], vv[TT][DT], dov[TT][DT];
    float lsev[TT];
    // The next row's Q, K, LSE (and, unless TAGAN_V4_SPLIT, V and dO) are prefetched during this one.
    auto load_qk = [&](int64_t rr, int c, int g) {
        const int64_t hb = rr * A.s_row + (int64_t)h * d;
#pragma unroll
        for (int t = 0; t < TT; ++t) {
            const int i = t * 16 + c;
#pragma unroll
            for (int dt = 0; dt < DT; ++dt) {
                const int64_t off = hb + (int64_t)i * A.s_t + dt * 16 + 4 * g;
                qv[t][dt] = ldr4<S>(q, off, i < T);
                kv[t][dt] = ldr4<S>(k, off, i < T);
            }
            lsev[t] = (i < T) ? lse[(rr * A.heads + h) * T + i] : 0.f;
        }
    };
    auto load_vd = [&](int64_t rr, int c, int g) {
        const int64_t hb = rr * A.s_row + (int64_t)h * d;
#pragma unroll
        for (int t = 0; t < TT; ++t) {
            const int i = t * 16 + c;
#pragma unroll
            for (int dt = 0; dt < DT; ++dt) {
                vv[t][dt] = ldr4<S>(v, hb + (int64_t)i * A.s_t + dt * 16 + 4 * g, i < T);
                dov[t][dt] = ldr4<S>(dout, rr * A.do_row + (int64_t)h * d + (int64_t)i * A.do_t + dt * 16 + 4 * g,
                                     i < T);
            }
        }
    };
    if (TAGAN_V4_PREFETCH && rg < A.rows) {
        load_qk(rg, c0, g0);
        if (!TAGAN_V4_SPLIT) load_vd(rg, c0, g0);
    }
    for (int64_t r = rg; r < A.rows; r += G) {
        // The lane indices are re-derived per row behind an empty asm: otherwise the compiler hoists
        // every per-element constant built from them (mask / dropout counters, store offsets) out of
        // the row loop into dozens of live registers, and occupancy drops.
        int c = c0, g = g0;
        if (TAGAN_V4_NOHOIST) asm volatile("" : "+v"(c), "+v"(g));
        if (!TAGAN_V4_PREFETCH) load_qk(r, c, g);
        if (!TAGAN_V4_PREFETCH || TAGAN_V4_SPLIT) load_vd(r, c, g);
        const uint32_t drk = tkey(A, r, h);
        f4v s[TT][TT], dp[TT][TT];   // [jt][it]: Sᵀ -> P -> P' (dropped P), dPᵀ -> dSᵀ
        float lse_i[TT];
#pragma unroll
        for (int t = 0; t < TT; ++t) lse_i[t] = lsev[t];
#pragma unroll
        for (int jt = 0; jt < TT; ++jt)
#pragma unroll
            for (int it = 0; it < TT; ++it) {
                s[jt][it] = f4v{0.f, 0.f, 0.f, 0.f};
                dp[jt][it] = f4v{0.f, 0.f, 0.f, 0.f};
            }
        v4_scores<TT, DT, bf_scores<S>(), S>(kv, qv, s);
        v4_scores<TT, DT, bf_scores<S>(), S>(vv, dov, dp);
        wave_sync();   // the previous unit's reads of Kt / Qt / Ot / X are done
        v4_stage_t<TT, DT, LD>(Kt, kv, c, g);
        v4_stage_t<TT, DT, LD>(Qt, qv, c, g);
        v4_stage_t<TT, DT, LD>(Ot, dov, c, g);
        if (TAGAN_V4_PREFETCH && r + G < A.rows) {
            load_qk(r + G, c, g);
            if (!TAGAN_V4_SPLIT) load_vd(r + G, c, g);
        }   // next unit's rows in flight during this one
        // P = exp(S - lse); dP·m (m = drop_scale); delta_i = Σ_j P·dP·m (= Σ_c dO∘O, so O is not read);
        // dS = P·(dP·m - delta); P' = P·m
        if constexpr (MODE != 0) {   // fast path (v5_fast_shape): log2 units, keep bit in the sign of P
            const float sc2 = A.inv_sqrt_d * LOG2E_F;
#pragma unroll
            for (int it = 0; it < TT; ++it) {
                const int i = it * 16 + c;
                const float lse2 = lse_i[it] * LOG2E_F;
                const uint32_t cb = (uint32_t)(i * T + 4 * g);
                float dl = 0.f;
#pragma unroll
                for (int jt = 0; jt < TT; ++jt) {
                    uint32_t pw[2] = {0u, 0u};
                    if constexpr (MODE == 2) tpair(drk, cb, jt, pw);
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float p = __builtin_amdgcn_exp2f(fmaf(s[jt][it][e], sc2, bst[jt][it][e]) - lse2);
                        float dpv = dp[jt][it][e];
                        if constexpr (MODE == 2) {
                            uint32_t km;
                            if (e == 0) km = tkeepmask<0>(pw, thr - 1u);
                            else if (e == 1) km = tkeepmask<1>(pw, thr - 1u);
                            else if (e == 2) km = tkeepmask<2>(pw, thr - 1u);
                            else km = tkeepmask<3>(pw, thr - 1u);
                            dpv = fand(dpv * msc, km);
                            s[jt][it][e] = fsignkeep(p, km);
                        } else {
                            s[jt][it][e] = p;
                        }
                        dp[jt][it][e] = dpv;
                        dl = fmaf(p, dpv, dl);
                    }
                }
                dl = rows_sum(dl);
#pragma unroll
                for (int jt = 0; jt < TT; ++jt)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float sv = s[jt][it][e];
                        dp[jt][it][e] = fabsf(sv) * (dp[jt][it][e] - dl);
                        if constexpr (MODE == 2) s[jt][it][e] = fmaxf(sv, 0.f) * msc;
                    }
            }
        } else {
        uint32_t keep = 0;   // bit (jt*TT + it)*4 + e: element kept by the dropout
#pragma unroll
        for (int it = 0; it < TT; ++it) {
            const int i = it * 16 + c;
            float dl = 0.f;
#pragma unroll
            for (int jt = 0; jt < TT; ++jt)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int j = jt * 16 + 4 * g + e;
                    const float sc = v4_score(A, bst[jt][it][e], r, h, i, j, s[jt][it][e]);
                    const float p = (sc == -INFINITY) ? 0.f : __expf(sc - lse_i[it]);
                    const float m = drop_scale(A, drk, i, j);
                    keep |= (m != 0.f ? 1u : 0u) << ((jt * TT + it) * 4 + e);
                    s[jt][it][e] = p;
                    dp[jt][it][e] *= m;
                    dl = fmaf(p, dp[jt][it][e], dl);
                }
            dl = rows_sum(dl);
#pragma unroll
            for (int jt = 0; jt < TT; ++jt)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int j = jt * 16 + 4 * g + e;
                    const float p = s[jt][it][e];
                    const float dsv = p * (dp[jt][it][e] - dl);
                    dp[jt][it][e] = dsv;
                    s[jt][it][e] = ((keep >> ((jt * TT + it) * 4 + e)) & 1u) ? p * msc : 0.f;
                    if (A.dbias_dense && i < T && j < T)
                        A.dbias_dense[((r * A.heads + h) * T + i) * (int64_t)T + j] = dsv;
                }
        }
        }
        if (A.part) {
#pragma unroll
            for (int jt = 0; jt < TT; ++jt)
#pragma unroll
                for (int it = 0; it < TT; ++it) gsum[jt][it] += dp[jt][it];
        }
        // dSᵀ -> X[j][i]
#pragma unroll
        for (int jt = 0; jt < TT; ++jt)
#pragma unroll
            for (int it = 0; it < TT; ++it)
#pragma unroll
                for (int e = 0; e < 4; ++e) X[(jt * 16 + 4 * g + e) * LD + it * 16 + c] = dp[jt][it][e];
        wave_sync();
        // dQᵀ = Kᵀ·dSᵀ: A = K[jt*16+4g+e][dt*16+c] (Kt), B = dSᵀ accumulators
        {
            f4v acc[DT][TT];
#pragma unroll
            for (int dt = 0; dt < DT; ++dt)
#pragma unroll
                for (int it = 0; it < TT; ++it) acc[dt][it] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int jt = 0; jt < TT; ++jt)
#pragma unroll
                for (int dt = 0; dt < DT; ++dt) {
                    const f4v ka = lds4(Kt + (dt * 16 + c) * LD + jt * 16 + 4 * g);
#pragma unroll
                    for (int e = 0; e < 4; ++e)
#pragma unroll
                        for (int it = 0; it < TT; ++it) acc[dt][it] = mfma4(ka[e], dp[jt][it][e], acc[dt][it]);
                }
#pragma unroll
            for (int it = 0; it < TT; ++it) {
                const int i = it * 16 + c;
                if (i >= T) continue;
#pragma unroll
                for (int dt = 0; dt < DT; ++dt)
                    st4v<S>(A.dq, r * A.d_row + (int64_t)i * A.d_t + h * d + dt * 16 + 4 * g, acc[dt][it],
                            A.inv_sqrt_d);
            }
            if (A.qkv_part) {   // padded steps contribute exact zeros (dS = 0 there)
#pragma unroll
                for (int it = 0; it < TT; ++it)
#pragma unroll
                    for (int dt = 0; dt < DT; ++dt) bsum[0][dt] += acc[dt][it] * A.inv_sqrt_d;
            }
        }
        // dKᵀ = Qᵀ·dS (A = Qt, B = X), then dVᵀ = dOᵀ·P' (A = Ot, B = X after P' replaces dS)
#pragma unroll
        for (int pass = 0; pass < 2; ++pass) {
            if (pass == 1) {
                wave_sync();   // dK's reads of X are done
#pragma unroll
                for (int jt = 0; jt < TT; ++jt)
#pragma unroll
                    for (int it = 0; it < TT; ++it)
#pragma unroll
                        for (int e = 0; e < 4; ++e) X[(jt * 16 + 4 * g + e) * LD + it * 16 + c] = s[jt][it][e];
                wave_sync();
            }
            const float* At = pass == 0 ? Qt : Ot;
            f4v acc[DT][TT];
#pragma unroll
            for (int dt = 0; dt < DT; ++dt)
#pragma unroll
                for (int jt = 0; jt < TT; ++jt) acc[dt][jt] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int it = 0; it < TT; ++it) {
                f4v xa[DT], xb[TT];
#pragma unroll
                for (int dt = 0; dt < DT; ++dt) xa[dt] = lds4(At + (dt * 16 + c) * LD + it * 16 + 4 * g);
#pragma unroll
                for (int jt = 0; jt < TT; ++jt) xb[jt] = lds4(X + (jt * 16 + c) * LD + it * 16 + 4 * g);
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int jt = 0; jt < TT; ++jt)
#pragma unroll
                        for (int dt = 0; dt < DT; ++dt) acc[dt][jt] = mfma4(xa[dt][e], xb[jt][e], acc[dt][jt]);
            }
            float* dst = pass == 0 ? A.dk : A.dv;
            const float sc = pass == 0 ? A.inv_sqrt_d : 1.f;
#pragma unroll
            for (int jt = 0; jt < TT; ++jt) {
                const int j = jt * 16 + c;
                if (j >= T) continue;
#pragma unroll
                for (int dt = 0; dt < DT; ++dt)
                    st4v<S>(dst, r * A.d_row + (int64_t)j * A.d_t + h * d + dt * 16 + 4 * g, acc[dt][jt], sc);
            }
            if (A.qkv_part) {
#pragma unroll
                for (int jt = 0; jt < TT; ++jt)
#pragma unroll
                    for (int dt = 0; dt < DT; ++dt) bsum[1 + pass][dt] += acc[dt][jt] * sc;
            }
        }
    }
    if (A.qkv_part) {
        // reduce over the 16 step lanes (fixed butterfly order), lanes c == 0 write features 16dt + 4g + e
        float* prow = A.qkv_part + rg * 3 * (int64_t)A.H + (int64_t)h * d;
#pragma unroll
        for (int t3 = 0; t3 < 3; ++t3)
#pragma unroll
            for (int dt = 0; dt < DT; ++dt)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float v = bsum[t3][dt][e];
                    v = lane_sum<16>(v);
                    if (c0 == 0) prow[t3 * (int64_t)A.H + dt * 16 + 4 * g0 + e] = v;
                }
    }
    if (A.part) {
        // diagonal sums (t = i - j + T - 1) of the summed dS tile in j order; partial row
        // rg holds head h's columns: part[rg][h][t]
        wave_sync();   // the last unit's reads of X are done
#pragma unroll
        for (int jt = 0; jt < TT; ++jt)
#pragma unroll
            for (int it = 0; it < TT; ++it)
#pragma unroll
                for (int e = 0; e < 4; ++e) X[(jt * 16 + 4 * g0 + e) * LD + it * 16 + c0] = gsum[jt][it][e];
        wave_sync();
        float* prow = A.part + rg * A.heads * NB + (int64_t)h * NB;
        for (int t = lane; t < NB; t += WAVE) {
            const int off = t - (T - 1);
            const int j0 = off < 0 ? -off : 0, j1 = off < 0 ? T : T - off;
            float a = 0.f;
            for (int j = j0; j < j1; ++j) a += X[j * LD + j + off];
            prow[t] = a;
        }
    }
}

// ---------------------------------------------------------------------------------------------------------
// v6 (T <= 32, d in {16, 32}: C1, C2, C4): the v4 per-head products, fed through head-group SLABS.  At d = 16 every
// (row, step, head) slice of the time-major [T, N, 3H] projection is a 64-B half line, and the v4 lane -> (step,
// 4 features) loads cap even a compute-free copy of the backward's traffic at 3.3-3.7 TB/s (tools/probes/
// tattn_copy.hip); 256-B+ runs per step reach 5+ TB/s.  So one workgroup of GH waves takes (node row, group of GH
// heads): the whole workgroup streams the row's [T, GH·d] slices of Q | K | V (| dO) with flat float4 loads into one
// LDS slab (issued one unit ahead, held in registers meanwhile), wave w computes head w of the group exactly as v4
// (operands from the slab: b128 rows for the register operands, four b32 reads for the transposed ones; dS / P'
// through a private [TP][TP+8] tile), parks its outputs in its own slab columns, and the workgroup stores the slab
// back as flat float4 runs.
// ---------------------------------------------------------------------------------------------------------
// Build knobs: PREFETCH=1 holds the next unit's slab share in registers during this one (else the slab is loaded
// at the unit's start and the other workgroups on the CU cover the latency); WPE = minimum waves per SIMD.
#ifndef TAGAN_V6_PREFETCH
#define TAGAN_V6_PREFETCH 0
#endif
#ifndef TAGAN_V6_WPE
#define TAGAN_V6_WPE 2
#endif
#ifndef TAGAN_V6_WPE_B
#define TAGAN_V6_WPE_B 3
#endif
// slab pitch: (4 or 3)·GH·DP + 8 floats = 4m with m = 2 (mod 4): conflict-free ds_read_b128 of lanes (c, g)
template <int NT, int GH, int DP>
constexpr int v6_pitch() { return NT * GH * DP + 8; }
size_t v6_fwd_lds(int TT, int DT, int GH) { return (size_t)(16 * TT) * (3 * GH * 16 * DT + 8) * 4; }
size_t v6_bwd_lds(int TT, int DT, int GH) {
    return ((size_t)(16 * TT) * (4 * GH * 16 * DT + 8) + (size_t)GH * 16 * TT * v4_ld(16 * TT)) * 4;
}

// the workgroup's share of one unit's slab: thread tid holds float4 number tid + n·(64·GH), n < NPF
template <int TT, int DT, int GH, int NT, typename S>
struct V6Slab {
    static constexpr int TP = 16 * TT, DP = 16 * DT, C4 = NT * GH * DP / 4, NPF = TP * C4 / (WAVE * GH);
    static constexpr int SP = v6_pitch<NT, GH, DP>();
    Raw4<S> pf[NPF];
    // tensor x of the slab: 0..2 = Q, K, V (row stride s_row, step stride s_t), 3 = dO
    __device__ __forceinline__ void load(const TArgs& A, const void* q, const void* k, const void* v, const void* dout,
                                         int64_t r, int hg) {
#pragma unroll
        for (int n = 0; n < NPF; ++n) {
            const int e = threadIdx.x + n * WAVE * GH, t = e / C4, col = 4 * (e % C4);
            const int x = col / (GH * DP), cc = col % (GH * DP);
            const bool ok = t < A.T;
            if (x < 3) {
                const void* src = x == 0 ? q : x == 1 ? k : v;
                pf[n] = ldr4<S>(src, r * A.s_row + (int64_t)t * A.s_t + hg * GH * DP + cc, ok);
            } else {
                pf[n] = ldr4<S>(dout, r * A.do_row + (int64_t)t * A.do_t + hg * GH * DP + cc, ok);
            }
        }
    }
    __device__ __forceinline__ void park(float* slab) const {
#pragma unroll
        for (int n = 0; n < NPF; ++n) {
            const int e = threadIdx.x + n * WAVE * GH;
            *(f4v*)(slab + (e / C4) * SP + 4 * (e % C4)) = pf[n].f();
        }
    }
};

// v4_scores for one feature tile whose operands were read from the slab
template <int TT, bool BF>
__device__ __forceinline__ void v6_scores(const f4v (&a)[TT], const f4v (&b)[TT], f4v (&acc)[TT][TT]) {
    if constexpr (BF) {
        s16x4 pa[TT], pb[TT];
#pragma unroll
        for (int t = 0; t < TT; ++t) {
            pa[t] = pk4bf(a[t]);
            pb[t] = pk4bf(b[t]);
        }
#pragma unroll
        for (int jt = 0; jt < TT; ++jt)
#pragma unroll
            for (int it = 0; it < TT; ++it) acc[jt][it] = mfma16bf(pa[jt], pb[it], acc[jt][it]);
    } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int jt = 0; jt < TT; ++jt)
#pragma unroll
                for (int it = 0; it < TT; ++it) acc[jt][it] = mfma4(a[jt][e], b[it][e], acc[jt][it]);
    }
}

template <int TT, int DT, int GH, typename S>
__global__ void __launch_bounds__(WAVE * GH, TAGAN_V6_WPE) k_tattn_fwd_v6(TArgs A, const float* __restrict__ q,
                                                            const float* __restrict__ k,
                                                            const float* __restrict__ v) {
    TAGAN_LIVE_SEED(A);
    using Slab = V6Slab<TT, DT, GH, 3, S>;
    constexpr int DP = 16 * DT, SP = Slab::SP;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* slab = sm;   // [TP][SP]: Q | K | V of the group's heads, then O in the Q columns
    const int T = A.T;
    const int w = threadIdx.x / WAVE, lane = threadIdx.x % WAVE, c0 = lane & 15, g0 = lane >> 4;
    const int hgc = A.heads / GH, hg = blockIdx.x % hgc, h = hg * GH + w;
    const int64_t rg = blockIdx.x / hgc, G = gridDim.x / hgc;
    float bst[TT][TT][4];
    v4_static_bias<TT>(A, h, c0, g0, bst);
    Slab io;
    if (TAGAN_V6_PREFETCH && rg < A.rows) io.load(A, q, k, v, nullptr, rg, hg);
    for (int64_t r = rg; r < A.rows; r += G) {
        int c = c0, g = g0;
        asm volatile("" : "+v"(c), "+v"(g));   // see k_tattn_fwd_v4
        if (!TAGAN_V6_PREFETCH) io.load(A, q, k, v, nullptr, r, hg);
        __syncthreads();   // the previous unit's stores have read the slab
        io.park(slab);
        __syncthreads();
        if (TAGAN_V6_PREFETCH && r + G < A.rows) io.load(A, q, k, v, nullptr, r + G, hg);
        const float* sq = slab + w * DP;
        const float* sk = slab + GH * DP + w * DP;
        const float* sv = slab + 2 * GH * DP + w * DP;
        f4v s[TT][TT];
#pragma unroll
        for (int jt = 0; jt < TT; ++jt)
#pragma unroll
            for (int it = 0; it < TT; ++it) s[jt][it] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
            f4v qv[TT], kv[TT];
#pragma unroll
            for (int t = 0; t < TT; ++t) {
                qv[t] = lds4(sq + (t * 16 + c) * SP + dt * 16 + 4 * g);
                kv[t] = lds4(sk + (t * 16 + c) * SP + dt * 16 + 4 * g);
            }
            v6_scores<TT, bf_scores<S>()>(kv, qv, s);
        }
        const uint32_t drk = tkey(A, r, h);
        float inv_l[TT];
#pragma unroll
        for (int it = 0; it < TT; ++it) {
            const int i = it * 16 + c;
            float mx = -INFINITY;
#pragma unroll
            for (int jt = 0; jt < TT; ++jt)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float sc = v4_score(A, bst[jt][it][e], r, h, i, jt * 16 + 4 * g + e, s[jt][it][e]);
                    s[jt][it][e] = sc;
                    mx = fmaxf(mx, sc);
                }
            mx = rows_max(mx);
            float l = 0.f;
#pragma unroll
            for (int jt = 0; jt < TT; ++jt)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float sc = s[jt][it][e];
                    const float p = (sc == -INFINITY) ? 0.f : __expf(sc - mx);
                    l += p;
                    s[jt][it][e] = p * drop_scale(A, drk, i, jt * 16 + 4 * g + e);
                }
            l = rows_sum(l);
            inv_l[it] = (l > 0.f) ? 1.f / l : NAN;
            if (g == 0 && i < T) A.lse[(r * A.heads + h) * T + i] = mx + __logf(l);
        }
        // Oᵀ = Vᵀ·P'ᵀ: A = V[16jt + 4g + e][16dt + c] (four b32 reads of the slab), B = the P'ᵀ accumulators
        f4v o[DT][TT];
#pragma unroll
        for (int dt = 0; dt < DT; ++dt)
#pragma unroll
            for (int it = 0; it < TT; ++it) o[dt][it] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int jt = 0; jt < TT; ++jt)
#pragma unroll
            for (int dt = 0; dt < DT; ++dt)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float va = sv[(jt * 16 + 4 * g + e) * SP + dt * 16 + c];
#pragma unroll
                    for (int it = 0; it < TT; ++it) o[dt][it] = mfma4(va, s[jt][it][e], o[dt][it]);
                }
        __syncthreads();   // every wave is done reading the slab
#pragma unroll
        for (int it = 0; it < TT; ++it)
#pragma unroll
            for (int dt = 0; dt < DT; ++dt)
                *(f4v*)(slab + (it * 16 + c) * SP + w * DP + dt * 16 + 4 * g) = o[dt][it] * inv_l[it];
        __syncthreads();
        // O of the group's heads: the slab's first GH·DP columns, flat float4 runs
        constexpr int OC4 = GH * DP / 4;
        for (int e = threadIdx.x; e < T * OC4; e += WAVE * GH) {
            const int t = e / OC4, col = 4 * (e % OC4);
            st4v<S>(A.out, r * A.o_row + (int64_t)t * A.o_t + hg * GH * DP + col, lds4(slab + t * SP + col), 1.f);
        }
    }
}

template <int TT, int DT, int GH, typename S>
__global__ void __launch_bounds__(WAVE * GH, (TT == 2 && DT == 2) ? 2 : TAGAN_V6_WPE_B) k_tattn_bwd_v6(TArgs A, const float* __restrict__ q,
                                                            const float* __restrict__ k,
                                                            const float* __restrict__ v,
                                                            const float* __restrict__ dout,
                                                            const float* __restrict__ lse) {
    TAGAN_LIVE_SEED(A);
    using Slab = V6Slab<TT, DT, GH, 4, S>;
    constexpr int TP = 16 * TT, LD = v4_ld(TP), DP = 16 * DT, SP = Slab::SP;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* slab = sm;                       // [TP][SP]: Q | K | V | dO, then dQ | dK | dV in the first three
    const int T = A.T, NB = 2 * T - 1, d = A.d;
    const int w = threadIdx.x / WAVE, lane = threadIdx.x % WAVE, c0 = lane & 15, g0 = lane >> 4;
    const int hgc = A.heads / GH, hg = blockIdx.x % hgc, h = hg * GH + w;
    const int64_t rg = blockIdx.x / hgc, G = gridDim.x / hgc;
    float* X = sm + TP * SP + w * TP * LD;   // this wave's [TP][LD] transpose tile (dS, then P')
    // static score part: registers at TT = 1; at TT = 2 the head's bias-table row lives in the unused padding
    // columns TP..TP+7 of this wave's X tile (row t/8, column TP + t%8; 2T-1 <= 63 entries), which keeps the
    // kernel inside 168 VGPRs (3 waves/SIMD) -- with 54 KB of LDS per 4-wave workgroup, 3 fit per CU
    constexpr bool BREG = TT == 1;
    float bst[BREG ? TT : 1][BREG ? TT : 1][4];
    if constexpr (BREG) {
        v4_static_bias<TT>(A, h, c0, g0, bst);
    } else {
        for (int t = lane; t < NB; t += WAVE) X[(t >> 3) * LD + TP + (t & 7)] = A.bias_table ? A.bias_table[h * NB + t] : 0.f;
    }
    const float msc = A.p_drop > 0.f ? A.inv_keep : 1.f;
    f4v gsum[TT][TT];
#pragma unroll
    for (int jt = 0; jt < TT; ++jt)
#pragma unroll
        for (int it = 0; it < TT; ++it) gsum[jt][it] = f4v{0.f, 0.f, 0.f, 0.f};
    f4v bsum[3][DT];
#pragma unroll
    for (int t3 = 0; t3 < 3; ++t3)
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) bsum[t3][dt] = f4v{0.f, 0.f, 0.f, 0.f};
    Slab io;
    float lsev[TT];
    auto load_lse = [&](int64_t rr) {
#pragma unroll
        for (int t = 0; t < TT; ++t) {
            const int i = t * 16 + c0;
            lsev[t] = (i < T) ? lse[(rr * A.heads + h) * T + i] : 0.f;
        }
    };
    if (TAGAN_V6_PREFETCH && rg < A.rows) {
        io.load(A, q, k, v, dout, rg, hg);
        load_lse(rg);
    }
    for (int64_t r = rg; r < A.rows; r += G) {
        int c = c0, g = g0;
        asm volatile("" : "+v"(c), "+v"(g));   // see k_tattn_fwd_v4
        if (!TAGAN_V6_PREFETCH) {
            io.load(A, q, k, v, dout, r, hg);
            load_lse(r);
        }
        __syncthreads();   // the previous unit's stores have read the slab
        io.park(slab);
        float lse_i[TT];
#pragma unroll
        for (int t = 0; t < TT; ++t) lse_i[t] = lsev[t];
        __syncthreads();
        if (TAGAN_V6_PREFETCH && r + G < A.rows) {
            io.load(A, q, k, v, dout, r + G, hg);
            load_lse(r + G);
        }
        const float* sq = slab + w * DP;
        const float* sk = slab + GH * DP + w * DP;
        const float* sv = slab + 2 * GH * DP + w * DP;
        const float* so = slab + 3 * GH * DP + w * DP;
        const uint32_t drk = tkey(A, r, h);
        f4v s[TT][TT], dp[TT][TT];
#pragma unroll
        for (int jt = 0; jt < TT; ++jt)
#pragma unroll
            for (int it = 0; it < TT; ++it) {
                s[jt][it] = f4v{0.f, 0.f, 0.f, 0.f};
                dp[jt][it] = f4v{0.f, 0.f, 0.f, 0.f};
            }
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
            f4v xa[TT], xb[TT];
#pragma unroll
            for (int t = 0; t < TT; ++t) {
                xa[t] = lds4(sk + (t * 16 + c) * SP + dt * 16 + 4 * g);
                xb[t] = lds4(sq + (t * 16 + c) * SP + dt * 16 + 4 * g);
            }
            v6_scores<TT, bf_scores<S>()>(xa, xb, s);
#pragma unroll
            for (int t = 0; t < TT; ++t) {
                xa[t] = lds4(sv + (t * 16 + c) * SP + dt * 16 + 4 * g);
                xb[t] = lds4(so + (t * 16 + c) * SP + dt * 16 + 4 * g);
            }
            v6_scores<TT, bf_scores<S>()>(xa, xb, dp);
        }
        uint32_t keep = 0;
#pragma unroll
        for (int it = 0; it < TT; ++it) {
            const int i = it * 16 + c;
            float dl = 0.f;
#pragma unroll
            for (int jt = 0; jt < TT; ++jt)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int j = jt * 16 + 4 * g + e;
                    float b0;
                    if constexpr (BREG) {
                        b0 = bst[jt][it][e];
                    } else {
                        const int tb = i - j + T - 1;
                        b0 = (i < T && j < T && !(A.causal && j > i)) ? X[(tb >> 3) * LD + TP + (tb & 7)] : -INFINITY;
                    }
                    const float sc = v4_score(A, b0, r, h, i, j, s[jt][it][e]);
                    const float p = (sc == -INFINITY) ? 0.f : __expf(sc - lse_i[it]);
                    const float m = drop_scale(A, drk, i, j);
                    keep |= (m != 0.f ? 1u : 0u) << ((jt * TT + it) * 4 + e);
                    s[jt][it][e] = p;
                    dp[jt][it][e] *= m;
                    dl = fmaf(p, dp[jt][it][e], dl);
                }
            dl = rows_sum(dl);
#pragma unroll
            for (int jt = 0; jt < TT; ++jt)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int j = jt * 16 + 4 * g + e;
                    const float p = s[jt][it][e];
                    const float dsv = p * (dp[jt][it][e] - dl);
                    dp[jt][it][e] = dsv;
                    s[jt][it][e] = ((keep >> ((jt * TT + it) * 4 + e)) & 1u) ? p * msc : 0.f;
                    if (A.dbias_dense && i < T && j < T)
                        A.dbias_dense[((r * A.heads + h) * T + i) * (int64_t)T + j] = dsv;
                }
        }
        if (A.part) {
#pragma unroll
            for (int jt = 0; jt < TT; ++jt)
#pragma unroll
                for (int it = 0; it < TT; ++it) gsum[jt][it] += dp[jt][it];
        }
#pragma unroll
        for (int jt = 0; jt < TT; ++jt)
#pragma unroll
            for (int it = 0; it < TT; ++it)
#pragma unroll
                for (int e = 0; e < 4; ++e) X[(jt * 16 + 4 * g + e) * LD + it * 16 + c] = dp[jt][it][e];
        // dQᵀ = Kᵀ·dSᵀ: A = K[16jt + 4g + e][16dt + c] (four b32 reads), B = the dSᵀ accumulators
        f4v aq[DT][TT];
#pragma unroll
        for (int dt = 0; dt < DT; ++dt)
#pragma unroll
            for (int it = 0; it < TT; ++it) aq[dt][it] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int jt = 0; jt < TT; ++jt)
#pragma unroll
            for (int dt = 0; dt < DT; ++dt)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float ka = sk[(jt * 16 + 4 * g + e) * SP + dt * 16 + c];
#pragma unroll
                    for (int it = 0; it < TT; ++it) aq[dt][it] = mfma4(ka, dp[jt][it][e], aq[dt][it]);
                }
        wave_sync();   // X (dSᵀ) written by the whole wave
        // dKᵀ = Qᵀ·dS (B = X), then dVᵀ = dOᵀ·P' (B = X after P'ᵀ replaces dSᵀ).  Each output is parked in this
        // head's slab columns as soon as its source columns are dead for this wave (only wave w reads head w's
        // columns): dK over K (K last read by dQ), then dQ over Q (Q last read by dK), dV over V (V last read by dP).
#pragma unroll
        for (int pass = 0; pass < 2; ++pass) {
            if (pass == 1) {
                wave_sync();   // dK's reads of X are done
#pragma unroll
                for (int jt = 0; jt < TT; ++jt)
#pragma unroll
                    for (int it = 0; it < TT; ++it)
#pragma unroll
                        for (int e = 0; e < 4; ++e) X[(jt * 16 + 4 * g + e) * LD + it * 16 + c] = s[jt][it][e];
                wave_sync();
            }
            const float* At = pass == 0 ? sq : so;
            f4v acc[DT][TT];
#pragma unroll
            for (int dt = 0; dt < DT; ++dt)
#pragma unroll
                for (int jt = 0; jt < TT; ++jt) acc[dt][jt] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int it = 0; it < TT; ++it) {
                f4v xb[TT];
#pragma unroll
                for (int jt = 0; jt < TT; ++jt) xb[jt] = lds4(X + (jt * 16 + c) * LD + it * 16 + 4 * g);
#pragma unroll
                for (int dt = 0; dt < DT; ++dt)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float xa = At[(it * 16 + 4 * g + e) * SP + dt * 16 + c];
#pragma unroll
                        for (int jt = 0; jt < TT; ++jt) acc[dt][jt] = mfma4(xa, xb[jt][e], acc[dt][jt]);
                    }
            }
            const float sc = pass == 0 ? A.inv_sqrt_d : 1.f;
            float* dst = slab + (pass == 0 ? GH * DP : 2 * GH * DP) + w * DP;   // dK over K, dV over V
#pragma unroll
            for (int t = 0; t < TT; ++t)
#pragma unroll
                for (int dt = 0; dt < DT; ++dt) {
                    const f4v vv = acc[dt][t] * sc;
                    *(f4v*)(dst + (t * 16 + c) * SP + dt * 16 + 4 * g) = vv;
                    if (A.qkv_part) bsum[1 + pass][dt] += vv;   // padded steps add exact zeros
                }
            if (pass == 0) {   // Q is dead for this wave: dQ over Q
#pragma unroll
                for (int t = 0; t < TT; ++t)
#pragma unroll
                    for (int dt = 0; dt < DT; ++dt) {
                        const f4v vq = aq[dt][t] * A.inv_sqrt_d;
                        *(f4v*)(slab + (t * 16 + c) * SP + w * DP + dt * 16 + 4 * g) = vq;
                        if (A.qkv_part) bsum[0][dt] += vq;
                    }
            }
        }
        __syncthreads();   // every head's dQ | dK | dV is parked
        // dQ | dK | dV of the group's heads as flat float4 runs (the layout of Q | K | V)
        constexpr int OC4 = 3 * GH * DP / 4;
        for (int e = threadIdx.x; e < T * OC4; e += WAVE * GH) {
            const int t = e / OC4, col = 4 * (e % OC4);
            const int x = col / (GH * DP), cc = col % (GH * DP);
            float* dst = x == 0 ? A.dq : x == 1 ? A.dk : A.dv;
            st4v<S>(dst, r * A.d_row + (int64_t)t * A.d_t + hg * GH * DP + cc, lds4(slab + t * SP + col), 1.f);
        }
    }
    if (A.qkv_part) {
        float* prow = A.qkv_part + rg * 3 * (int64_t)A.H + (int64_t)h * d;
#pragma unroll
        for (int t3 = 0; t3 < 3; ++t3)
#pragma unroll
            for (int dt = 0; dt < DT; ++dt)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float v = bsum[t3][dt][e];
                    v = lane_sum<16>(v);
                    if (c0 == 0) prow[t3 * (int64_t)A.H + dt * 16 + 4 * g0 + e] = v;
                }
    }
    if (A.part) {
        wave_sync();   // the last unit's reads of X are done
#pragma unroll
        for (int jt = 0; jt < TT; ++jt)
#pragma unroll
            for (int it = 0; it < TT; ++it)
#pragma unroll
                for (int e = 0; e < 4; ++e) X[(jt * 16 + 4 * g0 + e) * LD + it * 16 + c0] = gsum[jt][it][e];
        wave_sync();
        float* prow = A.part + rg * A.heads * NB + (int64_t)h * NB;
        for (int t = lane; t < NB; t += WAVE) {
            const int off = t - (T - 1);
            const int j0 = off < 0 ? -off : 0, j1 = off < 0 ? T : T - off;
            float a = 0.f;
            for (int j = j0; j < j1; ++j) a += X[j * LD + j + off];
            prow[t] = a;
        }
    }
}

// ---------------------------------------------------------------------------------------------------------
// v5 (T in (16, 128], d in {16, 32}: C3's T = 64, C5's T = 128): one WORKGROUP of TT waves per (node row, head)
// unit, TP = 16·TT >= T steps (TT in {2, 4, 8}).  Wave w owns query tile w (steps 16w .. 16w+15) in the score,
// softmax and dQ products and key tile w in the dK / dV products, so no wave holds more than one 16-step
// column of the T x T score matrix (v4 keeps all of it in one wave: > 256 VGPRs at T = 64).  Per unit the
// waves stage their K | V rows (row-major, the A operand of Sᵀ = K·Qᵀ and dPᵀ = V·dOᵀ) and Kᵀ, Qᵀ, dOᵀ (the A
// operands of dQᵀ, dKᵀ, dVᵀ) once into the workgroup's LDS; dSᵀ and then P'ᵀ pass between the query-tile and
// key-tile phases through one shared [TP][LD] tile.  Five T x T x d products per unit (none recomputed), all on
// v_mfma_f32_16x16x4_f32; no atomics (every sum has a fixed order), so results are bitwise reproducible.
// ---------------------------------------------------------------------------------------------------------
// Row stride of the row-major K | V tiles: lane (c, g) reads 16 B at row c, column 4g, and with stride 4m
// dwords (m = DP/4 + 2 = 6 or 10, i.e. m = 2 mod 4) the 16-lane groups of ds_read_b128 hit distinct bank slots
// (the same argument as v4_ld).
constexpr int v5_lk(int DP) { return DP + 8; }
#ifndef TAGAN_V5B_IL
#define TAGAN_V5B_IL 1   // 0: the fast-path backward without the software pipelining of phase 1 (A/B builds)
#endif
size_t v5_fwd_lds(int TT, int DT) { return (size_t)(16 * TT * v5_lk(16 * DT) + 16 * DT * v4_ld(16 * TT) + 32 * TT) * 4; }
size_t v5_bwd_lds(int TT, int DT) {
    const int TP = 16 * TT, DP = 16 * DT;
    return (size_t)(TP * v4_ld(TP) + 3 * DP * v4_ld(TP) + 2 * TP * v5_lk(DP) + 2 * TP) * 4;
}

// static score part of the lane's elements of query tile it (i = 16·it + c, j = 16·jt + 4g + e): see v4_static_bias
template <int TT>
__device__ __forceinline__ void v5_static_bias(const TArgs& A, int h, int it, int c, int g, float (&bst)[TT][4]) {
    const int T = A.T, NB = 2 * T - 1;
    const int i = it * 16 + c;
#pragma unroll
    for (int jt = 0; jt < TT; ++jt)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int j = jt * 16 + 4 * g + e;
            const bool ok = i < T && j < T && !(A.causal && j > i);
            bst[jt][e] = ok ? (A.bias_table ? A.bias_table[h * NB + i - j + T - 1] : 0.f) : -INFINITY;
        }
}

// log2-scaled bias-table values of the lane's elements (fast path: every element valid)
template <int TT>
__device__ __forceinline__ void v5_fast_bias(const TArgs& A, int h, int it, int c, int g, float (&bst)[TT][4]) {
    const int T = A.T, i = it * 16 + c;
#pragma unroll
    for (int jt = 0; jt < TT; ++jt)
#pragma unroll
        for (int e = 0; e < 4; ++e)
            bst[jt][e] = A.bias_table ? A.bias_table[h * (2 * T - 1) + i - (jt * 16 + 4 * g + e) + T - 1] * LOG2E_F : 0.f;
}

// the head's table row staged REVERSED and log2-scaled (TT = 8): element (i, j) at Br[T - 1 - i + j], so a lane's
// elements sit at one per-lane base + compile-time offsets (immediate-offset LDS reads)
__device__ __forceinline__ void v5_stage_bias_rev(const TArgs& A, int h, float* Br, int nthreads) {
    const int NB = 2 * A.T - 1;
    for (int t = threadIdx.x; t < NB; t += nthreads) Br[t] = A.bias_table ? A.bias_table[h * NB + NB - 1 - t] * LOG2E_F : 0.f;
}

template <int TT, int DT, typename S, int MODE>
__global__ void __launch_bounds__(WAVE * TT) k_tattn_fwd_v5(TArgs A, const float* __restrict__ q,
                                                            const float* __restrict__ k,
                                                            const float* __restrict__ v) {
    TAGAN_LIVE_SEED(A);
    constexpr int TP = 16 * TT, LT = v4_ld(TP), DP = 16 * DT, LK = v5_lk(DP);
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* Kr = sm;              // [TP][LK] K row-major
    float* Vt = Kr + TP * LK;    // [DP][LT] V transposed
    float* Bt = Vt + DP * LT;    // [2TP] the head's bias-table row (BREG false)
    const int T = A.T, d = A.d;
    const int w = threadIdx.x / WAVE, lane = threadIdx.x % WAVE, c0 = lane & 15, g0 = lane >> 4;
    int h;
    int64_t rg;
    v4_wave_map(A.heads, h, rg);
    const int64_t G = gridDim.x / A.heads;
    constexpr bool BREG = TT <= 4;   // as in k_tattn_bwd_v5: at TT = 8 the table row is read from LDS
    float bst[BREG ? TT : 1][4];
    if constexpr (MODE != 0) {
        if constexpr (BREG) v5_fast_bias<TT>(A, h, w, c0, g0, bst);
        else v5_stage_bias_rev(A, h, Bt, WAVE * TT);
    } else if constexpr (BREG) {
        v5_static_bias<TT>(A, h, w, c0, g0, bst);
    } else {
        for (int t = threadIdx.x; t < 2 * T - 1; t += WAVE * TT) Bt[t] = A.bias_table ? A.bias_table[h * (2 * T - 1) + t] : 0.f;
    }
    const uint32_t thr = MODE >= 2 ? tthr(A.p_drop) : 0u;
    Raw4<S> qv[DT], kv[DT], vv[DT];
    auto load = [&](int64_t rr) {
        const int i = w * 16 + c0;
        const int64_t off = rr * A.s_row + (int64_t)h * d + (int64_t)i * A.s_t + 4 * g0;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
            qv[dt] = ldr4<S>(q, off + dt * 16, i < T);
            kv[dt] = ldr4<S>(k, off + dt * 16, i < T);
            vv[dt] = ldr4<S>(v, off + dt * 16, i < T);
        }
    };
    if (rg < A.rows) load(rg);
    for (int64_t r = rg; r < A.rows; r += G) {
        int c = c0, g = g0;
        asm volatile("" : "+v"(c), "+v"(g));   // see k_tattn_fwd_v4
        const int i = w * 16 + c;
        __syncthreads();   // the previous unit's reads of Kr / Vt are done
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
            *(f4v*)(Kr + i * LK + dt * 16 + 4 * g) = kv[dt].f();
            const f4v vf = vv[dt].f();
#pragma unroll
            for (int e = 0; e < 4; ++e) Vt[(dt * 16 + 4 * g + e) * LT + i] = vf[e];
        }
        constexpr bool BFS = bf_scores<S>();
        f4v qc[BFS ? 1 : DT];
        s16x4 qb[BFS ? DT : 1];
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
            if constexpr (BFS) qb[dt] = pk4(qv[dt]);
            else qc[dt] = qv[dt].f();
        }
        __syncthreads();
        if (r + G < A.rows) load(r + G);   // the next unit's rows in flight during this one
        f4v s[TT];   // Sᵀ tiles [jt] of query tile w
#pragma unroll
        for (int jt = 0; jt < TT; ++jt) {
            s[jt] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int dt = 0; dt < DT; ++dt) {
                const f4v ka = lds4(Kr + (jt * 16 + c) * LK + dt * 16 + 4 * g);   // K[16jt + c][16dt + 4g + e]
                if constexpr (BFS) {
                    s[jt] = mfma16bf(pk4bf(ka), qb[dt], s[jt]);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) s[jt] = mfma4(ka[e], qc[dt][e], s[jt]);
                }
            }
        }
        const uint32_t drk = tkey(A, r, h);
        float inv_l;
        f4v o[DT][2];   // Oᵀ, two accumulator chains per feature tile
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) o[dt][0] = o[dt][1] = f4v{0.f, 0.f, 0.f, 0.f};
        if constexpr (MODE != 0) {   // fast path: scores in log2 units, every element valid
            const float sc2 = A.inv_sqrt_d * LOG2E_F;
            const int rb = T - 1 - i + 4 * g;
            float mx = -INFINITY;
#pragma unroll
            for (int jt = 0; jt < TT; ++jt)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float b2 = BREG ? bst[jt][e] : Bt[rb + jt * 16 + e];
                    const float sc = fmaf(s[jt][e], sc2, b2);
                    s[jt][e] = sc;
                    mx = fmaxf(mx, sc);
                }
            mx = rows_max(mx);
            const uint32_t cb = (uint32_t)(i * T + 4 * g);   // dropout counter of element (jt, e): cb + 16 jt + e
            float l = 0.f;
            uint32_t kw = 0;   // MODE 3: keep bit of element (jt, e) at bit 4 jt + e, for the backward
            auto soft = [&](int jt) {
                uint32_t pw[2] = {0u, 0u};
                if constexpr (MODE >= 2) tpair(drk, cb, jt, pw);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float p = __builtin_amdgcn_exp2f(s[jt][e] - mx);
                    l += p;
                    if constexpr (MODE >= 2) {
                        uint32_t km;
                        if (e == 0) km = tkeepmask<0>(pw, thr - 1u);
                        else if (e == 1) km = tkeepmask<1>(pw, thr - 1u);
                        else if (e == 2) km = tkeepmask<2>(pw, thr - 1u);
                        else km = tkeepmask<3>(pw, thr - 1u);
                        if constexpr (MODE == 3) kw |= km & (1u << (jt * 4 + e));
                        s[jt][e] = fand(p, km);
                    } else {
                        s[jt][e] = p;
                    }
                }
            };
            // Oᵀ = Vᵀ·P'ᵀ: the products of key tile jt issued between the softmax instructions of tile jt+1
            soft(0);
#pragma unroll
            for (int jt = 0; jt < TT; ++jt) {
                if (jt + 1 < TT) soft(jt + 1);
#pragma unroll
                for (int dt = 0; dt < DT; ++dt) {
                    const f4v va = lds4(Vt + (dt * 16 + c) * LT + jt * 16 + 4 * g);   // V[16jt + 4g + e][16dt + c]
#pragma unroll
                    for (int e = 0; e < 4; ++e) o[dt][jt & 1] = mfma4(va[e], s[jt][e], o[dt][jt & 1]);
                }
                if (jt + 1 < TT) {
#pragma unroll
                    for (int k2 = 0; k2 < 4 * DT; ++k2) {
                        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            l = rows_sum(l);
            inv_l = (MODE >= 2 ? A.inv_keep : 1.f) / l;
            if (g == 0) A.lse[(r * A.heads + h) * T + i] = (mx + __log2f(l)) * LN2_F;
            if constexpr (MODE == 3) A.keep[((r * A.heads + h) * TT + w) * WAVE + lane] = kw;
        } else {
        float mx = -INFINITY;
#pragma unroll
        for (int jt = 0; jt < TT; ++jt)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int j = jt * 16 + 4 * g + e;
                float b0;
                if constexpr (BREG) {
                    b0 = bst[jt][e];
                } else {
                    b0 = (i < T && j < T && !(A.causal && j > i)) ? Bt[i - j + T - 1] : -INFINITY;
                }
                const float sc = v4_score(A, b0, r, h, i, j, s[jt][e]);
                s[jt][e] = sc;
                mx = fmaxf(mx, sc);
            }
        mx = rows_max(mx);
        float l = 0.f;
#pragma unroll
        for (int jt = 0; jt < TT; ++jt)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float sc = s[jt][e];
                const float p = (sc == -INFINITY) ? 0.f : __expf(sc - mx);
                l += p;
                s[jt][e] = p * drop_scale(A, drk, i, jt * 16 + 4 * g + e);
            }
        l = rows_sum(l);
        inv_l = (l > 0.f) ? 1.f / l : NAN;
        if (g == 0 && i < T) A.lse[(r * A.heads + h) * T + i] = mx + __logf(l);
#pragma unroll
        for (int jt = 0; jt < TT; ++jt)
#pragma unroll
            for (int dt = 0; dt < DT; ++dt) {
                const f4v va = lds4(Vt + (dt * 16 + c) * LT + jt * 16 + 4 * g);   // V[16jt + 4g + e][16dt + c]
#pragma unroll
                for (int e = 0; e < 4; ++e) o[dt][jt & 1] = mfma4(va[e], s[jt][e], o[dt][jt & 1]);
            }
        }
        if (i < T) {
#pragma unroll
            for (int dt = 0; dt < DT; ++dt)
                st4v<S>(A.out, r * A.o_row + (int64_t)i * A.o_t + h * d + dt * 16 + 4 * g, o[dt][0] + o[dt][1], inv_l);
        }
    }
}

template <int TT, int DT, typename S, int MODE>
__global__ void __launch_bounds__(WAVE * TT) k_tattn_bwd_v5(TArgs A, const float* __restrict__ q,
                                                            const float* __restrict__ k,
                                                            const float* __restrict__ v,
                                                            const float* __restrict__ dout,
                                                            const float* __restrict__ lse) {
    TAGAN_LIVE_SEED(A);
    constexpr int TP = 16 * TT, LD = v4_ld(TP), DP = 16 * DT, LK = v5_lk(DP);
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* X = sm;               // [TP][LD]: dSᵀ[j][i], then P'ᵀ[j][i]
    float* Kt = X + TP * LD;     // [DP][LD] Kᵀ
    float* Qt = Kt + DP * LD;    // [DP][LD] Qᵀ
    float* Ot = Qt + DP * LD;    // [DP][LD] dOᵀ
    float* Kr = Ot + DP * LD;    // [TP][LK] K row-major
    float* Vr = Kr + TP * LK;    // [TP][LK] V row-major
    float* Bt = Vr + TP * LK;    // [2TP] the head's bias-table row (BREG false)
    const int T = A.T, NB = 2 * T - 1, d = A.d;
    const int w = threadIdx.x / WAVE, lane = threadIdx.x % WAVE, c0 = lane & 15, g0 = lane >> 4;
    int h;
    int64_t rg;
    v4_wave_map(A.heads, h, rg);
    const int64_t G = gridDim.x / A.heads;
    // static score part in registers up to TT = 4; at TT = 8 those 32 VGPRs would spill, so the head's
    // bias-table row is read from LDS per element instead
    constexpr bool BREG = TT <= 4;
    float bst[BREG ? TT : 1][4];
    if constexpr (MODE != 0) {
        if constexpr (BREG) v5_fast_bias<TT>(A, h, w, c0, g0, bst);
        else v5_stage_bias_rev(A, h, Bt, WAVE * TT);   // (visible after the first unit's staging barrier)
    } else if constexpr (BREG) {
        v5_static_bias<TT>(A, h, w, c0, g0, bst);
    } else {
        for (int t = threadIdx.x; t < NB; t += WAVE * TT) Bt[t] = A.bias_table ? A.bias_table[h * NB + t] : 0.f;
        // (visible to all waves after the first unit's staging barrier)
    }
    const float msc = A.p_drop > 0.f ? A.inv_keep : 1.f;
    // the pipelined MODE 3 path carries dS and P' without the 1 / (1 - p) factor and applies it to dQ, dK, dV and the
    // bias-table sums instead (one multiply per output instead of two per element)
    const float fsc = (MODE == 3 && TAGAN_V5B_IL) ? msc : 1.f;
    const uint32_t thr = MODE >= 2 ? tthr(A.p_drop) : 0u;
    f4v gsum[TT];   // Σ over units of dSᵀ[jt tiles][query tile w]: the bias-table gradient before its diagonal sums
#pragma unroll
    for (int jt = 0; jt < TT; ++jt) gsum[jt] = f4v{0.f, 0.f, 0.f, 0.f};
    f4v bsum[3][DT];   // Σ of the stored dq (query tile w) | dk | dv (key tile w): the QKV bias gradient
#pragma unroll
    for (int t3 = 0; t3 < 3; ++t3)
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) bsum[t3][dt] = f4v{0.f, 0.f, 0.f, 0.f};
    Raw4<S> qv[DT], kv[DT], vv[DT], dov[DT];
    float lsev;
    uint32_t kwv = 0;   // MODE 3: the forward's keep bits of this lane's elements (bit 4 jt + e)
    auto load = [&](int64_t rr) {
        const int i = w * 16 + c0;
        const int64_t off = rr * A.s_row + (int64_t)h * d + (int64_t)i * A.s_t + 4 * g0;
        const int64_t offd = rr * A.do_row + (int64_t)h * d + (int64_t)i * A.do_t + 4 * g0;
        if constexpr (MODE == 3) kwv = A.keep[((rr * A.heads + h) * TT + w) * WAVE + lane];
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
            qv[dt] = ldr4<S>(q, off + dt * 16, i < T);
            kv[dt] = ldr4<S>(k, off + dt * 16, i < T);
            vv[dt] = ldr4<S>(v, off + dt * 16, i < T);
            dov[dt] = ldr4<S>(dout, offd + dt * 16, i < T);
        }
        lsev = (i < T) ? lse[(rr * A.heads + h) * T + i] : 0.f;
    };
    if (rg < A.rows) load(rg);
    for (int64_t r = rg; r < A.rows; r += G) {
        int c = c0, g = g0;
        asm volatile("" : "+v"(c), "+v"(g));   // see k_tattn_fwd_v4
        const int i = w * 16 + c;   // this lane's query step (phase 1) and key step (phase 2)
        __syncthreads();   // the previous unit's reads of every LDS tile are done
        f4v qf[DT], df[DT];   // this unit's Q and dO rows as fp32 (the f32-instruction score products read them)
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
            const f4v kf = kv[dt].f();
            qf[dt] = qv[dt].f();
            df[dt] = dov[dt].f();
            *(f4v*)(Kr + i * LK + dt * 16 + 4 * g) = kf;
            *(f4v*)(Vr + i * LK + dt * 16 + 4 * g) = vv[dt].f();
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                Kt[(dt * 16 + 4 * g + e) * LD + i] = kf[e];
                Qt[(dt * 16 + 4 * g + e) * LD + i] = qf[dt][e];
                Ot[(dt * 16 + 4 * g + e) * LD + i] = df[dt][e];
            }
        }
        const float lse_i = lsev;
        const uint32_t kw = kwv;
        constexpr bool BFS = bf_scores<S>();
        s16x4 qb[BFS ? DT : 1], db[BFS ? DT : 1];   // the query tile's Q and dO as packed bf16 operands
        if constexpr (BFS) {
#pragma unroll
            for (int dt = 0; dt < DT; ++dt) {
                qb[dt] = pk4(qv[dt]);
                db[dt] = pk4(dov[dt]);
            }
        }
        // Sᵀ and dPᵀ of key tile jt (A = K | V rows of the key tile from LDS, B = this lane's query row)
        auto sdp0 = [&](int jt, f4v& sj, f4v& dpj) {
            sj = f4v{0.f, 0.f, 0.f, 0.f};
            dpj = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int dt = 0; dt < DT; ++dt) {
                const f4v ka = lds4(Kr + (jt * 16 + c) * LK + dt * 16 + 4 * g);
                const f4v va = lds4(Vr + (jt * 16 + c) * LK + dt * 16 + 4 * g);
                if constexpr (BFS) {
                    sj = mfma16bf(pk4bf(ka), qb[dt], sj);
                    dpj = mfma16bf(pk4bf(va), db[dt], dpj);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        sj = mfma4(ka[e], qf[dt][e], sj);
                        dpj = mfma4(va[e], df[dt][e], dpj);
                    }
                }
            }
        };
        __syncthreads();
        // ---- phase 1, query tile w: Sᵀ, dPᵀ (all key tiles), P, δ, dS, P', dQ
        f4v s[TT], dp[TT];
        if constexpr (MODE != 0 && TAGAN_V5B_IL) {
            // fast path, software-pipelined: the softmax / dropout VALU work of key tile jt issues between the
            // S / dP products of tile jt + 1, and dS of tile jt + 1 between the dQ products of tile jt
            auto sdp = [&](int jt) { sdp0(jt, s[jt], dp[jt]); };
            const uint32_t drk = tkey(A, r, h);
            const float sc2 = A.inv_sqrt_d * LOG2E_F, lse2 = lse_i * LOG2E_F;
            const int rb = T - 1 - i + 4 * g;
            const uint32_t cb = (uint32_t)(i * T + 4 * g);
            float dl = 0.f;
            auto softA = [&](int jt) {   // P, the keep decision (sign of P), masked dP, Σ P·dP
                uint32_t pw[2] = {0u, 0u};
                if constexpr (MODE == 2) tpair(drk, cb, jt, pw);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float b2 = BREG ? bst[jt][e] : Bt[rb + jt * 16 + e];
                    const float p = __builtin_amdgcn_exp2f(fmaf(s[jt][e], sc2, b2) - lse2);
                    float dpv = dp[jt][e];
                    if constexpr (MODE == 3) {   // keep bits at hand: no sign trick; 1 / (1 - p) folded into the outputs
                        dpv = fand(dpv, tbitmask(kw, jt * 4 + e));
                        s[jt][e] = p;
                    } else if constexpr (MODE == 2) {
                        uint32_t km;
                        if (e == 0) km = tkeepmask<0>(pw, thr - 1u);
                        else if (e == 1) km = tkeepmask<1>(pw, thr - 1u);
                        else if (e == 2) km = tkeepmask<2>(pw, thr - 1u);
                        else km = tkeepmask<3>(pw, thr - 1u);
                        dpv = fand(dpv * msc, km);
                        s[jt][e] = fsignkeep(p, km);
                    } else {
                        s[jt][e] = p;
                    }
                    dp[jt][e] = dpv;
                    dl = fmaf(p, dpv, dl);
                }
            };
            constexpr int NM = (BFS ? 2 : 8) * DT;         // products per key tile
            constexpr int VA = (MODE == 3 ? 40 : 64) / NM;  // VALU of softA per product slot
            sdp(0);
#pragma unroll
            for (int jt = 0; jt < TT; ++jt) {
                if (jt + 1 < TT) sdp(jt + 1);
                softA(jt);
                if (jt + 1 < TT) {
#pragma unroll
                    for (int k2 = 0; k2 < NM; ++k2) {
                        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x002, VA, 0);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            if (r + G < A.rows) load(r + G);   // the next unit's rows in flight during the rest of this one
            dl = rows_sum(dl);
            auto softB = [&](int jt) {   // dS (to X, transposed, and kept for dQ), P' in s, the bias-table sum
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float sv = s[jt][e];
                    const float dsv = (MODE == 3 ? sv : fabsf(sv)) * (dp[jt][e] - dl);   // (MODE 3: dS (1 - p))
                    dp[jt][e] = dsv;
                    if constexpr (MODE == 3) s[jt][e] = fand(sv, tbitmask(kw, jt * 4 + e));   // P' (1 - p)
                    else if constexpr (MODE == 2) s[jt][e] = fmaxf(sv, 0.f) * msc;
                    X[(jt * 16 + 4 * g + e) * LD + i] = dsv;   // dSᵀ[j][i]
                }
                gsum[jt] += dp[jt];   // (unused when A.part is null)
            };
            f4v acc[DT][2];
#pragma unroll
            for (int dt = 0; dt < DT; ++dt) acc[dt][0] = acc[dt][1] = f4v{0.f, 0.f, 0.f, 0.f};
            softB(0);
#pragma unroll
            for (int jt = 0; jt < TT; ++jt) {
                if (jt + 1 < TT) softB(jt + 1);
#pragma unroll
                for (int dt = 0; dt < DT; ++dt) {   // dQᵀ += Kᵀ[dt tile][key tile jt] · dSᵀ[jt]
                    const f4v ka = lds4(Kt + (dt * 16 + c) * LD + jt * 16 + 4 * g);
#pragma unroll
                    for (int e = 0; e < 4; ++e) acc[dt][jt & 1] = mfma4(ka[e], dp[jt][e], acc[dt][jt & 1]);
                }
                if (jt + 1 < TT) {
#pragma unroll
                    for (int k2 = 0; k2 < 4 * DT; ++k2) {
                        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x002, 6 / DT + 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int dt = 0; dt < DT; ++dt) {
                const f4v a = acc[dt][0] + acc[dt][1];
                st4v<S>(A.dq, r * A.d_row + (int64_t)i * A.d_t + h * d + dt * 16 + 4 * g, a, A.inv_sqrt_d * fsc);
                bsum[0][dt] += a * (A.inv_sqrt_d * fsc);
            }
        } else {
#pragma unroll
        for (int jt = 0; jt < TT; ++jt) sdp0(jt, s[jt], dp[jt]);
        if (r + G < A.rows) load(r + G);   // the next unit's rows in flight during the rest of this one
        const uint32_t drk = tkey(A, r, h);
        if constexpr (MODE != 0) {   // fast path (see v5_fast_shape): log2 units, keep bit in the sign of P
            const float sc2 = A.inv_sqrt_d * LOG2E_F, lse2 = lse_i * LOG2E_F;
            const int rb = T - 1 - i + 4 * g;
            const uint32_t cb = (uint32_t)(i * T + 4 * g);
            float dl = 0.f;
#pragma unroll
            for (int jt = 0; jt < TT; ++jt) {
                uint32_t pw[2] = {0u, 0u};
                if constexpr (MODE == 2) tpair(drk, cb, jt, pw);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float b2 = BREG ? bst[jt][e] : Bt[rb + jt * 16 + e];
                    const float p = __builtin_amdgcn_exp2f(fmaf(s[jt][e], sc2, b2) - lse2);
                    float dpv = dp[jt][e];
                    if constexpr (MODE >= 2) {
                        uint32_t km;
                        if constexpr (MODE == 3) km = tbitmask(kw, jt * 4 + e);
                        else if (e == 0) km = tkeepmask<0>(pw, thr - 1u);
                        else if (e == 1) km = tkeepmask<1>(pw, thr - 1u);
                        else if (e == 2) km = tkeepmask<2>(pw, thr - 1u);
                        else km = tkeepmask<3>(pw, thr - 1u);
                        dpv = fand(dpv * msc, km);
                        s[jt][e] = fsignkeep(p, km);
                    } else {
                        s[jt][e] = p;
                    }
                    dp[jt][e] = dpv;
                    dl = fmaf(p, dpv, dl);
                }
            }
            dl = rows_sum(dl);
#pragma unroll
            for (int jt = 0; jt < TT; ++jt)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float sv = s[jt][e];
                    const float dsv = fabsf(sv) * (dp[jt][e] - dl);
                    dp[jt][e] = dsv;
                    if constexpr (MODE >= 2) s[jt][e] = fmaxf(sv, 0.f) * msc;
                    X[(jt * 16 + 4 * g + e) * LD + i] = dsv;   // dSᵀ[j][i]
                }
        } else {
        uint32_t keep = 0;   // bit jt*4 + e: element kept by the dropout
        float dl = 0.f;
#pragma unroll
        for (int jt = 0; jt < TT; ++jt)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int j = jt * 16 + 4 * g + e;
                float b0;
                if constexpr (BREG) {
                    b0 = bst[jt][e];
                } else {
                    b0 = (i < T && j < T && !(A.causal && j > i)) ? Bt[i - j + T - 1] : -INFINITY;
                }
                const float sc = v4_score(A, b0, r, h, i, j, s[jt][e]);
                const float p = (sc == -INFINITY) ? 0.f : __expf(sc - lse_i);
                const float m = drop_scale(A, drk, i, j);
                keep |= (m != 0.f ? 1u : 0u) << (jt * 4 + e);
                s[jt][e] = p;
                dp[jt][e] *= m;
                dl = fmaf(p, dp[jt][e], dl);
            }
        dl = rows_sum(dl);
#pragma unroll
        for (int jt = 0; jt < TT; ++jt)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int j = jt * 16 + 4 * g + e;
                const float p = s[jt][e];
                const float dsv = p * (dp[jt][e] - dl);
                dp[jt][e] = dsv;
                s[jt][e] = ((keep >> (jt * 4 + e)) & 1u) ? p * msc : 0.f;
                if (A.dbias_dense && i < T && j < T)
                    A.dbias_dense[((r * A.heads + h) * T + i) * (int64_t)T + j] = dsv;
                X[j * LD + i] = dsv;   // dSᵀ[j][i]
            }
        }
        if (A.part) {
#pragma unroll
            for (int jt = 0; jt < TT; ++jt) gsum[jt] += dp[jt];
        }
        {   // dQᵀ = Kᵀ·dSᵀ: A = Kᵀ[16dt + c][16jt + 4g + e], B = the dSᵀ accumulators
            f4v acc[DT][2];
#pragma unroll
            for (int dt = 0; dt < DT; ++dt) acc[dt][0] = acc[dt][1] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int jt = 0; jt < TT; ++jt)
#pragma unroll
                for (int dt = 0; dt < DT; ++dt) {
                    const f4v ka = lds4(Kt + (dt * 16 + c) * LD + jt * 16 + 4 * g);
#pragma unroll
                    for (int e = 0; e < 4; ++e) acc[dt][jt & 1] = mfma4(ka[e], dp[jt][e], acc[dt][jt & 1]);
                }
#pragma unroll
            for (int dt = 0; dt < DT; ++dt) {
                const f4v a = acc[dt][0] + acc[dt][1];
                if (i < T) st4v<S>(A.dq, r * A.d_row + (int64_t)i * A.d_t + h * d + dt * 16 + 4 * g, a, A.inv_sqrt_d);
                if (A.qkv_part) bsum[0][dt] += a * A.inv_sqrt_d;   // padded steps add exact zeros (dS = 0)
            }
        }
        }
        __syncthreads();   // dSᵀ complete in X
        // ---- phase 2, key tile w: dKᵀ = Qᵀ·dS (B = X[16w + c][i]), then dVᵀ = dOᵀ·P' (B = X after P'ᵀ replaces dSᵀ)
#pragma unroll
        for (int pass = 0; pass < 2; ++pass) {
            if (pass == 1) {
                __syncthreads();   // dK's reads of X are done
#pragma unroll
                for (int jt = 0; jt < TT; ++jt)
#pragma unroll
                    for (int e = 0; e < 4; ++e) X[(jt * 16 + 4 * g + e) * LD + i] = s[jt][e];
                __syncthreads();
            }
            const float* At = pass == 0 ? Qt : Ot;
            f4v acc[DT][2];
#pragma unroll
            for (int dt = 0; dt < DT; ++dt) acc[dt][0] = acc[dt][1] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int it = 0; it < TT; ++it) {
                const f4v xb = lds4(X + i * LD + it * 16 + 4 * g);   // B[k = 16it + 4g + e][n = key 16w + c]
#pragma unroll
                for (int dt = 0; dt < DT; ++dt) {
                    const f4v xa = lds4(At + (dt * 16 + c) * LD + it * 16 + 4 * g);
#pragma unroll
                    for (int e = 0; e < 4; ++e) acc[dt][it & 1] = mfma4(xa[e], xb[e], acc[dt][it & 1]);
                }
            }
            float* dst = pass == 0 ? A.dk : A.dv;
            const float sc = (pass == 0 ? A.inv_sqrt_d : 1.f) * fsc;
#pragma unroll
            for (int dt = 0; dt < DT; ++dt) {
                const f4v a = acc[dt][0] + acc[dt][1];
                if (i < T) st4v<S>(dst, r * A.d_row + (int64_t)i * A.d_t + h * d + dt * 16 + 4 * g, a, sc);
                if (A.qkv_part) bsum[1 + pass][dt] += a * sc;
            }
        }
    }
    __syncthreads();   // the last unit's reads of X and the staged tiles are done
    if (A.qkv_part) {
        // over the 16 step lanes (fixed butterfly), then over the waves in wave order through Kr
        float* red = Kr;   // [TT][3·DP]
#pragma unroll
        for (int t3 = 0; t3 < 3; ++t3)
#pragma unroll
            for (int dt = 0; dt < DT; ++dt)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float x = bsum[t3][dt][e];
                    x = lane_sum<16>(x);
                    if (c0 == 0) red[w * 3 * DP + t3 * DP + dt * 16 + 4 * g0 + e] = x;
                }
        __syncthreads();
        float* prow = A.qkv_part + rg * 3 * (int64_t)A.H + (int64_t)h * d;
        for (int t = threadIdx.x; t < 3 * DP; t += WAVE * TT) {
            float x = 0.f;
            for (int ww = 0; ww < TT; ++ww) x += red[ww * 3 * DP + t];
            if (t % DP < d) prow[(t / DP) * (int64_t)A.H + t % DP] = x;
        }
    }
    if (A.part) {
        // diagonal sums (t = i - j + T - 1) of the summed dSᵀ tile in j order: part[rg][h][t]
#pragma unroll
        for (int jt = 0; jt < TT; ++jt)
#pragma unroll
            for (int e = 0; e < 4; ++e) X[(jt * 16 + 4 * g0 + e) * LD + w * 16 + c0] = gsum[jt][e] * fsc;
        __syncthreads();
        float* prow = A.part + rg * A.heads * NB + (int64_t)h * NB;
        for (int t = threadIdx.x; t < NB; t += WAVE * TT) {
            const int off = t - (T - 1);
            const int j0 = off < 0 ? -off : 0, j1 = off < 0 ? T : T - off;
            float a = 0.f;
            for (int j = j0; j < j1; ++j) a += X[j * LD + j + off];
            prow[t] = a;
        }
    }
}

// T <= 32 (TT <= 2); at TT = 4 the backward needs > 256 VGPRs (spills) and T in (32, 128] keeps v3
int v4_tiles(int T) { return T <= 16 ? 1 : T <= 32 ? 2 : 0; }

#ifndef TAGAN_TATTN_V4
#define TAGAN_TATTN_V4 1
#endif
bool v4_enabled() {   // TAGAN_TATTN_V4=0 selects the v3 kernels (A/B runs, v3-vs-v4 parity test)
    const char* e = getenv("TAGAN_TATTN_V4");
    return (e && e[0] == '0') ? false : TAGAN_TATTN_V4 != 0;
}
bool v4_ok(int T, int d) { return v4_enabled() && v4_tiles(T) != 0 && (d == 16 || d == 32); }

// v5 (one workgroup of TT waves per unit) for T in (32, 128]; TAGAN_TATTN_V5=2 also takes T in (16, 32]
// (TT = 2, the A/B against v4), 0 leaves T > 32 on v3
int v5_tiles(int T) { return T <= 16 ? 0 : T <= 32 ? 2 : T <= 64 ? 4 : T <= 128 ? 8 : 0; }
int v5_mode() {   // read per call, like TAGAN_TATTN_V4, so a test can switch kernels within one process
    const char* e = getenv("TAGAN_TATTN_V5");
    return e ? atoi(e) : 1;
}
bool v5_ok(int T, int d) {
    const int m = v5_mode();
    return m > 0 && v5_tiles(T) != 0 && (d == 16 || d == 32) && (T > 32 || (m == 2 && v4_enabled()));
}

// v6 (head-group slabs) for the v4 range; TAGAN_TATTN_V6=0 keeps v4, TAGAN_V6_GH=2|4 forces the group width
int v6_group(int T, int heads, int d) {
    const char* e = getenv("TAGAN_TATTN_V6");
    if (e && e[0] == '0') return 0;
    if (!v4_ok(T, d)) return 0;
    const char* f = getenv("TAGAN_V6_GH");
    const int want = f ? atoi(f) : 4;
    if (want >= 8 && heads % 8 == 0) return 8;
    if (want >= 4 && heads % 4 == 0) return 4;
    return (want >= 2 && heads % 2 == 0) ? 2 : 0;
}
// the v6 backward only where it measured faster than v4: head_dim 32 (C4: 12.0 vs 15.9 ms) or T <= 16; at
// T in (16, 32] with head_dim 16 (C2) its 168+ VGPRs cost a wave per SIMD against v4 (0.43 vs 0.36 ms)
bool v6_bwd_ok(int T, int d) {
    const char* e = getenv("TAGAN_TATTN_V6");
    if (e && e[0] == '2') return true;   // force (A/B runs, parity tests)
    return d == 32 || v4_tiles(T) == 1;
}

// the keep-bit cache where it wins: at TT = 8 (C5: fwd + bwd 80.2 -> 76.7 ms); at TT = 4 (C3) the forward's bit
// stores cost more than the backward saves (21.8 -> 22.0 ms; profiles/r4m_tattn.txt)
bool v5_keep_tiles(int TT) { return TT >= 8; }

// > 64 KB of dynamic LDS needs the per-kernel opt-in (once per instantiation)
template <typename K>
int lds_optin(K* kern, size_t bytes) {
    if (bytes <= 64 * 1024) return TAGAN_OK;
    // once per kernel, to the full 160 KB (later launches of any size skip the runtime call)
    static std::mutex mu;
    static std::unordered_set<const void*> done;
    const void* key = reinterpret_cast<const void*>(kern);
    std::lock_guard<std::mutex> lock(mu);
    if (done.count(key)) return TAGAN_OK;
    TAGAN_REQUIRE(bytes <= 160 * 1024, TAGAN_ERR_UNSUPPORTED, "temporal_attn: %zu B of LDS", bytes);
    hipError_t e = hipFuncSetAttribute(key, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    TAGAN_REQUIRE(e == hipSuccess, TAGAN_ERR_LAUNCH, "temporal_attn: LDS opt-in %zu B: %s", bytes, hipGetErrorString(e));
    done.insert(key);
    return TAGAN_OK;
}

// waves: G partial rows x heads (G <= grid_rows(rows), the bias-gradient workspace rows)
// (a multiple of 8 from 8 rows up, for the XCD-aware wave map)
// 1024 row groups: 2048 / 4096 / 8192 measured 0.344 / 0.359 / 0.401 ms against 0.346 ms for the C2 backward
// 
int64_t v4_groups(int64_t rows) {
    constexpr int64_t cap = 1024;
    return rows >= 8 ? std::min<int64_t>(rows, cap) & ~(int64_t)7 : rows;
}

int v3_lanes(int T) { return T <= 16 ? 16 : T <= 32 ? 32 : T <= 128 ? 64 : 0; }
int v3_wph(int T) { return T > 64 ? 2 : 1; }

#ifndef TAGAN_TATTN_V3
#define TAGAN_TATTN_V3 1
#endif
bool v3_ok(int T, int d) {
    return TAGAN_TATTN_V3 && v3_lanes(T) != 0 && (d == 8 || d == 16 || d == 32 || d == 64);
}

int pick_D(int d) {
    if (d <= 8) return 8;
    if (d <= 16) return 16;
    if (d <= 32) return 32;
    if (d <= 64) return 64;
    if (d <= 128) return 128;
    return 0;
}

int grid_rows(int64_t rows) { return (int)std::min<int64_t>(rows, 256 * 4); }
// partial rows of the backward workspace: every kernel generation's row groups fit
int64_t ws_rows(int64_t rows) { return std::max<int64_t>(grid_rows(rows), v4_groups(rows)); }

int check(int dtype, int64_t rows, int T, int heads, int d, float p_drop) {
    TAGAN_REQUIRE(dtype == TAGAN_F32 || dtype == TAGAN_BF16, TAGAN_ERR_UNSUPPORTED, "temporal_attn: dtype %d",
                  dtype);
    TAGAN_REQUIRE(rows > 0 && T > 0 && heads > 0 && d > 0, TAGAN_ERR_ARG, "temporal_attn: bad sizes");
    TAGAN_REQUIRE(pick_D(d) != 0, TAGAN_ERR_UNSUPPORTED, "temporal_attn: head_dim %d > 128", d);
    TAGAN_REQUIRE(p_drop >= 0.f && p_drop < 1.f, TAGAN_ERR_ARG, "temporal_attn: p_drop %f", (double)p_drop);
    return TAGAN_OK;
}

TArgs make(int64_t rows, int T, int heads, int d, int64_t s_row, int64_t s_t, const float* bias_table,
           const float* bias_dense, int64_t bias_bstride, const uint8_t* mask, int64_t mb, int64_t mh, int causal,
           float p_drop, uint64_t seed) {
    TArgs A{};
    A.rows = rows;
    A.T = T;
    A.heads = heads;
    A.d = d;
    A.H = heads * d;
    A.s_row = s_row;
    A.s_t = s_t;
    A.bias_table = bias_table;
    A.bias_dense = bias_dense;
    A.bias_bstride = bias_bstride;
    A.mask = mask;
    A.mask_bstride = mb;
    A.mask_hstride = mh;
    A.causal = causal;
    A.p_drop = p_drop;
    A.inv_keep = 1.f / (1.f - p_drop);
    A.inv_sqrt_d = 1.f / sqrtf((float)d);
    A.seed = seed; A.seed_ctr = seed_counter();
    return A;
}

}  // namespace
}  // namespace tagan

extern "C" {

size_t tagan_temporal_attn_keep_bytes(int64_t rows, int32_t T, int32_t heads, int32_t head_dim, int causal,
                                      int has_mask, int has_bias_dense, float p_drop) {
    using namespace tagan;
    if (rows <= 0 || heads <= 0 || !(p_drop > 0.f) || !v5_ok(T, head_dim)) return 0;
    const int TT = v5_tiles(T);
    if (!v5_keep_tiles(TT)) return 0;
    const int one = 1;   // any non-null pointer: v5_fast_shape tests presence only
    if (!v5_fast_shape(T, TT, causal, has_mask ? &one : nullptr, has_bias_dense ? &one : nullptr, nullptr, p_drop))
        return 0;
    return (size_t)rows * heads * TT * WAVE * sizeof(uint32_t);
}

int tagan_temporal_attn_fwd(int dtype, int64_t rows, int32_t T, int32_t heads, int32_t head_dim, const void* q,
                            const void* k, const void* v, int64_t s_row, int64_t s_t, const float* bias_table,
                            const float* bias_dense, int64_t bias_bstride, const uint8_t* mask,
                            int64_t mask_bstride, int64_t mask_hstride, int causal, float p_drop, uint64_t seed,
                            void* out, int64_t o_row, int64_t o_t, float* lse, float* attn, void* stream) {
    return tagan_temporal_attn_fwd_keep(dtype, rows, T, heads, head_dim, q, k, v, s_row, s_t, bias_table, bias_dense,
                                        bias_bstride, mask, mask_bstride, mask_hstride, causal, p_drop, seed, out,
                                        o_row, o_t, lse, attn, nullptr, 0, nullptr, stream);
}

int tagan_temporal_attn_fwd_keep(int dtype, int64_t rows, int32_t T, int32_t heads, int32_t head_dim, const void* q,
                                 const void* k, const void* v, int64_t s_row, int64_t s_t, const float* bias_table,
                                 const float* bias_dense, int64_t bias_bstride, const uint8_t* mask,
                                 int64_t mask_bstride, int64_t mask_hstride, int causal, float p_drop, uint64_t seed,
                                 void* out, int64_t o_row, int64_t o_t, float* lse, float* attn, uint32_t* keep,
                                 size_t keep_bytes, int32_t* keep_written, void* stream) {
    using namespace tagan;
    if (keep_written) *keep_written = 0;
    int rc = check(dtype, rows, T, heads, head_dim, p_drop);
    if (rc) return rc;
    TAGAN_REQUIRE(q && k && v && out && lse, TAGAN_ERR_ARG, "temporal_attn_fwd: null pointer");
    TArgs A = make(rows, T, heads, head_dim, s_row, s_t, bias_table, bias_dense, bias_bstride, mask, mask_bstride,
                   mask_hstride, causal, p_drop, seed);
    A.out = (float*)out;
    A.o_row = o_row;
    A.o_t = o_t;
    A.lse = lse;
    A.attn = attn;
    hipStream_t s = as_stream(stream);
    const dim3 g(grid_rows(rows));
    const float* qf = (const float*)q;
    const float* kf = (const float*)k;
    const float* vf = (const float*)v;
    const bool al4 = s_t % 4 == 0 && s_row % 4 == 0 && o_t % 4 == 0 && o_row % 4 == 0;
    const bool bf = dtype == TAGAN_BF16;
    TAGAN_REQUIRE(!bf || (al4 && !attn && (v3_ok(T, head_dim) || v4_ok(T, head_dim) || v5_ok(T, head_dim))),
                  TAGAN_ERR_UNSUPPORTED,
                  "temporal_attn_fwd: bf16 storage needs the v3 kernels (T <= 128, head_dim 8..64, no attn output)");
    if (al4 && !attn && v6_group(T, heads, head_dim)) {
        const int TT = v4_tiles(T), GH = v6_group(T, heads, head_dim);
        const dim3 g6((unsigned)(v4_groups(rows) * (heads / GH)));
        const size_t lds = v6_fwd_lds(TT, head_dim / 16, GH);
#define TAGAN_V6F(TTT, DDT, GGH) { auto kern = bf ? k_tattn_fwd_v6<TTT, DDT, GGH, bf16s> : k_tattn_fwd_v6<TTT, DDT, GGH, float>; \
                                   rc = lds_optin(kern, lds); if (rc) return rc; kern<<<g6, WAVE * GGH, lds, s>>>(A, qf, kf, vf); }
#define TAGAN_V6F_G(TTT, DDT) if (GH == 8) TAGAN_V6F(TTT, DDT, 8) else if (GH == 4) TAGAN_V6F(TTT, DDT, 4) else TAGAN_V6F(TTT, DDT, 2)
#define TAGAN_V6F_D(TTT) if (head_dim == 16) { TAGAN_V6F_G(TTT, 1) } else { TAGAN_V6F_G(TTT, 2) }
        if (TT == 1) { TAGAN_V6F_D(1) } else { TAGAN_V6F_D(2) }
#undef TAGAN_V6F_D
#undef TAGAN_V6F_G
#undef TAGAN_V6F
        TAGAN_CHECK_LAUNCH("temporal_attn_fwd_v6");
        return TAGAN_OK;
    }
    if (al4 && !attn && v5_ok(T, head_dim)) {
        const int TT = v5_tiles(T);
        const dim3 g5((unsigned)(v4_groups(rows) * heads));
        const size_t lds = v5_fwd_lds(TT, head_dim / 16);
        int mode = v5_fast_shape(T, TT, causal, mask, bias_dense, nullptr, p_drop) ? (p_drop > 0.f ? 2 : 1) : 0;
        // MODE 3: also store the keep bits for the backward (one word per row, head, wave and lane)
        if (mode == 2 && v5_keep_tiles(TT) && keep && keep_bytes >= (size_t)rows * heads * TT * WAVE * sizeof(uint32_t)) {
            mode = 3;
            A.keep = keep;
        }
#define TAGAN_V5F_M(TTT, DDT, MM) { auto kern = bf ? k_tattn_fwd_v5<TTT, DDT, bf16s, MM> : k_tattn_fwd_v5<TTT, DDT, float, MM>; \
                              rc = lds_optin(kern, lds); if (rc) return rc; kern<<<g5, WAVE * TTT, lds, s>>>(A, qf, kf, vf); }
#define TAGAN_V5F(TTT, DDT) { if (mode == 3) TAGAN_V5F_M(TTT, DDT, 3) else if (mode == 2) TAGAN_V5F_M(TTT, DDT, 2) \
                              else if (mode == 1) TAGAN_V5F_M(TTT, DDT, 1) else TAGAN_V5F_M(TTT, DDT, 0) }
#define TAGAN_V5F_D(TTT) if (head_dim == 16) TAGAN_V5F(TTT, 1) else TAGAN_V5F(TTT, 2)
        if (TT == 2) TAGAN_V5F_D(2) else if (TT == 4) TAGAN_V5F_D(4) else TAGAN_V5F_D(8)
#undef TAGAN_V5F_D
#undef TAGAN_V5F
#undef TAGAN_V5F_M
        TAGAN_CHECK_LAUNCH("temporal_attn_fwd_v5");
        if (keep_written) *keep_written = mode == 3;
        return TAGAN_OK;
    }
    if (al4 && !attn && v4_ok(T, head_dim)) {
        const int TT = v4_tiles(T);
        const dim3 g4((unsigned)(v4_groups(rows) * heads));
        const size_t lds = v4_fwd_lds(TT, head_dim / 16);
#define TAGAN_V4F(TTT, DDT) (bf ? k_tattn_fwd_v4<TTT, DDT, bf16s> : k_tattn_fwd_v4<TTT, DDT, float>)<<<g4, WAVE, lds, s>>>(A, qf, kf, vf)
#define TAGAN_V4F_D(TTT) if (head_dim == 16) { TAGAN_V4F(TTT, 1); } else { TAGAN_V4F(TTT, 2); }
        if (TT == 1) { TAGAN_V4F_D(1) } else { TAGAN_V4F_D(2) }
#undef TAGAN_V4F_D
#undef TAGAN_V4F
        TAGAN_CHECK_LAUNCH("temporal_attn_fwd_v4");
        return TAGAN_OK;
    }
    if (al4 && !attn && v3_ok(T, head_dim)) {
        const int LG = v3_lanes(T), HPW = WAVE / LG, n_hg = (heads + HPW - 1) / HPW, WPH = v3_wph(T);
        const dim3 g3((unsigned)(grid_rows(rows) * n_hg));
        const size_t lds = v3_fwd_lds(T, head_dim, HPW);
#define TAGAN_V3F(DD, LL, W) (bf ? k_tattn_fwd_v3<DD, LL, bf16s, W> : k_tattn_fwd_v3<DD, LL, float, W>)<<<g3, V3_BLK * W, lds, s>>>(A, qf, kf, vf, n_hg)
#define TAGAN_V3F_D(LL, W) switch (head_dim) { case 8: TAGAN_V3F(8, LL, W); break; case 16: TAGAN_V3F(16, LL, W); break; \
                                               case 32: TAGAN_V3F(32, LL, W); break; default: TAGAN_V3F(64, LL, W); break; }
        if (LG == 16) { TAGAN_V3F_D(16, 1) } else if (LG == 32) { TAGAN_V3F_D(32, 1) }
        else if (WPH == 1) { TAGAN_V3F_D(64, 1) } else { TAGAN_V3F_D(64, 2) }
#undef TAGAN_V3F_D
#undef TAGAN_V3F
        TAGAN_CHECK_LAUNCH("temporal_attn_fwd_v3");
        return TAGAN_OK;
    }
    const int G = al4 ? v2_groups(false, T, head_dim, heads) : 0;
    if (G > 0) {
        const size_t lds = v2_fwd_lds(G, T, head_dim);
        switch (head_dim) {
            case 4: k_tattn_fwd_v2<4><<<g, BLK, lds, s>>>(A, qf, kf, vf, G); break;
            case 8: k_tattn_fwd_v2<8><<<g, BLK, lds, s>>>(A, qf, kf, vf, G); break;
            case 16: k_tattn_fwd_v2<16><<<g, BLK, lds, s>>>(A, qf, kf, vf, G); break;
            case 32: k_tattn_fwd_v2<32><<<g, BLK, lds, s>>>(A, qf, kf, vf, G); break;
            case 64: k_tattn_fwd_v2<64><<<g, BLK, lds, s>>>(A, qf, kf, vf, G); break;
            default: k_tattn_fwd_v2<128><<<g, BLK, lds, s>>>(A, qf, kf, vf, G); break;
        }
        TAGAN_CHECK_LAUNCH("temporal_attn_fwd_v2");
        return TAGAN_OK;
    }
    switch (pick_D(head_dim)) {
        case 8: k_tattn_fwd<8><<<g, BLK, 0, s>>>(A, qf, kf, vf); break;
        case 16: k_tattn_fwd<16><<<g, BLK, 0, s>>>(A, qf, kf, vf); break;
        case 32: k_tattn_fwd<32><<<g, BLK, 0, s>>>(A, qf, kf, vf); break;
        case 64: k_tattn_fwd<64><<<g, BLK, 0, s>>>(A, qf, kf, vf); break;
        default: k_tattn_fwd<128><<<g, BLK, 0, s>>>(A, qf, kf, vf); break;
    }
    TAGAN_CHECK_LAUNCH("temporal_attn_fwd");
    return TAGAN_OK;
}

size_t tagan_temporal_attn_bwd_workspace(int64_t rows, int32_t T, int32_t heads, int32_t head_dim) {
    using namespace tagan;
    if (rows <= 0 || T <= 0 || heads <= 0 || head_dim <= 0) return 0;
    return align_up((size_t)ws_rows(rows) * heads * (2 * T - 1) * sizeof(float), 256) +
           align_up((size_t)ws_rows(rows) * 3 * heads * head_dim * sizeof(float), 256);
}

int tagan_temporal_attn_bwd(int dtype, int64_t rows, int32_t T, int32_t heads, int32_t head_dim, const void* q,
                            const void* k, const void* v, int64_t s_row, int64_t s_t, const float* bias_table,
                            const float* bias_dense, int64_t bias_bstride, const uint8_t* mask,
                            int64_t mask_bstride, int64_t mask_hstride, int causal, float p_drop, uint64_t seed,
                            const void* out, int64_t o_row, int64_t o_t, const float* lse, const void* dout,
                            int64_t do_row, int64_t do_t, void* dq, void* dk, void* dv, int64_t d_row, int64_t d_t,
                            float* dbias_table, float* dbias_dense, float* dsum_qkv, void* workspace,
                            size_t workspace_bytes, void* stream) {
    return tagan_temporal_attn_bwd_keep(dtype, rows, T, heads, head_dim, q, k, v, s_row, s_t, bias_table, bias_dense,
                                        bias_bstride, mask, mask_bstride, mask_hstride, causal, p_drop, seed, out,
                                        o_row, o_t, lse, dout, do_row, do_t, dq, dk, dv, d_row, d_t, dbias_table,
                                        dbias_dense, dsum_qkv, nullptr, 0, workspace, workspace_bytes, stream);
}

int tagan_temporal_attn_bwd_keep(int dtype, int64_t rows, int32_t T, int32_t heads, int32_t head_dim, const void* q,
                                 const void* k, const void* v, int64_t s_row, int64_t s_t, const float* bias_table,
                                 const float* bias_dense, int64_t bias_bstride, const uint8_t* mask,
                                 int64_t mask_bstride, int64_t mask_hstride, int causal, float p_drop, uint64_t seed,
                                 const void* out, int64_t o_row, int64_t o_t, const float* lse, const void* dout,
                                 int64_t do_row, int64_t do_t, void* dq, void* dk, void* dv, int64_t d_row,
                                 int64_t d_t, float* dbias_table, float* dbias_dense, float* dsum_qkv,
                                 const uint32_t* keep, size_t keep_bytes, void* workspace, size_t workspace_bytes,
                                 void* stream) {
    using namespace tagan;
    int rc = check(dtype, rows, T, heads, head_dim, p_drop);
    if (rc) return rc;
    TAGAN_REQUIRE(q && k && v && out && lse && dout && dq && dk && dv, TAGAN_ERR_ARG,
                  "temporal_attn_bwd: null pointer");
    const size_t lds = ((size_t)heads * (2 * T - 1) + (size_t)NW * T) * sizeof(float);
    TAGAN_REQUIRE(lds <= 160 * 1024, TAGAN_ERR_UNSUPPORTED, "temporal_attn_bwd: T=%d heads=%d exceed LDS", T, heads);
    TArgs A = make(rows, T, heads, head_dim, s_row, s_t, bias_table, bias_dense, bias_bstride, mask, mask_bstride,
                   mask_hstride, causal, p_drop, seed);
    A.o_in = (const float*)out;
    A.o_row = o_row;
    A.o_t = o_t;
    A.lse_in = lse;
    A.do_row = do_row;
    A.do_t = do_t;
    A.dq = (float*)dq;
    A.dk = (float*)dk;
    A.dv = (float*)dv;
    A.d_row = d_row;
    A.d_t = d_t;
    A.dbias_dense = dbias_dense;
    const int nblk = grid_rows(rows);
    {
        const bool al4_ = s_t % 4 == 0 && s_row % 4 == 0 && o_t % 4 == 0 && o_row % 4 == 0 && do_t % 4 == 0 &&
                          do_row % 4 == 0 && d_t % 4 == 0 && d_row % 4 == 0;
        TAGAN_REQUIRE(!dsum_qkv || (al4_ && (v4_ok(T, head_dim) || v5_ok(T, head_dim))), TAGAN_ERR_UNSUPPORTED,
                      "temporal_attn_bwd: dsum_qkv needs the matrix-core path (T <= 128, head_dim 16/32, aligned)");
    }
    if (dbias_table || dsum_qkv) {
        const size_t need = tagan_temporal_attn_bwd_workspace(rows, T, heads, head_dim);
        TAGAN_REQUIRE(workspace && workspace_bytes >= need, TAGAN_ERR_WORKSPACE,
                      "temporal_attn_bwd: workspace %zu < %zu", workspace_bytes, need);
        if (dbias_table) A.part = (float*)workspace;
        if (dsum_qkv)
            A.qkv_part = (float*)((char*)workspace +
                                  align_up((size_t)ws_rows(rows) * heads * (2 * T - 1) * sizeof(float), 256));
    }
    hipStream_t s = as_stream(stream);
    const dim3 g(nblk);
    const float* qf = (const float*)q;
    const float* kf = (const float*)k;
    const float* vf = (const float*)v;
    const float* df = (const float*)dout;
    const bool al4 = s_t % 4 == 0 && s_row % 4 == 0 && o_t % 4 == 0 && o_row % 4 == 0 && do_t % 4 == 0 &&
                     do_row % 4 == 0 && d_t % 4 == 0 && d_row % 4 == 0;
    const bool bf = dtype == TAGAN_BF16;
    TAGAN_REQUIRE(!bf || (al4 && (v3_ok(T, head_dim) || v4_ok(T, head_dim) || v5_ok(T, head_dim))),
                  TAGAN_ERR_UNSUPPORTED,
                  "temporal_attn_bwd: bf16 storage needs the v3 kernels (T <= 128, head_dim 8..64)");
    if (al4 && v6_group(T, heads, head_dim) && v6_bwd_ok(T, head_dim)) {
        // grid = G6 partial rows x head groups; workgroup b keeps head group b % (heads / GH)
        const int TT = v4_tiles(T), GH = v6_group(T, heads, head_dim);
        const int64_t G6 = v4_groups(rows);   // <= nblk: the workspace rows
        const dim3 g6((unsigned)(G6 * (heads / GH)));
        const size_t lds = v6_bwd_lds(TT, head_dim / 16, GH);
#define TAGAN_V6B(TTT, DDT, GGH) { auto kern = bf ? k_tattn_bwd_v6<TTT, DDT, GGH, bf16s> : k_tattn_bwd_v6<TTT, DDT, GGH, float>; \
                                   rc = lds_optin(kern, lds); if (rc) return rc; kern<<<g6, WAVE * GGH, lds, s>>>(A, qf, kf, vf, df, lse); }
#define TAGAN_V6B_G(TTT, DDT) if (GH == 8) TAGAN_V6B(TTT, DDT, 8) else if (GH == 4) TAGAN_V6B(TTT, DDT, 4) else TAGAN_V6B(TTT, DDT, 2)
#define TAGAN_V6B_D(TTT) if (head_dim == 16) { TAGAN_V6B_G(TTT, 1) } else { TAGAN_V6B_G(TTT, 2) }
        if (TT == 1) { TAGAN_V6B_D(1) } else { TAGAN_V6B_D(2) }
#undef TAGAN_V6B_D
#undef TAGAN_V6B_G
#undef TAGAN_V6B
        TAGAN_CHECK_LAUNCH("temporal_attn_bwd_v6");
        if (dbias_table) {
            const int n = heads * (2 * T - 1);
            launch_colsum(A.part, (int)G6, n, dbias_table, nullptr, n, s);
            TAGAN_CHECK_LAUNCH("temporal_attn_bwd_sum");
        }
        if (dsum_qkv) {
            const int n = 3 * heads * head_dim;
            launch_colsum(A.qkv_part, (int)G6, n, dsum_qkv, nullptr, n, s);
            TAGAN_CHECK_LAUNCH("temporal_attn_bwd_qkv_sum");
        }
        return TAGAN_OK;
    }
    if (al4 && v5_ok(T, head_dim)) {
        // grid = G5 partial rows x heads; each workgroup keeps one head (v4_wave_map)
        const int TT = v5_tiles(T);
        const int64_t G5 = v4_groups(rows);   // <= nblk: the workspace rows
        const dim3 g5((unsigned)(G5 * heads));
        const size_t lds = v5_bwd_lds(TT, head_dim / 16);
        int mode = v5_fast_shape(T, TT, causal, mask, bias_dense, dbias_dense, p_drop) ? (p_drop > 0.f ? 2 : 1) : 0;
        // MODE 3: the forward's keep bits (tagan_temporal_attn_fwd_keep reported them written) instead of the hash
        if (mode == 2 && v5_keep_tiles(TT) && keep && keep_bytes >= (size_t)rows * heads * TT * WAVE * sizeof(uint32_t)) {
            mode = 3;
            A.keep = const_cast<uint32_t*>(keep);
        }
#define TAGAN_V5B_M(TTT, DDT, MM) { auto kern = bf ? k_tattn_bwd_v5<TTT, DDT, bf16s, MM> : k_tattn_bwd_v5<TTT, DDT, float, MM>; \
                              rc = lds_optin(kern, lds); if (rc) return rc; kern<<<g5, WAVE * TTT, lds, s>>>(A, qf, kf, vf, df, lse); }
#define TAGAN_V5B(TTT, DDT) { if (mode == 3) TAGAN_V5B_M(TTT, DDT, 3) else if (mode == 2) TAGAN_V5B_M(TTT, DDT, 2) \
                              else if (mode == 1) TAGAN_V5B_M(TTT, DDT, 1) else TAGAN_V5B_M(TTT, DDT, 0) }
#define TAGAN_V5B_D(TTT) if (head_dim == 16) TAGAN_V5B(TTT, 1) else TAGAN_V5B(TTT, 2)
        if (TT == 2) TAGAN_V5B_D(2) else if (TT == 4) TAGAN_V5B_D(4) else TAGAN_V5B_D(8)
#undef TAGAN_V5B_D
#undef TAGAN_V5B
#undef TAGAN_V5B_M
        TAGAN_CHECK_LAUNCH("temporal_attn_bwd_v5");
        if (dbias_table) {
            const int n = heads * (2 * T - 1);
            launch_colsum(A.part, (int)G5, n, dbias_table, nullptr, n, s);
            TAGAN_CHECK_LAUNCH("temporal_attn_bwd_sum");
        }
        if (dsum_qkv) {
            const int n = 3 * heads * head_dim;
            launch_colsum(A.qkv_part, (int)G5, n, dsum_qkv, nullptr, n, s);
            TAGAN_CHECK_LAUNCH("temporal_attn_bwd_qkv_sum");
        }
        return TAGAN_OK;
    }
    if (al4 && v4_ok(T, head_dim)) {
        // grid = G4 partial rows x heads; each block keeps one head (v4_wave_map)
        const int TT = v4_tiles(T);
        const int64_t G4 = v4_groups(rows);   // <= nblk: the workspace rows
        const dim3 g4((unsigned)(G4 * heads));
        const size_t lds = v4_bwd_lds(TT, head_dim / 16);
        const int mode4 = v5_fast_shape(T, TT, causal, mask, bias_dense, dbias_dense, p_drop) ? (p_drop > 0.f ? 2 : 1) : 0;
#define TAGAN_V4B_M(TTT, DDT, MM) (bf ? k_tattn_bwd_v4<TTT, DDT, bf16s, MM> : k_tattn_bwd_v4<TTT, DDT, float, MM>)<<<g4, WAVE, lds, s>>>(A, qf, kf, vf, df, lse)
#define TAGAN_V4B(TTT, DDT) { if (mode4 == 2) TAGAN_V4B_M(TTT, DDT, 2); else if (mode4 == 1) TAGAN_V4B_M(TTT, DDT, 1); else TAGAN_V4B_M(TTT, DDT, 0); }
#define TAGAN_V4B_D(TTT) if (head_dim == 16) { TAGAN_V4B(TTT, 1); } else { TAGAN_V4B(TTT, 2); }
        if (TT == 1) { TAGAN_V4B_D(1) } else { TAGAN_V4B_D(2) }
#undef TAGAN_V4B_D
#undef TAGAN_V4B
#undef TAGAN_V4B_M
        TAGAN_CHECK_LAUNCH("temporal_attn_bwd_v4");
        if (dbias_table) {
            const int n = heads * (2 * T - 1);
            launch_colsum(A.part, (int)G4, n, dbias_table, nullptr, n, s);
            TAGAN_CHECK_LAUNCH("temporal_attn_bwd_sum");
        }
        if (dsum_qkv) {
            const int n = 3 * heads * head_dim;
            launch_colsum(A.qkv_part, (int)G4, n, dsum_qkv, nullptr, n, s);
            TAGAN_CHECK_LAUNCH("temporal_attn_bwd_qkv_sum");
        }
        return TAGAN_OK;
    }
    if (al4 && v3_ok(T, head_dim)) {
        // grid = nblk partial rows x n_hg head groups; block b keeps head group b % n_hg
        const int LG = v3_lanes(T), HPW = WAVE / LG, n_hg = (heads + HPW - 1) / HPW, WPH = v3_wph(T);
        const dim3 g3((unsigned)(nblk * n_hg));
        const size_t lds = v3_bwd_lds(T, head_dim, HPW, WPH);
#define TAGAN_V3B(DD, LL, W) (bf ? k_tattn_bwd_v3<DD, LL, bf16s, W> : k_tattn_bwd_v3<DD, LL, float, W>)<<<g3, V3_BLK * W, lds, s>>>(A, qf, kf, vf, df, lse, n_hg)
#define TAGAN_V3B_D(LL, W) switch (head_dim) { case 8: TAGAN_V3B(8, LL, W); break; case 16: TAGAN_V3B(16, LL, W); break; \
                                               case 32: TAGAN_V3B(32, LL, W); break; default: TAGAN_V3B(64, LL, W); break; }
        if (LG == 16) { TAGAN_V3B_D(16, 1) } else if (LG == 32) { TAGAN_V3B_D(32, 1) }
        else if (WPH == 1) { TAGAN_V3B_D(64, 1) } else { TAGAN_V3B_D(64, 2) }
#undef TAGAN_V3B_D
#undef TAGAN_V3B
        TAGAN_CHECK_LAUNCH("temporal_attn_bwd_v3");
        if (dbias_table) {
            const int n = heads * (2 * T - 1);
            launch_colsum(A.part, nblk, n, dbias_table, nullptr, n, s);
            TAGAN_CHECK_LAUNCH("temporal_attn_bwd_sum");
        }
        return TAGAN_OK;
    }
    const int G = al4 ? v2_groups(true, T, head_dim, heads) : 0;
    if (G > 0) {
        const size_t l2 = v2_bwd_lds(G, T, head_dim, heads);
        switch (head_dim) {
            case 4: k_tattn_bwd_v2<4><<<g, BLK, l2, s>>>(A, qf, kf, vf, df, lse, G); break;
            case 8: k_tattn_bwd_v2<8><<<g, BLK, l2, s>>>(A, qf, kf, vf, df, lse, G); break;
            case 16: k_tattn_bwd_v2<16><<<g, BLK, l2, s>>>(A, qf, kf, vf, df, lse, G); break;
            case 32: k_tattn_bwd_v2<32><<<g, BLK, l2, s>>>(A, qf, kf, vf, df, lse, G); break;
            case 64: k_tattn_bwd_v2<64><<<g, BLK, l2, s>>>(A, qf, kf, vf, df, lse, G); break;
            default: k_tattn_bwd_v2<128><<<g, BLK, l2, s>>>(A, qf, kf, vf, df, lse, G); break;
        }
    } else switch (pick_D(head_dim)) {
        case 8: k_tattn_bwd<8><<<g, BLK, lds, s>>>(A, qf, kf, vf, df, lse); break;
        case 16: k_tattn_bwd<16><<<g, BLK, lds, s>>>(A, qf, kf, vf, df, lse); break;
        case 32: k_tattn_bwd<32><<<g, BLK, lds, s>>>(A, qf, kf, vf, df, lse); break;
        case 64: k_tattn_bwd<64><<<g, BLK, lds, s>>>(A, qf, kf, vf, df, lse); break;
        default: k_tattn_bwd<128><<<g, BLK, lds, s>>>(A, qf, kf, vf, df, lse); break;
    }
    TAGAN_CHECK_LAUNCH("temporal_attn_bwd");
    if (dbias_table) {
        const int n = heads * (2 * T - 1);
        launch_colsum(A.part, nblk, n, dbias_table, nullptr, n, s);
        TAGAN_CHECK_LAUNCH("temporal_attn_bwd_sum");
    }
    return TAGAN_OK;
}

}  // extern "C"
