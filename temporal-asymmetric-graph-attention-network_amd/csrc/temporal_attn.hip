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

__device__ __forceinline__ float drop_scale(const TArgs& A, int64_t r, int h, int i, int j) {
    if (A.p_drop <= 0.f) return 1.f;
    const uint64_t idx = (((uint64_t)r * A.heads + h) * A.T + i) * (uint64_t)A.T + j;
    return uniform01(A.seed, idx) >= A.p_drop ? A.inv_keep : 0.f;
}

template <int D>
__device__ __forceinline__ void load_row(const float* __restrict__ p, int d, float (&r)[D]) {
#pragma unroll
    for (int c = 0; c < D; ++c) r[c] = (c < d) ? p[c] : 0.f;
}

template <int D>
__global__ void __launch_bounds__(BLK) k_tattn_fwd(TArgs A, const float* __restrict__ q,
                                                   const float* __restrict__ k, const float* __restrict__ v) {
    const int lane = threadIdx.x & (WAVE - 1);
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int T = A.T, d = A.d;
    for (int64_t r = blockIdx.x; r < A.rows; r += gridDim.x) {
        for (int h = wid; h < A.heads; h += NW) {
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
                    const float pw = p * drop_scale(A, r, h, ii, j);
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
                                a = __expf(s - ls) * drop_scale(A, r, h, i, j);
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
                        ds = p * (dp * drop_scale(A, r, h, ii, j) - Di);
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
                        const float sc = drop_scale(A, r, h, i, jj);
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

__global__ void __launch_bounds__(BLK) k_sum_parts(const float* __restrict__ part, int nblk, int n,
                                                   float* __restrict__ out) {
    const int x = blockIdx.x * BLK + threadIdx.x;
    if (x >= n) return;
    float s = 0.f;
    for (int b = 0; b < nblk; ++b) s += part[(int64_t)b * n + x];
    out[x] = s;
}

int pick_D(int d) {
    if (d <= 8) return 8;
    if (d <= 16) return 16;
    if (d <= 32) return 32;
    if (d <= 64) return 64;
    if (d <= 128) return 128;
    return 0;
}

int grid_rows(int64_t rows) { return (int)std::min<int64_t>(rows, 256 * 8); }

int check(int dtype, int64_t rows, int T, int heads, int d, float p_drop) {
    TAGAN_REQUIRE(dtype == TAGAN_F32, TAGAN_ERR_UNSUPPORTED, "temporal_attn: dtype %d unsupported", dtype);
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
    A.seed = seed;
    return A;
}

}  // namespace
}  // namespace tagan

extern "C" {

int tagan_temporal_attn_fwd(int dtype, int64_t rows, int32_t T, int32_t heads, int32_t head_dim, const void* q,
                            const void* k, const void* v, int64_t s_row, int64_t s_t, const float* bias_table,
                            const float* bias_dense, int64_t bias_bstride, const uint8_t* mask,
                            int64_t mask_bstride, int64_t mask_hstride, int causal, float p_drop, uint64_t seed,
                            void* out, int64_t o_row, int64_t o_t, float* lse, float* attn, void* stream) {
    using namespace tagan;
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

size_t tagan_temporal_attn_bwd_workspace(int64_t rows, int32_t T, int32_t heads) {
    using namespace tagan;
    if (rows <= 0 || T <= 0 || heads <= 0) return 0;
    return align_up((size_t)grid_rows(rows) * heads * (2 * T - 1) * sizeof(float), 256);
}

int tagan_temporal_attn_bwd(int dtype, int64_t rows, int32_t T, int32_t heads, int32_t head_dim, const void* q,
                            const void* k, const void* v, int64_t s_row, int64_t s_t, const float* bias_table,
                            const float* bias_dense, int64_t bias_bstride, const uint8_t* mask,
                            int64_t mask_bstride, int64_t mask_hstride, int causal, float p_drop, uint64_t seed,
                            const void* out, int64_t o_row, int64_t o_t, const float* lse, const void* dout,
                            int64_t do_row, int64_t do_t, void* dq, void* dk, void* dv, int64_t d_row, int64_t d_t,
                            float* dbias_table, float* dbias_dense, void* workspace, size_t workspace_bytes,
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
    if (dbias_table) {
        const size_t need = tagan_temporal_attn_bwd_workspace(rows, T, heads);
        TAGAN_REQUIRE(workspace && workspace_bytes >= need, TAGAN_ERR_WORKSPACE,
                      "temporal_attn_bwd: workspace %zu < %zu", workspace_bytes, need);
        A.part = (float*)workspace;
    }
    hipStream_t s = as_stream(stream);
    const dim3 g(nblk);
    const float* qf = (const float*)q;
    const float* kf = (const float*)k;
    const float* vf = (const float*)v;
    const float* df = (const float*)dout;
    switch (pick_D(head_dim)) {
        case 8: k_tattn_bwd<8><<<g, BLK, lds, s>>>(A, qf, kf, vf, df, lse); break;
        case 16: k_tattn_bwd<16><<<g, BLK, lds, s>>>(A, qf, kf, vf, df, lse); break;
        case 32: k_tattn_bwd<32><<<g, BLK, lds, s>>>(A, qf, kf, vf, df, lse); break;
        case 64: k_tattn_bwd<64><<<g, BLK, lds, s>>>(A, qf, kf, vf, df, lse); break;
        default: k_tattn_bwd<128><<<g, BLK, lds, s>>>(A, qf, kf, vf, df, lse); break;
    }
    TAGAN_CHECK_LAUNCH("temporal_attn_bwd");
    if (dbias_table) {
        const int n = heads * (2 * T - 1);
        k_sum_parts<<<(n + BLK - 1) / BLK, BLK, 0, s>>>(A.part, nblk, n, dbias_table);
        TAGAN_CHECK_LAUNCH("temporal_attn_bwd_sum");
    }
    return TAGAN_OK;
}

}  // extern "C"
