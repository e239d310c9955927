// Row LayerNorm with fused residual + dropout for the TAGAN layers on gfx950.
//
// Replaces, per layer, the ATen chain  output_dropout(proj) + identity -> LayerNorm
// (geometric_attention.py:586-596, temporal_attention.py:1190-1200) and the plain
// layer_norm1 (:541-542, :985-986).  HBM-bound elementwise/reduction work: a group
// of LPR = H/(4*NV) lanes owns one row (NV float4 per lane), mean / variance are
// XOR-butterfly reductions inside the group, two-pass in registers (no Welford
// round-off), rstd = 1/sqrt(var+eps).  Backward recomputes x̂ from the saved LN
// input and (mean, rstd); dγ/dβ are per-block partials summed in block order.
#include <stdlib.h>

#include "common.cuh"

namespace tagan {
namespace {

constexpr int BLK = 256;

template <int LPR>
__device__ __forceinline__ float row_sum(float x) { return lane_sum<LPR>(x); }   // DPP / permlane (common.cuh)

struct LnArgs {
    int64_t M;
    int H;
    const float* a;
    const float* a_bias;   // optional [H] added to a before the dropout (the projection's bias)
    const float* b;
    float p_drop, inv_keep;
    uint64_t seed;
    const uint64_t* seed_ctr;   // graph-replay seed source (tagan_set_seed_counter) or null
    const float* gamma;
    const float* beta;
    float eps;
    float* s_out;
    float* y;
    float* mean;
    float* rstd;
    // backward
    const float* s_in;
    const float* dy;
    const float* dres;   // optional gradient added to ds (the other consumer of the LN input)
    float* ds;
    float* da;
    float* part;   // [gridDim.x, 3H]: dgamma | dbeta | column sums of da (projection-bias gradient)
    int want_dsa;  // accumulate the column sums of da
    int64_t ldy;   // forward output row stride (>= H)
    int ones_col;  // ldy >= H + 4: write (1, 0, 0, 0) at columns H..H+3 of y (bias folded into the next GEMM)
    // forward skip branch (model.py:258-262): y += LN_s(b) with its own gamma/beta/eps/statistics
    const float* gamma_s;
    const float* beta_s;
    float eps_s;
    float* mean_s;
    float* rstd_s;
};

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

// dropout stream = row, counter = column
__device__ __forceinline__ float4 drop4(const LnArgs& A, float4 v, int64_t row, int c) {
    if (A.p_drop <= 0.f) return v;
    const uint32_t key = drop_key(A.seed, (uint64_t)row);
    v.x = drop_u(key, (uint32_t)c + 0) >= A.p_drop ? v.x * A.inv_keep : 0.f;
    v.y = drop_u(key, (uint32_t)c + 1) >= A.p_drop ? v.y * A.inv_keep : 0.f;
    v.z = drop_u(key, (uint32_t)c + 2) >= A.p_drop ? v.z * A.inv_keep : 0.f;
    v.w = drop_u(key, (uint32_t)c + 3) >= A.p_drop ? v.w * A.inv_keep : 0.f;
    return v;
}

// U row groups per wave: all U rows' loads are issued before the first reduction, so one
// wave keeps U x NV x (1 or 2) KB in flight instead of one load's worth.  At C2's H = 128 a
// single row pair per wave left the LN passes latency-bound at ~50 % of the HBM roofline.
template <int LPR, int NV, int U, typename S>
__global__ void __launch_bounds__(BLK) k_ln_fwd(LnArgs A) {
    TAGAN_LIVE_SEED(A);
    constexpr int RPW = WAVE / LPR;
    const int lane = threadIdx.x & (WAVE - 1), sl = lane % LPR;
    const int64_t wave = blockIdx.x * (int64_t)(BLK / WAVE) + (threadIdx.x >> 6);
    const int64_t row0 = wave * (RPW * U) + lane / LPR;
    if (row0 >= A.M) return;   // whole row groups leave together (the butterflies stay inside a group)
    const int H = A.H;
    float4 v[U][NV], rb[U][NV];
    float sum[U], sum_b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t row = row0 + u * RPW;
        const int64_t r = row < A.M ? row : A.M - 1;   // dead rows reload the last row; never stored
        sum[u] = 0.f; sum_b[u] = 0.f;
#pragma unroll
        for (int n = 0; n < NV; ++n) {
            const int c = (n * LPR + sl) * 4;
            v[u][n] = ld4(A.a + r * H + c);
            rb[u][n] = A.b ? ld4(A.b + r * H + c) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t row = row0 + u * RPW;
        const bool live = row < A.M;
#pragma unroll
        for (int n = 0; n < NV; ++n) {
            const int c = (n * LPR + sl) * 4;
            float4 x = v[u][n];
            if (A.a_bias) {
                const float4 ab = ld4(A.a_bias + c);
                x.x += ab.x; x.y += ab.y; x.z += ab.z; x.w += ab.w;
            }
            x = drop4(A, x, row, c);
            if (A.b) {
                const float4 rr = rb[u][n];
                x.x += rr.x; x.y += rr.y; x.z += rr.z; x.w += rr.w;
                sum_b[u] += (rr.x + rr.y) + (rr.z + rr.w);
            }
            v[u][n] = x;
            if (A.s_out && live) st4(A.s_out + row * H + c, x);
            sum[u] += (x.x + x.y) + (x.z + x.w);
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t row = row0 + u * RPW;
        const bool live = row < A.M;
        const float mean = row_sum<LPR>(sum[u]) / (float)H;
        float sq = 0.f;
#pragma unroll
        for (int n = 0; n < NV; ++n) {
            const float dx = v[u][n].x - mean, dyv = v[u][n].y - mean, dz = v[u][n].z - mean, dw = v[u][n].w - mean;
            sq += (dx * dx + dyv * dyv) + (dz * dz + dw * dw);
        }
        const float var = row_sum<LPR>(sq) / (float)H;
        const float rstd = 1.f / sqrtf(var + A.eps);
        float mean_s = 0.f, rstd_s = 0.f;
        if (A.gamma_s) {                     // skip branch: statistics of b alone (two-pass, like the main one)
            mean_s = row_sum<LPR>(sum_b[u]) / (float)H;
            float sqb = 0.f;
#pragma unroll
            for (int n = 0; n < NV; ++n) {
                const float dx = rb[u][n].x - mean_s, dyv = rb[u][n].y - mean_s, dz = rb[u][n].z - mean_s,
                            dw = rb[u][n].w - mean_s;
                sqb += (dx * dx + dyv * dyv) + (dz * dz + dw * dw);
            }
            rstd_s = 1.f / sqrtf(row_sum<LPR>(sqb) / (float)H + A.eps_s);
        }
        if (!live) continue;
#pragma unroll
        for (int n = 0; n < NV; ++n) {
            const int c = (n * LPR + sl) * 4;
            const float4 g = ld4(A.gamma + c), be = ld4(A.beta + c);
            float4 o;
            o.x = (v[u][n].x - mean) * rstd * g.x + be.x;
            o.y = (v[u][n].y - mean) * rstd * g.y + be.y;
            o.z = (v[u][n].z - mean) * rstd * g.z + be.z;
            o.w = (v[u][n].w - mean) * rstd * g.w + be.w;
            if (A.gamma_s) {   // same rounding as the reference's separate  y + LN_s(b)
                const float4 gs = ld4(A.gamma_s + c), bs = ld4(A.beta_s + c);
                o.x += (rb[u][n].x - mean_s) * rstd_s * gs.x + bs.x;
                o.y += (rb[u][n].y - mean_s) * rstd_s * gs.y + bs.y;
                o.z += (rb[u][n].z - mean_s) * rstd_s * gs.z + bs.z;
                o.w += (rb[u][n].w - mean_s) * rstd_s * gs.w + bs.w;
            }
            Io<S>::st(A.y, row * A.ldy + c, o);     // y in the storage type (bf16 feeds a GEMM)
        }
        if (A.ones_col && sl == 0) Io<S>::st(A.y, row * A.ldy + H, make_float4(1.f, 0.f, 0.f, 0.f));
        if (sl == 0) {
            A.mean[row] = mean;
            A.rstd[row] = rstd;
            if (A.gamma_s) {
                A.mean_s[row] = mean_s;
                A.rstd_s[row] = rstd_s;
            }
        }
    }
}

// SK: the skip branch of model.py:258-262 in the same pass -- y = LN(s) + LN_s(b) shares dy, so ds gets LN_s's
// input gradient too (b = A.b with statistics A.mean_s / A.rstd_s and gamma A.gamma_s), and the partial rows carry
// its dgamma_s | dbeta_s (5H per block instead of 3H).  One read of dy and one write of ds instead of two.
template <int LPR, int NV, int U, typename S, bool SK = false>
__global__ void __launch_bounds__(BLK) k_ln_bwd(LnArgs A) {
    TAGAN_LIVE_SEED(A);
    constexpr int RPW = WAVE / LPR, NP = SK ? 5 : 3;
    __shared__ float red[BLK / WAVE][RPW][NP * 4 * NV * LPR];
    const int lane = threadIdx.x & (WAVE - 1), sl = lane % LPR, sub = lane / LPR, w = threadIdx.x >> 6;
    const int H = A.H;
    float4 dg[NV], db[NV], dsa[NV], dgs[SK ? NV : 1], dbs[SK ? NV : 1];
#pragma unroll
    for (int n = 0; n < NV; ++n) {
        dg[n] = make_float4(0.f, 0.f, 0.f, 0.f);
        db[n] = make_float4(0.f, 0.f, 0.f, 0.f);
        dsa[n] = make_float4(0.f, 0.f, 0.f, 0.f);
        if constexpr (SK) {
            dgs[n] = make_float4(0.f, 0.f, 0.f, 0.f);
            dbs[n] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    const int64_t nwaves = (int64_t)gridDim.x * (BLK / WAVE);
    for (int64_t wave = blockIdx.x * (int64_t)(BLK / WAVE) + w; wave * (RPW * U) < A.M; wave += nwaves) {
        float4 sv[U][NV], dv[U][NV], ev[U][NV], bv[SK ? U : 1][NV];
        float mean[U], rstd[U], mean_s[SK ? U : 1], rstd_s[SK ? U : 1];
#pragma unroll
        for (int u = 0; u < U; ++u) {        // every load of the U row groups first
            const int64_t row = wave * (RPW * U) + u * RPW + sub;
            const int64_t r = row < A.M ? row : A.M - 1;
            mean[u] = A.mean[r];
            rstd[u] = A.rstd[r];
            if constexpr (SK) {
                mean_s[u] = A.mean_s[r];
                rstd_s[u] = A.rstd_s[r];
            }
#pragma unroll
            for (int n = 0; n < NV; ++n) {
                const int c = (n * LPR + sl) * 4;
                sv[u][n] = ld4(A.s_in + r * H + c);
                dv[u][n] = ld4(A.dy + r * H + c);
                ev[u][n] = (A.ds && A.dres) ? ld4(A.dres + r * H + c) : make_float4(0.f, 0.f, 0.f, 0.f);
                if constexpr (SK) bv[u][n] = ld4(A.b + r * H + c);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t row = wave * (RPW * U) + u * RPW + sub;
            const bool live = row < A.M;
            float4 xh[NV], gd[NV];
            float c1 = 0.f, c2 = 0.f;
#pragma unroll
            for (int n = 0; n < NV; ++n) {
                const int c = (n * LPR + sl) * 4;
                const float4 s = sv[u][n], d = dv[u][n], g = ld4(A.gamma + c);
                const float m = mean[u], rs = rstd[u];
                xh[n] = make_float4((s.x - m) * rs, (s.y - m) * rs, (s.z - m) * rs, (s.w - m) * rs);
                gd[n] = make_float4(d.x * g.x, d.y * g.y, d.z * g.z, d.w * g.w);
                c1 += (gd[n].x * xh[n].x + gd[n].y * xh[n].y) + (gd[n].z * xh[n].z + gd[n].w * xh[n].w);
                c2 += (gd[n].x + gd[n].y) + (gd[n].z + gd[n].w);
                if (live) {
                    dg[n].x += d.x * xh[n].x; dg[n].y += d.y * xh[n].y; dg[n].z += d.z * xh[n].z; dg[n].w += d.w * xh[n].w;
                    db[n].x += d.x; db[n].y += d.y; db[n].z += d.z; db[n].w += d.w;
                }
            }
            c1 = row_sum<LPR>(c1) / (float)H;
            c2 = row_sum<LPR>(c2) / (float)H;
            // skip branch: x̂_s, g_s·dy and its two row sums
            float4 xs[SK ? NV : 1], gs[SK ? NV : 1];
            float c1s = 0.f, c2s = 0.f;
            if constexpr (SK) {
#pragma unroll
                for (int n = 0; n < NV; ++n) {
                    const int c = (n * LPR + sl) * 4;
                    const float4 b = bv[u][n], d = dv[u][n], g = ld4(A.gamma_s + c);
                    const float m = mean_s[u], rs = rstd_s[u];
                    xs[n] = make_float4((b.x - m) * rs, (b.y - m) * rs, (b.z - m) * rs, (b.w - m) * rs);
                    gs[n] = make_float4(d.x * g.x, d.y * g.y, d.z * g.z, d.w * g.w);
                    c1s += (gs[n].x * xs[n].x + gs[n].y * xs[n].y) + (gs[n].z * xs[n].z + gs[n].w * xs[n].w);
                    c2s += (gs[n].x + gs[n].y) + (gs[n].z + gs[n].w);
                    if (live) {
                        dgs[n].x += d.x * xs[n].x; dgs[n].y += d.y * xs[n].y; dgs[n].z += d.z * xs[n].z; dgs[n].w += d.w * xs[n].w;
                        dbs[n].x += d.x; dbs[n].y += d.y; dbs[n].z += d.z; dbs[n].w += d.w;
                    }
                }
                c1s = row_sum<LPR>(c1s) / (float)H;
                c2s = row_sum<LPR>(c2s) / (float)H;
            }
            if (!live) continue;
            const float rs = rstd[u];
#pragma unroll
            for (int n = 0; n < NV; ++n) {
                const int c = (n * LPR + sl) * 4;
                float4 o;
                o.x = rs * (gd[n].x - c1 * xh[n].x - c2);
                o.y = rs * (gd[n].y - c1 * xh[n].y - c2);
                o.z = rs * (gd[n].z - c1 * xh[n].z - c2);
                o.w = rs * (gd[n].w - c1 * xh[n].w - c2);
                if (A.da || A.want_dsa) {
                    const float4 a = drop4(A, o, row, c);
                    if (A.da) Io<S>::st(A.da, row * H + c, a);   // da in the storage type
                    dsa[n].x += a.x; dsa[n].y += a.y; dsa[n].z += a.z; dsa[n].w += a.w;
                }
                if (A.ds) {
                    const float4 e = ev[u][n];
                    o.x += e.x; o.y += e.y; o.z += e.z; o.w += e.w;
                    if constexpr (SK) {   // + LN_s's input gradient (same rounding order as the two-pass form)
                        const float r2 = rstd_s[u];
                        o.x += r2 * (gs[n].x - c1s * xs[n].x - c2s);
                        o.y += r2 * (gs[n].y - c1s * xs[n].y - c2s);
                        o.z += r2 * (gs[n].z - c1s * xs[n].z - c2s);
                        o.w += r2 * (gs[n].w - c1s * xs[n].w - c2s);
                    }
                    st4(A.ds + row * H + c, o);
                }
            }
        }
    }
    if (A.part) {
#pragma unroll
        for (int n = 0; n < NV; ++n) {
            const int c = (n * LPR + sl) * 4;
            st4(&red[w][sub][c], dg[n]);
            st4(&red[w][sub][H + c], db[n]);
            st4(&red[w][sub][2 * H + c], dsa[n]);
            if constexpr (SK) {
                st4(&red[w][sub][3 * H + c], dgs[n]);
                st4(&red[w][sub][4 * H + c], dbs[n]);
            }
        }
        __syncthreads();
        for (int x = threadIdx.x; x < NP * H; x += BLK) {
            float s = 0.f;
            for (int ww = 0; ww < BLK / WAVE; ++ww)
                for (int ss = 0; ss < RPW; ++ss) s += red[ww][ss][x];
            A.part[(int64_t)blockIdx.x * NP * H + x] = s;
        }
    }
}

// Geometry: H = 4 * LPR * NV with LPR in {8,16,32,64}, NV in {1,2}.
bool geometry(int H, int& lpr, int& nv) {
    switch (H) {
        case 32: lpr = 8; nv = 1; return true;
        case 64: lpr = 16; nv = 1; return true;
        case 128: lpr = 32; nv = 1; return true;
        case 256: lpr = 64; nv = 1; return true;
        case 512: lpr = 64; nv = 2; return true;
        default: return false;
    }
}

// Backward grid (persistent blocks, one [3H] partial row each): 1024 blocks (4 waves / SIMD); 1280 / 2048 / 4096 were
// 3 / 10 / 27 % slower on the full backward (profiles/r1_ln_bwd_blocks_ab.txt).
#ifndef TAGAN_LN_BWD_BLOCKS
#define TAGAN_LN_BWD_BLOCKS 1024
#endif
int ln_bwd_blocks() { return TAGAN_LN_BWD_BLOCKS; }

// Row groups per wave (U): 4.  Round 1 measured 2 best at C2 (profiles/r1_ln_rows_ab.txt); round 5 re-measured the
// backward at 4: C2 shape 162-163 vs 166 us, H = 256 (3.2M rows) 3.24 vs 3.41-3.48 ms, the C2 step within noise
// (profiles/r5w_ln_bwd_ab.txt; a register prefetch of the next iteration's rows measured no gain and is not built).
// NV = 2 (H = 512) is instantiated for U <= 2 only.
#ifndef TAGAN_LN_ROWS
#define TAGAN_LN_ROWS 4
#endif
static_assert(TAGAN_LN_ROWS == 1 || TAGAN_LN_ROWS == 2 || TAGAN_LN_ROWS == 4, "TAGAN_LN_ROWS: 1, 2 or 4 (instantiated)");
int ln_rows(int nv) { return nv == 2 && TAGAN_LN_ROWS > 2 ? 2 : TAGAN_LN_ROWS; }

// the fused LN2 + skip-LN backward (one float4 per lane and row: H = 128 (LPR 32) and, round 6, H = 256 (LPR 64);
// any U).  Both launchers run exactly the U the caller sized the grid for, or launch nothing and return false.
template <typename S>
bool launch_ln_skip_bwd(int lpr, int u, dim3 g, hipStream_t s, const LnArgs& A) {
#define TAGAN_LN_SK(L)                                                       \
    do {                                                                     \
        if (u == 1) k_ln_bwd<L, 1, 1, S, true><<<g, BLK, 0, s>>>(A);         \
        else if (u == 2) k_ln_bwd<L, 1, 2, S, true><<<g, BLK, 0, s>>>(A);    \
        else if (u == 4) k_ln_bwd<L, 1, 4, S, true><<<g, BLK, 0, s>>>(A);    \
        else return false;                                                   \
    } while (0)
    if (lpr == 32) TAGAN_LN_SK(32);
    else if (lpr == 64) TAGAN_LN_SK(64);
    else return false;
#undef TAGAN_LN_SK
    return true;
}

template <typename S, bool FWD>
bool launch_ln(int lpr, int nv, int u, dim3 g, hipStream_t s, const LnArgs& A) {
#define TAGAN_LN_K(L, N, U) (FWD ? k_ln_fwd<L, N, U, S> : k_ln_bwd<L, N, U, S>)<<<g, BLK, 0, s>>>(A)
#define TAGAN_LN_U(L, N)                          \
    do {                                          \
        if (u == 1) TAGAN_LN_K(L, N, 1);          \
        else if (u == 2) TAGAN_LN_K(L, N, 2);     \
        else if (u == 4) TAGAN_LN_K(L, N, 4);     \
        else return false;                        \
    } while (0)
    if (lpr == 8) TAGAN_LN_U(8, 1);
    else if (lpr == 16) TAGAN_LN_U(16, 1);
    else if (lpr == 32) TAGAN_LN_U(32, 1);
    else if (nv == 1) TAGAN_LN_U(64, 1);
    else if (u == 1) TAGAN_LN_K(64, 2, 1);
    else if (u == 2) TAGAN_LN_K(64, 2, 2);
    else return false;
#undef TAGAN_LN_U
#undef TAGAN_LN_K
    return true;
}

}  // namespace
}  // namespace tagan

extern "C" {

int tagan_layernorm_supported(int32_t H) {
    int l, n;
    return tagan::geometry(H, l, n) ? 1 : 0;
}

int tagan_add_layernorm_fwd(int dtype, int64_t M, int32_t H, const float* a, const float* a_bias, const float* b,
                            float p_drop,
                            uint64_t seed, const float* gamma, const float* beta, float eps, float* s_out, float* y,
                            int64_t ldy, float* mean, float* rstd, void* stream) {
    using namespace tagan;
    int lpr, nv;
    TAGAN_REQUIRE(dtype == TAGAN_F32 || dtype == TAGAN_BF16, TAGAN_ERR_UNSUPPORTED, "layernorm: dtype %d", dtype);
    TAGAN_REQUIRE(geometry(H, lpr, nv), TAGAN_ERR_UNSUPPORTED, "layernorm: H=%d unsupported", H);
    TAGAN_REQUIRE(M > 0 && a && gamma && beta && y && mean && rstd, TAGAN_ERR_ARG, "layernorm_fwd: bad args");
    TAGAN_REQUIRE(p_drop >= 0.f && p_drop < 1.f, TAGAN_ERR_ARG, "layernorm_fwd: p_drop");
    LnArgs A{};
    A.M = M; A.H = H; A.a = a; A.a_bias = a_bias; A.b = b; A.p_drop = p_drop; A.inv_keep = 1.f / (1.f - p_drop); A.seed = seed; A.seed_ctr = seed_counter();
    A.gamma = gamma; A.beta = beta; A.eps = eps; A.s_out = s_out; A.y = y; A.mean = mean; A.rstd = rstd;
    A.ldy = ldy > 0 ? ldy : H;
    TAGAN_REQUIRE(A.ldy >= H && A.ldy % 4 == 0, TAGAN_ERR_ARG, "layernorm_fwd: ldy %lld", (long long)ldy);
    A.ones_col = A.ldy >= H + 4;
    const int u = ln_rows(nv);
    const int64_t rpw = (WAVE / lpr) * u;
    const dim3 g((unsigned)(((M + rpw - 1) / rpw + (BLK / WAVE) - 1) / (BLK / WAVE)));
    hipStream_t s = as_stream(stream);
    const bool ok = dtype == TAGAN_BF16 ? launch_ln<bf16s, true>(lpr, nv, u, g, s, A)
                                        : launch_ln<float, true>(lpr, nv, u, g, s, A);
    TAGAN_REQUIRE(ok, TAGAN_ERR_UNSUPPORTED, "layernorm_fwd: no kernel for H=%d with %d row groups per wave", H, u);
    TAGAN_CHECK_LAUNCH("layernorm_fwd");
    return TAGAN_OK;
}

int tagan_add_layernorm_skip_fwd(int64_t M, int32_t H, const float* a, const float* a_bias, const float* b,
                                 float p_drop, uint64_t seed,
                                 const float* gamma, const float* beta, float eps, const float* gamma_s,
                                 const float* beta_s, float eps_s, float* s_out, float* y, float* mean, float* rstd,
                                 float* mean_s, float* rstd_s, void* stream) {
    using namespace tagan;
    int lpr, nv;
    TAGAN_REQUIRE(geometry(H, lpr, nv), TAGAN_ERR_UNSUPPORTED, "layernorm: H=%d unsupported", H);
    TAGAN_REQUIRE(M > 0 && a && b && gamma && beta && gamma_s && beta_s && y && mean && rstd && mean_s && rstd_s,
                  TAGAN_ERR_ARG, "layernorm_skip_fwd: bad args");
    TAGAN_REQUIRE(p_drop >= 0.f && p_drop < 1.f, TAGAN_ERR_ARG, "layernorm_skip_fwd: p_drop");
    LnArgs A{};
    A.M = M; A.H = H; A.a = a; A.a_bias = a_bias; A.b = b; A.p_drop = p_drop; A.inv_keep = 1.f / (1.f - p_drop); A.seed = seed; A.seed_ctr = seed_counter();
    A.gamma = gamma; A.beta = beta; A.eps = eps; A.s_out = s_out; A.y = y; A.mean = mean; A.rstd = rstd;
    A.ldy = H;
    A.gamma_s = gamma_s; A.beta_s = beta_s; A.eps_s = eps_s; A.mean_s = mean_s; A.rstd_s = rstd_s;
    const int u = ln_rows(nv);
    const int64_t rpw = (WAVE / lpr) * u;
    const dim3 g((unsigned)(((M + rpw - 1) / rpw + (BLK / WAVE) - 1) / (BLK / WAVE)));
    TAGAN_REQUIRE((launch_ln<float, true>(lpr, nv, u, g, as_stream(stream), A)), TAGAN_ERR_UNSUPPORTED,
                  "layernorm_skip_fwd: no kernel for H=%d with %d row groups per wave", H, u);
    TAGAN_CHECK_LAUNCH("layernorm_skip_fwd");
    return TAGAN_OK;
}

size_t tagan_layernorm_bwd_workspace(int64_t M, int32_t H) {
    (void)M;
    return (size_t)tagan::ln_bwd_blocks() * 3 * H * sizeof(float);
}

int tagan_layernorm_bwd(int dtype, int64_t M, int32_t H, const float* s_in, const float* mean, const float* rstd,
                        const float* gamma, const float* dy, const float* dres, float p_drop, uint64_t seed,
                        float* ds, float* da, float* dgamma, float* dbeta, float* dsum_a, void* workspace,
                        size_t workspace_bytes, void* stream) {
    using namespace tagan;
    int lpr, nv;
    TAGAN_REQUIRE(dtype == TAGAN_F32 || dtype == TAGAN_BF16, TAGAN_ERR_UNSUPPORTED, "layernorm: dtype %d", dtype);
    TAGAN_REQUIRE(geometry(H, lpr, nv), TAGAN_ERR_UNSUPPORTED, "layernorm: H=%d unsupported", H);
    TAGAN_REQUIRE(M > 0 && s_in && mean && rstd && gamma && dy, TAGAN_ERR_ARG, "layernorm_bwd: bad args");
    const bool want = dgamma || dbeta || dsum_a;
    TAGAN_REQUIRE(!want || (workspace && workspace_bytes >= tagan_layernorm_bwd_workspace(M, H)),
                  TAGAN_ERR_WORKSPACE, "layernorm_bwd: workspace");
    LnArgs A{};
    A.M = M; A.H = H; A.gamma = gamma; A.s_in = s_in; A.mean = (float*)mean; A.rstd = (float*)rstd; A.dy = dy;
    A.dres = dres; A.ds = ds; A.da = da; A.p_drop = p_drop; A.inv_keep = 1.f / (1.f - p_drop); A.seed = seed; A.seed_ctr = seed_counter();
    A.part = want ? (float*)workspace : nullptr;
    A.want_dsa = dsum_a != nullptr;
    const int u = ln_rows(nv);
    const int64_t rpw = (WAVE / lpr) * u;
    const int64_t need = ((M + rpw - 1) / rpw + (BLK / WAVE) - 1) / (BLK / WAVE);
    const int nblk = (int)std::min<int64_t>(need, ln_bwd_blocks());
    hipStream_t s = as_stream(stream);
    const bool ok = dtype == TAGAN_BF16 ? launch_ln<bf16s, false>(lpr, nv, u, dim3(nblk), s, A)
                                        : launch_ln<float, false>(lpr, nv, u, dim3(nblk), s, A);
    TAGAN_REQUIRE(ok, TAGAN_ERR_UNSUPPORTED, "layernorm_bwd: no kernel for H=%d with %d row groups per wave", H, u);
    TAGAN_CHECK_LAUNCH("layernorm_bwd");
    if (dgamma || dbeta) {
        launch_colsum(A.part, nblk, 2 * H, dgamma, dbeta, H, s, 1.f, 3 * H);
        TAGAN_CHECK_LAUNCH("layernorm_bwd_sum");
    }
    if (dsum_a) {
        launch_colsum(A.part + 2 * H, nblk, H, dsum_a, nullptr, H, s, 1.f, 3 * H);
        TAGAN_CHECK_LAUNCH("layernorm_bwd_sum_a");
    }
    return TAGAN_OK;
}

size_t tagan_layernorm_skip_bwd_workspace(int64_t M, int32_t H) {
    (void)M;
    return (size_t)tagan::ln_bwd_blocks() * 5 * H * sizeof(float);
}

int tagan_layernorm_skip_bwd(int dtype, int64_t M, int32_t H, const float* s_in, const float* mean, const float* rstd,
                             const float* gamma, const float* b, const float* mean_s, const float* rstd_s,
                             const float* gamma_s, const float* dy, float p_drop, uint64_t seed, float* ds, float* da,
                             float* dgamma, float* dbeta, float* dsum_a, float* dgamma_s, float* dbeta_s,
                             void* workspace, size_t workspace_bytes, void* stream) {
    using namespace tagan;
    TAGAN_REQUIRE(dtype == TAGAN_F32 || dtype == TAGAN_BF16, TAGAN_ERR_UNSUPPORTED, "layernorm: dtype %d", dtype);
    int lpr, nv;
    TAGAN_REQUIRE(geometry(H, lpr, nv) && nv == 1 && (lpr == 32 || lpr == 64), TAGAN_ERR_UNSUPPORTED,
                  "layernorm_skip_bwd: H=%d (H = 128 or 256)", H);
    TAGAN_REQUIRE(M > 0 && s_in && mean && rstd && gamma && b && mean_s && rstd_s && gamma_s && dy && ds && da &&
                      dgamma && dbeta && dsum_a && dgamma_s && dbeta_s,
                  TAGAN_ERR_ARG, "layernorm_skip_bwd: bad args");
    TAGAN_REQUIRE(workspace && workspace_bytes >= tagan_layernorm_skip_bwd_workspace(M, H), TAGAN_ERR_WORKSPACE,
                  "layernorm_skip_bwd: workspace");
    LnArgs A{};
    A.M = M; A.H = H; A.gamma = gamma; A.s_in = s_in; A.mean = (float*)mean; A.rstd = (float*)rstd; A.dy = dy;
    A.b = b; A.mean_s = (float*)mean_s; A.rstd_s = (float*)rstd_s; A.gamma_s = gamma_s;
    A.dres = nullptr; A.ds = ds; A.da = da; A.p_drop = p_drop; A.inv_keep = 1.f / (1.f - p_drop); A.seed = seed;
    A.seed_ctr = seed_counter();
    A.part = (float*)workspace;
    A.want_dsa = 1;
    const int u = ln_rows(1);
    const int64_t rpw = (WAVE / lpr) * u;
    const int64_t need = ((M + rpw - 1) / rpw + (BLK / WAVE) - 1) / (BLK / WAVE);
    const int nblk = (int)std::min<int64_t>(need, ln_bwd_blocks());
    hipStream_t s = as_stream(stream);
    const bool ok = dtype == TAGAN_BF16 ? launch_ln_skip_bwd<bf16s>(lpr, u, dim3(nblk), s, A)
                                        : launch_ln_skip_bwd<float>(lpr, u, dim3(nblk), s, A);
    TAGAN_REQUIRE(ok, TAGAN_ERR_UNSUPPORTED, "layernorm_skip_bwd: no kernel with %d row groups per wave", u);
    TAGAN_CHECK_LAUNCH("layernorm_skip_bwd");
    launch_colsum(A.part, nblk, 2 * H, dgamma, dbeta, H, s, 1.f, 5 * H);
    TAGAN_CHECK_LAUNCH("layernorm_skip_bwd_sum");
    launch_colsum(A.part + 2 * H, nblk, H, dsum_a, nullptr, H, s, 1.f, 5 * H);
    TAGAN_CHECK_LAUNCH("layernorm_skip_bwd_sum_a");
    launch_colsum(A.part + 3 * H, nblk, 2 * H, dgamma_s, dbeta_s, H, s, 1.f, 5 * H);
    TAGAN_CHECK_LAUNCH("layernorm_skip_bwd_sum_s");
    return TAGAN_OK;
}

}  // extern "C"
