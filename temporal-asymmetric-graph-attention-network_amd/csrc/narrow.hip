// Narrow-input projection y = x·Wᵀ + b (K <= 31 input features, N = 64, 128 or 256 outputs, fp32) and its parameter
// gradients: TAGAN's node embedding, model.py:233 (nn.Linear(node_feature_dim, hidden_dim) applied to every
// snapshot's x; C2: [320000, 27] -> [320000, 128]).
//
// Both directions run on the exact-f32 matrix core (v_mfma_f32_16x16x4_f32: a k-ordered fmaf chain, bitwise
// deterministic): the problem is HBM-bound (y / dY are 4.7x the bytes of x), and at K = 27 the f32 VALU would sit
// at the same time as the traffic.
//   forward : a wave owns 16-row tiles (grid-stride); A = x rows (lane: row l & 15, feature l >> 4 + 4 s),
//             B = Wᵀ from LDS; the bias is the accumulator's initial value; 64-B output segments per row.
//   backward: [dW | db]ᵀ = x_augᵀ · dY over the rows, x_aug = [x | 1 | 0 ...] (feature K is a column of ones, so the
//             accumulator row K is Σ dY = db): A = x_aug (lane: feature l & 15 + 16 kt, row l >> 4), B = dY rows;
//             each workgroup sums a contiguous row range (its waves interleave 4-row groups in a fixed order), the
//             waves meet in LDS in a fixed order, and the per-workgroup partials [N·K | N] are folded by the
//             ordered column sum (k_colsum_parts) -- the same result on every run.
// Replaces the library GEMM + split-K batched GEMM + sum + bias column sum of the projection (4 launches, ~150 us
// per C2 step; profiles/r6r_c2_kernel_stats.csv) with 1 + 2 launches over y / dY once each.
#include <algorithm>
#include <cstdlib>

#include "common.cuh"

namespace tagan {
namespace {

typedef float nf32x4 __attribute__((ext_vector_type(4)));
constexpr int NBLK = 256;     // 4 waves
constexpr int NKMAX = 31;     // K + 1 <= 32 (the backward's ones column)
constexpr int NNMAX = 256;

__device__ __forceinline__ nf32x4 mfma4(float a, float b, nf32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Virtual n-tiles: MFMA tile (blk, c) of a 64-column block takes columns 64 blk + 4 j + c (j = the tile's column
// index 0..15), so lane li holds columns 64 blk + 4 li + [0, 4) of the four tiles c = 0..3: the forward stores and
// the backward's dY loads are whole float4 per lane (256-B row runs) instead of 64-B dword segments.

// y[r][n] = b[n] + Σ_k x[r][k] w[n][k]
template <int NB, int KS>   // N / 64 column blocks, ceil(K / 4) feature steps
__global__ void __launch_bounds__(NBLK) k_narrow_fwd(int64_t M, int K, const float* __restrict__ x, int64_t ldx,
                                                     const float* __restrict__ w, const float* __restrict__ b,
                                                     float* __restrict__ y, int64_t ldy) {
    constexpr int N = NB * 64;
    __shared__ float wt[4 * KS][N];   // Wᵀ, features >= K zero
    for (int i = threadIdx.x; i < 4 * KS * N; i += NBLK) {
        const int k = i / N, n = i % N;
        wt[k][n] = k < K ? w[(int64_t)n * K + k] : 0.f;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
    nf32x4 bias[NB];
#pragma unroll
    for (int bk = 0; bk < NB; ++bk)
        bias[bk] = b ? *reinterpret_cast<const nf32x4*>(b + 64 * bk + 4 * li) : nf32x4{0.f, 0.f, 0.f, 0.f};
    const int64_t ntiles = (M + 15) / 16;
    const int64_t nw = (int64_t)gridDim.x * (NBLK / 64);
    // the next tile's x is loaded before this tile's MFMAs (a wave's tiles are a dependent chain otherwise)
    float a[KS], an[KS];
    auto load = [&](int64_t t, float (&av)[KS]) {
        const int64_t rw = t * 16 + li;
        const int64_t ra = rw < M ? rw : M - 1;   // rows past M reload the last row (never stored)
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int k = 4 * s + g;
            av[s] = k < K ? x[ra * ldx + k] : 0.f;
        }
    };
    int64_t tile = blockIdx.x * (int64_t)(NBLK / 64) + (threadIdx.x >> 6);
    if (tile < ntiles) load(tile, a);
    for (; tile < ntiles; tile += nw) {
        const int64_t r0 = tile * 16;
        if (tile + nw < ntiles) load(tile + nw, an);
        nf32x4 acc[NB][4];
#pragma unroll
        for (int bk = 0; bk < NB; ++bk)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[bk][c] = nf32x4{bias[bk][c], bias[bk][c], bias[bk][c], bias[bk][c]};
#pragma unroll
        for (int s = 0; s < KS; ++s) {
#pragma unroll
            for (int bk = 0; bk < NB; ++bk) {
                const nf32x4 wv = *reinterpret_cast<const nf32x4*>(&wt[4 * s + g][64 * bk + 4 * li]);
#pragma unroll
                for (int c = 0; c < 4; ++c) acc[bk][c] = mfma4(a[s], wv[c], acc[bk][c]);
            }
        }
        // D[i][j] of tile (bk, c): lane holds rows 4 g + e, column 64 bk + 4 li + c
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int64_t r = r0 + 4 * g + e;
            if (r < M) {
#pragma unroll
                for (int bk = 0; bk < NB; ++bk)
                    *reinterpret_cast<nf32x4*>(y + r * ldy + 64 * bk + 4 * li) =
                        nf32x4{acc[bk][0][e], acc[bk][1][e], acc[bk][2][e], acc[bk][3][e]};
            }
        }
#pragma unroll
        for (int s = 0; s < KS; ++s) a[s] = an[s];
    }
}

// part[blockIdx.x] = [ dW (n-major: n K + k) | db ] over the workgroup's rows [r0, r1)
template <int NB>
__global__ void __launch_bounds__(NBLK) k_narrow_bwd(int64_t M, int K, const float* __restrict__ x, int64_t ldx,
                                                     const float* __restrict__ dy, int64_t lddy,
                                                     int64_t rows_per_wg, float* __restrict__ part) {
    constexpr int N = NB * 64;
    __shared__ float red[32][N + 4];
    const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4, w = threadIdx.x >> 6;
    const int64_t r0 = blockIdx.x * rows_per_wg;
    const int64_t r1 = r0 + rows_per_wg < M ? r0 + rows_per_wg : M;
    nf32x4 acc[2][NB][4];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int bk = 0; bk < NB; ++bk)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[kt][bk][c] = nf32x4{0.f, 0.f, 0.f, 0.f};
    // wave w takes the 4-row groups w, w + 4, ... of the range (lane row g); a dead row contributes exact zeros
    // (a = 0).  A ring of PD groups' operands: group i's slot is reloaded with group i + PD right after its MFMAs,
    // so PD groups of loads are in flight (one group of prefetch left the loop latency-bound: 62.7 us at C2).
    constexpr int PD = 4;
    float a[PD][2];
    nf32x4 bv[PD][NB];
    auto load = [&](int64_t q, float (&av)[2], nf32x4 (&dv)[NB]) {
        const int64_t r = q + g;
        const bool live = r < r1;
        const int64_t rr = live ? r : (r1 > 0 ? r1 - 1 : 0);
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
            const int k = kt * 16 + li;
            const float xv = k < K ? x[rr * ldx + k] : (k == K ? 1.f : 0.f);
            av[kt] = live ? xv : 0.f;
        }
#pragma unroll
        for (int bk = 0; bk < NB; ++bk) dv[bk] = *reinterpret_cast<const nf32x4*>(dy + rr * lddy + 64 * bk + 4 * li);
    };
    constexpr int64_t STEP = 4 * (NBLK / 64);
    const int64_t q0 = r0 + 4 * w;
#pragma unroll
    for (int u = 0; u < PD; ++u) load(q0 + u * STEP, a[u], bv[u]);
    for (int64_t q = q0; q < r1; q += PD * STEP) {
#pragma unroll
        for (int u = 0; u < PD; ++u) {
#pragma unroll
            for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                for (int bk = 0; bk < NB; ++bk)
#pragma unroll
                    for (int c = 0; c < 4; ++c) acc[kt][bk][c] = mfma4(a[u][kt], bv[u][bk][c], acc[kt][bk][c]);
            load(q + (u + PD) * STEP, a[u], bv[u]);
        }
    }
    // D[i = feature][j]: lane holds features 16 kt + 4 g + e, column 64 bk + 4 li + c; the waves meet in one LDS
    // image in wave order (fixed: bitwise reproducible)
    for (int ww = 0; ww < NBLK / 64; ++ww) {
        if (w == ww) {
#pragma unroll
            for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                for (int bk = 0; bk < NB; ++bk)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        nf32x4* d = reinterpret_cast<nf32x4*>(&red[16 * kt + 4 * g + e][64 * bk + 4 * li]);
                        const nf32x4 v{acc[kt][bk][0][e], acc[kt][bk][1][e], acc[kt][bk][2][e], acc[kt][bk][3][e]};
                        *d = ww == 0 ? v : *d + v;
                    }
        }
        __syncthreads();
    }
    float* p = part + (int64_t)blockIdx.x * (N * K + N);
    for (int i = threadIdx.x; i < (K + 1) * N; i += NBLK) {
        const int k = i / N, n = i % N;
        if (k < K) p[n * K + k] = red[k][n];
        else p[N * K + n] = red[k][n];
    }
}

// backward workgroups (row ranges): at most TAGAN_NARROW_BWD_GROUPS (A/B knob, default 512), >= 256 rows each
int narrow_groups(int64_t M) {
    static const int64_t gmax = [] {
        const char* e = std::getenv("TAGAN_NARROW_BWD_GROUPS");
        return (int64_t)(e && std::atoi(e) > 0 ? std::atoi(e) : 512);
    }();
    const int64_t g = (M + 255) / 256;
    return (int)(g < gmax ? (g > 0 ? g : 1) : gmax);
}

}  // namespace
}  // namespace tagan

extern "C" {

int tagan_narrow_linear_supported(int32_t K, int32_t N) {
    return K >= 1 && K <= tagan::NKMAX && (N == 64 || N == 128 || N == tagan::NNMAX) ? 1 : 0;
}

int tagan_narrow_linear_fwd(int64_t M, int32_t K, int32_t N, const float* x, int64_t ldx, const float* w,
                            const float* b, float* y, int64_t ldy, void* stream) {
    using namespace tagan;
    TAGAN_REQUIRE(tagan_narrow_linear_supported(K, N), TAGAN_ERR_UNSUPPORTED, "narrow_linear: K=%d N=%d", K, N);
    TAGAN_REQUIRE(M >= 0 && (M == 0 || (x && w && y)) && ldx >= K && ldy >= N && ldy % 4 == 0 &&
                      (uintptr_t)y % 16 == 0 && (!b || (uintptr_t)b % 16 == 0), TAGAN_ERR_ARG,
                  "narrow_linear_fwd: bad args");
    if (M == 0) return TAGAN_OK;
    const int64_t tiles = (M + 15) / 16;
    // persistent: one workgroup per CU (256 / 512 / 768 / 1024: 43.8 / 47.3 / 54.9 / 48.2 us at C2,
    // profiles/r6ac_narrow_grid.txt), each stages Wᵀ once (a workgroup per 4
    // tiles re-read it 4096 times and spent its life in the staging: 69 us at C2)
    static const int64_t gmax = [] {
        const char* e = std::getenv("TAGAN_NARROW_GRID");   // A/B knob (workgroups, default 256)
        return (int64_t)(e && std::atoi(e) > 0 ? std::atoi(e) : 256);
    }();
    const unsigned grid = (unsigned)std::min<int64_t>((tiles + 3) / 4, gmax);
    hipStream_t s = as_stream(stream);
#define TAGAN_NF(NB, KS) k_narrow_fwd<NB, KS><<<grid, NBLK, 0, s>>>(M, K, x, ldx, wc, bc, yc, ldy)
#define TAGAN_NFK(NB) if (K <= 16) TAGAN_NF(NB, 4); else if (K <= 28) TAGAN_NF(NB, 7); else TAGAN_NF(NB, 8)
    // N = 256 as two 128-column launches (a four-block kernel takes 308 registers: one wave per SIMD)
    for (int c0 = 0; c0 < N; c0 += 128) {
        const float* wc = w + (int64_t)c0 * K;
        const float* bc = b ? b + c0 : nullptr;
        float* yc = y + c0;
        if (N == 64) TAGAN_NFK(1);
        else TAGAN_NFK(2);
    }
#undef TAGAN_NFK
#undef TAGAN_NF
    TAGAN_CHECK_LAUNCH("narrow_linear_fwd");
    return TAGAN_OK;
}

size_t tagan_narrow_linear_bwd_workspace(int64_t M, int32_t K, int32_t N) {
    const int NC = N <= 128 ? N : 128;   // per column pass
    return (size_t)tagan::narrow_groups(M) * (size_t)(NC * K + NC) * sizeof(float);
}

int tagan_narrow_linear_bwd(int64_t M, int32_t K, int32_t N, const float* x, int64_t ldx, const float* dy,
                            int64_t lddy, float* dw, float* db, void* workspace, size_t workspace_bytes,
                            void* stream) {
    using namespace tagan;
    TAGAN_REQUIRE(tagan_narrow_linear_supported(K, N), TAGAN_ERR_UNSUPPORTED, "narrow_linear: K=%d N=%d", K, N);
    TAGAN_REQUIRE(M > 0 && x && dy && (dw || db) && ldx >= K && lddy >= N && lddy % 4 == 0 &&
                      (uintptr_t)dy % 16 == 0, TAGAN_ERR_ARG,
                  "narrow_linear_bwd: bad args");
    TAGAN_REQUIRE(workspace && workspace_bytes >= tagan_narrow_linear_bwd_workspace(M, K, N), TAGAN_ERR_WORKSPACE,
                  "narrow_linear_bwd: workspace");
    const int G = narrow_groups(M);
    const int64_t per = ((M + G - 1) / G + 3) / 4 * 4;
    hipStream_t s = as_stream(stream);
    float* part = (float*)workspace;
    // N = 256 as two 128-column passes, each with its own partials and ordered column sum
    const int NC = N == 64 ? 64 : 128;
    for (int c0 = 0; c0 < N; c0 += NC) {
        const float* dyc = dy + c0;
        if (NC == 64) k_narrow_bwd<1><<<G, NBLK, 0, s>>>(M, K, x, ldx, dyc, lddy, per, part);
        else k_narrow_bwd<2><<<G, NBLK, 0, s>>>(M, K, x, ldx, dyc, lddy, per, part);
        TAGAN_CHECK_LAUNCH("narrow_linear_bwd");
        launch_colsum(part, G, NC * K + NC, dw ? dw + (int64_t)c0 * K : nullptr, db ? db + c0 : nullptr, NC * K, s);
        TAGAN_CHECK_LAUNCH("narrow_linear_bwd_sum");
    }
    return TAGAN_OK;
}

}  // extern "C"
