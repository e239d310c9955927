// Projection GEMMs of the attention blocks on the gfx950 bf16 matrix cores (v_mfma_f32_16x16x32_bf16).
//
// Every projection of the hot path (GeometricAttention.forward, geometric_attention.py:541-596; the temporal
// layer's q/k/v/out projections, temporal_attention.py:985-1200) is a STREAMING shape: M = rows of the block
// (320k at C2), K and N = H or 3H (128 / 384), so the weights are small and every activation byte is touched once.
// Two kernels cover the six products of a block:
//
//   k_sgemm_nt  C[M, N] = A[M, K] · B[N, K]ᵀ (+ bias[N])   forward projections (B = W) and input gradients
//               (B = Wᵀ, prepared once per call): WEIGHT-STATIONARY — each wave keeps the bf16 fragments of its
//               16-column slabs of B for all of K in registers for the whole kernel, the workgroup streams A
//               tiles (BM rows) HBM -> registers -> bf16 planes in LDS (double-buffered: tile i+1's loads are in
//               flight while tile i's MFMAs run) and the accumulators go straight to HBM.
//   k_sgemm_tn  dW[N, K] = dYᵀ · X and db[N] = Σ_m dY  weight / bias gradients: split over M across the
//               workgroups; a 32-row tile of dY and X is staged as row-major bf16 planes in LDS and read back
//               column-major with ds_read_b64_tr_b16; per-workgroup partials are summed by k_sgemm_tn_reduce in
//               a fixed order (bitwise reproducible).
//
// fp32 ("planes" = 3): both operands are split into three bf16 planes, x = x0 + x1 + x2 (each the round-to-
// nearest bf16 of the previous remainder, so |x - x0 - x1 - x2| <= 2^-24 |x|), and every product keeps the six
// terms of weight up to 2^-16: a0b0 + a0b1 + a1b0 + a0b2 + a1b1 + a2b0 (the dropped a1b2, a2b1, a2b2 are
// <= 2^-24 |a||b| each), accumulated in fp32 by the matrix core.  The result differs from an fp32 GEMM by the
// same order as two fp32 GEMMs with different summation orders differ (tests/test_gpu_sgemm.py pins it against
// fp64 and against torch's fp32 GEMM).  Six bf16 MFMAs cost 6/16 of one fp32 MFMA's cycles, so the fp32 products
// run at 2.7x the fp32 matrix-core peak and these shapes become HBM-bound.
// bf16 ("planes" = 1): one plane (the bf16 activation mode's operands), fp32 accumulate.
#include <stdlib.h>

#include <algorithm>

#include "common.cuh"

namespace tagan {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// two fp32 -> two bf16 (round to nearest even, v_cvt_pk_bf16_f32), packed low | high
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
    const f32x2 v = {a, b};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
}
__device__ __forceinline__ float bf_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }

// planes of a pair (a, b): out[p] = packed bf16 pair of plane p (P = 1 or 3)
template <int P>
__device__ __forceinline__ void split2(float a, float b, uint32_t (&out)[P]) {
    out[0] = pk_bf16(a, b);
    if constexpr (P == 3) {
        const float ra = a - bf_lo(out[0]), rb = b - bf_hi(out[0]);
        out[1] = pk_bf16(ra, rb);
        out[2] = pk_bf16(ra - bf_lo(out[1]), rb - bf_hi(out[1]));
    }
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its global loads and
// stores (__syncthreads() emits s_waitcnt vmcnt(0), which would drain the next tile's prefetch and the output
// stores at every tile).  The asm's memory clobber keeps the compiler from moving LDS accesses across it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// acc += Σ over the kept plane products of a·b (a, b: P planes each)
template <int P>
__device__ __forceinline__ f32x4 mfma_planes(const bf16x8 (&a)[P], const bf16x8 (&b)[P], f32x4 acc) {
    if constexpr (P == 3) {
        acc = mfma(a[2], b[0], acc);
        acc = mfma(a[1], b[1], acc);
        acc = mfma(a[0], b[2], acc);
        acc = mfma(a[1], b[0], acc);
        acc = mfma(a[0], b[1], acc);
    }
    return mfma(a[0], b[0], acc);
}

// ------------------------------------------------------------------------------------------- weight planes
// wp[((ns * KK + kk) * P + p) * 64 + lane] = plane p of the MFMA fragment of lane `lane`:
//   B[n = 16 ns + (lane & 15)][k = 32 kk + 8 (lane >> 4) + e], e = 0..7,
// B[n][k] = kmajor ? w[k * ldw + n] : w[n * ldw + k].
__global__ void k_sgemm_wprep(int N, int K, const float* __restrict__ w, int64_t ldw, int kmajor, int P,
                              uint4* __restrict__ wp) {
    const int KK = K / 32;
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)(N / 16) * KK * 64) return;
    const int lane = (int)(idx & 63);
    const int64_t f = idx >> 6;
    const int kk = (int)(f % KK), ns = (int)(f / KK);
    const int n = ns * 16 + (lane & 15), k0 = kk * 32 + 8 * (lane >> 4);
    float x[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = kmajor ? w[(int64_t)(k0 + e) * ldw + n] : w[(int64_t)n * ldw + k0 + e];
    uint32_t pl[3][4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        uint32_t t[3];
        split2<3>(x[2 * e], x[2 * e + 1], t);
        pl[0][e] = t[0]; pl[1][e] = t[1]; pl[2][e] = t[2];
    }
    for (int p = 0; p < P; ++p)
        wp[((int64_t)(ns * KK + kk) * P + p) * 64 + lane] = make_uint4(pl[p][0], pl[p][1], pl[p][2], pl[p][3]);
}

// the four weight preparations of an attention block in one launch (blockIdx.y = job): the forward operands of
// the QKV and out projections and the transposed (k-major) operands of their input gradients
struct PrepJob {
    int N, K, kmajor;
    const float* w;
    int64_t ldw;
    uint4* wp;
};
struct PrepJobs {
    PrepJob j[4];
};
__global__ void k_sgemm_wprep4(PrepJobs J, int P) {
    const PrepJob& jb = J.j[blockIdx.y];
    const int KK = jb.K / 32;
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)(jb.N / 16) * KK * 64) return;
    const int lane = (int)(idx & 63);
    const int64_t f = idx >> 6;
    const int kk = (int)(f % KK), ns = (int)(f / KK);
    const int n = ns * 16 + (lane & 15), k0 = kk * 32 + 8 * (lane >> 4);
    float x[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = jb.kmajor ? jb.w[(int64_t)(k0 + e) * jb.ldw + n] : jb.w[(int64_t)n * jb.ldw + k0 + e];
    uint32_t pl[3][4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        uint32_t t[3];
        split2<3>(x[2 * e], x[2 * e + 1], t);
        pl[0][e] = t[0]; pl[1][e] = t[1]; pl[2][e] = t[2];
    }
    for (int p = 0; p < P; ++p)
        jb.wp[((int64_t)(ns * KK + kk) * P + p) * 64 + lane] = make_uint4(pl[p][0], pl[p][1], pl[p][2], pl[p][3]);
}

// ------------------------------------------------------------------------------------------- NT: C = A·Bᵀ
struct NtArgs {
    int64_t M;
    const void* a;           // [M, K] rows, row stride lda (fp32 or bf16)
    int64_t lda;
    const uint4* wp;         // k_sgemm_wprep planes of B [N, K]
    const float* bias;       // [N] or null
    void* c;                 // [M, N] rows, row stride ldc (fp32 or bf16)
    int64_t ldc;
    // MODE_LN_IN (K = H): a = x fp32 and the staged operand is h = LN(x) = (x - mean) rstd ln_g + ln_b; the row
    // statistics go to mean / rstd (the LayerNorm backward and the LN-recomputing weight gradient read them)
    const float* ln_g;
    const float* ln_b;
    float eps;
    float* mean;
    float* rstd;
    // MODE_LN_OUT (N = H): v = dropout(acc + bias) + res -> s_out; c = LN(v) (ln_g, ln_b, eps; statistics -> mean,
    // rstd) [+ LN_s(res) (gs, bs, eps_s; statistics -> mean_s, rstd_s)]
    // MODE_LN_BWD (N = H): acc = dh, the gradient of h = LN(x) (x = res, statistics mean / rstd as inputs, gamma =
    // ln_g); c = dx = rstd (g dh - mean(g dh x̂) x̂ - mean(g dh)) + dres; part[blockIdx.x][2H] = Σ dh x̂ | Σ dh
    const float* res;
    int64_t ldr;
    float p_drop, inv_keep;
    uint64_t seed;
    const uint64_t* seed_ctr;
    float* s_out;
    const float* gs;
    const float* bs;
    float eps_s;
    float* mean_s;
    float* rstd_s;
    const float* dres;
    float* part;
    // split-K: B's fragments are k-blocks [kk0, kk0 + K / 32) of a panel prepared with kkt k-blocks per n-subtile
    // (kkt = 0: K / 32); MODE_ACC adds the product to the fp32 C already there
    int kkt, kk0;
};

// MODE_ACC: MODE_PLAIN whose epilogue adds C's old value (the second half of a split-K product; a separate
// instantiation: a runtime "add the old C" branch beside the output stores made the plain kernels wait for every
// outstanding load before each store)
enum { MODE_PLAIN = 0, MODE_LN_IN = 1, MODE_LN_OUT = 2, MODE_LN_BWD = 3, MODE_ACC = 4 };


// h = LN(x) element: one expression shared by the prologue and the weight gradient's recompute (bitwise equal)
__device__ __forceinline__ float ln_apply(float x, float m, float rs, float g, float b) {
    return __builtin_fmaf((x - m) * rs, g, b);
}

// sums over aligned lane groups (DPP / permlane swaps, common.cuh: no LDS round trips)
template <int G>
__device__ __forceinline__ float xsum(float x) { return lane_sum<G>(x); }
// sum over the four 16-lane groups of a wave (lanes l, l ^ 16, l ^ 32, l ^ 48: same MFMA output row)
__device__ __forceinline__ float gsum4(float x) { return rows_sum(x); }

// Workgroup: NW waves; wave w owns columns [16 NSUB (NW blockIdx.y + w), +16 NSUB) and keeps their B planes
// (NSUB x K/32 x P fragments) in registers.  A tile = BM rows x K; thread chunk = 8 consecutive k of one row.
// LDS image of a tile (per buffer): entry ((p * KK + kk) * J + j) * 64 + slot holds plane p of the B-operand
// fragment of rows 16 j + (slot & 15), k = 32 kk + 8 (slot >> 4) + [0, 8) — one conflict-free ds_read_b128 per
// (kk, j, plane) and wave.
//
// MODE_LN_IN maps a tile chunk to (row = c / 16, q = c % 16): the 16 lanes of a DPP row hold one whole row of x, so
// its LayerNorm statistics are two butterflies in registers (two-pass, like k_ln_fwd).  Those lanes would all hit
// the same LDS banks in the fragment image, so every mode stores slot (row r, k-group t) of a 64-entry block at
// 16 t + (r ^ (t + 4 (kk & 3))): a permutation inside each 16-lane group, conflict-free for both chunk maps.
// MODE_LN_OUT / MODE_LN_BWD need whole output rows: each wave reduces its 16 NSUB columns of a row (two-pass mean
// and M2 for the forward, plain sums for the backward), the NW wave partials meet in LDS behind one barrier per
// tile, and the forward merges them with Chan's pairwise formula (no E[x²] - E[x]² cancellation).
template <int K, int NSUB, int NW, int BM, int P, bool ABF, bool CBF, int MODE, int MINB>
__global__ void __launch_bounds__(NW * 64, MINB) k_sgemm_nt(NtArgs g) {
    constexpr int KK = K / 32, J = BM / 16, NT = NW * 64, QK = K / 8;
    constexpr int CPT = BM * QK / NT;
    static_assert(BM * QK % NT == 0, "tile chunks must divide over the workgroup");
    static_assert(!ABF || P == 1, "bf16 operands have one plane");
    static_assert(MODE != MODE_LN_IN || ((QK == 16 || QK == 32) && !ABF), "LN prologue: K = 128 or 256 fp32 rows");
    // LN_IN chunk map: QK consecutive lanes (one or two DPP rows) hold one whole row of x
    constexpr int LQ = MODE == MODE_LN_IN ? QK : 16;
    constexpr bool EPI = MODE == MODE_LN_OUT || MODE == MODE_LN_BWD;
    constexpr int BUF = P * KK * J * 64;
    extern __shared__ uint4 sg_lds[];
    float* red = reinterpret_cast<float*>(sg_lds + 2 * BUF);   // EPI: [BM][NW][4] wave partials of the rows
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int nsub0 = (blockIdx.y * NW + w) * NSUB;
    if constexpr (MODE == MODE_LN_OUT) {
        if (g.seed_ctr) g.seed ^= *g.seed_ctr * 0x9E3779B97F4A7C15ull;   // TAGAN_LIVE_SEED
    }
    // LN prologue: gamma | beta in LDS after the two tile buffers
    float* lgb = reinterpret_cast<float*>(sg_lds + 2 * BUF);
    if constexpr (MODE == MODE_LN_IN) {
        for (int i = threadIdx.x; i < 2 * K; i += NT) lgb[i] = i < K ? g.ln_g[i] : g.ln_b[i - K];
        __syncthreads();
    }
    // epilogues: the LayerNorm parameters in LDS after the row partials: [4][HN] = gamma | beta | gamma_s | beta_s
    // (this lane's columns: 16 (nsub0 + s) + 4 (lane >> 4) + [0, 4))
    constexpr int HNE = NW * NSUB * 16;
    const f32x4* eprm = reinterpret_cast<const f32x4*>(red + BM * NW * 4);
    f32x4 dgacc[MODE == MODE_LN_BWD ? NSUB : 1], dbacc[MODE == MODE_LN_BWD ? NSUB : 1];
    if constexpr (EPI) {
        float* ep = red + BM * NW * 4;
        for (int i = threadIdx.x; i < 4 * HNE; i += NT) {
            const int q = i / HNE, c = i % HNE;
            const float* src = q == 0 ? g.ln_g : q == 1 ? g.ln_b : q == 2 ? g.gs : g.bs;
            ep[i] = (src && (MODE == MODE_LN_OUT || q == 0)) ? src[c] : 0.f;
        }
        __syncthreads();
        if constexpr (MODE == MODE_LN_BWD) {
#pragma unroll
            for (int s = 0; s < NSUB; ++s) dgacc[s] = dbacc[s] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
    }
    auto eprm_at = [&](int q, int s) { return eprm[(q * HNE + (nsub0 + s) * 16 + 4 * (lane >> 4)) / 4]; };

    bf16x8 wr[NSUB][KK][P];
#pragma unroll
    for (int s = 0; s < NSUB; ++s)
#pragma unroll
        for (int kk = 0; kk < KK; ++kk)
#pragma unroll
            for (int p = 0; p < P; ++p)
                wr[s][kk][p] = __builtin_bit_cast(
                    bf16x8, g.wp[((int64_t)((nsub0 + s) * (g.kkt ? g.kkt : KK) + g.kk0 + kk) * P + p) * 64 + lane]);
    f32x4 bias[NSUB];
#pragma unroll
    for (int s = 0; s < NSUB; ++s) {
        bias[s] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (g.bias) bias[s] = *reinterpret_cast<const f32x4*>(g.bias + (nsub0 + s) * 16 + 4 * (lane >> 4));
    }

    const int64_t ntiles = (g.M + BM - 1) / BM;
    int64_t tile = blockIdx.x;
    if (tile >= ntiles) return;   // uniform over the workgroup (the host launches at most ntiles workgroups)

    // ---- staging: global -> registers (pf) -> planes in LDS.  A lane loads one whole 8-k chunk (32 B) per piece;
    // the 64 lanes of an instruction spread over 16 rows.  (A whole-row map -- 1 KB of contiguous lines per
    // instruction, fp32 float4 pieces stored as half slots -- measured slower in the step: C2 fp32 6.84 vs 6.79 ms,
    // dC 71 vs 67 us, profiles/r4i_*; the A tile is mostly cache-resident there, written by the kernel before.)
    float pf[ABF ? 1 : CPT][8];
    uint4 pb[ABF ? CPT : 1];
    auto load = [&](int64_t t) {
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
            const int c = i * NT + threadIdx.x;
            const int rl = MODE == MODE_LN_IN ? (c / LQ) & 15 : c & 15;
            const int q = MODE == MODE_LN_IN ? c % LQ : (c >> 4) % QK;
            const int rh = MODE == MODE_LN_IN ? c / (16 * LQ) : (c >> 4) / QK;
            // rows past M reload row M - 1: they only feed output rows that are never stored, and an unconditional
            // load needs no zero-filled destination (a conditional one made the compiler drain every store of the
            // previous tile -- s_waitcnt vmcnt(0) -- before this prefetch could issue)
            const int64_t row0 = t * BM + rh * 16 + rl;
            const int64_t row = row0 < g.M ? row0 : g.M - 1;
            if constexpr (ABF) {
                pb[i] = *reinterpret_cast<const uint4*>((const uint16_t*)g.a + row * g.lda + 8 * q);
            } else {
                float4 v0, v1;
                {
                    const float* src = (const float*)g.a + row * g.lda + 8 * q;
                    v0 = *reinterpret_cast<const float4*>(src);
                    v1 = *reinterpret_cast<const float4*>(src + 4);
                }
                pf[i][0] = v0.x; pf[i][1] = v0.y; pf[i][2] = v0.z; pf[i][3] = v0.w;
                pf[i][4] = v1.x; pf[i][5] = v1.y; pf[i][6] = v1.z; pf[i][7] = v1.w;
            }
        }
    };
    auto stash = [&](uint4* buf, int64_t t) {
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
            const int c = i * NT + threadIdx.x;
            const int rl = MODE == MODE_LN_IN ? (c / LQ) & 15 : c & 15;
            const int q = MODE == MODE_LN_IN ? c % LQ : (c >> 4) % QK;
            const int rh = MODE == MODE_LN_IN ? c / (16 * LQ) : (c >> 4) / QK;
            const int e0 = ((q >> 2) * J + rh) * 64 + 16 * (q & 3) + (rl ^ ((q & 3) + 4 * ((q >> 2) & 3)));
            if constexpr (MODE == MODE_LN_IN) {   // the LQ lanes of one or two DPP rows hold the whole row
                float sm = (pf[i][0] + pf[i][1]) + (pf[i][2] + pf[i][3]) + ((pf[i][4] + pf[i][5]) + (pf[i][6] + pf[i][7]));
                const float mean = xsum<LQ>(sm) / (float)K;
                float sq = 0.f;
#pragma unroll
                for (int e = 0; e < 8; ++e) sq += (pf[i][e] - mean) * (pf[i][e] - mean);
                const float rstd = 1.f / sqrtf(xsum<LQ>(sq) / (float)K + g.eps);
#pragma unroll
                for (int e = 0; e < 8; ++e) pf[i][e] = ln_apply(pf[i][e], mean, rstd, lgb[8 * q + e], lgb[K + 8 * q + e]);
                const int64_t row = t * BM + rh * 16 + rl;
                if (q == 0 && row < g.M) {
                    g.mean[row] = mean;
                    g.rstd[row] = rstd;
                }
            }
            if constexpr (ABF) {
                buf[e0] = pb[i];
            } else {
                uint32_t pl[4][P];
#pragma unroll
                for (int e = 0; e < 4; ++e) split2<P>(pf[i][2 * e], pf[i][2 * e + 1], pl[e]);
#pragma unroll
                for (int p = 0; p < P; ++p)
                    buf[p * KK * J * 64 + e0] = make_uint4(pl[0][p], pl[1][p], pl[2][p], pl[3][p]);
            }
        }
    };

    // fragment slot of this lane in a 64-entry block of k-block kk (the swizzle of stash)
    int rslot[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) rslot[u] = 16 * (lane >> 4) + ((lane & 15) ^ ((lane >> 4) + 4 * u));

    load(tile);
    stash(sg_lds, tile);
    // the prefetch is unconditional (the last tile re-stages itself into the idle buffer): with a conditional one
    // the compiler could not prove the loads drained at the back edge and waited for every store of the tile
    // (s_waitcnt vmcnt(0)) before the next prefetch could issue
    __syncthreads();
    for (int it = 0;; ++it) {
        const int64_t next = tile + gridDim.x;
        const int64_t pre = next < ntiles ? next : tile;
        load(pre);
        __builtin_amdgcn_sched_barrier(0);
        // epilogue operands of this tile (in flight under the MFMAs): the residual rows (LN_OUT: res, LN_BWD: the LN
        // input x and dres) and the LN_BWD row statistics
        f32x4 er[EPI ? J : 1][EPI ? NSUB : 1], ed[MODE == MODE_LN_BWD ? J : 1][MODE == MODE_LN_BWD ? NSUB : 1];
        float em[MODE == MODE_LN_BWD ? J : 1], es[MODE == MODE_LN_BWD ? J : 1];
        if constexpr (EPI) {
#pragma unroll
            for (int j = 0; j < J; ++j) {
                const int64_t row = tile * BM + j * 16 + (lane & 15);
                const int64_t r = row < g.M ? row : g.M - 1;
#pragma unroll
                for (int s = 0; s < NSUB; ++s) {
                    const int col = (nsub0 + s) * 16 + 4 * (lane >> 4);
                    er[j][s] = *reinterpret_cast<const f32x4*>(g.res + r * g.ldr + col);
                }
                if constexpr (MODE == MODE_LN_BWD) {
                    em[j] = g.mean[r];
                    es[j] = g.rstd[r];
                }
            }
        }
        const uint4* buf = sg_lds + (it & 1) * BUF;
        f32x4 acc[J][NSUB];
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
            for (int s = 0; s < NSUB; ++s) acc[j][s] = bias[s];
        if constexpr (P == 1) {
            // one plane: a fragment feeds only NSUB MFMAs, so the fragments of k-block kk + 1 are read while kk's
            // MFMAs run (otherwise every read's LDS latency sits in front of its 1-3 MFMAs)
            bf16x8 af[2][J];
#pragma unroll
            for (int j = 0; j < J; ++j) af[0][j] = __builtin_bit_cast(bf16x8, buf[j * 64 + rslot[0]]);
#pragma unroll
            for (int kk = 0; kk < KK; ++kk) {
                if (kk + 1 < KK) {
#pragma unroll
                    for (int j = 0; j < J; ++j)
                        af[(kk + 1) & 1][j] = __builtin_bit_cast(bf16x8, buf[((kk + 1) * J + j) * 64 + rslot[(kk + 1) & 3]]);
                }
                __builtin_amdgcn_sched_barrier(0);   // keep the reads ahead of the MFMAs (the scheduler sinks them)
#pragma unroll
                for (int j = 0; j < J; ++j)
#pragma unroll
                    for (int s = 0; s < NSUB; ++s) acc[j][s] = mfma(wr[s][kk][0], af[kk & 1][j], acc[j][s]);
            }
        } else {
#pragma unroll
            for (int kk = 0; kk < KK; ++kk) {
#pragma unroll
                for (int j = 0; j < J; ++j) {
                    bf16x8 a[P];
#pragma unroll
                    for (int p = 0; p < P; ++p)
                        a[p] = __builtin_bit_cast(bf16x8, buf[((p * KK + kk) * J + j) * 64 + rslot[kk & 3]]);
#pragma unroll
                    for (int s = 0; s < NSUB; ++s) acc[j][s] = mfma_planes<P>(wr[s][kk], a, acc[j][s]);
                }
            }
        }
        // stage the next tile first: its loads were issued before this tile's MFMAs, and waiting for them after
        // the output stores would wait for the stores too.  Scheduling barriers pin the order prefetch -> MFMAs ->
        // stash: otherwise the scheduler sinks the prefetch loads to their use or hoists the stash (it writes the
        // other LDS buffer) above the MFMAs, and either way the loads no longer overlap the matrix work; the empty
        // asm statements keep the IR passes from moving the plane split of the prefetched values up to the loads
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
            for (int s = 0; s < NSUB; ++s) asm volatile("" : "+v"(acc[j][s]));
        if constexpr (ABF) {
#pragma unroll
            for (int i = 0; i < CPT; ++i) asm volatile("" : "+v"(pb[i].x), "+v"(pb[i].y), "+v"(pb[i].z), "+v"(pb[i].w));
        } else {
#pragma unroll
            for (int i = 0; i < CPT; ++i)
#pragma unroll
                for (int e = 0; e < 8; ++e) asm volatile("" : "+v"(pf[i][e]));
        }
        stash(sg_lds + ((it + 1) & 1) * BUF, pre);
        if constexpr (EPI) {
            if constexpr (MODE == MODE_LN_BWD) {   // dres is read in pass 2 only: its loads fly under pass 1
#pragma unroll
                for (int j = 0; j < J; ++j) {
                    const int64_t row = tile * BM + j * 16 + (lane & 15);
                    const int64_t r = row < g.M ? row : g.M - 1;
#pragma unroll
                    for (int s = 0; s < NSUB; ++s)
                        ed[j][s] = g.dres ? *reinterpret_cast<const f32x4*>(g.dres + r * g.ldc + (nsub0 + s) * 16 +
                                                                            4 * (lane >> 4))
                                          : f32x4{0.f, 0.f, 0.f, 0.f};
                }
            }
            constexpr int HN = NW * NSUB * 16;      // the whole row (gridDim.y == 1 in the LN modes)
            constexpr float WC = (float)(NSUB * 16);
            float v[MODE == MODE_LN_OUT ? J : 1][NSUB][4];
            // pass 1: this wave's share of every row -> red[row][w]
#pragma unroll
            for (int j = 0; j < J; ++j) {
                const int64_t row = tile * BM + j * 16 + (lane & 15);
                const bool live = row < g.M;
                float p0 = 0.f, p1 = 0.f, p2 = 0.f, p3 = 0.f;
                if constexpr (MODE == MODE_LN_OUT) {
                    const uint32_t key = drop_key(g.seed, (uint64_t)row);
#pragma unroll
                    for (int s = 0; s < NSUB; ++s) {
                        const int col = (nsub0 + s) * 16 + 4 * (lane >> 4);
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            float x = acc[j][s][e];
                            if (g.p_drop > 0.f) x = drop_u(key, (uint32_t)(col + e)) >= g.p_drop ? x * g.inv_keep : 0.f;
                            x += er[j][s][e];
                            v[j][s][e] = x;
                            p0 += x;
                            p2 += er[j][s][e];
                        }
                        if (live) *reinterpret_cast<f32x4*>(g.s_out + row * g.ldc + col) =
                                      f32x4{v[j][s][0], v[j][s][1], v[j][s][2], v[j][s][3]};
                    }
                    const float mw = gsum4(p0) / WC, ms = gsum4(p2) / WC;
#pragma unroll
                    for (int s = 0; s < NSUB; ++s)
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            p1 += (v[j][s][e] - mw) * (v[j][s][e] - mw);
                            p3 += (er[j][s][e] - ms) * (er[j][s][e] - ms);
                        }
                    p0 = mw; p1 = gsum4(p1); p2 = ms; p3 = gsum4(p3);
                } else {
                    const float m = em[j], rs = es[j];
#pragma unroll
                    for (int s = 0; s < NSUB; ++s)
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const float d = acc[j][s][e];
                            const float xv = (er[j][s][e] - m) * rs, gd = d * eprm_at(0, s)[e];
                            p0 += gd * xv;
                            p1 += gd;
                            if (live) {
                                dgacc[s][e] += d * xv;
                                dbacc[s][e] += d;
                            }
                        }
                    p0 = gsum4(p0); p1 = gsum4(p1);
                }
                if ((lane >> 4) == 0) {
                    float* rp = red + ((j * 16 + (lane & 15)) * NW + w) * 4;
                    rp[0] = p0; rp[1] = p1; rp[2] = p2; rp[3] = p3;
                }
            }
            lds_barrier();
            // pass 2: whole-row statistics, outputs
#pragma unroll
            for (int j = 0; j < J; ++j) {
                const int64_t row = tile * BM + j * 16 + (lane & 15);
                const bool live = row < g.M;
                const float* rp = red + (j * 16 + (lane & 15)) * NW * 4;
                if constexpr (MODE == MODE_LN_OUT) {
                    float mean = 0.f, means = 0.f;
#pragma unroll
                    for (int ww = 0; ww < NW; ++ww) { mean += rp[ww * 4]; means += rp[ww * 4 + 2]; }
                    mean /= (float)NW;
                    means /= (float)NW;
                    float m2 = 0.f, m2s = 0.f;
#pragma unroll
                    for (int ww = 0; ww < NW; ++ww) {
                        const float d = rp[ww * 4] - mean, ds = rp[ww * 4 + 2] - means;
                        m2 += rp[ww * 4 + 1] + WC * d * d;
                        m2s += rp[ww * 4 + 3] + WC * ds * ds;
                    }
                    const float rstd = 1.f / sqrtf(m2 / (float)HN + g.eps);
                    const float rstds = 1.f / sqrtf(m2s / (float)HN + g.eps_s);
                    if (!live) continue;
#pragma unroll
                    for (int s = 0; s < NSUB; ++s) {
                        const int col = (nsub0 + s) * 16 + 4 * (lane >> 4);
                        f32x4 y;
                        const f32x4 eg = eprm_at(0, s), eb = eprm_at(1, s);
#pragma unroll
                        for (int e = 0; e < 4; ++e) y[e] = (v[j][s][e] - mean) * rstd * eg[e] + eb[e];
                        if (g.gs) {
                            const f32x4 egs = eprm_at(2, s), ebs = eprm_at(3, s);
#pragma unroll
                            for (int e = 0; e < 4; ++e) y[e] += (er[j][s][e] - means) * rstds * egs[e] + ebs[e];
                        }
                        *reinterpret_cast<f32x4*>((float*)g.c + row * g.ldc + col) = y;
                    }
                    if ((lane >> 4) == 0 && w == 0) {
                        g.mean[row] = mean;
                        g.rstd[row] = rstd;
                        if (g.gs) {
                            g.mean_s[row] = means;
                            g.rstd_s[row] = rstds;
                        }
                    }
                } else {
                    float c1 = 0.f, c2 = 0.f;
#pragma unroll
                    for (int ww = 0; ww < NW; ++ww) { c1 += rp[ww * 4]; c2 += rp[ww * 4 + 1]; }
                    c1 /= (float)HN;
                    c2 /= (float)HN;
                    if (!live) continue;
                    const float rs = es[j];
#pragma unroll
                    for (int s = 0; s < NSUB; ++s) {
                        const int col = (nsub0 + s) * 16 + 4 * (lane >> 4);
                        f32x4 dx;
                        const f32x4 eg = eprm_at(0, s);
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const float xv = (er[j][s][e] - em[j]) * rs, gd = acc[j][s][e] * eg[e];
                            dx[e] = rs * (gd - c1 * xv - c2) + ed[j][s][e];
                        }
                        *reinterpret_cast<f32x4*>((float*)g.c + row * g.ldc + col) = dx;
                    }
                }
            }
            if (next >= ntiles) break;
            lds_barrier();
            tile = next;
            continue;
        }
        // D[n][m] of the MFMA = C[m][n]: lane holds C[row 16 j + (lane & 15)][4 consecutive n]
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const int64_t row = tile * BM + j * 16 + (lane & 15);
            if (row < g.M) {
#pragma unroll
                for (int s = 0; s < NSUB; ++s) {
                    const int64_t off = row * g.ldc + (nsub0 + s) * 16 + 4 * (lane >> 4);
                    f32x4 v = acc[j][s];
                    if constexpr (MODE == MODE_ACC) v += *reinterpret_cast<const f32x4*>((const float*)g.c + off);
                    if constexpr (CBF) {
                        *reinterpret_cast<uint2*>((uint16_t*)g.c + off) = make_uint2(pk_bf16(v[0], v[1]),
                                                                                     pk_bf16(v[2], v[3]));
                    } else {
                        *reinterpret_cast<f32x4*>((float*)g.c + off) = v;
                    }
                }
            }
        }
        if (next >= ntiles) break;
        lds_barrier();
        tile = next;
    }
    if constexpr (MODE == MODE_LN_BWD) {
        // Σ over this workgroup's rows of dh x̂ and dh for the lane's columns: lanes l ^ 1..8 share them
#pragma unroll
        for (int s = 0; s < NSUB; ++s)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float a = xsum<16>(dgacc[s][e]), b = xsum<16>(dbacc[s][e]);
                if ((lane & 15) == 0) {
                    const int col = (nsub0 + s) * 16 + 4 * (lane >> 4) + e;
                    g.part[(int64_t)blockIdx.x * 2 * NW * NSUB * 16 * gridDim.y + col] = a;
                    g.part[(int64_t)blockIdx.x * 2 * NW * NSUB * 16 * gridDim.y + NW * NSUB * 16 * gridDim.y + col] = b;
                }
            }
    }
}

// ------------------------------------------------------------------------------------------- ping-pong NT
#ifndef TAGAN_SG_PF
#define TAGAN_SG_PF 0
#endif
// k_sgemm_nt's plain / split-K / LN-prologue forms with the two waves of each SIMD half a period apart (round 6).  In
// k_sgemm_nt all eight waves run the MFMAs of a tile together and then all stage the next one together, so each
// SIMD's matrix pipe idles through every staging phase (PMC: 3-4 % of MFMA-busy cycles co-executing VALU, round 5).
// Here waves 0-3 (group 0) and 4-7 (group 1; wave w runs on SIMD w % 4, so each SIMD holds one of each) alternate:
//   phase X: group 0 runs tile t's MFMAs; group 1 stages its half (rows 16 J/2 ..) of tile t + 1 into the other
//            buffer from the registers its loads filled a period ago, issues the loads of its half of tile t + 2 and
//            stores its outputs of tile t - 1;
//   phase Y: the same with the groups swapped (group 0 stores tile t's outputs).
// One barrier between the phases and one per period; a buffer is read in X and Y of its period and rewritten only in
// the next period, so two buffers suffice.  Each wave still owns 16 NSUB output columns (weights in registers) and
// stages half a tile per period, i.e. as many chunks per thread as in k_sgemm_nt: no extra registers.
template <int K, int NSUB, int BM, int P, bool ABF, bool CBF, int MODE>
__global__ void __launch_bounds__(512, 1) k_sgemm_nt_pp(NtArgs g) {
    constexpr int NW = 8, KK = K / 32, J = BM / 16, JH = J / 2, QK = K / 8, GT = 256;
    constexpr int CPT = (BM / 2) * QK / GT;
    static_assert(J % 2 == 0 && (BM / 2) * QK % GT == 0, "each group stages whole 16-row blocks");
    static_assert(MODE == MODE_PLAIN || MODE == MODE_ACC || MODE == MODE_LN_IN, "no row-wide epilogues here");
    static_assert(!ABF || P == 1, "bf16 operands have one plane");
    static_assert(MODE != MODE_LN_IN || ((QK == 16 || QK == 32) && !ABF), "LN prologue: K = 128 or 256 fp32 rows");
    constexpr int LQ = MODE == MODE_LN_IN ? QK : 16;
    constexpr int BUF = P * KK * J * 64;
    extern __shared__ uint4 sg_lds[];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, grp = w >> 2, gtid = threadIdx.x & (GT - 1);
    const int nsub0 = (blockIdx.y * NW + w) * NSUB;
    float* lgb = reinterpret_cast<float*>(sg_lds + 2 * BUF);
    if constexpr (MODE == MODE_LN_IN)
        for (int i = threadIdx.x; i < 2 * K; i += NW * 64) lgb[i] = i < K ? g.ln_g[i] : g.ln_b[i - K];
    bf16x8 wr[NSUB][KK][P];
#pragma unroll
    for (int s = 0; s < NSUB; ++s)
#pragma unroll
        for (int kk = 0; kk < KK; ++kk)
#pragma unroll
            for (int p = 0; p < P; ++p)
                wr[s][kk][p] = __builtin_bit_cast(
                    bf16x8, g.wp[((int64_t)((nsub0 + s) * (g.kkt ? g.kkt : KK) + g.kk0 + kk) * P + p) * 64 + lane]);
    if constexpr (MODE == MODE_LN_IN) __syncthreads();
    f32x4 bias[NSUB];
#pragma unroll
    for (int s = 0; s < NSUB; ++s) {
        bias[s] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (g.bias) bias[s] = *reinterpret_cast<const f32x4*>(g.bias + (nsub0 + s) * 16 + 4 * (lane >> 4));
    }
    const int64_t ntiles = (g.M + BM - 1) / BM;
    int64_t tile = blockIdx.x;
    if (tile >= ntiles) return;   // uniform over the workgroup

    // this thread's staging chunks: rows of its group's half of the tile (k_sgemm_nt's maps within the half)
    auto chunk = [&](int i, int& rl, int& q, int& rh) {
        const int c = i * GT + gtid;
        rl = MODE == MODE_LN_IN ? (c / LQ) & 15 : c & 15;
        q = MODE == MODE_LN_IN ? c % LQ : (c >> 4) % QK;
        rh = grp * JH + (MODE == MODE_LN_IN ? c / (16 * LQ) : (c >> 4) / QK);
    };
    float pf[ABF ? 1 : CPT][8];
    uint4 pb[ABF ? CPT : 1];
    auto load = [&](int64_t t) {
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
            int rl, q, rh;
            chunk(i, rl, q, rh);
            const int64_t row0 = t * BM + rh * 16 + rl;
            const int64_t row = row0 < g.M ? row0 : g.M - 1;   // rows past M reload row M - 1 (never stored)
            if constexpr (ABF) {
                pb[i] = *reinterpret_cast<const uint4*>((const uint16_t*)g.a + row * g.lda + 8 * q);
            } else {
                const float* src = (const float*)g.a + row * g.lda + 8 * q;
                const float4 v0 = *reinterpret_cast<const float4*>(src);
                const float4 v1 = *reinterpret_cast<const float4*>(src + 4);
                pf[i][0] = v0.x; pf[i][1] = v0.y; pf[i][2] = v0.z; pf[i][3] = v0.w;
                pf[i][4] = v1.x; pf[i][5] = v1.y; pf[i][6] = v1.z; pf[i][7] = v1.w;
            }
        }
    };
    auto stash = [&](uint4* buf, int64_t t) {
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
            int rl, q, rh;
            chunk(i, rl, q, rh);
            const int e0 = ((q >> 2) * J + rh) * 64 + 16 * (q & 3) + (rl ^ ((q & 3) + 4 * ((q >> 2) & 3)));
            if constexpr (MODE == MODE_LN_IN) {
                const float sm = (pf[i][0] + pf[i][1]) + (pf[i][2] + pf[i][3]) + ((pf[i][4] + pf[i][5]) + (pf[i][6] + pf[i][7]));
                const float mean = xsum<LQ>(sm) / (float)K;
                float sq = 0.f;
#pragma unroll
                for (int e = 0; e < 8; ++e) sq += (pf[i][e] - mean) * (pf[i][e] - mean);
                const float rstd = 1.f / sqrtf(xsum<LQ>(sq) / (float)K + g.eps);
#pragma unroll
                for (int e = 0; e < 8; ++e) pf[i][e] = ln_apply(pf[i][e], mean, rstd, lgb[8 * q + e], lgb[K + 8 * q + e]);
                const int64_t row = t * BM + rh * 16 + rl;
                if (q == 0 && row < g.M) {
                    g.mean[row] = mean;
                    g.rstd[row] = rstd;
                }
            }
            if constexpr (ABF) {
                buf[e0] = pb[i];
            } else {
                uint32_t pl[4][P];
#pragma unroll
                for (int e = 0; e < 4; ++e) split2<P>(pf[i][2 * e], pf[i][2 * e + 1], pl[e]);
#pragma unroll
                for (int p = 0; p < P; ++p)
                    buf[p * KK * J * 64 + e0] = make_uint4(pl[0][p], pl[1][p], pl[2][p], pl[3][p]);
            }
        }
    };
    int rslot[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) rslot[u] = 16 * (lane >> 4) + ((lane & 15) ^ ((lane >> 4) + 4 * u));
    f32x4 acc[J][NSUB];
    auto compute = [&](const uint4* buf) {
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
            for (int s = 0; s < NSUB; ++s) acc[j][s] = bias[s];
        if constexpr (P == 1) {
            bf16x8 af[2][J];
#pragma unroll
            for (int j = 0; j < J; ++j) af[0][j] = __builtin_bit_cast(bf16x8, buf[j * 64 + rslot[0]]);
#pragma unroll
            for (int kk = 0; kk < KK; ++kk) {
                if (kk + 1 < KK) {
#pragma unroll
                    for (int j = 0; j < J; ++j)
                        af[(kk + 1) & 1][j] = __builtin_bit_cast(bf16x8, buf[((kk + 1) * J + j) * 64 + rslot[(kk + 1) & 3]]);
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int j = 0; j < J; ++j)
#pragma unroll
                    for (int s = 0; s < NSUB; ++s) acc[j][s] = mfma(wr[s][kk][0], af[kk & 1][j], acc[j][s]);
            }
        } else {
#pragma unroll
            for (int kk = 0; kk < KK; ++kk) {
#pragma unroll
                for (int j = 0; j < J; ++j) {
                    bf16x8 a[P];
#pragma unroll
                    for (int p = 0; p < P; ++p)
                        a[p] = __builtin_bit_cast(bf16x8, buf[((p * KK + kk) * J + j) * 64 + rslot[kk & 3]]);
#pragma unroll
                    for (int s = 0; s < NSUB; ++s) acc[j][s] = mfma_planes<P>(wr[s][kk], a, acc[j][s]);
                }
            }
        }
    };
    // outputs through a buffer resource over the tile's valid rows: rows past M are dropped by the range check, so
    // the stores are unconditional instructions and the staging phase's wait for its loads counts them exactly (a
    // row < M branch made the compiler wait for every store too: s_waitcnt vmcnt(0)).  store(-1) issues the same
    // instructions over an empty range: the prologue and group 1's first period end with it, so every path into a
    // staging phase has the same number of stores behind its loads (else the merged count is vmcnt(0) again).
    auto store = [&](int64_t t) {
        constexpr int ES = CBF ? 2 : 4;
        const int64_t r0 = t < 0 ? 0 : t * BM;
        const int64_t nv = t < 0 ? 0 : g.M - r0 < BM ? g.M - r0 : BM;   // t < 0: a phantom batch (all dropped)
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (char*)g.c + r0 * g.ldc * ES, (short)0, (int)(nv * g.ldc * ES), 0x00020000);
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
            for (int s = 0; s < NSUB; ++s) {
                const int off = (int)(((j * 16 + (lane & 15)) * g.ldc + (nsub0 + s) * 16 + 4 * (lane >> 4)) * ES);
                f32x4 v = acc[j][s];
                if constexpr (MODE == MODE_ACC)
                    v += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
                if constexpr (CBF) {
                    const uint2 pk = make_uint2(pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3]));
                    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, pk), rs, off, 0, 0);
                } else {
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, off, 0, 0);
                }
            }
    };
    // TAGAN_SG_PF: also pull tile nx2 + 1 (this group's half) into L2 one period early: one dword per 128-B line
    // into a sink register consumed a period later, so the loads of the next period hit L2
    float sink = 0.f;
    auto stage = [&](uint4* buf, int64_t nx, int64_t nx2, int64_t nx3) {
        __builtin_amdgcn_sched_barrier(0);
        stash(buf, nx);
        load(nx2);
        if constexpr (TAGAN_SG_PF) {
            asm volatile("" ::"v"(sink));
            constexpr int LPR = K * (ABF ? 2 : 4) / 128;          // 128-B lines per row
            constexpr int LINES = (BM / 2) * LPR;                 // lines of the group's half tile
            if (gtid < LINES) {
                const int64_t row0 = nx3 * BM + grp * (BM / 2) + gtid / LPR;
                const int64_t row = row0 < g.M ? row0 : g.M - 1;
                sink = *(reinterpret_cast<const volatile float*>(
                    (const char*)g.a + (row * g.lda) * (ABF ? 2 : 4) + (gtid % LPR) * 128));
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    };

    load(tile);
    stash(sg_lds, tile);
    {
        const int64_t n1 = tile + gridDim.x;
        load(n1 < ntiles ? n1 : tile);
        store(-1);
    }
    __syncthreads();
    // Each group runs its own copy of the period loop (straight-line phases, the same barriers in the same order): in
    // one loop with the phases in grp branches the compiler merged the staging registers at every join and drained
    // the fresh loads (s_waitcnt vmcnt(0)) at the end of each staging phase.
    // phase boundaries: the MFMAs must not drift across a barrier (they touch no memory, so the asm's clobber does
    // not hold them)
    auto pp_barrier = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        lds_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    if (grp == 0) {
        for (int it = 0;; ++it) {
            const int64_t next = tile + gridDim.x, next2 = next + gridDim.x, next3 = next2 + gridDim.x;
            const int64_t sx = next < ntiles ? next : tile;   // unconditional staging (see k_sgemm_nt)
            const int64_t lx = next2 < ntiles ? next2 : sx;
            const int64_t px = next3 < ntiles ? next3 : lx;
            compute(sg_lds + (it & 1) * BUF);                 // phase X
            pp_barrier();
            stage(sg_lds + ((it + 1) & 1) * BUF, sx, lx, px);  // phase Y
            store(tile);
            if (next >= ntiles) break;
            pp_barrier();
            tile = next;
        }
    } else {
        int64_t prev = -1;   // the tile whose outputs this group still holds
        for (int it = 0;; ++it) {
            const int64_t next = tile + gridDim.x, next2 = next + gridDim.x, next3 = next2 + gridDim.x;
            const int64_t sx = next < ntiles ? next : tile;
            const int64_t lx = next2 < ntiles ? next2 : sx;
            const int64_t px = next3 < ntiles ? next3 : lx;
            stage(sg_lds + ((it + 1) & 1) * BUF, sx, lx, px);  // phase X
            store(prev);
            pp_barrier();
            compute(sg_lds + (it & 1) * BUF);                 // phase Y
            prev = tile;
            if (next >= ntiles) break;
            pp_barrier();
            tile = next;
        }
        store(prev);
    }
}

// ------------------------------------------------------------------------------------------- row-owner NT (N = 128)
// For the N = H = 128 products (out-projection forward, its input gradient, the QKV input gradient) and their
// LayerNorm-fused forms: ONE WAVE OWNS WHOLE 16-ROW OUTPUT TILES.  B's bf16 planes sit in LDS (staged once per
// workgroup in k_sgemm_wprep's fragment order, read back with one conflict-free ds_read_b128 per fragment); each wave
// loads its A fragments straight from HBM into MFMA operand registers (lane (c, t): row c, k = 32 kk + 8 t + [0, 8):
// 32 or 16 contiguous bytes), splits them into planes in registers, and runs 8 n-subtiles x K/32 x (6 | 1) MFMAs.
// The finished row is then entirely inside the wave (lanes c, c ^ 16, c ^ 32, c ^ 48 hold 4 columns of each
// n-subtile), so a LayerNorm's row statistics are two shuffles: no LDS hand-off and no workgroup barrier in the tile
// loop -- the W waves of a CU run their tiles independently and overlap each other's memory and matrix phases (the
// weight-stationary k_sgemm_nt needs one barrier per tile for a row-wide epilogue and measured slower there).
//
// MODE_LN_IN (N = 3H = 384, one plane: the bf16 QKV projection): LN1 in the prologue -- the lane's 32 values of x
// (row c, k = 32 kk + 8 t + [0, 8)) and the other three lane groups hold the whole row, so its two-pass statistics
// are in-lane sums and two shuffles; h = ln_apply(x) exactly as k_sgemm_nt's prologue makes it.
template <int K, int P, bool ABF, bool CBF, int MODE, int W, int NN = 128>
__global__ void __launch_bounds__(W * 64) k_rowgemm(NtArgs g) {
    constexpr int N = NN, NS = N / 16, KK = K / 32;
    static_assert(MODE != MODE_LN_IN || (!ABF && K == 128), "LN prologue: fp32 rows of K = 128");
    static_assert(MODE == MODE_LN_IN || N == 128 || (MODE == MODE_LN_OUT && N == 256 && P == 1),
                  "row-wide epilogues: N = 128 (LN2 epilogue: also N = 256 with one plane)");
    constexpr int NB = NS * KK * P * 64;             // B fragments (uint4) in LDS
    static_assert(!ABF || P == 1, "bf16 operands have one plane");
    extern __shared__ uint4 sg_lds[];
    float* prm = reinterpret_cast<float*>(sg_lds + NB);   // [5][N]: gamma | beta | gamma_s | beta_s | bias
    float* wred = prm + 5 * N;                            // LN_BWD: [W][2N] wave partials of dgamma | dbeta
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = lane & 15, gq = lane >> 4;
    for (int i = threadIdx.x; i < NB; i += W * 64) sg_lds[i] = g.wp[i];
    for (int i = threadIdx.x; i < 5 * N; i += W * 64) {
        const int q = i / N, col = i % N;
        const float* src = q == 0 ? g.ln_g : q == 1 ? g.ln_b : q == 2 ? g.gs : q == 3 ? g.bs : g.bias;
        const bool use = q == 4 || MODE == MODE_LN_OUT || (MODE == MODE_LN_BWD && q == 0) ||
                         (MODE == MODE_LN_IN && q < 2 && col < K);
        prm[i] = (src && use) ? src[col] : 0.f;
    }
    __syncthreads();
    if constexpr (MODE == MODE_LN_OUT) {
        if (g.seed_ctr) g.seed ^= *g.seed_ctr * 0x9E3779B97F4A7C15ull;   // TAGAN_LIVE_SEED
    }
    auto pv = [&](int q, int s) { return *reinterpret_cast<const f32x4*>(prm + q * N + 16 * s + 4 * gq); };
    f32x4 dgacc[MODE == MODE_LN_BWD ? NS : 1], dbacc[MODE == MODE_LN_BWD ? NS : 1];
    if constexpr (MODE == MODE_LN_BWD) {
#pragma unroll
        for (int s = 0; s < NS; ++s) dgacc[s] = dbacc[s] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const int64_t ntiles = (g.M + 15) / 16;
    for (int64_t t = (int64_t)blockIdx.x * W + w; t < ntiles; t += (int64_t)gridDim.x * W) {
        const int64_t row0 = t * 16 + c;
        const bool live = row0 < g.M;
        const int64_t row = live ? row0 : g.M - 1;   // dead rows recompute row M - 1 and store nothing
        // B's LDS reads are the same every tile: behind an opaque copy of the lane index the compiler cannot hoist
        // them out of the tile loop (it would hold every fragment in registers and spill)
        int lb = lane;
        asm volatile("" : "+v"(lb));
        uint4 ar[ABF ? KK : 1];
        float4 af[ABF ? 1 : KK][2];
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) {
            if constexpr (ABF) {
                ar[kk] = *reinterpret_cast<const uint4*>((const uint16_t*)g.a + row * g.lda + 32 * kk + 8 * gq);
            } else {
                const float* src = (const float*)g.a + row * g.lda + 32 * kk + 8 * gq;
                af[kk][0] = *reinterpret_cast<const float4*>(src);
                af[kk][1] = *reinterpret_cast<const float4*>(src + 4);
            }
        }
        // LN_OUT: the residual row is read with the A fragments (in flight under the MFMAs)
        f32x4 er[MODE == MODE_LN_OUT ? NS : 1];
        if constexpr (MODE == MODE_LN_OUT) {
#pragma unroll
            for (int s = 0; s < NS; ++s) er[s] = *reinterpret_cast<const f32x4*>(g.res + row * g.ldr + 16 * s + 4 * gq);
        }
        if constexpr (MODE == MODE_LN_IN) {   // h = LN1(x) in place
            float sm = 0.f;
#pragma unroll
            for (int kk = 0; kk < KK; ++kk)
                sm += (af[kk][0].x + af[kk][0].y) + (af[kk][0].z + af[kk][0].w) +
                      ((af[kk][1].x + af[kk][1].y) + (af[kk][1].z + af[kk][1].w));
            const float mean = gsum4(sm) / (float)K;
            float sq = 0.f;
#pragma unroll
            for (int kk = 0; kk < KK; ++kk)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const float4 v = af[kk][h];
                    sq += ((v.x - mean) * (v.x - mean) + (v.y - mean) * (v.y - mean)) +
                          ((v.z - mean) * (v.z - mean) + (v.w - mean) * (v.w - mean));
                }
            const float rstd = 1.f / sqrtf(gsum4(sq) / (float)K + g.eps);
#pragma unroll
            for (int kk = 0; kk < KK; ++kk)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int k0 = 32 * kk + 8 * gq + 4 * h;
                    float4& v = af[kk][h];
                    v.x = ln_apply(v.x, mean, rstd, prm[k0], prm[N + k0]);
                    v.y = ln_apply(v.y, mean, rstd, prm[k0 + 1], prm[N + k0 + 1]);
                    v.z = ln_apply(v.z, mean, rstd, prm[k0 + 2], prm[N + k0 + 2]);
                    v.w = ln_apply(v.w, mean, rstd, prm[k0 + 3], prm[N + k0 + 3]);
                }
            if (live && gq == 0) {
                g.mean[row] = mean;
                g.rstd[row] = rstd;
            }
        }
        f32x4 acc[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) acc[s] = pv(4, s);
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) {
            bf16x8 ap[P];
            if constexpr (ABF) {
                ap[0] = __builtin_bit_cast(bf16x8, ar[kk]);
            } else {
                uint32_t pl[4][P];
                split2<P>(af[kk][0].x, af[kk][0].y, pl[0]);
                split2<P>(af[kk][0].z, af[kk][0].w, pl[1]);
                split2<P>(af[kk][1].x, af[kk][1].y, pl[2]);
                split2<P>(af[kk][1].z, af[kk][1].w, pl[3]);
#pragma unroll
                for (int p = 0; p < P; ++p)
                    ap[p] = __builtin_bit_cast(bf16x8, make_uint4(pl[0][p], pl[1][p], pl[2][p], pl[3][p]));
            }
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                bf16x8 bp[P];
#pragma unroll
                for (int p = 0; p < P; ++p) bp[p] = __builtin_bit_cast(bf16x8, sg_lds[((s * KK + kk) * P + p) * 64 + lb]);
                acc[s] = mfma_planes<P>(bp, ap, acc[s]);
            }
        }
        // lane holds C[row][16 s + 4 gq + e], e = 0..3, for every n-subtile s
        if constexpr (MODE == MODE_PLAIN || MODE == MODE_LN_IN) {
            if (live) {
#pragma unroll
                for (int s = 0; s < NS; ++s) {
                    const int64_t off = row * g.ldc + 16 * s + 4 * gq;
                    if constexpr (CBF) {
                        *reinterpret_cast<uint2*>((uint16_t*)g.c + off) = make_uint2(pk_bf16(acc[s][0], acc[s][1]),
                                                                                     pk_bf16(acc[s][2], acc[s][3]));
                    } else {
                        *reinterpret_cast<f32x4*>((float*)g.c + off) = acc[s];
                    }
                }
            }
        } else if constexpr (MODE == MODE_LN_OUT) {
            const uint32_t key = drop_key(g.seed, (uint64_t)row0);
            float sm = 0.f, sr = 0.f;
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                const int col = 16 * s + 4 * gq;
                const f32x4 r = er[s];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float x = acc[s][e];
                    if (g.p_drop > 0.f) x = drop_u(key, (uint32_t)(col + e)) >= g.p_drop ? x * g.inv_keep : 0.f;
                    x += r[e];
                    acc[s][e] = x;
                    sm += x;
                    sr += r[e];
                }
                if (live) *reinterpret_cast<f32x4*>(g.s_out + row * g.ldc + col) = acc[s];
            }
            const float mean = gsum4(sm) / (float)N;
            float sq = 0.f;
#pragma unroll
            for (int s = 0; s < NS; ++s)
#pragma unroll
                for (int e = 0; e < 4; ++e) sq += (acc[s][e] - mean) * (acc[s][e] - mean);
            const float rstd = 1.f / sqrtf(gsum4(sq) / (float)N + g.eps);
            float means = 0.f, rstds = 0.f;
            if (g.gs) {   // skip branch: statistics of the residual rows (re-read: L1 / L2 hits)
                means = gsum4(sr) / (float)N;
                float sqs = 0.f;
#pragma unroll
                for (int s = 0; s < NS; ++s)
#pragma unroll
                    for (int e = 0; e < 4; ++e) sqs += (er[s][e] - means) * (er[s][e] - means);
                rstds = 1.f / sqrtf(gsum4(sqs) / (float)N + g.eps_s);
            }
            if (live) {
#pragma unroll
                for (int s = 0; s < NS; ++s) {
                    const int col = 16 * s + 4 * gq;
                    const f32x4 ga = pv(0, s), be = pv(1, s);
                    f32x4 y;
#pragma unroll
                    for (int e = 0; e < 4; ++e) y[e] = (acc[s][e] - mean) * rstd * ga[e] + be[e];
                    if (g.gs) {
                        const f32x4 gs = pv(2, s), bs = pv(3, s);
#pragma unroll
                        for (int e = 0; e < 4; ++e) y[e] += (er[s][e] - means) * rstds * gs[e] + bs[e];
                    }
                    *reinterpret_cast<f32x4*>((float*)g.c + row * g.ldc + col) = y;
                }
                if (gq == 0) {
                    g.mean[row] = mean;
                    g.rstd[row] = rstd;
                    if (g.gs) {
                        g.mean_s[row] = means;
                        g.rstd_s[row] = rstds;
                    }
                }
            }
        } else {   // MODE_LN_BWD: acc = dh
            const float m = g.mean[row], rs = g.rstd[row];
            float c1 = 0.f, c2 = 0.f;
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                const f32x4 x = *reinterpret_cast<const f32x4*>(g.res + row * g.ldr + 16 * s + 4 * gq);
                const f32x4 ga = pv(0, s);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float xv = (x[e] - m) * rs, gd = acc[s][e] * ga[e];
                    c1 += gd * xv;
                    c2 += gd;
                    if (live) {
                        dgacc[s][e] += acc[s][e] * xv;
                        dbacc[s][e] += acc[s][e];
                    }
                }
            }
            c1 = gsum4(c1) / (float)N;
            c2 = gsum4(c2) / (float)N;
            if (live) {
#pragma unroll
                for (int s = 0; s < NS; ++s) {
                    const int col = 16 * s + 4 * gq;
                    const f32x4 x = *reinterpret_cast<const f32x4*>(g.res + row * g.ldr + col);
                    const f32x4 d = g.dres ? *reinterpret_cast<const f32x4*>(g.dres + row * g.ldc + col)
                                           : f32x4{0.f, 0.f, 0.f, 0.f};
                    const f32x4 ga = pv(0, s);
                    f32x4 dx;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float xv = (x[e] - m) * rs, gd = acc[s][e] * ga[e];
                        dx[e] = rs * (gd - c1 * xv - c2) + d[e];
                    }
                    *reinterpret_cast<f32x4*>((float*)g.c + row * g.ldc + col) = dx;
                }
            }
        }
    }
    if constexpr (MODE == MODE_LN_BWD) {
        // Σ over the wave's rows (lanes c = 0..15 share the columns), the waves' sums in wave order -> one partial
        // row per workgroup (fixed order: bitwise reproducible)
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float a = xsum<16>(dgacc[s][e]), b = xsum<16>(dbacc[s][e]);
                if (c == 0) {
                    wred[w * 2 * N + 16 * s + 4 * gq + e] = a;
                    wred[w * 2 * N + N + 16 * s + 4 * gq + e] = b;
                }
            }
        __syncthreads();
        for (int i = threadIdx.x; i < 2 * N; i += W * 64) {
            float a = 0.f;
            for (int ww = 0; ww < W; ++ww) a += wred[ww * 2 * N + i];
            g.part[(int64_t)blockIdx.x * 2 * N + i] = a;
        }
    }
}

// ------------------------------------------------------------------------------------------- TN: dW = dYᵀ·X
#ifndef TAGAN_SG_TN_ILOAD
#define TAGAN_SG_TN_ILOAD 1
#endif
struct TnArgs {
    int64_t M;
    const void* dy;          // [M, N] rows, row stride ldy
    int64_t ldy;
    const void* x;           // [M, K] rows, row stride ldx
    int64_t ldx;
    int64_t tiles_per_wg;    // 32-row tiles per workgroup (contiguous range)
    float* part;             // [gridDim.x][N * K + N] partial dW | db
    // LNX: x is the fp32 LayerNorm input and the X operand is h = LN(x), recomputed from the forward's row
    // statistics exactly as the LN prologue of k_sgemm_nt made it (ln_apply)
    const float* ln_g;
    const float* ln_b;
    const float* mean;
    const float* rstd;
};

// One 32-row tile per step.  Workgroup (blockIdx.x, blockIdx.y): rows of m-group blockIdx.x, dY columns
// [NL blockIdx.y, NL (blockIdx.y + 1)), NL = N / NG (NG > 1 halves the LDS image so two workgroups share a CU and one
// stages while the other multiplies).  LDS: P planes of dY [32][NL + 16] and of X [32][K + 16] bf16 (row strides
// of an odd multiple of 8 dwords mod 64 banks).  MFMA reduction index = the tile row: element e of lane group g is row 4 g + (e & 3) + 16 (e >> 2)
// for BOTH operands (a permutation of the sum), so each ds_read_b64_tr_b16 of a 32-lane half covers 8 adjacent rows:
// conflict-free.  Wave w owns n-subtiles [NSN w, NSN (w + 1)) and all K / 16 k-subtiles; db comes from one more
// MFMA per plane against a fragment of ones.
template <int N, int K, int NSN, int NW, int NG, int P, bool ABF, int MINB, bool LNX>
__global__ void __launch_bounds__(NW * 64, MINB) k_sgemm_tn(TnArgs g) {
    constexpr int NL = N / NG;
    static_assert(NL == NW * NSN * 16, "waves must cover the workgroup's columns");
    static_assert(!ABF || P == 1, "bf16 operands have one plane");
    constexpr int NT = NW * 64, KS = K / 16;
    constexpr int SY = NL + 16, SX = K + 16;                // bf16 elements per LDS row
    constexpr int PY = 32 * SY, PX = 32 * SX;               // elements per plane
    constexpr int Q4 = 32 * (NL + K) / 4;                   // 4-element chunks per tile
    const int ncol0 = blockIdx.y * NL;
    constexpr int CPT = (Q4 + NT - 1) / NT;
    extern __shared__ uint4 sg_lds[];
    uint16_t* ly = reinterpret_cast<uint16_t*>(sg_lds);
    uint16_t* lx = ly + P * PY;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int grp = lane >> 4, li = lane & 15;

    f32x4 acc[NSN][KS], accb[NSN];
#pragma unroll
    for (int s = 0; s < NSN; ++s) {
        accb[s] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < KS; ++k) acc[s][k] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    bf16x8 ones;
#pragma unroll
    for (int e = 0; e < 8; ++e) ones[e] = (__bf16)1.0f;

    const int64_t t0 = (int64_t)blockIdx.x * g.tiles_per_wg;
    const int64_t t1 = min(t0 + g.tiles_per_wg, (g.M + 31) / 32);

    // LNX: an x chunk's 4 columns are fixed per thread (NT and the dY part of a tile are multiples of K / 4)
    static_assert(!LNX || (NT % (K / 4) == 0 && (8 * NL) % (K / 4) == 0), "LNX: thread-fixed x columns");
    float4 lng = make_float4(0.f, 0.f, 0.f, 0.f), lnb = lng;
    if constexpr (LNX) {
        const int col = 4 * (threadIdx.x % (K / 4));
        lng = *reinterpret_cast<const float4*>(g.ln_g + col);
        lnb = *reinterpret_cast<const float4*>(g.ln_b + col);
    }
    // LNX: chunks [0, CY) are dY's, [CY, CPT) X's (compile-time split)
    constexpr int CY = LNX ? 8 * NL / NT : 0, CX = LNX ? CPT - CY : 1;
    static_assert(!LNX || (8 * NL % NT == 0 && Q4 % NT == 0), "LNX: whole chunk rounds per operand");
    float4 pf[(ABF && !LNX) ? 1 : CPT];
    uint2 pb[ABF ? CPT : 1];
    float pm[CX], pr[CX];
    auto load1 = [&](int64_t t, const int i) {
        {
            const int c = i * NT + threadIdx.x;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            uint2 u = make_uint2(0, 0);
            if constexpr (LNX) {
                if (i >= CY) { pm[i - CY] = 0.f; pr[i - CY] = 0.f; }
            }
            if (c < Q4) {
                const bool isy = LNX ? i < CY : c < 32 * NL / 4;
                const int cc = isy ? c : c - 32 * NL / 4;
                const int W4 = (isy ? NL : K) / 4;
                const int r = cc / W4, col = 4 * (cc % W4);
                const int64_t row = t * 32 + r;
                if (row < g.M) {
                    const void* base = isy ? g.dy : g.x;
                    const int64_t ld = isy ? g.ldy : g.ldx;
                    const int64_t o = row * ld + col + (isy ? ncol0 : 0);
                    if (LNX && !isy) {
                        v = *reinterpret_cast<const float4*>((const float*)base + o);
                        pm[LNX ? i - CY : 0] = g.mean[row];
                        pr[LNX ? i - CY : 0] = g.rstd[row];
                    } else if constexpr (ABF) {
                        u = *reinterpret_cast<const uint2*>((const uint16_t*)base + o);
                    } else {
                        v = *reinterpret_cast<const float4*>((const float*)base + o);
                    }
                }
            }
            if constexpr (ABF) pb[i] = u;
            if constexpr (!ABF || LNX) pf[i] = v;
        }
    };
    auto load = [&](int64_t t) {
#pragma unroll
        for (int i = 0; i < CPT; ++i) load1(t, i);
    };
    auto stash1 = [&](const int i) {
        {
            const int c = i * NT + threadIdx.x;
            if (c < Q4) {
                const bool isy = LNX ? i < CY : c < 32 * NL / 4;
                const int cc = isy ? c : c - 32 * NL / 4;
                const int W4 = (isy ? NL : K) / 4;
                const int r = cc / W4, col = 4 * (cc % W4);
                uint16_t* dst = isy ? ly + r * SY + col : lx + r * SX + col;
                const int pstride = isy ? PY : PX;
                if (LNX && !isy) {
                    const float4 x = pf[i];
                    const float m = pm[LNX ? i - CY : 0], rs = pr[LNX ? i - CY : 0];
                    uint32_t lo[P], hi[P];
                    split2<P>(ln_apply(x.x, m, rs, lng.x, lnb.x), ln_apply(x.y, m, rs, lng.y, lnb.y), lo);
                    split2<P>(ln_apply(x.z, m, rs, lng.z, lnb.z), ln_apply(x.w, m, rs, lng.w, lnb.w), hi);
#pragma unroll
                    for (int p = 0; p < P; ++p) *reinterpret_cast<uint2*>(dst + p * pstride) = make_uint2(lo[p], hi[p]);
                } else if constexpr (ABF) {
                    *reinterpret_cast<uint2*>(dst) = pb[i];
                } else {
                    uint32_t lo[P], hi[P];
                    split2<P>(pf[i].x, pf[i].y, lo);
                    split2<P>(pf[i].z, pf[i].w, hi);
#pragma unroll
                    for (int p = 0; p < P; ++p) *reinterpret_cast<uint2*>(dst + p * pstride) = make_uint2(lo[p], hi[p]);
                }
            }
        }
    };
    // TAGAN_SG_TN_ILOAD: chunk i of the next tile is loaded as soon as chunk i of this one is stashed (the next
    // tile's loads start during the stash instead of after it; no extra registers)
    auto stash_reload = [&](int64_t tn, bool more) {
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
            stash1(i);
            if (TAGAN_SG_TN_ILOAD && more) load1(tn, i);
        }
    };
    // transposed fragment of columns [c0, c0 + 16) of a plane with row stride S: rows 4 grp + q and 16 + 4 grp + q
    auto frag = [&](const uint16_t* plane, int S, int c0) {
        const int q = li >> 2, p4 = li & 3;
        const uint16_t* a0 = plane + (4 * grp + q) * S + c0 + 4 * p4;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a0);
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 16 * S));
        const short __attribute__((ext_vector_type(8))) v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        return __builtin_bit_cast(bf16x8, v);
    };

    if (t0 < t1) load(t0);
    for (int64_t t = t0; t < t1; ++t) {
        lds_barrier();                   // the previous tile's fragments are read
        stash_reload(t + 1, t + 1 < t1);
        lds_barrier();
        if (!TAGAN_SG_TN_ILOAD && t + 1 < t1) load(t + 1);
        bf16x8 ya[NSN][P];
#pragma unroll
        for (int s = 0; s < NSN; ++s)
#pragma unroll
            for (int p = 0; p < P; ++p) ya[s][p] = frag(ly + p * PY, SY, (w * NSN + s) * 16);
#pragma unroll
        for (int s = 0; s < NSN; ++s)
#pragma unroll
            for (int p = 0; p < P; ++p) accb[s] = mfma(ya[s][p], ones, accb[s]);
#pragma unroll
        for (int k = 0; k < KS; ++k) {
            bf16x8 xb[P];
#pragma unroll
            for (int p = 0; p < P; ++p) xb[p] = frag(lx + p * PX, SX, k * 16);
#pragma unroll
            for (int s = 0; s < NSN; ++s) acc[s][k] = mfma_planes<P>(ya[s], xb, acc[s][k]);
        }
    }
    // D[n][k]: lane holds rows n = 4 grp + r, column k = li of each 16 x 16 tile
    float* part = g.part + (int64_t)blockIdx.x * (N * K + N);
#pragma unroll
    for (int s = 0; s < NSN; ++s) {
        const int nb = ncol0 + (w * NSN + s) * 16 + 4 * grp;
#pragma unroll
        for (int k = 0; k < KS; ++k)
#pragma unroll
            for (int r = 0; r < 4; ++r) part[(int64_t)(nb + r) * K + 16 * k + li] = acc[s][k][r];
        if (li == 0)
#pragma unroll
            for (int r = 0; r < 4; ++r) part[N * K + nb + r] = accb[s][r];
    }
}

// dw[n * lddw + k] = Σ_g part[g][n K + k], db[n] likewise.  A 256-thread block owns 64 consecutive outputs; its four
// waves sum the four quarters of the partial range (g ascending, 4 interleaved accumulators each: 16 loads in
// flight per lane) and the quarters meet in LDS in a fixed order (bitwise reproducible).  One thread per output
// with a serial loop over every partial left the reduction latency-bound at ~1.7 TB/s.
constexpr int TNR_COLS = 64, TNR_SLICES = 4;
__global__ void __launch_bounds__(TNR_COLS * TNR_SLICES) k_sgemm_tn_reduce(const float* __restrict__ part, int G, int N,
                                                                         int K, float* __restrict__ dw, int64_t lddw,
                                                                         float* __restrict__ db) {
    __shared__ float q4[TNR_SLICES][TNR_COLS];
    const int L = N * K + N;
    const int col = threadIdx.x % TNR_COLS, sl = threadIdx.x / TNR_COLS;
    const int idx = blockIdx.x * TNR_COLS + col;
    const int per = (G + TNR_SLICES - 1) / TNR_SLICES;
    const int g0 = min(G, sl * per), g1 = min(G, g0 + per);
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    if (idx < L) {
        int gi = g0;
        for (; gi + 3 < g1; gi += 4) {
            s0 += part[(int64_t)gi * L + idx];
            s1 += part[(int64_t)(gi + 1) * L + idx];
            s2 += part[(int64_t)(gi + 2) * L + idx];
            s3 += part[(int64_t)(gi + 3) * L + idx];
        }
        for (; gi < g1; ++gi) s0 += part[(int64_t)gi * L + idx];
    }
    q4[sl][col] = (s0 + s1) + (s2 + s3);
    __syncthreads();
    if (sl != 0 || idx >= L) return;
    const float v = (q4[0][col] + q4[1][col]) + (q4[2][col] + q4[3][col]);
    if (idx < N * K) {
        if (dw) dw[(int64_t)(idx / K) * lddw + idx % K] = v;
    } else if (db) {
        db[idx - N * K] = v;
    }
}

// ------------------------------------------------------------------------------------------- LN2 backward + out-projection
// The first three steps of an attention block's backward (geometric_attention.py:586-596, temporal_attention.py:
// 1190-1200 reversed) in ONE pass over the rows, H = 128:
//   LN2 backward   ds = rstd (g dy - mean(g dy x̂) x̂ - mean(g dy)) [+ the skip LayerNorm's input gradient] -> dres,
//                  do = dropout(ds) (the forward's mask: stream = row, counter = column), dγ, dβ [, dγ_s, dβ_s]
//   dC = do · W_o  (the out-projection input gradient)                                     -> dc
//   dW_o = doᵀ · c, db_o = Σ do  (its weight and bias gradients)                           -> per-workgroup partials
// Separately these were a LayerNorm pass (s, dy in; dres, do out), an NT GEMM (do in; dc out) and a TN GEMM (do, c
// in): 8 row-sized HBM passes.  Here do never reaches HBM: 5 passes (dy, s, c in; dres, dc out).
// Workgroup: 8 waves over contiguous 32-row tiles (fixed ranges: the partials are summed in workgroup order, bitwise
// reproducible).  Thread c owns row c >> 4 of the tile and columns 8 (c & 15) + [0, 8) for the row math (the 16 lanes
// of a DPP row hold a whole row: row sums by butterflies); do and c go to LDS as row-major bf16 planes ([32][H + 16]);
// wave w then runs the dW_o rows 16 w.. (k_sgemm_tn's transposed reads, the db_o sum against a ones fragment) and the
// dc columns 16 w.. (B = W_oᵀ fragments in registers, A = do rows straight from the planes).
struct L2Args {
    int64_t M;
    int64_t tiles_per_wg;
    const float* dy;          // [M, H] gradient of the block output
    const float* s;           // [M, H] LN2 input (saved by the forward)
    const float* mean;
    const float* rstd;
    const float* gamma;
    float p_drop, inv_keep;
    uint64_t seed;
    const uint64_t* seed_ctr;
    const float* xs;          // skip branch: LN_s input [M, H], statistics, gamma (null: no skip LayerNorm)
    const float* mean_s;
    const float* rstd_s;
    const float* gamma_s;
    const void* c;            // [M, H] out-projection input (fp32, or bf16 with ABF)
    const uint4* wp;          // W_oᵀ fragment planes (tagan_sgemm_wprep(w_o, kmajor = 1))
    float* dres;              // [M, H] gradient of the block input through the residual (+ skip) path
    void* dc;                 // [M, H] (fp32, or bf16 with ABF)
    float* part_w;            // [G][H * H + H]: dW_o | db_o partials (k_sgemm_tn_reduce layout)
    float* part_ln;           // [G][NPL * H]: dγ | dβ [| dγ_s | dβ_s]
};

// TAGAN_LN2_FORM (A/B builds only): 0 shipped; 1 the next tile's loads after the plane-writing barriers; 2 as 1 with
// dead rows branched around in the LN sums (the round-5 first form, profiles/r5d_ln2_probe.txt).
#ifndef TAGAN_LN2_FORM
#define TAGAN_LN2_FORM 0
#endif
template <int P, bool ABF, bool SK>
__global__ void __launch_bounds__(512, 1) k_ln2_bwd_out(L2Args g) {
    constexpr int H = 128, BM = 32, NW = 8, KK = H / 32, KS = H / 16, S = H + 16, PL = BM * S;
    static_assert(!ABF || P == 1, "bf16 operands have one plane");
    extern __shared__ uint4 sg_lds[];
    uint16_t* ldo = reinterpret_cast<uint16_t*>(sg_lds);   // P planes of do [BM][S]
    uint16_t* lcp = ldo + P * PL;                          // P planes of c
    float* red = reinterpret_cast<float*>(lcp + P * PL);   // [NW][NPL * H] wave partials of the LN sums (end)
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int grp = lane >> 4, li = lane & 15;
    const int rr = threadIdx.x >> 4, q = threadIdx.x & 15;   // row-math chunk: tile row, 8-column group
    TAGAN_LIVE_SEED(g);

    // this thread's 8 columns of gamma (and gamma_s)
    float gm[8], gms[SK ? 8 : 1];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        gm[e] = g.gamma[8 * q + e];
        if constexpr (SK) gms[e] = g.gamma_s[8 * q + e];
    }
    // dc columns 16 w..: B fragments of W_oᵀ
    bf16x8 wr[KK][P];
#pragma unroll
    for (int kk = 0; kk < KK; ++kk)
#pragma unroll
        for (int p = 0; p < P; ++p) wr[kk][p] = __builtin_bit_cast(bf16x8, g.wp[((int64_t)(w * KK + kk) * P + p) * 64 + lane]);
    bf16x8 ones;
#pragma unroll
    for (int e = 0; e < 8; ++e) ones[e] = (__bf16)1.0f;

    float dg[8], db[8], dgs[SK ? 8 : 1], dbs[SK ? 8 : 1];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        dg[e] = db[e] = 0.f;
        if constexpr (SK) dgs[e] = dbs[e] = 0.f;
    }
    f32x4 accw[KS], accb = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < KS; ++k) accw[k] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int64_t t0 = (int64_t)blockIdx.x * g.tiles_per_wg;
    const int64_t t1 = min(t0 + g.tiles_per_wg, (g.M + BM - 1) / BM);

    // the tile's operands of this thread (row rr, columns 8 q..)
    float4 vdy[2], vs[2], vx[SK ? 2 : 1];
    float4 vc[ABF ? 1 : 2];
    uint4 vcb;
    float mrow = 0.f, rrow = 0.f, mrs = 0.f, rrs = 0.f;
    auto load = [&](int64_t t) {
        const int64_t row0 = t * BM + rr;
        const int64_t r = row0 < g.M ? row0 : g.M - 1;
        const float* pdy = g.dy + r * H + 8 * q;
        const float* ps = g.s + r * H + 8 * q;
        vdy[0] = *reinterpret_cast<const float4*>(pdy);
        vdy[1] = *reinterpret_cast<const float4*>(pdy + 4);
        vs[0] = *reinterpret_cast<const float4*>(ps);
        vs[1] = *reinterpret_cast<const float4*>(ps + 4);
        if constexpr (ABF) {
            vcb = *reinterpret_cast<const uint4*>((const uint16_t*)g.c + r * H + 8 * q);
        } else {
            const float* pc = (const float*)g.c + r * H + 8 * q;
            vc[0] = *reinterpret_cast<const float4*>(pc);
            vc[1] = *reinterpret_cast<const float4*>(pc + 4);
        }
        mrow = g.mean[r];
        rrow = g.rstd[r];
        if constexpr (SK) {
            const float* px = g.xs + r * H + 8 * q;
            vx[0] = *reinterpret_cast<const float4*>(px);
            vx[1] = *reinterpret_cast<const float4*>(px + 4);
            mrs = g.mean_s[r];
            rrs = g.rstd_s[r];
        }
    };
    // transposed fragment of columns [c0, c0 + 16) of a plane (k_sgemm_tn's frag)
    auto frag = [&](const uint16_t* plane, int c0) {
        const int qq = li >> 2, p4 = li & 3;
        const uint16_t* a0 = plane + (4 * grp + qq) * S + c0 + 4 * p4;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a0);
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 16 * S));
        const short __attribute__((ext_vector_type(8))) v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        return __builtin_bit_cast(bf16x8, v);
    };

    if (t0 < t1) load(t0);
    for (int64_t t = t0; t < t1; ++t) {
        const int64_t row = t * BM + rr;
        const bool live = row < g.M;
        // ---- LN2 backward of this thread's 8 columns
        const float d[8] = {vdy[0].x, vdy[0].y, vdy[0].z, vdy[0].w, vdy[1].x, vdy[1].y, vdy[1].z, vdy[1].w};
        const float sv[8] = {vs[0].x, vs[0].y, vs[0].z, vs[0].w, vs[1].x, vs[1].y, vs[1].z, vs[1].w};
        float xh[8], gd[8];
        float c1 = 0.f, c2 = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            xh[e] = (sv[e] - mrow) * rrow;
            gd[e] = d[e] * gm[e];
        }
        // the LayerNorm kernel's association: (x0 + x1) + (x2 + x3) per float4, then the float4 halves
        c1 = ((gd[0] * xh[0] + gd[1] * xh[1]) + (gd[2] * xh[2] + gd[3] * xh[3])) +
             ((gd[4] * xh[4] + gd[5] * xh[5]) + (gd[6] * xh[6] + gd[7] * xh[7]));
        c2 = ((gd[0] + gd[1]) + (gd[2] + gd[3])) + ((gd[4] + gd[5]) + (gd[6] + gd[7]));
        c1 = xsum<16>(c1) / (float)H;
        c2 = xsum<16>(c2) / (float)H;
        float xsk[SK ? 8 : 1], gsk[SK ? 8 : 1], c1s = 0.f, c2s = 0.f;
        if constexpr (SK) {
            const float xv[8] = {vx[0].x, vx[0].y, vx[0].z, vx[0].w, vx[1].x, vx[1].y, vx[1].z, vx[1].w};
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                xsk[e] = (xv[e] - mrs) * rrs;
                gsk[e] = d[e] * gms[e];
            }
            c1s = ((gsk[0] * xsk[0] + gsk[1] * xsk[1]) + (gsk[2] * xsk[2] + gsk[3] * xsk[3])) +
                  ((gsk[4] * xsk[4] + gsk[5] * xsk[5]) + (gsk[6] * xsk[6] + gsk[7] * xsk[7]));
            c2s = ((gsk[0] + gsk[1]) + (gsk[2] + gsk[3])) + ((gsk[4] + gsk[5]) + (gsk[6] + gsk[7]));
            c1s = xsum<16>(c1s) / (float)H;
            c2s = xsum<16>(c2s) / (float)H;
        }
        const uint32_t key = drop_key(g.seed, (uint64_t)row);
        float dov[8], dsv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float o = rrow * (gd[e] - c1 * xh[e] - c2);
            float a = o;
            if (g.p_drop > 0.f) a = drop_u(key, (uint32_t)(8 * q + e)) >= g.p_drop ? o * g.inv_keep : 0.f;
            dov[e] = live ? a : 0.f;    // dead rows add nothing to dW_o / db_o
            float sres = o;
            if constexpr (SK) sres += rrs * (gsk[e] - c1s * xsk[e] - c2s);
            dsv[e] = sres;
            if (TAGAN_LN2_FORM == 2) {   // round-5 first form: dead rows branched around (A/B only)
                if (live) {
                    dg[e] += d[e] * xh[e];
                    db[e] += d[e];
                    if constexpr (SK) {
                        dgs[e] += d[e] * xsk[e];
                        dbs[e] += d[e];
                    }
                }
            } else {
            const float dl = live ? d[e] : 0.f;   // dead rows add exact zeros (their operands are row M - 1's)
            dg[e] += dl * xh[e];
            db[e] += dl;
            if constexpr (SK) {
                dgs[e] += dl * xsk[e];
                dbs[e] += dl;
            }
            }
        }
        if (live) {
            float* pr = g.dres + row * H + 8 * q;
            *reinterpret_cast<float4*>(pr) = make_float4(dsv[0], dsv[1], dsv[2], dsv[3]);
            *reinterpret_cast<float4*>(pr + 4) = make_float4(dsv[4], dsv[5], dsv[6], dsv[7]);
        }
        // The next tile's loads go out here, right after this tile's row math, into the same variables (c is copied
        // first).  Round 5's first form (loads after the plane-writing barriers, dead rows branched around in the LN
        // sums: TAGAN_LN2_FORM=2) gave nondeterministic dgamma columns 8q + 4 / 8q + 6: not a load hazard, but the
        // compiler encoding those two products as v_pk_mul_f32 with src1's high register in the low lane, a form that
        // drops low-lane results on gfx950 (tools/isa_audit.py now rejects it at every build).
        float4 vc_cur[ABF ? 1 : 2];
        const uint4 vcb_cur = vcb;
        if constexpr (!ABF) { vc_cur[0] = vc[0]; vc_cur[1] = vc[1]; }
        if (TAGAN_LN2_FORM == 0 && t + 1 < t1) load(t + 1);
        // ---- do and c -> row-major bf16 planes
        lds_barrier();   // the previous tile's fragments are read
        {
            uint32_t pd[4][P], pc[4][P];
#pragma unroll
            for (int e = 0; e < 4; ++e) split2<P>(dov[2 * e], dov[2 * e + 1], pd[e]);
            const uint4 cb = vcb_cur;
            const float4* cv = vc_cur;
            if constexpr (ABF) {
                pc[0][0] = cb.x; pc[1][0] = cb.y; pc[2][0] = cb.z; pc[3][0] = cb.w;
            } else {
                split2<P>(cv[0].x, cv[0].y, pc[0]);
                split2<P>(cv[0].z, cv[0].w, pc[1]);
                split2<P>(cv[1].x, cv[1].y, pc[2]);
                split2<P>(cv[1].z, cv[1].w, pc[3]);
            }
#pragma unroll
            for (int p = 0; p < P; ++p) {
                *reinterpret_cast<uint4*>(ldo + p * PL + rr * S + 8 * q) = make_uint4(pd[0][p], pd[1][p], pd[2][p], pd[3][p]);
                *reinterpret_cast<uint4*>(lcp + p * PL + rr * S + 8 * q) = make_uint4(pc[0][p], pc[1][p], pc[2][p], pc[3][p]);
            }
        }
        lds_barrier();
        if (TAGAN_LN2_FORM != 0 && t + 1 < t1) load(t + 1);   // round-5 first form (A/B only)
        // ---- dW_o rows 16 w.., db_o
        {
            bf16x8 ya[P];
#pragma unroll
            for (int p = 0; p < P; ++p) ya[p] = frag(ldo + p * PL, 16 * w);
#pragma unroll
            for (int p = 0; p < P; ++p) accb = mfma(ya[p], ones, accb);
#pragma unroll
            for (int k = 0; k < KS; ++k) {
                bf16x8 xb[P];
#pragma unroll
                for (int p = 0; p < P; ++p) xb[p] = frag(lcp + p * PL, 16 * k);
                accw[k] = mfma_planes<P>(ya, xb, accw[k]);
            }
        }
        // ---- dc columns 16 w.. for the tile's two 16-row halves
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kk = 0; kk < KK; ++kk) {
                bf16x8 a[P];
#pragma unroll
                for (int p = 0; p < P; ++p)
                    a[p] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(
                                                          ldo + p * PL + (16 * j + li) * S + 32 * kk + 8 * grp));
                acc = mfma_planes<P>(wr[kk], a, acc);
            }
            const int64_t orow = t * BM + 16 * j + li;
            if (orow < g.M) {
                const int64_t off = orow * H + 16 * w + 4 * grp;
                if constexpr (ABF) {
                    *reinterpret_cast<uint2*>((uint16_t*)g.dc + off) = make_uint2(pk_bf16(acc[0], acc[1]),
                                                                                  pk_bf16(acc[2], acc[3]));
                } else {
                    *reinterpret_cast<f32x4*>((float*)g.dc + off) = acc;
                }
            }
        }
    }
    // ---- partials: dW_o | db_o (k_sgemm_tn layout: lane holds rows n = 16 w + 4 grp + r, column k = 16 k + li)
    float* pw = g.part_w + (int64_t)blockIdx.x * (H * H + H);
#pragma unroll
    for (int k = 0; k < KS; ++k)
#pragma unroll
        for (int r = 0; r < 4; ++r) pw[(int64_t)(16 * w + 4 * grp + r) * H + 16 * k + li] = accw[k][r];
    if (li == 0)
#pragma unroll
        for (int r = 0; r < 4; ++r) pw[H * H + 16 * w + 4 * grp + r] = accb[r];
    // LN sums: lanes l, l ^ 16, l ^ 32, l ^ 48 share columns; then the 8 waves in order through LDS
    constexpr int NPL = SK ? 4 : 2;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const float a0 = gsum4(dg[e]), a1 = gsum4(db[e]);
        float a2 = 0.f, a3 = 0.f;
        if constexpr (SK) {
            a2 = gsum4(dgs[e]);
            a3 = gsum4(dbs[e]);
        }
        if (grp == 0) {
            float* rw = red + w * NPL * H + 8 * q + e;
            rw[0] = a0;
            rw[H] = a1;
            if constexpr (SK) {
                rw[2 * H] = a2;
                rw[3 * H] = a3;
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < NPL * H; i += NW * 64) {
        float a = 0.f;
#pragma unroll
        for (int ww = 0; ww < NW; ++ww) a += red[ww * NPL * H + i];
        g.part_ln[(int64_t)blockIdx.x * NPL * H + i] = a;
    }
}

// ------------------------------------------------------------------------------------------- LN2 backward + out-projection, H = 256
#ifndef TAGAN_SG_LN2_256
#define TAGAN_SG_LN2_256 1
#endif
// k_ln2_bwd_out at H = 256 with one plane (the bf16 activation mode, C5; round 6).  A whole 256-wide W_o^T panel and
// dW_o's 256 x 256 accumulators do not fit one 8-wave workgroup's registers, so the work is split over TWO column
// groups cg (grid = 2 G, adjacent on one XCD: block b -> cg = (b / 8) % 2, row range (b / 16) * 8 + b % 8): both run
// the LN2 row math over whole rows (the row sums need all 256 columns; the second group's reads of dy / s / x hit
// the L2 the first one just filled), and group cg then owns
//   dW_o rows n in [128 cg, 128 cg + 128) (wave w: 16 rows x all 256 k: 16 accumulator tiles), db_o of those rows,
//   dc columns in [128 cg, 128 cg + 128) (wave w: 16 columns, K = 256: 8 W_o^T fragments in registers),
//   dres columns of its half; group 0 also accumulates the LN column sums (dgamma | dbeta [| dgamma_s | dbeta_s]).
// Thread = (row, 8 columns), 32 lanes per row (two DPP rows: lane_sum<32>), 16 rows per pass, two passes per
// 32-row tile (the MFMA K of dW_o); the operands of the next pass are loaded while this one's planes are built.
template <bool ABF, bool SK>
__global__ void __launch_bounds__(512, 1) k_ln2_bwd_out256(L2Args g) {
    constexpr int H = 256, BM = 32, NW = 8, KK = H / 32, S = H + 16, PL = BM * S;
    extern __shared__ uint4 sg_lds[];
    uint16_t* ldo = reinterpret_cast<uint16_t*>(sg_lds);   // do plane [BM][S]
    uint16_t* lcp = ldo + PL;                              // c plane
    float* red = reinterpret_cast<float*>(lcp + PL);       // [NW][NPL * H] wave partials of the LN sums (end)
    float* lgm = red + NW * (SK ? 4 : 2) * H;              // gamma | gamma_s (read per row: 16 VGPRs fewer)
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int grp = lane >> 4, li = lane & 15;
    const int rr = threadIdx.x >> 5, q = threadIdx.x & 31;   // row math: pass row, 8-column group
    const int cg = (blockIdx.x >> 3) & 1;
    const int64_t rb = ((int64_t)(blockIdx.x >> 4) << 3) | (blockIdx.x & 7);
    TAGAN_LIVE_SEED(g);

    for (int i = threadIdx.x; i < (SK ? 2 : 1) * H; i += NW * 64) lgm[i] = i < H ? g.gamma[i] : g.gamma_s[i - H];
    __syncthreads();
    bf16x8 wr[KK];
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) wr[kk] = __builtin_bit_cast(bf16x8, g.wp[((int64_t)((8 * cg + w) * KK + kk)) * 64 + lane]);
    // column sums over the rows, fp32: group 0 the LN ones (dg: dgamma, db: dbeta [, dgs, dbs]), group 1 db_o
    // (in dg: the exact sum of the fp32 do, not of its bf16 plane)
    // (dbeta_s = Σ dy = dbeta: one array serves both)
    float dg[8], db[8], dgs[SK ? 8 : 1];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        dg[e] = db[e] = 0.f;
        if constexpr (SK) dgs[e] = 0.f;
    }
    f32x4 accw[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) accw[k] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int64_t t0 = rb * g.tiles_per_wg;
    const int64_t t1 = min(t0 + g.tiles_per_wg, (g.M + BM - 1) / BM);

    // one pass-row's operands (row r = 32 t + 16 pass + rr, columns 8 q..)
    float4 vdy[2], vs[2], vx[SK ? 2 : 1], vc[ABF ? 1 : 2];
    uint4 vcb;
    float mrow = 0.f, rrow = 0.f, mrs = 0.f, rrs = 0.f;
    auto load = [&](int64_t row0) {
        const int64_t r = row0 < g.M ? row0 : g.M - 1;
        const float* pdy = g.dy + r * H + 8 * q;
        const float* ps = g.s + r * H + 8 * q;
        vdy[0] = *reinterpret_cast<const float4*>(pdy);
        vdy[1] = *reinterpret_cast<const float4*>(pdy + 4);
        vs[0] = *reinterpret_cast<const float4*>(ps);
        vs[1] = *reinterpret_cast<const float4*>(ps + 4);
        if constexpr (ABF) {
            vcb = *reinterpret_cast<const uint4*>((const uint16_t*)g.c + r * H + 8 * q);
        } else {
            const float* pc = (const float*)g.c + r * H + 8 * q;
            vc[0] = *reinterpret_cast<const float4*>(pc);
            vc[1] = *reinterpret_cast<const float4*>(pc + 4);
        }
        mrow = g.mean[r];
        rrow = g.rstd[r];
        if constexpr (SK) {
            const float* px = g.xs + r * H + 8 * q;
            vx[0] = *reinterpret_cast<const float4*>(px);
            vx[1] = *reinterpret_cast<const float4*>(px + 4);
            mrs = g.mean_s[r];
            rrs = g.rstd_s[r];
        }
    };
    auto frag = [&](const uint16_t* plane, int c0) {
        const int qq = li >> 2, p4 = li & 3;
        const uint16_t* a0 = plane + (4 * grp + qq) * S + c0 + 4 * p4;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a0);
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 16 * S));
        const short __attribute__((ext_vector_type(8))) v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        return __builtin_bit_cast(bf16x8, v);
    };
    // the LN2 backward of this thread's 8 columns of one row -> its do and c plane words (4 + 4 packed bf16 pairs)
    auto rowmath = [&](int64_t row, uint32_t (&pd)[4], uint32_t (&pc)[4]) {
        const bool live = row < g.M;
        const float d[8] = {vdy[0].x, vdy[0].y, vdy[0].z, vdy[0].w, vdy[1].x, vdy[1].y, vdy[1].z, vdy[1].w};
        const float sv[8] = {vs[0].x, vs[0].y, vs[0].z, vs[0].w, vs[1].x, vs[1].y, vs[1].z, vs[1].w};
        float xh[8], gd[8];
        const float4 g0 = *reinterpret_cast<const float4*>(lgm + 8 * q), g1 = *reinterpret_cast<const float4*>(lgm + 8 * q + 4);
        const float gm[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            xh[e] = (sv[e] - mrow) * rrow;
            gd[e] = d[e] * gm[e];
        }
        float c1 = ((gd[0] * xh[0] + gd[1] * xh[1]) + (gd[2] * xh[2] + gd[3] * xh[3])) +
                   ((gd[4] * xh[4] + gd[5] * xh[5]) + (gd[6] * xh[6] + gd[7] * xh[7]));
        float c2 = ((gd[0] + gd[1]) + (gd[2] + gd[3])) + ((gd[4] + gd[5]) + (gd[6] + gd[7]));
        c1 = xsum<32>(c1) / (float)H;
        c2 = xsum<32>(c2) / (float)H;
        float xsk[SK ? 8 : 1], gsk[SK ? 8 : 1], c1s = 0.f, c2s = 0.f;
        if constexpr (SK) {
            const float xv[8] = {vx[0].x, vx[0].y, vx[0].z, vx[0].w, vx[1].x, vx[1].y, vx[1].z, vx[1].w};
            const float4 h0 = *reinterpret_cast<const float4*>(lgm + H + 8 * q);
            const float4 h1 = *reinterpret_cast<const float4*>(lgm + H + 8 * q + 4);
            const float gms[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                xsk[e] = (xv[e] - mrs) * rrs;
                gsk[e] = d[e] * gms[e];
            }
            c1s = ((gsk[0] * xsk[0] + gsk[1] * xsk[1]) + (gsk[2] * xsk[2] + gsk[3] * xsk[3])) +
                  ((gsk[4] * xsk[4] + gsk[5] * xsk[5]) + (gsk[6] * xsk[6] + gsk[7] * xsk[7]));
            c2s = ((gsk[0] + gsk[1]) + (gsk[2] + gsk[3])) + ((gsk[4] + gsk[5]) + (gsk[6] + gsk[7]));
            c1s = xsum<32>(c1s) / (float)H;
            c2s = xsum<32>(c2s) / (float)H;
        }
        const uint32_t key = drop_key(g.seed, (uint64_t)row);
        float dov[8], dsv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float o = rrow * (gd[e] - c1 * xh[e] - c2);
            float a = o;
            if (g.p_drop > 0.f) a = drop_u(key, (uint32_t)(8 * q + e)) >= g.p_drop ? o * g.inv_keep : 0.f;
            dov[e] = live ? a : 0.f;
            float sres = o;
            if constexpr (SK) sres += rrs * (gsk[e] - c1s * xsk[e] - c2s);
            dsv[e] = sres;
            // the column sums, branch-free (a branch here sent the arrays to scratch): group 0 the LN ones (dead
            // rows add exact zeros), group 1 db_o
            const float dl = (live && cg == 0) ? d[e] : 0.f;
            dg[e] += cg == 0 ? dl * xh[e] : dov[e];
            db[e] += dl;
            if constexpr (SK) dgs[e] += dl * xsk[e];
        }
        if (live && (q >> 4) == cg) {   // dres: each group its half of the columns
            float* pr = g.dres + row * H + 8 * q;
            *reinterpret_cast<float4*>(pr) = make_float4(dsv[0], dsv[1], dsv[2], dsv[3]);
            *reinterpret_cast<float4*>(pr + 4) = make_float4(dsv[4], dsv[5], dsv[6], dsv[7]);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) pd[e] = pk_bf16(dov[2 * e], dov[2 * e + 1]);
        if constexpr (ABF) {
            pc[0] = vcb.x; pc[1] = vcb.y; pc[2] = vcb.z; pc[3] = vcb.w;
        } else {
            pc[0] = pk_bf16(vc[0].x, vc[0].y);
            pc[1] = pk_bf16(vc[0].z, vc[0].w);
            pc[2] = pk_bf16(vc[1].x, vc[1].y);
            pc[3] = pk_bf16(vc[1].z, vc[1].w);
        }
    };

    if (t0 < t1) load(t0 * BM + rr);
    for (int64_t t = t0; t < t1; ++t) {
        uint32_t pd[2][4], pc[2][4];
#pragma unroll
        for (int pass = 0; pass < 2; ++pass) {
            rowmath(t * BM + 16 * pass + rr, pd[pass], pc[pass]);
            // next pass-row: row rr + 16 of this tile, then row rr of the next one (t1 - 1's second pass reloads
            // itself: unconditional loads)
            const int64_t nrow = pass == 0 ? t * BM + 16 + rr : (t + 1 < t1 ? (t + 1) * BM + rr : t * BM + rr);
            load(nrow);
        }
        lds_barrier();   // the previous tile's fragments are read
#pragma unroll
        for (int pass = 0; pass < 2; ++pass) {
            *reinterpret_cast<uint4*>(ldo + (16 * pass + rr) * S + 8 * q) = make_uint4(pd[pass][0], pd[pass][1], pd[pass][2], pd[pass][3]);
            *reinterpret_cast<uint4*>(lcp + (16 * pass + rr) * S + 8 * q) = make_uint4(pc[pass][0], pc[pass][1], pc[pass][2], pc[pass][3]);
        }
        lds_barrier();
        // ---- dW_o rows 128 cg + 16 w.. (all 256 k)
        {
            const bf16x8 ya = frag(ldo, 128 * cg + 16 * w);
#pragma unroll
            for (int k = 0; k < 16; ++k) accw[k] = mfma(ya, frag(lcp, 16 * k), accw[k]);
        }
        // ---- dc columns 128 cg + 16 w.. for the tile's two 16-row halves
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kk = 0; kk < KK; ++kk) {
                const bf16x8 a = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(
                                                                ldo + (16 * j + li) * S + 32 * kk + 8 * grp));
                acc = mfma(wr[kk], a, acc);
            }
            const int64_t orow = t * BM + 16 * j + li;
            if (orow < g.M) {
                const int64_t off = orow * H + 128 * cg + 16 * w + 4 * grp;
                if constexpr (ABF) {
                    *reinterpret_cast<uint2*>((uint16_t*)g.dc + off) = make_uint2(pk_bf16(acc[0], acc[1]),
                                                                                  pk_bf16(acc[2], acc[3]));
                } else {
                    *reinterpret_cast<f32x4*>((float*)g.dc + off) = acc;
                }
            }
        }
    }
    // ---- partials of row range rb: dW_o rows of this group (k_sgemm_tn_reduce layout)
    float* pw = g.part_w + rb * (H * H + H);
#pragma unroll
    for (int k = 0; k < 16; ++k)
#pragma unroll
        for (int r = 0; r < 4; ++r) pw[(int64_t)(128 * cg + 16 * w + 4 * grp + r) * H + 16 * k + li] = accw[k][r];
    // column sums: lanes l and l ^ 32 share columns (two rows per wave); then the 8 waves in order through LDS.
    // Group 0: the LN sums -> part_ln; group 1: db_o -> the bias slot of part_w.
    const int NPL = cg == 0 ? (SK ? 4 : 2) : 1;
    auto sum2 = [](float x) {
        float a, b;
        swap32(x, a, b);
        return a + b;
    };
    lds_barrier();
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const float a0 = sum2(dg[e]), a1 = sum2(db[e]);
        float a2 = 0.f, a3 = 0.f;
        if constexpr (SK) {
            a2 = sum2(dgs[e]);
            a3 = a1;
        }
        if (lane < 32) {
            float* rw = red + w * NPL * H + 8 * q + e;
            rw[0] = a0;
            if (cg == 0) {
                rw[H] = a1;
                if constexpr (SK) {
                    rw[2 * H] = a2;
                    rw[3 * H] = a3;
                }
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < NPL * H; i += NW * 64) {
        float a = 0.f;
#pragma unroll
        for (int ww = 0; ww < NW; ++ww) a += red[ww * NPL * H + i];
        if (cg == 0) g.part_ln[rb * NPL * H + i] = a;
        else pw[H * H + i] = a;
    }
}

// ------------------------------------------------------------------------------------------- dispatch
int g_num_cu = 0;
int num_cu() {
    if (!g_num_cu) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
            g_num_cu = n;
        else
            g_num_cu = 256;
    }
    return g_num_cu;
}

typedef void (*nt_fn)(NtArgs);
struct NtCfg {
    int K, N, P, abf, cbf, mode;   // shape / storage / fusion key
    nt_fn fn;
    int nw, nsub, bm;
    size_t lds;
    int wg_per_cu;
};

// MINB: waves per SIMD the register allocation must allow (4 = two 8-wave workgroups per CU: the LN epilogues
// serialise each workgroup's memory and matrix phases, a second workgroup per CU overlaps them)
// TAGAN_SG_PP: the three-plane 8-wave plain / split-K forms run on the ping-pong kernel (k_sgemm_nt_pp).  C2 QKV
// input gradient 173.8 -> 163.1 us (profiles/r6k_pp_ab.txt).  The LN-prologue QKV forward stays on k_sgemm_nt: on
// the ping-pong kernel it measured 175.8 -> 196.8 us; an L2 prefetch of the tile after next (TAGAN_SG_PF) slowed
// both (dX 185.8, QKV 234.8 us).
#ifndef TAGAN_SG_PP
#define TAGAN_SG_PP 1
#endif
template <int K, int NSUB, int NW, int BM, int P, bool ABF, bool CBF, int MODE, int MINB>
constexpr nt_fn nt_kernel() {
    if constexpr (TAGAN_SG_PP && P == 3 && NW == 8 && MINB == 1 && (BM / 16) % 2 == 0 &&
                  (MODE == MODE_PLAIN || MODE == MODE_ACC))
        return k_sgemm_nt_pp<K, NSUB, BM, P, ABF, CBF, MODE>;
    else
        return k_sgemm_nt<K, NSUB, NW, BM, P, ABF, CBF, MODE, MINB>;
}
template <int K, int NSUB, int NW, int BM, int P, bool ABF, bool CBF, int MODE = MODE_PLAIN, int MINB = 1>
constexpr NtCfg nt_cfg(int N, int wg_per_cu) {
    return NtCfg{K, N, P, ABF, CBF, MODE, nt_kernel<K, NSUB, NW, BM, P, ABF, CBF, MODE, MINB>(), NW, NSUB, BM,
                 (size_t)2 * P * (K / 32) * (BM / 16) * 64 * 16 +
                     ((MODE == MODE_LN_OUT || MODE == MODE_LN_BWD) ? (size_t)(BM * NW * 4 + 4 * N) * 4 : 0) +
                     (MODE == MODE_LN_IN ? (size_t)2 * K * 4 : 0) + (size_t)NW * NSUB * 16 * 4,
                 wg_per_cu};
}

// (K, N) of the attention blocks at H = 128: QKV forward (128, 384), out-projection forward and its input
// gradient (128, 128), QKV input gradient (384, 128).
// One configuration per key (compile-time alternatives are A/B'd as variant libraries: make variant NAME=.. EXTRA=..).
// fp32 (three planes): MFMA-bound, tiles sized by the registers the weight fragments leave; one plane: HBM-bound,
// taller tiles so that more bytes are in flight per workgroup.
// H = 256 (C3, C5): a K = 256 three-plane panel is 96 VGPRs per 16 columns, so one n-subtile per wave and the
// columns spread over grid.y (N / 128 workgroup columns; each re-reads A, mostly from L2); K = 768 three-plane (the
// QKV input gradient, 288 VGPRs per 16 columns) runs as two K = 384 halves, the second accumulating into C
// (tagan_sgemm_nt splits it).  H = 64 (C1): 4-wave workgroups cover N = 192 / 64 in one grid column.
// H = 256 three-plane NT: two n-subtiles per wave over 16-row tiles (248 VGPRs).  With one n-subtile over 32-row
// tiles (TAGAN_SG_H256N2=0, the round-4 form) each A fragment read from LDS fed 6 MFMAs -- as many LDS cycles as
// matrix cycles per tile -- and six workgroup columns re-read A for N = 768; now 12 MFMAs per read, three columns:
// QKV forward 3.11 -> 2.78 ms, out-projection / dC 1.12 -> 1.04 ms at 1.6M rows, C3 step 467 -> 462 ms
// (profiles/r5za_h256_nt_ab.txt)
#ifndef TAGAN_SG_H256N2
#define TAGAN_SG_H256N2 1
#endif
#if TAGAN_SG_H256N2
#define NT_H256_F32 nt_cfg<256, 2, 8, 16, 3, false, false>(768, 1), nt_cfg<256, 2, 8, 16, 3, false, false>(256, 1),
#else
#define NT_H256_F32 nt_cfg<256, 1, 8, 32, 3, false, false>(768, 1), nt_cfg<256, 1, 8, 32, 3, false, false>(256, 1),
#endif
#define NT_SET3                                                                                              \
    nt_cfg<128, 3, 8, 32, 3, false, false>(384, 1), nt_cfg<128, 1, 8, 32, 3, false, false>(128, 2),            \
    nt_cfg<384, 1, 8, 32, 3, false, false>(128, 1),                                                            \
    NT_H256_F32                                                                                              \
    nt_cfg<384, 1, 8, 32, 3, false, false>(256, 1), nt_cfg<384, 1, 8, 32, 3, false, false, MODE_ACC>(256, 1),   \
    nt_cfg<64, 3, 4, 32, 3, false, false>(192, 1), nt_cfg<64, 1, 4, 32, 3, false, false>(64, 2),               \
    nt_cfg<192, 1, 4, 32, 3, false, false>(64, 2)
// the one-plane H = 256 QKV input gradient (K = 768, N = 256) with bf16 dqkv: all 256 columns in one workgroup
// column (two n-subtiles per wave, 16-row tiles), so dqkv is read once instead of by two column groups -- C5 bf16
// 504.5 / 504.9 -> 496.6 / 496.0 ms (profiles/r5ze_dh256_wide_ab.txt); =0: two columns of one n-subtile
#ifndef TAGAN_SG_DH256_WIDE
#define TAGAN_SG_DH256_WIDE 1
#endif
#if TAGAN_SG_DH256_WIDE
#define NT_DH256(ABF, CBF) nt_cfg<768, (ABF ? 2 : 1), 8, (ABF ? 16 : 32), 1, ABF, CBF>(256, 1),   // (fp32 A spills)
#else
#define NT_DH256(ABF, CBF) nt_cfg<768, 1, 8, 32, 1, ABF, CBF>(256, 1),
#endif
#define NT_SET1(ABF, CBF)                                                                                    \
    nt_cfg<128, 3, 8, 64, 1, ABF, CBF>(384, 1), nt_cfg<128, 1, 8, 128, 1, ABF, CBF>(128, 2),                  \
    nt_cfg<384, 1, 8, 64, 1, ABF, CBF>(128, 1),                                                                \
    nt_cfg<256, 2, 8, 64, 1, ABF, CBF>(768, 1), nt_cfg<256, 2, 8, 64, 1, ABF, CBF>(256, 1),                   \
    NT_DH256(ABF, CBF)                                                                                       \
    nt_cfg<64, 3, 4, 64, 1, ABF, CBF>(192, 1), nt_cfg<64, 1, 4, 64, 1, ABF, CBF>(64, 2),                      \
    nt_cfg<192, 1, 4, 64, 1, ABF, CBF>(64, 2)
// The LayerNorm-fused forms (H = 128): LN1 prologue of the QKV projection (x fp32 in; qkv fp32, or bf16 in the
// bf16 activation mode), dropout + residual + LN2 [+ skip LN] epilogue of the out-projection (y fp32), LN1 backward
// epilogue of the QKV input gradient (dx fp32).  At H = 256 (C3, C5) the LN1 prologue (32 lanes per row) with its
// LN-recomputing weight gradient, and in the one-plane (bf16 activation) mode the LN2 epilogue of the out-projection
// (MODE_LN_OUT row-owner kernels with N = 256); LN1's backward stays standalone there, LN2's backward is fused with the
// out-projection's gradients in one plane (k_ln2_bwd_out256) and standalone in three.
// (The LN2 epilogue and the one-plane LN1-backward epilogue run on the row-owner kernels, RG_TABLE; the three-plane
// LN1-backward epilogue lost its A/B -- fp32 step 6.99 vs 6.75 ms, profiles/r3d_ab_step.txt -- and is not built.)
#ifndef TAGAN_SG_LN256
#define TAGAN_SG_LN256 1
#endif
#if TAGAN_SG_LN256
// (one plane only: the three-plane C3 form lost its A/B -- C3 fp32 547 vs 540 ms, its LN-recomputing weight gradient
// re-reads the fp32 x six times, profiles/r5i_h256_ln_ab.txt)
// two column groups of three n-subtiles per wave: the fp32 x (and its LN1 statistics) is read by two workgroup
// columns instead of three -- 3.2M rows 3.07 -> 2.55 ms, C5 bf16 504-508 -> 500 ms (profiles/r5zd_ln256_wide_ab.txt);
// six n-subtiles in one column group spill.  =0: three groups of two.
#ifndef TAGAN_SG_LN256_WIDE
#define TAGAN_SG_LN256_WIDE 1
#endif
#if TAGAN_SG_LN256_WIDE
#define NT_LN256                                                                                             \
    , nt_cfg<256, 3, 8, 32, 1, false, true, MODE_LN_IN>(768, 1),                                                \
    nt_cfg<256, 3, 8, 32, 1, false, false, MODE_LN_IN>(768, 1)
#else
#define NT_LN256                                                                                             \
    , nt_cfg<256, 2, 8, 64, 1, false, true, MODE_LN_IN>(768, 1),                                                \
    nt_cfg<256, 2, 8, 64, 1, false, false, MODE_LN_IN>(768, 1)
#endif
#define TN_LN256 tn_cfg<768, 256, 2, 8, 3, 1, true, true>(1), tn_cfg<768, 256, 2, 8, 3, 1, false, true>(1),
#else
#define NT_LN256
#define TN_LN256
#endif
#define NT_SETLN                                                                                             \
    nt_cfg<128, 3, 8, 32, 3, false, false, MODE_LN_IN>(384, 1),                                                 \
    nt_cfg<128, 3, 8, 64, 1, false, true, MODE_LN_IN>(384, 1),                                                  \
    nt_cfg<128, 3, 8, 64, 1, false, false, MODE_LN_IN>(384, 1) NT_LN256
const NtCfg NT_TABLE[] = {
    NT_SET3,
    NT_SET1(false, false),
    NT_SET1(true, false),
    NT_SET1(true, true),
    NT_SETLN,
};
#undef NT_SETLN
#undef NT_SET3
#undef NT_SET1


const NtCfg* nt_find(int K, int N, int P, int abf, int cbf, int mode = MODE_PLAIN) {
    for (const NtCfg& c : NT_TABLE)
        if (c.K == K && c.N == N && c.P == P && c.abf == abf && c.cbf == cbf && c.mode == mode) return &c;
    return nullptr;
}

typedef void (*tn_fn)(TnArgs);
struct TnCfg {
    int N, K, P, abf, lnx;
    tn_fn fn;
    int nw, ng;
    size_t lds;
    int wg_per_cu;
};
template <int N, int K, int NSN, int NW, int NG, int P, bool ABF, bool LNX = false>
constexpr TnCfg tn_cfg(int wg_per_cu) {
    return TnCfg{N, K, P, ABF, LNX, k_sgemm_tn<N, K, NSN, NW, NG, P, ABF, NW == 4 ? 2 : 1, LNX>, NW, NG,
                 (size_t)P * 32 * ((N / NG + 16) + (K + 16)) * 2, wg_per_cu};
}
// abf = dY stored bf16 (and X too, unless lnx: X = LN(x) from the fp32 LayerNorm input)
// H = 256: one n-subtile per wave (the K = 256 accumulator row is 64 VGPRs), grid.y = N / 128 column groups.
// H = 64: 4-wave workgroups over the whole N.
// H = 256 three-plane weight gradients with two n-subtiles per wave (as TAGAN_SG_H256N2 for the NT): 12 MFMAs per
// X fragment read instead of 6 and half the column groups re-reading X -- dW_qkv 3.74 -> 3.19 ms, dW_o 1.30 -> 1.16
// ms at 1.6M rows, C3 463 -> 453 ms (profiles/r5zb_h256_tn_ab.txt); =0 restores one n-subtile
#ifndef TAGAN_SG_TN256N2
#define TAGAN_SG_TN256N2 1
#endif
#define TN_SETP(P, ABF)                                                                                      \
    tn_cfg<384, 128, 3, 8, 1, P, ABF>(1), tn_cfg<128, 128, 1, 8, 1, P, ABF>(2),                               \
    tn_cfg<768, 256, (P == 1 || TAGAN_SG_TN256N2 ? 2 : 1), 8, (P == 1 || TAGAN_SG_TN256N2 ? 3 : 6), P, ABF>(1),   \
    tn_cfg<256, 256, (P == 3 && TAGAN_SG_TN256N2 ? 2 : 1), 8, (P == 3 && TAGAN_SG_TN256N2 ? 1 : 2), P, ABF>(1),   \
    tn_cfg<192, 64, 3, 4, 1, P, ABF>(2), tn_cfg<64, 64, 1, 4, 1, P, ABF>(2)
const TnCfg TN_TABLE[] = {
    TN_SETP(3, false), TN_SETP(1, false), TN_SETP(1, true),
    tn_cfg<384, 128, 3, 8, 1, 3, false, true>(1),
    tn_cfg<384, 128, 3, 8, 1, 1, true, true>(1),
    tn_cfg<384, 128, 3, 8, 1, 1, false, true>(1),
    TN_LN256
};
#undef NT_LN256
#undef TN_LN256
#undef TN_SETP
const TnCfg* tn_find(int N, int K, int P, int abf, int lnx = 0) {
    for (const TnCfg& c : TN_TABLE)
        if (c.N == N && c.K == K && c.P == P && c.abf == abf && c.lnx == lnx) return &c;
    return nullptr;
}

// m-groups of a weight-gradient launch (grid.x): one workgroup per CU slot, each over a contiguous row range
int64_t tn_groups(int64_t M, const TnCfg* cfg) {
    const int64_t tiles = (M + 31) / 32;
    const int64_t g = (int64_t)num_cu() * cfg->wg_per_cu / cfg->ng;
    return tiles < g ? (tiles > 0 ? tiles : 1) : g;
}

struct RgCfg {
    int K, P, abf, cbf, mode, w;
    nt_fn fn;
    size_t lds;
    int n;
};
template <int K, int P, bool ABF, bool CBF, int MODE, int W = 16, int NN = 128>
constexpr RgCfg rg_cfg() {
    return RgCfg{K, P, ABF, CBF, MODE, W, k_rowgemm<K, P, ABF, CBF, MODE, W, NN>,
                 (size_t)(NN / 16) * (K / 32) * P * 64 * 16 + (size_t)(5 * NN + (MODE == MODE_LN_BWD ? W * 2 * NN : 0)) * 4,
                 NN};
}
// N = 128 only; B's planes must fit the LDS (K = 384 in fp32 would need 288 KB: k_sgemm_nt keeps that shape)
const RgCfg RG_TABLE[] = {
    rg_cfg<128, 3, false, false, MODE_LN_OUT>(), rg_cfg<128, 1, true, false, MODE_LN_OUT>(),
    rg_cfg<128, 1, false, false, MODE_LN_OUT>(),
    rg_cfg<384, 1, true, false, MODE_LN_BWD, 8>(), rg_cfg<384, 1, false, false, MODE_LN_BWD, 8>(),
#if TAGAN_SG_LN256
    // H = 256, one plane (bf16 operands): W_o's planes are 128 KB of LDS, 8 waves per CU
    rg_cfg<256, 1, true, false, MODE_LN_OUT, 8, 256>(), rg_cfg<256, 1, false, false, MODE_LN_OUT, 8, 256>(),
#endif
};

// Row-owner kernels take the LayerNorm-fused N = 128 products only.  The plain products measured faster on the
// weight-stationary k_sgemm_nt (C2 kernel stats, profiles/r3d_sgemm_table_fp32.md: fp32 K = 128 62 vs 77 us, bf16 41
// vs 46 us, bf16 K = 384 70 vs 78 us: without a row-wide epilogue the register-resident B wins), and so did the
// one-plane LN1 + QKV forward (bf16 step 5.18 vs 5.23-5.25 ms); those forms are not built.
const RgCfg* rg_find(int K, int N, int P, int abf, int cbf, int mode) {
    if (mode == MODE_PLAIN || mode == MODE_LN_IN) return nullptr;
    for (const RgCfg& c : RG_TABLE)
        if (c.n == N && c.K == K && c.P == P && c.abf == abf && c.cbf == cbf && c.mode == mode) return &c;
    return nullptr;
}

int64_t rg_groups(int64_t M, const RgCfg* cfg) {
    const int64_t tiles = (M + 15) / 16;
    int64_t gx = std::min<int64_t>(num_cu(), (tiles + cfg->w - 1) / cfg->w);
    return gx < 1 ? 1 : gx;
}

bool lds_ok(const void* fn, size_t lds);

int rg_launch(const RgCfg* cfg, const NtArgs& g, void* stream, const char* what, int64_t* groups = nullptr) {
    TAGAN_REQUIRE(lds_ok((const void*)cfg->fn, cfg->lds), TAGAN_ERR_LAUNCH, "%s: LDS attribute", what);
    const int64_t gx = rg_groups(g.M, cfg);
    if (groups) *groups = gx;
    hipLaunchKernelGGL(cfg->fn, dim3((unsigned)gx), dim3(cfg->w * 64), cfg->lds, as_stream(stream), g);
    TAGAN_CHECK_LAUNCH(what);
    return TAGAN_OK;
}

// workgroups of an NT launch along the rows (grid.x): one per CU slot, at most one per tile
int64_t nt_groups(int64_t M, const NtCfg* cfg, int gy) {
    const int64_t tiles = (M + cfg->bm - 1) / cfg->bm;
    int64_t gx = (int64_t)num_cu() * cfg->wg_per_cu / gy;
    if (gx > tiles) gx = tiles;
    return gx < 1 ? 1 : gx;
}

bool lds_ok(const void* fn, size_t lds);

int nt_launch(const NtCfg* cfg, const NtArgs& g, int N, void* stream, const char* what) {
    TAGAN_REQUIRE(lds_ok((const void*)cfg->fn, cfg->lds), TAGAN_ERR_LAUNCH, "%s: LDS attribute", what);
    const int gy = N / (cfg->nw * cfg->nsub * 16);
    const int64_t gx = nt_groups(g.M, cfg, gy);
    hipLaunchKernelGGL(cfg->fn, dim3((unsigned)gx, (unsigned)gy), dim3(cfg->nw * 64), cfg->lds, as_stream(stream), g);
    TAGAN_CHECK_LAUNCH(what);
    return TAGAN_OK;
}

bool lds_ok(const void* fn, size_t lds) {
    static const void* done[64];
    static int nd = 0;
    for (int i = 0; i < nd; ++i)
        if (done[i] == fn) return true;
    if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) return false;
    if (nd < 64) done[nd++] = fn;
    return true;
}

// split-K form of a plain fp32-output product without a kernel of its own: two K / 2 halves, the second (MODE_ACC)
// accumulating into C (K = 768 three-plane: the H = 256 QKV input gradient)
const NtCfg* nt_find_half(int K, int N, int P, int abf, int cbf, int mode = MODE_PLAIN) {
    if (cbf || K % 64 != 0 || nt_find(K, N, P, abf, cbf)) return nullptr;
    if (!nt_find(K / 2, N, P, abf, cbf, MODE_ACC)) return nullptr;
    return nt_find(K / 2, N, P, abf, cbf, mode);
}

}  // namespace
}  // namespace tagan

using namespace tagan;

extern "C" int tagan_sgemm_supported(int32_t N, int32_t K, int32_t planes, int32_t a_dtype, int32_t c_dtype) {
    const int ab = a_dtype == TAGAN_BF16, cb = c_dtype == TAGAN_BF16;
    return nt_find(K, N, planes, ab, cb) != nullptr || rg_find(K, N, planes, ab, cb, MODE_PLAIN) != nullptr ||
           nt_find_half(K, N, planes, ab, cb) != nullptr;
}

extern "C" int tagan_sgemm_tn_supported(int32_t N, int32_t K, int32_t planes, int32_t dtype) {
    return tn_find(N, K, planes, dtype == TAGAN_BF16) != nullptr;
}

extern "C" int tagan_sgemm_wprep(int32_t N, int32_t K, const float* w, int64_t ldw, int32_t kmajor, int32_t planes,
                                 void* wp, void* stream) {
    TAGAN_REQUIRE(N > 0 && K > 0 && N % 16 == 0 && K % 32 == 0, TAGAN_ERR_ARG,
                  "tagan_sgemm_wprep: N %% 16 and K %% 32 must be 0 (N=%d K=%d)", N, K);
    TAGAN_REQUIRE(planes == 1 || planes == 3, TAGAN_ERR_ARG, "tagan_sgemm_wprep: planes must be 1 or 3");
    TAGAN_REQUIRE(w && wp, TAGAN_ERR_ARG, "tagan_sgemm_wprep: null pointer");
    const int64_t total = (int64_t)(N / 16) * (K / 32) * 64;
    k_sgemm_wprep<<<(unsigned)((total + 255) / 256), 256, 0, as_stream(stream)>>>(N, K, w, ldw, kmajor, planes,
                                                                                   (uint4*)wp);
    TAGAN_CHECK_LAUNCH("tagan_sgemm_wprep");
    return TAGAN_OK;
}

extern "C" int tagan_sgemm_wprep_block(int32_t H, const float* w_qkv, int64_t ld_qkv, const float* w_o, int64_t ld_o,
                                       int32_t planes, void* wq_nt, void* wo_nt, void* wo_km, void* wq_km,
                                       void* stream) {
    TAGAN_REQUIRE(H > 0 && H % 32 == 0, TAGAN_ERR_ARG, "tagan_sgemm_wprep_block: H %% 32 must be 0 (H=%d)", H);
    TAGAN_REQUIRE(planes == 1 || planes == 3, TAGAN_ERR_ARG, "tagan_sgemm_wprep_block: planes must be 1 or 3");
    TAGAN_REQUIRE(w_qkv && w_o && wq_nt && wo_nt && wo_km && wq_km && ld_qkv >= H && ld_o >= H, TAGAN_ERR_ARG,
                  "tagan_sgemm_wprep_block: bad arguments");
    PrepJobs J;
    J.j[0] = PrepJob{3 * H, H, 0, w_qkv, ld_qkv, (uint4*)wq_nt};   // QKV forward: B = W_qkv [3H, H]
    J.j[1] = PrepJob{H, H, 0, w_o, ld_o, (uint4*)wo_nt};           // out forward: B = W_o [H, H]
    J.j[2] = PrepJob{H, H, 1, w_o, ld_o, (uint4*)wo_km};           // dC = dO·W_o: B = W_oᵀ
    J.j[3] = PrepJob{H, 3 * H, 1, w_qkv, ld_qkv, (uint4*)wq_km};   // dh = dqkv·W_qkv: B = W_qkvᵀ
    const int64_t most = (int64_t)(3 * H / 16) * (H / 32) * 64;
    k_sgemm_wprep4<<<dim3((unsigned)((most + 255) / 256), 4), 256, 0, as_stream(stream)>>>(J, planes);
    TAGAN_CHECK_LAUNCH("tagan_sgemm_wprep_block");
    return TAGAN_OK;
}

extern "C" int tagan_sgemm_nt(int32_t a_dtype, int32_t c_dtype, int64_t M, int32_t N, int32_t K, const void* a,
                              int64_t lda, const void* wp, int32_t planes, const float* bias, void* c, int64_t ldc,
                              void* stream) {
    const RgCfg* rcfg = rg_find(K, N, planes, a_dtype == TAGAN_BF16, c_dtype == TAGAN_BF16, MODE_PLAIN);
    const NtCfg* cfg = nt_find(K, N, planes, a_dtype == TAGAN_BF16, c_dtype == TAGAN_BF16);
    const NtCfg* half = (cfg || rcfg) ? nullptr : nt_find_half(K, N, planes, a_dtype == TAGAN_BF16, c_dtype == TAGAN_BF16);
    TAGAN_REQUIRE(cfg || rcfg || half, TAGAN_ERR_UNSUPPORTED,
                  "tagan_sgemm_nt: no kernel for N=%d K=%d planes=%d dtypes %d/%d", N, K, planes, a_dtype, c_dtype);
    TAGAN_REQUIRE(M >= 0 && wp, TAGAN_ERR_ARG, "tagan_sgemm_nt: bad arguments");
    if (M == 0) return TAGAN_OK;
    TAGAN_REQUIRE(a && c, TAGAN_ERR_ARG, "tagan_sgemm_nt: null operand");
    TAGAN_REQUIRE(lda >= K && ldc >= N, TAGAN_ERR_ARG, "tagan_sgemm_nt: lda %lld < K or ldc %lld < N",
                  (long long)lda, (long long)ldc);
    const int es = a_dtype == TAGAN_BF16 ? 2 : 4, ec = c_dtype == TAGAN_BF16 ? 2 : 4;
    TAGAN_REQUIRE(((uintptr_t)a % 16 == 0) && (lda * es) % 16 == 0 && ((uintptr_t)c % 8 == 0) &&
                      (ldc * ec) % 8 == 0 && (!bias || (uintptr_t)bias % 16 == 0),
                  TAGAN_ERR_ARG, "tagan_sgemm_nt: operands must be 16-byte aligned rows");
    NtArgs g{};
    g.M = M; g.a = a; g.lda = lda; g.wp = (const uint4*)wp; g.bias = bias; g.c = c; g.ldc = ldc;
    if (rcfg) return rg_launch(rcfg, g, stream, "tagan_sgemm_nt");
    if (half) {   // C = A[:, :K/2]·B[:, :K/2]ᵀ + bias, then C += A[:, K/2:]·B[:, K/2:]ᵀ
        g.kkt = K / 32;
        const int rc = nt_launch(half, g, N, stream, "tagan_sgemm_nt (first K half)");
        if (rc != TAGAN_OK) return rc;
        g.a = (const char*)a + (size_t)(K / 2) * es;
        g.bias = nullptr;
        g.kk0 = K / 64;
        return nt_launch(nt_find_half(K, N, planes, a_dtype == TAGAN_BF16, 0, MODE_ACC), g, N, stream,
                         "tagan_sgemm_nt (second K half)");
    }
    return nt_launch(cfg, g, N, stream, "tagan_sgemm_nt");
}

extern "C" int tagan_sgemm_ln_supported(int32_t H, int32_t planes, int32_t act_dtype, int32_t op) {
    const int ab = act_dtype == TAGAN_BF16;
    switch (op) {
        case 1: return nt_find(H, 3 * H, planes, 0, ab, MODE_LN_IN) && tn_find(3 * H, H, planes, ab, 1);
        case 2: return nt_find(H, H, planes, ab, 0, MODE_LN_OUT) || rg_find(H, H, planes, ab, 0, MODE_LN_OUT);
        case 3: return nt_find(3 * H, H, planes, ab, 0, MODE_LN_BWD) || rg_find(3 * H, H, planes, ab, 0, MODE_LN_BWD);
        default: return 0;
    }
}

extern "C" int tagan_sgemm_nt_ln_in(int32_t c_dtype, int64_t M, int32_t N, int32_t K, const float* x, int64_t ldx,
                                    const float* ln_g, const float* ln_b, float eps, const void* wp, int32_t planes,
                                    const float* bias, void* c, int64_t ldc, float* mean, float* rstd, void* stream) {
    const RgCfg* rcfg = rg_find(K, N, planes, 0, c_dtype == TAGAN_BF16, MODE_LN_IN);
    const NtCfg* cfg = nt_find(K, N, planes, 0, c_dtype == TAGAN_BF16, MODE_LN_IN);
    TAGAN_REQUIRE(cfg || rcfg, TAGAN_ERR_UNSUPPORTED, "tagan_sgemm_nt_ln_in: no kernel for N=%d K=%d planes=%d", N, K,
                  planes);
    TAGAN_REQUIRE(M >= 0 && wp && ln_g && ln_b, TAGAN_ERR_ARG, "tagan_sgemm_nt_ln_in: bad arguments");
    if (M == 0) return TAGAN_OK;
    TAGAN_REQUIRE(x && c && mean && rstd && ldx >= K && ldc >= N, TAGAN_ERR_ARG, "tagan_sgemm_nt_ln_in: bad operands");
    const int ec = c_dtype == TAGAN_BF16 ? 2 : 4;
    TAGAN_REQUIRE((uintptr_t)x % 16 == 0 && (ldx * 4) % 16 == 0 && (uintptr_t)c % 8 == 0 && (ldc * ec) % 8 == 0 &&
                      (!bias || (uintptr_t)bias % 16 == 0),
                  TAGAN_ERR_ARG, "tagan_sgemm_nt_ln_in: operands must be 16-byte aligned rows");
    NtArgs g{};
    g.M = M; g.a = x; g.lda = ldx; g.wp = (const uint4*)wp; g.bias = bias; g.c = c; g.ldc = ldc;
    g.ln_g = ln_g; g.ln_b = ln_b; g.eps = eps; g.mean = mean; g.rstd = rstd;
    if (rcfg) return rg_launch(rcfg, g, stream, "tagan_sgemm_nt_ln_in");
    return nt_launch(cfg, g, N, stream, "tagan_sgemm_nt_ln_in");
}

extern "C" int tagan_sgemm_nt_ln_out(int32_t a_dtype, int64_t M, int32_t H, const void* a, int64_t lda, const void* wp,
                                     int32_t planes, const float* bias, const float* res, float p_drop, uint64_t seed,
                                     const float* ln_g, const float* ln_b, float eps, const float* gs, const float* bs,
                                     float eps_s, float* s_out, float* y, float* mean, float* rstd, float* mean_s,
                                     float* rstd_s, void* stream) {
    const RgCfg* rcfg = rg_find(H, H, planes, a_dtype == TAGAN_BF16, 0, MODE_LN_OUT);
    const NtCfg* cfg = nt_find(H, H, planes, a_dtype == TAGAN_BF16, 0, MODE_LN_OUT);
    TAGAN_REQUIRE(cfg || rcfg, TAGAN_ERR_UNSUPPORTED, "tagan_sgemm_nt_ln_out: no kernel for H=%d planes=%d", H, planes);
    TAGAN_REQUIRE(M >= 0 && wp && ln_g && ln_b && p_drop >= 0.f && p_drop < 1.f && (!gs == !bs) &&
                      (!gs || (mean_s && rstd_s)),
                  TAGAN_ERR_ARG, "tagan_sgemm_nt_ln_out: bad arguments");
    if (M == 0) return TAGAN_OK;
    TAGAN_REQUIRE(a && res && s_out && y && mean && rstd && lda >= H, TAGAN_ERR_ARG, "tagan_sgemm_nt_ln_out: bad operands");
    const int es = a_dtype == TAGAN_BF16 ? 2 : 4;
    TAGAN_REQUIRE((uintptr_t)a % 16 == 0 && (lda * es) % 16 == 0 && (uintptr_t)res % 16 == 0 &&
                      (uintptr_t)s_out % 16 == 0 && (uintptr_t)y % 16 == 0 && (!bias || (uintptr_t)bias % 16 == 0),
                  TAGAN_ERR_ARG, "tagan_sgemm_nt_ln_out: operands must be 16-byte aligned rows");
    NtArgs g{};
    g.M = M; g.a = a; g.lda = lda; g.wp = (const uint4*)wp; g.bias = bias; g.c = y; g.ldc = H;
    g.ln_g = ln_g; g.ln_b = ln_b; g.eps = eps; g.mean = mean; g.rstd = rstd;
    g.res = res; g.ldr = H; g.p_drop = p_drop; g.inv_keep = 1.f / (1.f - p_drop); g.seed = seed;
    g.seed_ctr = seed_counter(); g.s_out = s_out;
    g.gs = gs; g.bs = bs; g.eps_s = eps_s; g.mean_s = mean_s; g.rstd_s = rstd_s;
    if (rcfg) return rg_launch(rcfg, g, stream, "tagan_sgemm_nt_ln_out");
    return nt_launch(cfg, g, H, stream, "tagan_sgemm_nt_ln_out");
}

extern "C" size_t tagan_sgemm_nt_ln_bwd_workspace(int64_t M, int32_t H, int32_t K) {
    int64_t g = 1;
    for (const NtCfg& c : NT_TABLE)
        if (c.mode == MODE_LN_BWD && c.N == H && c.K == K) g = std::max(g, nt_groups(M, &c, 1));
    for (const RgCfg& c : RG_TABLE)
        if (c.mode == MODE_LN_BWD && c.n == H && c.K == K) g = std::max(g, rg_groups(M, &c));
    return (size_t)g * 2 * H * sizeof(float);
}

extern "C" int tagan_sgemm_nt_ln_bwd(int32_t a_dtype, int64_t M, int32_t H, int32_t K, const void* a, int64_t lda,
                                     const void* wp, int32_t planes, const float* x, const float* mean,
                                     const float* rstd, const float* gamma, const float* dres, float* dx, float* dgamma,
                                     float* dbeta, void* ws, size_t ws_bytes, void* stream) {
    const RgCfg* rcfg = rg_find(K, H, planes, a_dtype == TAGAN_BF16, 0, MODE_LN_BWD);
    const NtCfg* cfg = nt_find(K, H, planes, a_dtype == TAGAN_BF16, 0, MODE_LN_BWD);
    TAGAN_REQUIRE(cfg || rcfg, TAGAN_ERR_UNSUPPORTED, "tagan_sgemm_nt_ln_bwd: no kernel for H=%d K=%d planes=%d", H, K,
                  planes);
    TAGAN_REQUIRE(M >= 0 && wp && gamma && dgamma && dbeta, TAGAN_ERR_ARG, "tagan_sgemm_nt_ln_bwd: bad arguments");
    TAGAN_REQUIRE(M > 0, TAGAN_ERR_ARG, "tagan_sgemm_nt_ln_bwd: M must be positive (no rows: dgamma = dbeta = 0)");
    TAGAN_REQUIRE(a && x && mean && rstd && dx && lda >= K, TAGAN_ERR_ARG, "tagan_sgemm_nt_ln_bwd: bad operands");
    const int es = a_dtype == TAGAN_BF16 ? 2 : 4;
    TAGAN_REQUIRE((uintptr_t)a % 16 == 0 && (lda * es) % 16 == 0 && (uintptr_t)x % 16 == 0 &&
                      (uintptr_t)dx % 16 == 0 && (!dres || (uintptr_t)dres % 16 == 0),
                  TAGAN_ERR_ARG, "tagan_sgemm_nt_ln_bwd: operands must be 16-byte aligned rows");
    const int64_t G = rcfg ? rg_groups(M, rcfg) : nt_groups(M, cfg, 1);
    TAGAN_REQUIRE(ws && ws_bytes >= (size_t)G * 2 * H * sizeof(float), TAGAN_ERR_ARG, "tagan_sgemm_nt_ln_bwd: workspace");
    NtArgs g{};
    g.M = M; g.a = a; g.lda = lda; g.wp = (const uint4*)wp; g.bias = nullptr; g.c = dx; g.ldc = H;
    g.ln_g = gamma; g.mean = (float*)mean; g.rstd = (float*)rstd; g.res = x; g.ldr = H; g.dres = dres;
    g.part = (float*)ws;
    const int rc = rcfg ? rg_launch(rcfg, g, stream, "tagan_sgemm_nt_ln_bwd") :
                          nt_launch(cfg, g, H, stream, "tagan_sgemm_nt_ln_bwd");
    if (rc != TAGAN_OK) return rc;
    launch_colsum((const float*)ws, (int)G, 2 * H, dgamma, dbeta, H, as_stream(stream), 1.f, 2 * H);
    TAGAN_CHECK_LAUNCH("tagan_sgemm_nt_ln_bwd_sum");
    return TAGAN_OK;
}

extern "C" size_t tagan_sgemm_tn_workspace(int64_t M, int32_t N, int32_t K) {
    // the largest over the configurations of this shape (any planes / dtype / variant)
    int64_t g = 1;
    for (const TnCfg& c : TN_TABLE)
        if (c.N == N && c.K == K) g = std::max(g, tn_groups(M, &c));
    return (size_t)g * ((size_t)N * K + N) * sizeof(float);
}

static int tn_run(int32_t dtype, int64_t M, int32_t N, int32_t K, const void* dy, int64_t ldy, const void* x,
                  int64_t ldx, int32_t planes, float* dw, int64_t lddw, float* db, void* ws, size_t ws_bytes,
                  void* stream, const float* ln_g, const float* ln_b, const float* mean, const float* rstd);

extern "C" int tagan_sgemm_tn(int32_t dtype, int64_t M, int32_t N, int32_t K, const void* dy, int64_t ldy,
                              const void* x, int64_t ldx, int32_t planes, float* dw, int64_t lddw, float* db,
                              void* ws, size_t ws_bytes, void* stream) {
    return tn_run(dtype, M, N, K, dy, ldy, x, ldx, planes, dw, lddw, db, ws, ws_bytes, stream, nullptr, nullptr,
                  nullptr, nullptr);
}

extern "C" int tagan_sgemm_tn_ln(int32_t dtype, int64_t M, int32_t N, int32_t K, const void* dy, int64_t ldy,
                                 const float* x, int64_t ldx, const float* ln_g, const float* ln_b, const float* mean,
                                 const float* rstd, int32_t planes, float* dw, int64_t lddw, float* db, void* ws,
                                 size_t ws_bytes, void* stream) {
    TAGAN_REQUIRE(ln_g && ln_b && mean && rstd, TAGAN_ERR_ARG, "tagan_sgemm_tn_ln: null LayerNorm operand");
    TAGAN_REQUIRE((uintptr_t)x % 16 == 0 && (ldx * 4) % 16 == 0, TAGAN_ERR_ARG,
                  "tagan_sgemm_tn_ln: x must be 16-byte aligned rows");
    return tn_run(dtype, M, N, K, dy, ldy, x, ldx, planes, dw, lddw, db, ws, ws_bytes, stream, ln_g, ln_b, mean, rstd);
}

static int tn_run(int32_t dtype, int64_t M, int32_t N, int32_t K, const void* dy, int64_t ldy, const void* x,
                  int64_t ldx, int32_t planes, float* dw, int64_t lddw, float* db, void* ws, size_t ws_bytes,
                  void* stream, const float* ln_g, const float* ln_b, const float* mean, const float* rstd) {
    const int lnx = ln_g != nullptr;
    const TnCfg* cfg = tn_find(N, K, planes, dtype == TAGAN_BF16, lnx);
    TAGAN_REQUIRE(cfg, TAGAN_ERR_UNSUPPORTED, "tagan_sgemm_tn: no kernel for N=%d K=%d planes=%d dtype %d", N, K,
                  planes, dtype);
    TAGAN_REQUIRE(M >= 0 && (M == 0 || (dy && x)) && (dw || db), TAGAN_ERR_ARG, "tagan_sgemm_tn: bad arguments");
    TAGAN_REQUIRE(ldy >= N && ldx >= K && (!dw || lddw >= K), TAGAN_ERR_ARG, "tagan_sgemm_tn: bad strides");
    const int es = dtype == TAGAN_BF16 ? 2 : 4;
    TAGAN_REQUIRE((uintptr_t)dy % 8 == 0 && (uintptr_t)x % 8 == 0 && (ldy * es) % 8 == 0 && (ldx * es) % 8 == 0,
                  TAGAN_ERR_ARG, "tagan_sgemm_tn: operands must be 8-byte aligned rows");
    const size_t need = tagan_sgemm_tn_workspace(M, N, K);
    TAGAN_REQUIRE(ws && ws_bytes >= need, TAGAN_ERR_ARG, "tagan_sgemm_tn: workspace %zu < %zu", ws_bytes, need);
    TAGAN_REQUIRE(lds_ok((const void*)cfg->fn, cfg->lds), TAGAN_ERR_LAUNCH, "tagan_sgemm_tn: LDS attribute");
    const int64_t G = tn_groups(M, cfg);
    const int64_t tiles = (M + 31) / 32;
    TnArgs g{M, dy, ldy, x, ldx, (tiles + G - 1) / G, (float*)ws, ln_g, ln_b, mean, rstd};
    hipLaunchKernelGGL(cfg->fn, dim3((unsigned)G, (unsigned)cfg->ng), dim3(cfg->nw * 64), cfg->lds, as_stream(stream),
                       g);
    TAGAN_CHECK_LAUNCH("tagan_sgemm_tn");
    const int L = N * K + N;
    k_sgemm_tn_reduce<<<(L + TNR_COLS - 1) / TNR_COLS, TNR_COLS * TNR_SLICES, 0, as_stream(stream)>>>(
        (const float*)ws, (int)G, N, K, dw, lddw, db);
    TAGAN_CHECK_LAUNCH("tagan_sgemm_tn_reduce");
    return TAGAN_OK;
}

// ------------------------------------------------------------------------------------------- LN2 backward + out-proj
namespace tagan {
namespace {
typedef void (*l2_fn)(L2Args);
// H = 256: one plane only (k_ln2_bwd_out256; the three-plane panel would not fit)
l2_fn l2_pick256(int planes, int abf, int skip) {
    if (planes != 1) return nullptr;
    if (abf) return skip ? k_ln2_bwd_out256<true, true> : k_ln2_bwd_out256<true, false>;
    return skip ? k_ln2_bwd_out256<false, true> : k_ln2_bwd_out256<false, false>;
}
size_t l2_lds256(int skip) {
    return (size_t)2 * 32 * (256 + 16) * 2 + (size_t)8 * (skip ? 4 : 2) * 256 * 4 + (size_t)(skip ? 2 : 1) * 256 * 4;
}
// row ranges of the H = 256 form: a multiple of 8 (the two column groups of a range share an XCD), 2 x <= the CUs
int64_t l2_groups256(int64_t M) {
    const int64_t tiles = (M + 31) / 32;
    int64_t g = num_cu() / 2;
    if (tiles < g) g = tiles;
    g = (g + 7) / 8 * 8;
    return g < 8 ? 8 : g;
}
l2_fn l2_pick(int planes, int abf, int skip) {
    if (planes == 3 && !abf) return skip ? k_ln2_bwd_out<3, false, true> : k_ln2_bwd_out<3, false, false>;
    if (planes == 1 && abf) return skip ? k_ln2_bwd_out<1, true, true> : k_ln2_bwd_out<1, true, false>;
    if (planes == 1 && !abf) return skip ? k_ln2_bwd_out<1, false, true> : k_ln2_bwd_out<1, false, false>;
    return nullptr;
}
size_t l2_lds(int planes, int skip) { return (size_t)2 * planes * 32 * (128 + 16) * 2 + (size_t)8 * (skip ? 4 : 2) * 128 * 4; }
int64_t l2_groups(int64_t M) {
    const int64_t tiles = (M + 31) / 32;
    const int64_t g = num_cu();
    return tiles < g ? (tiles > 0 ? tiles : 1) : g;
}
}  // namespace
}  // namespace tagan

extern "C" int tagan_ln2_bwd_out_supported(int32_t H, int32_t planes, int32_t act_dtype) {
    if (H == 256) return TAGAN_SG_LN2_256 && l2_pick256(planes, act_dtype == TAGAN_BF16, 0) != nullptr;
    return H == 128 && l2_pick(planes, act_dtype == TAGAN_BF16, 0) != nullptr;
}

extern "C" size_t tagan_ln2_bwd_out_workspace(int64_t M, int32_t H, int32_t skip) {
    const int64_t G = H == 256 ? l2_groups256(M) : l2_groups(M);
    return (size_t)G * ((size_t)H * H + H + (size_t)(skip ? 4 : 2) * H) * sizeof(float);
}

extern "C" int tagan_ln2_bwd_out(int32_t act_dtype, int32_t planes, int64_t M, int32_t H, const float* dy,
                                 const float* s, const float* mean, const float* rstd, const float* gamma, float p_drop,
                                 uint64_t seed, const float* xs, const float* mean_s, const float* rstd_s,
                                 const float* gamma_s, const void* c, const void* wp_km, float* dres, void* dc,
                                 float* dw_o, float* db_o, float* dgamma, float* dbeta, float* dgamma_s,
                                 float* dbeta_s, void* ws, size_t ws_bytes, void* stream) {
    const int abf = act_dtype == TAGAN_BF16, skip = xs != nullptr;
    const bool w256 = H == 256 && TAGAN_SG_LN2_256;
    const l2_fn fn = H == 128 ? l2_pick(planes, abf, skip) : w256 ? l2_pick256(planes, abf, skip) : nullptr;
    TAGAN_REQUIRE(fn, TAGAN_ERR_UNSUPPORTED, "tagan_ln2_bwd_out: no kernel for H=%d planes=%d act dtype %d", H, planes,
                  act_dtype);
    TAGAN_REQUIRE(M > 0 && dy && s && mean && rstd && gamma && c && wp_km && dres && dc && dgamma && dbeta &&
                      p_drop >= 0.f && p_drop < 1.f,
                  TAGAN_ERR_ARG, "tagan_ln2_bwd_out: bad arguments");
    TAGAN_REQUIRE(!skip || (mean_s && rstd_s && gamma_s && dgamma_s && dbeta_s), TAGAN_ERR_ARG,
                  "tagan_ln2_bwd_out: the skip LayerNorm needs its statistics, gamma and gradient outputs");
    TAGAN_REQUIRE((uintptr_t)dy % 16 == 0 && (uintptr_t)s % 16 == 0 && (uintptr_t)c % 16 == 0 &&
                      (uintptr_t)dres % 16 == 0 && (uintptr_t)dc % 16 == 0 && (!skip || (uintptr_t)xs % 16 == 0),
                  TAGAN_ERR_ARG, "tagan_ln2_bwd_out: operands must be 16-byte aligned (dense [M, H] rows)");
    const size_t need = tagan_ln2_bwd_out_workspace(M, H, skip);
    TAGAN_REQUIRE(ws && ws_bytes >= need, TAGAN_ERR_ARG, "tagan_ln2_bwd_out: workspace %zu < %zu", ws_bytes, need);
    const size_t lds = w256 ? l2_lds256(skip) : l2_lds(planes, skip);
    TAGAN_REQUIRE(lds_ok((const void*)fn, lds), TAGAN_ERR_LAUNCH, "tagan_ln2_bwd_out: LDS attribute");
    const int64_t G = w256 ? l2_groups256(M) : l2_groups(M), tiles = (M + 31) / 32;
    L2Args g{};
    g.M = M; g.tiles_per_wg = (tiles + G - 1) / G;
    g.dy = dy; g.s = s; g.mean = mean; g.rstd = rstd; g.gamma = gamma;
    g.p_drop = p_drop; g.inv_keep = 1.f / (1.f - p_drop); g.seed = seed; g.seed_ctr = seed_counter();
    g.xs = xs; g.mean_s = mean_s; g.rstd_s = rstd_s; g.gamma_s = gamma_s;
    g.c = c; g.wp = (const uint4*)wp_km; g.dres = dres; g.dc = dc;
    g.part_w = (float*)ws;
    g.part_ln = (float*)ws + (size_t)G * (H * H + H);
    hipLaunchKernelGGL(fn, dim3((unsigned)(w256 ? 2 * G : G)), dim3(512), lds, as_stream(stream), g);
    TAGAN_CHECK_LAUNCH("tagan_ln2_bwd_out");
    const int L = H * H + H;
    k_sgemm_tn_reduce<<<(L + TNR_COLS - 1) / TNR_COLS, TNR_COLS * TNR_SLICES, 0, as_stream(stream)>>>(
        g.part_w, (int)G, H, H, dw_o, H, db_o);
    TAGAN_CHECK_LAUNCH("tagan_ln2_bwd_out (dW_o reduce)");
    const int npl = skip ? 4 : 2;
    launch_colsum(g.part_ln, (int)G, 2 * H, dgamma, dbeta, H, as_stream(stream), 1.f, npl * H);
    if (skip) launch_colsum(g.part_ln + 2 * H, (int)G, 2 * H, dgamma_s, dbeta_s, H, as_stream(stream), 1.f, npl * H);
    TAGAN_CHECK_LAUNCH("tagan_ln2_bwd_out (LayerNorm sums)");
    return TAGAN_OK;
}
