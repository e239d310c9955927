// Fused projection GEMMs of the attention blocks on the gfx950 f32 matrix cores.
//
// Every attention block of the hot path (GeometricAttention.forward, geometric_attention.py:541-596;
// the temporal layer, temporal_attention.py:985-1200) is  LN1 -> QKV projection -> core ->
// out-projection -> dropout + residual + LN2.  With H = 128 every projection has K = H (or 3H) and an
// output row of H (or 3H) columns, so one workgroup can own whole rows:
//
//   * the A operand (x, the attention output, dqkv) is held in REGISTERS, 32 rows per wave: lane
//     (r, h) = (lane & 31, lane >> 5) keeps row r's columns [64h, 64h + 64) of the current 128-wide
//     K chunk (64 VGPRs);  row statistics are then one in-lane sum + one exchange with lane ^ 32,
//     which makes LN1 a free prologue of the QKV GEMM (the normalised rows never touch HBM);
//   * the weights, 128 x 128 per chunk (64 KB), are staged once per chunk in LDS (row stride 132
//     floats: conflict-free ds_read_b128 for the n-major operand, ds_read_b32 for the k-major one);
//   * v_mfma_f32_32x32x2_f32 (exact f32, 64 FLOP/clk/SIMD = the f32 peak): lane half h contributes
//     k = 64h + s at step s (a k-permutation shared by A and B, so the product is the same sum);
//     each wave keeps 4 independent 32 x 32 accumulators (one 32-row x 128-column output chunk);
//   * the accumulator layout (column = lane & 31, 16 rows per lane) holds whole output rows per wave,
//     so LN2 (forward) and LN1-backward are epilogues: row sums by DPP inside 16 lanes + one swizzle,
//     column sums (dgamma, dbeta) in-lane over the 16 rows.
//
// 256 threads (4 waves, 128 rows) and 67.6 KB of LDS per workgroup: two workgroups per CU, so one
// stages its weight chunk while the other multiplies.  fp32 storage and math (the parity mode).
#include <stdlib.h>

#include "common.cuh"

namespace tagan {
namespace {

constexpr int PG_BLK = 256;          // 4 waves
constexpr int PG_ROWS = 128;         // rows per workgroup (32 per wave)
constexpr int PG_H = 128;            // hidden width: K chunk and N chunk
constexpr int PG_LD = PG_H + 4;      // LDS row stride (floats)
constexpr size_t PG_LDS = (size_t)PG_H * PG_LD * sizeof(float);   // 67,584 B

typedef float f16v __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f16v mfma32(float a, float b, f16v c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

template <int CTRL>
__device__ __forceinline__ float dpp(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}

// Sum over the 32 lanes of a wave half (every lane of the half ends with the same value):
// quad xor1 / xor2, row_half_mirror, row_mirror (DPP), then lane ^ 16.
__device__ __forceinline__ float half_sum(float x) {
    x += dpp<0xB1>(x);
    x += dpp<0x4E>(x);
    x += dpp<0x141>(x);
    x += dpp<0x140>(x);
    x += __shfl_xor(x, 16, 64);
    return x;
}

enum { PRO_NONE = 0, PRO_LN = 1 };
enum { EPI_STORE = 0, EPI_LN_FWD = 1, EPI_LN_BWD = 2 };

struct PgArgs {
    int64_t M;
    int kch, nch;            // K and N in 128-wide chunks
    const float* a;          // A rows, row stride lda
    int64_t lda;
    const float* w;          // weights, row stride ldw: n-major [N][K] or k-major [K][N]
    int64_t ldw;
    const float* bias;       // [N] (EPI_STORE, EPI_LN_FWD) or null
    float* out;              // EPI_STORE: [M, N] (row stride ldo); EPI_LN_FWD: y; EPI_LN_BWD: dx
    int64_t ldo;
    // PRO_LN (LN1 forward folded into the A operand)
    const float* g1;
    const float* b1;
    float eps1;
    float* mean1;
    float* rstd1;
    float* h_out;            // optional LN1 output [M, ldh] (+ ones column at H when ldh >= H + 4)
    int64_t ldh;
    // EPI_LN_FWD: y = LN2(dropout(acc + bias) + res) [+ LN_s(res)]
    const float* res;
    float p_drop, inv_keep;
    uint64_t seed;
    const uint64_t* seed_ctr;   // graph-replay seed source (tagan_set_seed_counter) or null
    const float* g2;
    const float* b2;
    float eps2;
    float* s_out;
    float* mean2;
    float* rstd2;
    const float* gs;
    const float* bs;
    float eps_s;
    float* mean_s;
    float* rstd_s;
    // EPI_LN_BWD: dx = LN1ᵀ(acc) + dres  (x, mean, rstd of LN1's forward; res = x, g2 = gamma)
    const float* mean_in;
    const float* rstd_in;
    const float* dres;
    float* part;             // [gridDim.x, 2H] dgamma | dbeta partials
    int diag;                // probe only (TAGAN_PROJ_DIAG): 1 = no A loads, 2 = no epilogue (results dropped)
};

// Copy a 128 x 128 block (row stride ldw) into LDS (row stride PG_LD) with NT threads: all loads first.
template <int NT = PG_BLK>
__device__ __forceinline__ void stage_w(float* lds, const float* w, int64_t ldw) {
    constexpr int IT = PG_H * PG_H / 4 / NT;
    float4 v[IT];
#pragma unroll
    for (int i = 0; i < IT; ++i) {
        const int idx = i * NT + threadIdx.x, r = idx >> 5, c4 = (idx & 31) * 4;
        v[i] = *reinterpret_cast<const float4*>(w + (int64_t)r * ldw + c4);
    }
#pragma unroll
    for (int i = 0; i < IT; ++i) {
        const int idx = i * NT + threadIdx.x, r = idx >> 5, c4 = (idx & 31) * 4;
        *reinterpret_cast<float4*>(lds + r * PG_LD + c4) = v[i];
    }
}

// Lane (r, h): row `row` (clamped, dead rows are never stored), columns col0 + 64h + [0, 64).
__device__ __forceinline__ void load_a(float (&a)[64], const float* A, int64_t lda, int64_t row, int col0, int h) {
    const float* p = A + row * lda + col0 + 64 * h;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const float4 v = *reinterpret_cast<const float4*>(p + 4 * j);
        a[4 * j] = v.x; a[4 * j + 1] = v.y; a[4 * j + 2] = v.z; a[4 * j + 3] = v.w;
    }
}

// B fragments of 4 consecutive k-steps for the 4 column blocks: b[cb][j] = B[k = 64h + 4 s4 + j][n = 32 cb + (lane & 31)].
template <bool KMAJOR>
__device__ __forceinline__ void load_b(float (&b)[4][4], const float* bp, int s4) {
    if (!KMAJOR) {   // lds[n][k]: one ds_read_b128 per column block
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
            const float4 v = *reinterpret_cast<const float4*>(bp + cb * 32 * PG_LD + 4 * s4);
            b[cb][0] = v.x; b[cb][1] = v.y; b[cb][2] = v.z; b[cb][3] = v.w;
        }
    } else {         // lds[k][n]: ds_read_b32 per (k-step, column block)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int cb = 0; cb < 4; ++cb) b[cb][j] = bp[(4 * s4 + j) * PG_LD + cb * 32];
    }
}

__device__ __forceinline__ void mma_group(const float (&a)[64], const float (&b)[4][4], f16v (&acc)[4], int s4) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) acc[cb] = mfma32(a[4 * s4 + j], b[cb][j], acc[cb]);
}

// One 128-deep K chunk: the B fragments of the next 4 k-steps are read while the current 16 MFMAs issue
// (scheduling barriers keep the compiler from hoisting every LDS read of the chunk).
template <bool KMAJOR>
__device__ __forceinline__ void mma_chunk(const float (&a)[64], const float* lds, f16v (&acc)[4], int lane) {
    const int n = lane & 31, h = lane >> 5;
    const float* bp = KMAJOR ? lds + 64 * h * PG_LD + n : lds + n * PG_LD + 64 * h;
    float b0[4][4], b1[4][4];
    load_b<KMAJOR>(b0, bp, 0);
#pragma unroll
    for (int s4 = 0; s4 < 16; s4 += 2) {
        load_b<KMAJOR>(b1, bp, s4 + 1);
        mma_group(a, b0, acc, s4);
        __builtin_amdgcn_sched_barrier(0);
        if (s4 + 2 < 16) load_b<KMAJOR>(b0, bp, s4 + 2);
        mma_group(a, b1, acc, s4 + 1);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// LN1 over the A registers: lane (r, h) and lane (r, h ^ 1) together hold row r.
__device__ __forceinline__ void ln_prologue(float (&a)[64], const PgArgs& P, int64_t row, bool live, int h) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 64; ++j) s += a[j];
    s += __shfl_xor(s, 32, 64);
    const float mean = s / (float)PG_H;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < 64; ++j) {
        const float d = a[j] - mean;
        q += d * d;
    }
    q += __shfl_xor(q, 32, 64);
    const float rstd = 1.f / sqrtf(q / (float)PG_H + P.eps1);
    const float* g = P.g1 + 64 * h;
    const float* b = P.b1 + 64 * h;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const float4 gg = *reinterpret_cast<const float4*>(g + 4 * j);
        const float4 bb = *reinterpret_cast<const float4*>(b + 4 * j);
        a[4 * j] = (a[4 * j] - mean) * rstd * gg.x + bb.x;
        a[4 * j + 1] = (a[4 * j + 1] - mean) * rstd * gg.y + bb.y;
        a[4 * j + 2] = (a[4 * j + 2] - mean) * rstd * gg.z + bb.z;
        a[4 * j + 3] = (a[4 * j + 3] - mean) * rstd * gg.w + bb.w;
    }
    if (!live) return;
    if (h == 0) {
        P.mean1[row] = mean;
        P.rstd1[row] = rstd;
    }
    if (P.h_out) {
        float* hp = P.h_out + row * P.ldh + 64 * h;
#pragma unroll
        for (int j = 0; j < 16; ++j)
            *reinterpret_cast<float4*>(hp + 4 * j) = make_float4(a[4 * j], a[4 * j + 1], a[4 * j + 2], a[4 * j + 3]);
        if (h == 0 && P.ldh >= PG_H + 4)
            *reinterpret_cast<float4*>(P.h_out + row * P.ldh + PG_H) = make_float4(1.f, 0.f, 0.f, 0.f);
    }
}

// Accumulator register i of a 32 x 32 block holds row 8 * (i >> 2) + 4 * (lane >> 5) + (i & 3), column lane & 31.
__device__ __forceinline__ int acc_row(int i, int lane) { return 8 * (i >> 2) + 4 * (lane >> 5) + (i & 3); }

// 4 x 4 transpose inside each lane quad (DPP quad_perm xor 1, xor 2): registers x0..x3 = rows 0..3 at column
// (lane & 3) become, in lane j of the quad, row j at columns 0..3.
__device__ __forceinline__ float4 quad_transpose(float x0, float x1, float x2, float x3, int lane) {
    const bool o1 = lane & 1, o2 = lane & 2;
    float s0 = dpp<0xB1>(x0), s1 = dpp<0xB1>(x1), s2 = dpp<0xB1>(x2), s3 = dpp<0xB1>(x3);
    const float y0 = o1 ? s1 : x0, y1 = o1 ? x1 : s0, y2 = o1 ? s3 : x2, y3 = o1 ? x3 : s2;
    s0 = dpp<0x4E>(y0); s1 = dpp<0x4E>(y1); s2 = dpp<0x4E>(y2); s3 = dpp<0x4E>(y3);
    return make_float4(o2 ? s2 : y0, o2 ? s3 : y1, o2 ? y2 : s0, o2 ? y3 : s1);
}

// Sum over the 8 lanes holding one row after quad_transpose (lanes j, j+4, ..., j+28 of a wave half).
__device__ __forceinline__ float row_sum8(float x) {
    x += dpp<0x124>(x);   // row_ror:4
    x += dpp<0x128>(x);   // row_ror:8
    x += __shfl_xor(x, 16, 64);
    return x;
}

__device__ __forceinline__ float hsum4(float4 v) { return (v.x + v.y) + (v.z + v.w); }
__device__ __forceinline__ float4 ld4g(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4g(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

// Epilogue of one 32-row x 128-column output chunk nc (called with every lane of the wave active: the
// transposes and row sums read other lanes by DPP, which sees a disabled lane as zero).  After quad_transpose, lane (h, q, j) =
// (lane >> 5, (lane >> 2) & 7, lane & 3) holds v[g][cb] = row 8g + 4h + j, columns 32cb + 4q + [0, 4): every
// row is 8 lanes x 16 values, stores and residual loads are float4 (8 rows x 128 B per wave-instruction).
template <int EPI, bool SKIP>
__device__ __forceinline__ void load_res(const PgArgs& P, float4 (&rr)[4][4], int64_t row_w, int lane) {
    const int h = lane >> 5, q = (lane >> 2) & 7, j = lane & 3;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const int64_t row = row_w + 8 * g + 4 * h + j;
        const int64_t rc = row < P.M ? row : P.M - 1;
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) rr[g][cb] = ld4g(P.res + rc * PG_H + 32 * cb + 4 * q);
    }
}

template <int EPI, bool SKIP, bool PRE = false>
__device__ __forceinline__ void epilogue(const PgArgs& P, f16v (&acc)[4], int64_t row_w, int nc, int lane,
                                         float4 (&pg)[4], float4 (&pb)[4], const float4 (*pre)[4] = nullptr) {
    const int h = lane >> 5, q = (lane >> 2) & 7, j = lane & 3;
    // row group g of the transposed tile (transposed where it is used: fewer live registers)
    auto vt = [&](int g, int cb) {
        return quad_transpose(acc[cb][4 * g], acc[cb][4 * g + 1], acc[cb][4 * g + 2], acc[cb][4 * g + 3], lane);
    };
    if (EPI == EPI_STORE) {
        float4 bias[4];
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
            bias[cb] = P.bias ? ld4g(P.bias + nc * PG_H + 32 * cb + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int64_t row = row_w + 8 * g + 4 * h + j;
            float4 x[4];   // DPP reads other lanes: transpose with every lane active, then mask the stores
#pragma unroll
            for (int cb = 0; cb < 4; ++cb) x[cb] = vt(g, cb);
            if (row >= P.M) continue;
#pragma unroll
            for (int cb = 0; cb < 4; ++cb) {
                const float4 b = bias[cb];
                st4g(P.out + row * P.ldo + nc * PG_H + 32 * cb + 4 * q,
                     make_float4(x[cb].x + b.x, x[cb].y + b.y, x[cb].z + b.z, x[cb].w + b.w));
            }
        }
    } else if (EPI == EPI_LN_FWD) {
        float4 rl[4][4];   // residual rows (unless preloaded before the MMA): every load in flight together
        if (!PRE) load_res<EPI, SKIP>(P, rl, row_w, lane);
        const float4 (*rr)[4] = PRE ? pre : rl;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int64_t row = row_w + 8 * g + 4 * h + j;
            const uint32_t key = P.p_drop > 0.f ? drop_key(P.seed, (uint64_t)row) : 0u;
            float4 sv[4];
            float sum = 0.f, sum_r = 0.f;
#pragma unroll
            for (int cb = 0; cb < 4; ++cb) {
                const int col = 32 * cb + 4 * q;
                const float4 b = P.bias ? ld4g(P.bias + col) : make_float4(0.f, 0.f, 0.f, 0.f);
                const float4 vv = vt(g, cb);
                float4 o = make_float4(vv.x + b.x, vv.y + b.y, vv.z + b.z, vv.w + b.w);
                if (P.p_drop > 0.f) {
                    o.x = drop_u(key, (uint32_t)col + 0) >= P.p_drop ? o.x * P.inv_keep : 0.f;
                    o.y = drop_u(key, (uint32_t)col + 1) >= P.p_drop ? o.y * P.inv_keep : 0.f;
                    o.z = drop_u(key, (uint32_t)col + 2) >= P.p_drop ? o.z * P.inv_keep : 0.f;
                    o.w = drop_u(key, (uint32_t)col + 3) >= P.p_drop ? o.w * P.inv_keep : 0.f;
                }
                const float4 r = rr[g][cb];
                sv[cb] = make_float4(o.x + r.x, o.y + r.y, o.z + r.z, o.w + r.w);
                sum += hsum4(sv[cb]);
                sum_r += hsum4(r);
            }
            const float mean = row_sum8(sum) / (float)PG_H;
            float qq = 0.f;
#pragma unroll
            for (int cb = 0; cb < 4; ++cb) {
                const float4 d = make_float4(sv[cb].x - mean, sv[cb].y - mean, sv[cb].z - mean, sv[cb].w - mean);
                qq += (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
            }
            const float rstd = 1.f / sqrtf(row_sum8(qq) / (float)PG_H + P.eps2);
            float mean_s = 0.f, rstd_s = 0.f;
            if (SKIP) {
                mean_s = row_sum8(sum_r) / (float)PG_H;
                float qs = 0.f;
#pragma unroll
                for (int cb = 0; cb < 4; ++cb) {
                    const float4 r = rr[g][cb];
                    const float4 d = make_float4(r.x - mean_s, r.y - mean_s, r.z - mean_s, r.w - mean_s);
                    qs += (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
                }
                rstd_s = 1.f / sqrtf(row_sum8(qs) / (float)PG_H + P.eps_s);
            }
            if (row >= P.M) continue;
#pragma unroll
            for (int cb = 0; cb < 4; ++cb) {
                const int col = 32 * cb + 4 * q;
                const float4 gg = ld4g(P.g2 + col), be = ld4g(P.b2 + col), s4 = sv[cb];
                float4 y = make_float4((s4.x - mean) * rstd * gg.x + be.x, (s4.y - mean) * rstd * gg.y + be.y,
                                       (s4.z - mean) * rstd * gg.z + be.z, (s4.w - mean) * rstd * gg.w + be.w);
                if (SKIP) {
                    const float4 gs = ld4g(P.gs + col), bs = ld4g(P.bs + col), r = rr[g][cb];
                    y.x += (r.x - mean_s) * rstd_s * gs.x + bs.x;
                    y.y += (r.y - mean_s) * rstd_s * gs.y + bs.y;
                    y.z += (r.z - mean_s) * rstd_s * gs.z + bs.z;
                    y.w += (r.w - mean_s) * rstd_s * gs.w + bs.w;
                }
                st4g(P.out + row * PG_H + col, y);
                st4g(P.s_out + row * PG_H + col, s4);
            }
            if (q == 0) {
                P.mean2[row] = mean;
                P.rstd2[row] = rstd;
                if (SKIP) { P.mean_s[row] = mean_s; P.rstd_s[row] = rstd_s; }
            }
        }
    } else {   // EPI_LN_BWD: v = dh;  dx = rstd * (g - c1 * xhat - c2) + dres,  g = dh * gamma
        float4 gm[4];
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) gm[cb] = ld4g(P.g2 + 32 * cb + 4 * q);
#pragma unroll
        for (int g0 = 0; g0 < 4; g0 += 2) {   // two row groups at a time: their loads in flight together
            float4 xr[2][4], dr[2][4];
            float mr[2], sr[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int64_t row = row_w + 8 * (g0 + u) + 4 * h + j;
                const int64_t rc = row < P.M ? row : P.M - 1;
                mr[u] = P.mean_in[rc];
                sr[u] = P.rstd_in[rc];
#pragma unroll
                for (int cb = 0; cb < 4; ++cb) {
                    xr[u][cb] = ld4g(P.res + rc * PG_H + 32 * cb + 4 * q);
                    dr[u][cb] = P.dres ? ld4g(P.dres + rc * PG_H + 32 * cb + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
                }
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int g = g0 + u;
                const int64_t row = row_w + 8 * g + 4 * h + j;
                const bool live = row < P.M;
                const float m = mr[u], rs = sr[u];
                float4 xh[4], gd[4];
                float c1 = 0.f, c2 = 0.f;
#pragma unroll
                for (int cb = 0; cb < 4; ++cb) {
                    const float4 x = xr[u][cb], d = vt(g, cb), gg = gm[cb];
                    xh[cb] = make_float4((x.x - m) * rs, (x.y - m) * rs, (x.z - m) * rs, (x.w - m) * rs);
                    gd[cb] = make_float4(d.x * gg.x, d.y * gg.y, d.z * gg.z, d.w * gg.w);
                    c1 += (gd[cb].x * xh[cb].x + gd[cb].y * xh[cb].y) + (gd[cb].z * xh[cb].z + gd[cb].w * xh[cb].w);
                    c2 += hsum4(gd[cb]);
                    if (live) {
                        pg[cb].x += d.x * xh[cb].x; pg[cb].y += d.y * xh[cb].y;
                        pg[cb].z += d.z * xh[cb].z; pg[cb].w += d.w * xh[cb].w;
                        pb[cb].x += d.x; pb[cb].y += d.y; pb[cb].z += d.z; pb[cb].w += d.w;
                    }
                }
                c1 = row_sum8(c1) / (float)PG_H;
                c2 = row_sum8(c2) / (float)PG_H;
                if (!live) continue;
#pragma unroll
                for (int cb = 0; cb < 4; ++cb) {
                    const float4 e = dr[u][cb];
                    st4g(P.out + row * PG_H + 32 * cb + 4 * q,
                         make_float4(rs * (gd[cb].x - c1 * xh[cb].x - c2) + e.x,
                                     rs * (gd[cb].y - c1 * xh[cb].y - c2) + e.y,
                                     rs * (gd[cb].z - c1 * xh[cb].z - c2) + e.z,
                                     rs * (gd[cb].w - c1 * xh[cb].w - c2) + e.w));
                }
            }
        }
    }
}

// EPI_LN_BWD: column partials of the workgroup -> P.part[blk]: the 8 lanes sharing a column group (j, h), then
// the 4 waves in order.
template <int EPI>
__device__ __forceinline__ void block_partials(const PgArgs& P, float* lds, float4 (&pg)[4], float4 (&pb)[4], int w,
                                               int lane, int blk) {
    if (EPI == EPI_LN_BWD && P.part) {
        auto red = [](float x) {
            x += dpp<0xB1>(x);
            x += dpp<0x4E>(x);
            return x + __shfl_xor(x, 32, 64);
        };
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
            pg[cb] = make_float4(red(pg[cb].x), red(pg[cb].y), red(pg[cb].z), red(pg[cb].w));
            pb[cb] = make_float4(red(pb[cb].x), red(pb[cb].y), red(pb[cb].z), red(pb[cb].w));
        }
        __syncthreads();   // every wave is done with the weight chunk
        if (lane < 32 && (lane & 3) == 0) {
            const int q = lane >> 2;
#pragma unroll
            for (int cb = 0; cb < 4; ++cb) {
                st4g(lds + w * 2 * PG_H + 32 * cb + 4 * q, pg[cb]);
                st4g(lds + w * 2 * PG_H + PG_H + 32 * cb + 4 * q, pb[cb]);
            }
        }
        __syncthreads();
        const int x = threadIdx.x;   // 256 = 2H columns
        P.part[(int64_t)blk * 2 * PG_H + x] =
            (lds[x] + lds[2 * PG_H + x]) + (lds[4 * PG_H + x] + lds[6 * PG_H + x]);
    }
}


// One workgroup per 128 rows; KCH weight chunks staged per output chunk (the K = 3H input gradient).
template <int PRO, int EPI, bool KMAJOR, bool SKIP, int KCH, int NCH>
__global__ void __launch_bounds__(PG_BLK, 2) k_proj(PgArgs P) {
    TAGAN_LIVE_SEED(P);
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int lane = threadIdx.x & (WAVE - 1), w = threadIdx.x >> 6, h = lane >> 5, cl = lane & 31;
    const int64_t row_w = (int64_t)blockIdx.x * PG_ROWS + 32 * w;          // first row of this wave
    const int64_t arow = row_w + cl;                                        // this lane's A row
    const bool alive = arow < P.M;
    const int64_t arow_c = alive ? arow : P.M - 1;

    float a[64];
    load_a(a, P.a, P.lda, arow_c, 0, h);
    if (PRO == PRO_LN) ln_prologue(a, P, arow, alive, h);

    float4 pg[4], pb[4];   // EPI_LN_BWD column partials
    for (int cb = 0; cb < 4; ++cb) pg[cb] = pb[cb] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int nc = 0; nc < NCH; ++nc) {
        f16v acc[4];
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[cb][i] = 0.f;
#pragma unroll
        for (int kc = 0; kc < KCH; ++kc) {
            if (kc > 0) load_a(a, P.a, P.lda, arow_c, kc * PG_H, h);   // (kch > 1 only without a prologue)
            __syncthreads();   // the previous chunk's readers are done
            if (KMAJOR) stage_w(lds, P.w + (int64_t)kc * PG_H * P.ldw + nc * PG_H, P.ldw);
            else stage_w(lds, P.w + (int64_t)nc * PG_H * P.ldw + kc * PG_H, P.ldw);
            __syncthreads();
            mma_chunk<KMAJOR>(a, lds, acc, lane);
        }
        epilogue<EPI, SKIP>(P, acc, row_w, nc, lane, pg, pb);
    }
    block_partials<EPI>(P, lds, pg, pb, w, lane, blockIdx.x);
}

// Weight-resident persistent form (one K chunk): a workgroup stages ONE 128-column weight chunk (chunk type
// c of P.nch) once and its 4 waves then loop over 32-row panels without a barrier, so the two workgroups of
// a CU overlap one wave's loads / epilogue with the other's MFMAs.  Blocks are mapped XCD-aware: the P.nch
// workgroups sharing a slot sit on one XCD and walk the same panels (the LN1 prologue's x rows are L2 hits
// for the second and third chunk type).
template <int PRO, int EPI, bool KMAJOR, bool SKIP>
__global__ void __launch_bounds__(PG_BLK, 2) k_proj_res(PgArgs P, int nslots) {
    TAGAN_LIVE_SEED(P);
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int lane = threadIdx.x & (WAVE - 1), w = threadIdx.x >> 6, h = lane >> 5, cl = lane & 31;
    const int xcd = blockIdx.x & 7, q = blockIdx.x >> 3;
    const int nc = q % P.nch, slot = (q / P.nch) * 8 + xcd;
    if (KMAJOR) stage_w(lds, P.w + nc * PG_H, P.ldw);
    else stage_w(lds, P.w + (int64_t)nc * PG_H * P.ldw, P.ldw);
    __syncthreads();
    float4 pg[4], pb[4];
    for (int cb = 0; cb < 4; ++cb) pg[cb] = pb[cb] = make_float4(0.f, 0.f, 0.f, 0.f);
    const int64_t npanel = (P.M + 31) / 32, stride = (int64_t)nslots * 4;
    int64_t pnl = (int64_t)slot * 4 + w;
    // EPI_STORE: the next panel's A rows are loaded before this panel's MFMAs (in flight across them);
    // EPI_LN_FWD: this panel's residual rows are (the A rows then wait: registers)
    constexpr bool PF_A = EPI == EPI_STORE;
    float a[64];
    if (pnl < npanel && PF_A) load_a(a, P.a, P.lda, pnl * 32 + cl < P.M ? pnl * 32 + cl : P.M - 1, 0, h);
    for (; pnl < npanel; pnl += stride) {
        const int64_t row_w = pnl * 32, arow = row_w + cl;
        const bool alive = arow < P.M;
        float an[64];
        float4 rr[4][4];
        if (PF_A) {
            const int64_t nx = pnl + stride;
            if (nx < npanel) load_a(an, P.a, P.lda, nx * 32 + cl < P.M ? nx * 32 + cl : P.M - 1, 0, h);
        } else {
            if (EPI == EPI_LN_FWD) load_res<EPI, SKIP>(P, rr, row_w, lane);
            if (P.diag & 1) {
#pragma unroll
                for (int jj = 0; jj < 64; ++jj) a[jj] = (float)(lane + jj + (int)pnl);
            } else {
                load_a(a, P.a, P.lda, alive ? arow : P.M - 1, 0, h);
            }
        }
        if (PRO == PRO_LN) ln_prologue(a, P, arow, alive, h);
        f16v acc[4];
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[cb][i] = 0.f;
        mma_chunk<KMAJOR>(a, lds, acc, lane);
        if (P.diag & 2) {
            float t = 0.f;
#pragma unroll
            for (int cb = 0; cb < 4; ++cb)
#pragma unroll
                for (int i = 0; i < 16; ++i) t += acc[cb][i];
            if (t == 1234.5f) P.out[0] = t;
        } else if (EPI == EPI_LN_FWD) {
            epilogue<EPI, SKIP, true>(P, acc, row_w, nc, lane, pg, pb, rr);
        } else {
            epilogue<EPI, SKIP>(P, acc, row_w, nc, lane, pg, pb);
        }
        if (PF_A) {
#pragma unroll
            for (int jj = 0; jj < 64; ++jj) a[jj] = an[jj];
        }
    }
}


// Ping-pong form (one K chunk, weight-resident): 8 waves per workgroup, one workgroup per CU, two waves per
// SIMD.  Half 0 (waves 0-3) and half 1 (waves 4-7) alternate, barrier-separated, between a COMPUTE phase
// (the 256 MFMAs of one 32-row panel) and a MEMORY phase (the previous panel's epilogue: stores, LN math,
// residual loads; and the next panel's A rows + LN1 prologue), so each SIMD's matrix pipe is fed by one
// wave while its partner moves data (MI355X_MICROARCH.md: the matrix pipe is per SIMD and fully paced).
constexpr int PP_BLK = 512;

template <int PRO, int EPI, bool KMAJOR, bool SKIP>
__global__ void __launch_bounds__(PP_BLK, 1) k_proj_pp(PgArgs P, int nslots) {
    TAGAN_LIVE_SEED(P);
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int lane = threadIdx.x & (WAVE - 1), w = threadIdx.x >> 6, half = w >> 2, h = lane >> 5, cl = lane & 31;
    const int xcd = blockIdx.x & 7, q = blockIdx.x >> 3;
    const int nc = q % P.nch, slot = (q / P.nch) * 8 + xcd;
    if (KMAJOR) stage_w<PP_BLK>(lds, P.w + nc * PG_H, P.ldw);
    else stage_w<PP_BLK>(lds, P.w + (int64_t)nc * PG_H * P.ldw, P.ldw);
    float4 pg[4], pb[4];
    for (int cb = 0; cb < 4; ++cb) pg[cb] = pb[cb] = make_float4(0.f, 0.f, 0.f, 0.f);
    const int64_t npanel = (P.M + 31) / 32, stride = (int64_t)nslots * 8, first = (int64_t)slot * 8 + w;
    const int64_t nit = (npanel - (int64_t)slot * 8 + stride - 1) / stride;   // wave 0's count: the WG's max
    float a[64];
    f16v acc[4];
    int64_t acc_row = -1;   // panel row whose accumulators await their epilogue
    auto fetch = [&](int64_t pnl) {
        const int64_t arow = pnl * 32 + cl;
        const bool alive = arow < P.M;
        load_a(a, P.a, P.lda, alive ? arow : P.M - 1, 0, h);
        if (PRO == PRO_LN) ln_prologue(a, P, arow, alive, h);
    };
    if (half == 0 && first < npanel) fetch(first);
    __syncthreads();   // weights staged
    for (int64_t it = 0; it < nit; ++it) {
        const int64_t pnl = first + it * stride;
#pragma unroll 1
        for (int ph = 0; ph < 2; ++ph) {
            if (ph == half) {                     // compute
                if (pnl < npanel) {
#pragma unroll
                    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
                        for (int i = 0; i < 16; ++i) acc[cb][i] = 0.f;
                    mma_chunk<KMAJOR>(a, lds, acc, lane);
                    acc_row = pnl * 32;
                }
            } else {                              // memory
                if (acc_row >= 0) {
                    epilogue<EPI, SKIP>(P, acc, acc_row, nc, lane, pg, pb);
                    acc_row = -1;
                }
                const int64_t nx = half == 0 ? pnl + stride : pnl;
                if (nx < npanel) fetch(nx);
            }
            __syncthreads();
        }
    }
    if (acc_row >= 0) epilogue<EPI, SKIP>(P, acc, acc_row, nc, lane, pg, pb);
}

template <int PRO, int EPI, bool KMAJOR, bool SKIP, int KCH, int NCH>
hipError_t launch_proj(const PgArgs& P, hipStream_t s) {
    static bool attr = false;
    if (!attr) {   // > 64 KB of dynamic LDS per workgroup
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_proj<PRO, EPI, KMAJOR, SKIP, KCH, NCH>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)PG_LDS);
        if (e != hipSuccess) return e;
        attr = true;
    }
    const unsigned nblk = (unsigned)((P.M + PG_ROWS - 1) / PG_ROWS);
    k_proj<PRO, EPI, KMAJOR, SKIP, KCH, NCH><<<nblk, PG_BLK, PG_LDS, s>>>(P);
    return hipGetLastError();
}

int num_cus() {
    static int n = 0;
    if (!n) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
            hipSuccess || n <= 0)
            n = 256;
    }
    return n;
}

template <int PRO, int EPI, bool KMAJOR, bool SKIP>
hipError_t launch_proj_res(const PgArgs& P, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_proj_res<PRO, EPI, KMAJOR, SKIP>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)PG_LDS);
        if (e != hipSuccess) return e;
        attr = true;
    }
    // two workgroups per CU; slots = workgroups per chunk type, a multiple of 8 (one per XCD), no more than
    // the 4-panel groups there are
    const int64_t groups = (P.M + PG_ROWS - 1) / PG_ROWS;
    int nslots = (2 * num_cus() / P.nch) / 8 * 8;
    if (nslots < 8) nslots = 8;
    if (nslots > groups) nslots = (int)((groups + 7) / 8 * 8);
    static const int diag = [] { const char* e = getenv("TAGAN_PROJ_DIAG"); return e ? atoi(e) : 0; }();
    PgArgs Q = P;
    Q.diag = diag;
    k_proj_res<PRO, EPI, KMAJOR, SKIP><<<(unsigned)(nslots * P.nch), PG_BLK, PG_LDS, s>>>(Q, nslots);
    return hipGetLastError();
}

template <int PRO, int EPI, bool KMAJOR, bool SKIP>
hipError_t launch_proj_pp(const PgArgs& P, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_proj_pp<PRO, EPI, KMAJOR, SKIP>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)PG_LDS);
        if (e != hipSuccess) return e;
        attr = true;
    }
    const int64_t groups = (P.M + 255) / 256;   // 8-panel groups
    int nslots = (num_cus() / P.nch) / 8 * 8;
    if (nslots < 8) nslots = 8;
    if (nslots > groups) nslots = (int)((groups + 7) / 8 * 8);
    k_proj_pp<PRO, EPI, KMAJOR, SKIP><<<(unsigned)(nslots * P.nch), PP_BLK, PG_LDS, s>>>(P, nslots);
    return hipGetLastError();
}

// TAGAN_PROJ_RES=0 selects the one-workgroup-per-128-rows kernel for the one-chunk projections (A/B probe)
// Kernel form (TAGAN_PROJ_RES, A/B probes): 0 = one workgroup per 128 rows (every output chunk of a row block in
// one workgroup: the A rows are read once), 1 = weight-resident persistent, 2 = ping-pong; default (unset):
// form 0 for the three-chunk QKV projection, form 1 for the one-chunk kernels (fastest of the three at C2,
// tools/proj_probe.py).
int proj_form(int nch) {
    static const int v = [] { const char* e = getenv("TAGAN_PROJ_RES"); return e ? atoi(e) : -1; }();
    return v >= 0 ? v : (nch > 1 ? 0 : 1);
}

template <int PRO, int EPI, bool KMAJOR, bool SKIP>
hipError_t launch_one_chunk(const PgArgs& P, hipStream_t s) {
    const int f = proj_form(P.nch);
    if (f == 2) return launch_proj_pp<PRO, EPI, KMAJOR, SKIP>(P, s);
    if (f == 1) return launch_proj_res<PRO, EPI, KMAJOR, SKIP>(P, s);
    if (P.nch == 3) return launch_proj<PRO, EPI, KMAJOR, SKIP, 1, 3>(P, s);
    return launch_proj<PRO, EPI, KMAJOR, SKIP, 1, 1>(P, s);
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

}  // namespace
}  // namespace tagan

extern "C" {

int tagan_proj_supported(int32_t H) { return H == tagan::PG_H ? 1 : 0; }

int tagan_ln_qkv_fwd(int64_t M, int32_t H, int32_t N, const float* x, const float* gamma, const float* beta, float eps,
                     const float* w, const float* bias, float* out, int64_t ldo, float* h_out, int64_t ldh,
                     float* mean, float* rstd, void* stream) {
    using namespace tagan;
    TAGAN_REQUIRE(H == PG_H, TAGAN_ERR_UNSUPPORTED, "ln_qkv_fwd: H=%d (only %d)", H, PG_H);
    TAGAN_REQUIRE(N == 3 * PG_H, TAGAN_ERR_UNSUPPORTED, "ln_qkv_fwd: N=%d (only 3H)", N);
    TAGAN_REQUIRE(M > 0 && x && gamma && beta && w && out && mean && rstd && ldo >= N, TAGAN_ERR_ARG,
                  "ln_qkv_fwd: bad args");
    TAGAN_REQUIRE(!h_out || (ldh >= H && ldh % 4 == 0), TAGAN_ERR_ARG, "ln_qkv_fwd: ldh %lld", (long long)ldh);
    TAGAN_REQUIRE(aligned16(x) && aligned16(w) && aligned16(gamma) && aligned16(beta) && (!h_out || aligned16(h_out)),
                  TAGAN_ERR_ARG, "ln_qkv_fwd: operands must be 16-byte aligned");
    PgArgs P{};
    P.M = M; P.kch = 1; P.nch = N / PG_H; P.a = x; P.lda = H; P.w = w; P.ldw = H; P.bias = bias; P.out = out;
    P.ldo = ldo; P.g1 = gamma; P.b1 = beta; P.eps1 = eps; P.mean1 = mean; P.rstd1 = rstd; P.h_out = h_out;
    P.ldh = ldh;
    TAGAN_CHECK_HIP((launch_one_chunk<PRO_LN, EPI_STORE, false, false>(P, as_stream(stream))), "ln_qkv_fwd launch");
    return TAGAN_OK;
}

int tagan_proj_ln_fwd(int64_t M, int32_t H, const float* a, const float* w, const float* bias, const float* res,
                      float p_drop, uint64_t seed, const float* gamma, const float* beta, float eps,
                      const float* gamma_s, const float* beta_s, float eps_s, float* s_out, float* y, float* mean,
                      float* rstd, float* mean_s, float* rstd_s, void* stream) {
    using namespace tagan;
    TAGAN_REQUIRE(H == PG_H, TAGAN_ERR_UNSUPPORTED, "proj_ln_fwd: H=%d (only %d)", H, PG_H);
    TAGAN_REQUIRE(M > 0 && a && w && res && gamma && beta && s_out && y && mean && rstd, TAGAN_ERR_ARG,
                  "proj_ln_fwd: bad args");
    TAGAN_REQUIRE(p_drop >= 0.f && p_drop < 1.f, TAGAN_ERR_ARG, "proj_ln_fwd: p_drop");
    const bool skip = gamma_s != nullptr;
    TAGAN_REQUIRE(!skip || (beta_s && mean_s && rstd_s), TAGAN_ERR_ARG, "proj_ln_fwd: skip branch args");
    TAGAN_REQUIRE(aligned16(a) && aligned16(w), TAGAN_ERR_ARG, "proj_ln_fwd: operands must be 16-byte aligned");
    PgArgs P{};
    P.M = M; P.kch = 1; P.nch = 1; P.a = a; P.lda = H; P.w = w; P.ldw = H; P.bias = bias; P.out = y; P.ldo = H;
    P.res = res; P.p_drop = p_drop; P.inv_keep = 1.f / (1.f - p_drop); P.seed = seed; P.seed_ctr = seed_counter(); P.g2 = gamma; P.b2 = beta;
    P.eps2 = eps; P.s_out = s_out; P.mean2 = mean; P.rstd2 = rstd; P.gs = gamma_s; P.bs = beta_s; P.eps_s = eps_s;
    P.mean_s = mean_s; P.rstd_s = rstd_s;
    hipStream_t s = as_stream(stream);
    hipError_t e;
    e = skip ? launch_one_chunk<PRO_NONE, EPI_LN_FWD, false, true>(P, s)
             : launch_one_chunk<PRO_NONE, EPI_LN_FWD, false, false>(P, s);
    TAGAN_CHECK_HIP(e, "proj_ln_fwd launch");
    return TAGAN_OK;
}

int tagan_proj_gemm(int64_t M, int32_t H, int32_t K, const float* a, int64_t lda, const float* w, int w_kmajor,
                    float* out, int64_t ldo, void* stream) {
    using namespace tagan;
    TAGAN_REQUIRE(H == PG_H, TAGAN_ERR_UNSUPPORTED, "proj_gemm: H=%d (only %d)", H, PG_H);
    TAGAN_REQUIRE(K == PG_H || K == 3 * PG_H, TAGAN_ERR_UNSUPPORTED, "proj_gemm: K=%d (H or 3H only)", K);
    TAGAN_REQUIRE(M > 0 && a && w && out && lda >= K && lda % 4 == 0 && ldo >= H, TAGAN_ERR_ARG,
                  "proj_gemm: bad args");
    TAGAN_REQUIRE(aligned16(a) && aligned16(w), TAGAN_ERR_ARG, "proj_gemm: operands must be 16-byte aligned");
    PgArgs P{};
    P.M = M; P.kch = K / PG_H; P.nch = 1; P.a = a; P.lda = lda; P.w = w; P.ldw = w_kmajor ? H : K; P.out = out;
    P.ldo = ldo;
    hipStream_t s = as_stream(stream);
    hipError_t e;
    if (K == PG_H) e = w_kmajor ? launch_one_chunk<PRO_NONE, EPI_STORE, true, false>(P, s)
                                : launch_one_chunk<PRO_NONE, EPI_STORE, false, false>(P, s);
    else e = w_kmajor ? launch_proj<PRO_NONE, EPI_STORE, true, false, 3, 1>(P, s)
                      : launch_proj<PRO_NONE, EPI_STORE, false, false, 3, 1>(P, s);
    TAGAN_CHECK_HIP(e, "proj_gemm launch");
    return TAGAN_OK;
}

size_t tagan_proj_ln_bwd_workspace(int64_t M, int32_t H) {
    return (size_t)((M + tagan::PG_ROWS - 1) / tagan::PG_ROWS) * 2 * H * sizeof(float);
}

int tagan_proj_ln_bwd(int64_t M, int32_t H, int32_t K, const float* da, const float* w, const float* x,
                      const float* mean, const float* rstd, const float* gamma, const float* dres, float* dx,
                      float* dgamma, float* dbeta, void* workspace, size_t workspace_bytes, void* stream) {
    using namespace tagan;
    TAGAN_REQUIRE(H == PG_H, TAGAN_ERR_UNSUPPORTED, "proj_ln_bwd: H=%d (only %d)", H, PG_H);
    TAGAN_REQUIRE(K == PG_H || K == 3 * PG_H, TAGAN_ERR_UNSUPPORTED, "proj_ln_bwd: K=%d (H or 3H only)", K);
    TAGAN_REQUIRE(M > 0 && da && w && x && mean && rstd && gamma && dx, TAGAN_ERR_ARG, "proj_ln_bwd: bad args");
    const bool want = dgamma || dbeta;
    TAGAN_REQUIRE(!want || (workspace && workspace_bytes >= tagan_proj_ln_bwd_workspace(M, H)), TAGAN_ERR_WORKSPACE,
                  "proj_ln_bwd: workspace");
    TAGAN_REQUIRE(aligned16(da) && aligned16(w), TAGAN_ERR_ARG, "proj_ln_bwd: operands must be 16-byte aligned");
    PgArgs P{};
    P.M = M; P.kch = K / PG_H; P.nch = 1; P.a = da; P.lda = K; P.w = w; P.ldw = H; P.out = dx; P.ldo = H;
    P.res = x; P.mean_in = mean; P.rstd_in = rstd; P.g2 = gamma; P.dres = dres;
    P.part = want ? (float*)workspace : nullptr;
    hipStream_t s = as_stream(stream);
    TAGAN_CHECK_HIP((K == PG_H ? launch_proj<PRO_NONE, EPI_LN_BWD, true, false, 1, 1>(P, s)
                               : launch_proj<PRO_NONE, EPI_LN_BWD, true, false, 3, 1>(P, s)), "proj_ln_bwd launch");
    if (want) {
        const int nblk = (int)((M + PG_ROWS - 1) / PG_ROWS);
        launch_colsum(P.part, nblk, 2 * H, dgamma, dbeta, H, s);
        TAGAN_CHECK_LAUNCH("proj_ln_bwd_sum");
    }
    return TAGAN_OK;
}

}  // extern "C"
