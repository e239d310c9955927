// TemporalEvolutionLayer's GRU recurrence over T as ONE persistent kernel per direction (intended mode of
// TemporalPropagation): temporal_propagation.py:402-558 (TemporalGRUCell) inside the
// loop of :648-755, forward and backward (BPTT).
//
// The x-side of the three gates for all T steps is one GEMM done by the caller (gx [T, N, 3hc] = LN_x(x)·W_xᵀ
// + b).  Per step, per node row (rows are independent; T is sequential):
//   hn  = LN_h(h_{t-1}) · exp(-clamp(Δt, 0, 10))        (h_{-1} = 0 -> hn = 0: no LayerNorm, :490-493)
//   r   = σ(gx_r + W_r·hn),  z = σ(gx_z + W_z·hn)
//   h~  = tanh(gx_c + W_c·(r ⊙ hn))
//   u   = dropout((1 - z) ⊙ hn + z ⊙ h~)               (stream = row · T + t, counter = unit)
//   h_t = LN_out(u)                                     (LayerNorm eps as passed; use_layer_norm only)
// A workgroup owns R = 8·(256/hc) rows for all T steps: thread j <-> hidden unit j of its row group, the row
// states live in LDS between steps, row statistics are shuffle (+ LDS for hc > 64) reductions, the
// recurrent products are VALU dot products against W rows (fwd) / columns (bwd) streamed from L1/L2, the row
// states float4 LDS broadcasts.  For hc in {64, 128, 256} the forward is k_gru_fwd_mfma below instead.
// Saved for the backward: hn, r⊙hn, r, z, h~, u [T, N, hc] and the two LayerNorms' (mean, rstd) [T, N].
// Backward walks t = T-1..0 with dL/dh_t carried in LDS and writes dgx [T, N, 3hc] (the gate pre-activation
// gradients; the caller turns them into the W_h gradients with one GEMM each against the saved hn / r⊙hn)
// and per-workgroup LayerNorm parameter partials (ordered column sums).
#include "common.cuh"

namespace tagan {
namespace {

constexpr int GB = 256;   // threads per workgroup
constexpr int RPG = 8;    // rows per thread group (forward)
constexpr int RPB = 4;    // rows per thread group (backward: more live state per row)

struct GruArgs {
    int64_t N;
    int T, hc;
    const float* gx;                  // [T, N, 3hc]
    const float* Wrz;                 // [2hc, hc]  (W_r | W_z, the h-side columns; nn.Linear layout)
    const float* Wc;                  // [hc, hc]
    const float* gh; const float* bh; float eps_h;     // LN_h (null: no LayerNorm)
    const float* go; const float* bo; float eps_o;     // LN_out (null: no LayerNorm)
    const float* tscale;              // [T, N] exp(-clamp(Δt)) factors or null
    float p_drop, inv_keep;
    uint64_t seed;
    const uint64_t* seed_ctr;
    float* states;                    // [T, N, hc]  h_t
    float* s_hn; float* s_rh; float* s_r; float* s_z; float* s_ht; float* s_u;   // [T, N, hc]
    float* s_stat;                    // [T, N, 4]: mean_h, rstd_h, mean_o, rstd_o
    // backward
    const float* dstates;             // [T, N, hc]
    float* dgx;                       // [T, N, 3hc]
    float* part;                      // [gridDim, 4hc]: dγh | dβh | dγo | dβo
};

// Sum over the hc threads of a row group (hc <= 64: aligned lane groups; 128/256: waves + LDS).
template <int HC, int RP = RPG>
__device__ __forceinline__ void group_sum8(float (&v)[RP], float* red) {
    if (HC <= 64) {
#pragma unroll
        for (int i = 0; i < RP; ++i) v[i] = group_sum<HC>(v[i]);
    } else {
        constexpr int W = HC >= 64 ? HC / 64 : 1;   // waves per group
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
        for (int i = 0; i < RP; ++i) v[i] = wave_sum(v[i]);
        __syncthreads();
        if (lane == 0)
#pragma unroll
            for (int i = 0; i < RP; ++i) red[w * RP + i] = v[i];
        __syncthreads();
        const int g0 = (w / W) * W;
#pragma unroll
        for (int i = 0; i < RP; ++i) {
            float s = 0.f;
#pragma unroll
            for (int q = 0; q < W; ++q) s += red[(g0 + q) * RP + i];
            v[i] = s;
        }
    }
}

template <int HC>
__global__ void __launch_bounds__(GB) k_gru_fwd(GruArgs A) {
    TAGAN_LIVE_SEED(A);
    constexpr int G = GB / HC, R = G * RPG;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* hs = sm;                  // [R][HC] h_{t-1}, then hn
    float* rh = hs + R * HC;         // [R][HC] r ⊙ hn
    float* red = rh + R * HC;        // [GB/64 * RPG]
    const int j = threadIdx.x % HC, g = threadIdx.x / HC;
    const int64_t row0 = (int64_t)blockIdx.x * R + g * RPG;
    const int64_t N = A.N;
    const int T = A.T;
    for (int t = 0; t < T; ++t) {
        float hn[RPG];
        if (t == 0) {
#pragma unroll
            for (int i = 0; i < RPG; ++i) hn[i] = 0.f;
        } else {
            float hv[RPG], s[RPG], q[RPG];
#pragma unroll
            for (int i = 0; i < RPG; ++i) { hv[i] = hs[(g * RPG + i) * HC + j]; s[i] = hv[i]; }
            if (A.gh) {
                group_sum8<HC>(s, red);
#pragma unroll
                for (int i = 0; i < RPG; ++i) { s[i] /= (float)HC; q[i] = (hv[i] - s[i]) * (hv[i] - s[i]); }
                group_sum8<HC>(q, red);
            }
#pragma unroll
            for (int i = 0; i < RPG; ++i) {
                const int64_t row = row0 + i;
                const int64_t rc = row < N ? row : N - 1;
                float x = hv[i];
                float rs = 1.f;
                if (A.gh) {
                    rs = 1.f / sqrtf(q[i] / (float)HC + A.eps_h);
                    x = (x - s[i]) * rs * A.gh[j] + A.bh[j];
                }
                if (A.tscale) x *= A.tscale[(int64_t)t * N + rc];
                hn[i] = x;
                if (j == 0 && row < N) {
                    A.s_stat[((int64_t)t * N + row) * 4 + 0] = A.gh ? s[i] : 0.f;
                    A.s_stat[((int64_t)t * N + row) * 4 + 1] = rs;
                }
            }
        }
        __syncthreads();   // every thread has read h_{t-1}
#pragma unroll
        for (int i = 0; i < RPG; ++i) hs[(g * RPG + i) * HC + j] = hn[i];
        __syncthreads();
        // r, z
        float ar[RPG], az[RPG];
#pragma unroll
        for (int i = 0; i < RPG; ++i) {
            const int64_t rc = row0 + i < N ? row0 + i : N - 1;
            const float* gp = A.gx + ((int64_t)t * N + rc) * 3 * HC;
            ar[i] = gp[j];
            az[i] = gp[HC + j];
        }
        if (t > 0) {
            const float* wr = A.Wrz + (int64_t)j * HC;
            const float* wz = A.Wrz + (int64_t)(HC + j) * HC;
#pragma unroll 2
            for (int k = 0; k < HC; k += 4) {
                const float4 a = *reinterpret_cast<const float4*>(wr + k);
                const float4 b = *reinterpret_cast<const float4*>(wz + k);
#pragma unroll
                for (int i = 0; i < RPG; ++i) {
                    const float4 h = *reinterpret_cast<const float4*>(hs + (g * RPG + i) * HC + k);
                    ar[i] += (a.x * h.x + a.y * h.y) + (a.z * h.z + a.w * h.w);
                    az[i] += (b.x * h.x + b.y * h.y) + (b.z * h.z + b.w * h.w);
                }
            }
        }
        float r[RPG], z[RPG];
#pragma unroll
        for (int i = 0; i < RPG; ++i) {
            r[i] = 1.f / (1.f + expf(-ar[i]));
            z[i] = 1.f / (1.f + expf(-az[i]));
            rh[(g * RPG + i) * HC + j] = r[i] * hn[i];
        }
        __syncthreads();
        float ac[RPG];
#pragma unroll
        for (int i = 0; i < RPG; ++i) {
            const int64_t rc = row0 + i < N ? row0 + i : N - 1;
            ac[i] = A.gx[((int64_t)t * N + rc) * 3 * HC + 2 * HC + j];
        }
        if (t > 0) {
            const float* wc = A.Wc + (int64_t)j * HC;
#pragma unroll 2
            for (int k = 0; k < HC; k += 4) {
                const float4 a = *reinterpret_cast<const float4*>(wc + k);
#pragma unroll
                for (int i = 0; i < RPG; ++i) {
                    const float4 h = *reinterpret_cast<const float4*>(rh + (g * RPG + i) * HC + k);
                    ac[i] += (a.x * h.x + a.y * h.y) + (a.z * h.z + a.w * h.w);
                }
            }
        }
        float u[RPG], s[RPG], q[RPG];
#pragma unroll
        for (int i = 0; i < RPG; ++i) {
            const float ht = tanhf(ac[i]);
            float v = (1.f - z[i]) * hn[i] + z[i] * ht;
            const int64_t row = row0 + i;
            if (A.p_drop > 0.f) {
                const uint32_t key = drop_key(A.seed, (uint64_t)row * (uint64_t)T + (uint64_t)t);
                v = drop_u(key, (uint32_t)j) >= A.p_drop ? v * A.inv_keep : 0.f;
            }
            u[i] = v;
            s[i] = v;
            if (row < N) {
                const int64_t o = ((int64_t)t * N + row) * HC + j;
                A.s_hn[o] = hn[i];
                A.s_rh[o] = r[i] * hn[i];
                A.s_r[o] = r[i];
                A.s_z[o] = z[i];
                A.s_ht[o] = ht;
                A.s_u[o] = v;
            }
        }
        if (A.go) {
            group_sum8<HC>(s, red);
#pragma unroll
            for (int i = 0; i < RPG; ++i) { s[i] /= (float)HC; q[i] = (u[i] - s[i]) * (u[i] - s[i]); }
            group_sum8<HC>(q, red);
        }
        __syncthreads();   // rh / hs reads of this step are done
#pragma unroll
        for (int i = 0; i < RPG; ++i) {
            const int64_t row = row0 + i;
            float h = u[i];
            float rs = 1.f;
            if (A.go) {
                rs = 1.f / sqrtf(q[i] / (float)HC + A.eps_o);
                h = (h - s[i]) * rs * A.go[j] + A.bo[j];
            }
            hs[(g * RPG + i) * HC + j] = h;
            if (row < N) {
                A.states[((int64_t)t * N + row) * HC + j] = h;
                if (j == 0) {
                    A.s_stat[((int64_t)t * N + row) * 4 + 2] = A.go ? s[i] : 0.f;
                    A.s_stat[((int64_t)t * N + row) * 4 + 3] = rs;
                }
            }
        }
        __syncthreads();
    }
}

template <int HC>
__global__ void __launch_bounds__(GB) k_gru_bwd(GruArgs A) {
    TAGAN_LIVE_SEED(A);
    constexpr int G = GB / HC, R = G * RPB;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* da = sm;                   // [R][HC] d(pre-activation) of the gate being transposed
    float* db = da + R * HC;          // [R][HC] second gate (z) for the fused r/z transposed product
    float* red = db + R * HC;
    const int j = threadIdx.x % HC, g = threadIdx.x / HC;
    const int64_t row0 = (int64_t)blockIdx.x * R + g * RPB;
    const int64_t N = A.N;
    const int T = A.T;
    float carry[RPB];                 // dL/dh_t from step t+1
#pragma unroll
    for (int i = 0; i < RPB; ++i) carry[i] = 0.f;
    float pgh = 0.f, pbh = 0.f, pgo = 0.f, pbo = 0.f;
    const float gom = A.go ? A.go[j] : 1.f;
    const float ghm = A.gh ? A.gh[j] : 1.f;
    for (int t = T - 1; t >= 0; --t) {
        float gq[RPB], xh[RPB], c1[RPB], c2[RPB], rso[RPB];
#pragma unroll
        for (int i = 0; i < RPB; ++i) {
            const int64_t row = row0 + i;
            const int64_t rc = row < N ? row : N - 1;
            const int64_t o = ((int64_t)t * N + rc) * HC + j;
            const float gh = (row < N ? A.dstates[o] : 0.f) + carry[i];
            const float uu = A.s_u[o];
            if (A.go) {
                const float m = A.s_stat[((int64_t)t * N + rc) * 4 + 2];
                rso[i] = A.s_stat[((int64_t)t * N + rc) * 4 + 3];
                xh[i] = (uu - m) * rso[i];
                if (row < N) { pgo += gh * xh[i]; pbo += gh; }
                gq[i] = gh * gom;
                c1[i] = gq[i] * xh[i];
                c2[i] = gq[i];
            } else {
                gq[i] = gh;
            }
        }
        if (A.go) {
            group_sum8<HC, RPB>(c1, red);
            group_sum8<HC, RPB>(c2, red);
        }
        float dar[RPB], daz[RPB], dac[RPB], dhn[RPB], hn[RPB], r[RPB];
#pragma unroll
        for (int i = 0; i < RPB; ++i) {
            const int64_t row = row0 + i;
            const int64_t rc = row < N ? row : N - 1;
            const int64_t o = ((int64_t)t * N + rc) * HC + j;
            float du = A.go ? rso[i] * (gq[i] - xh[i] * c1[i] / (float)HC - c2[i] / (float)HC) : gq[i];
            if (A.p_drop > 0.f) {
                const uint32_t key = drop_key(A.seed, (uint64_t)row * (uint64_t)T + (uint64_t)t);
                du = drop_u(key, (uint32_t)j) >= A.p_drop ? du * A.inv_keep : 0.f;
            }
            hn[i] = A.s_hn[o];
            r[i] = A.s_r[o];
            const float z = A.s_z[o], ht = A.s_ht[o];
            const float dz = du * (ht - hn[i]);
            const float dht = du * z;
            dhn[i] = du * (1.f - z);
            dac[i] = dht * (1.f - ht * ht);
            daz[i] = dz * z * (1.f - z);
            if (row >= N) { dac[i] = 0.f; daz[i] = 0.f; }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < RPB; ++i) da[(g * RPB + i) * HC + j] = dac[i];
        __syncthreads();
        // d(r ⊙ hn)[k = j] = Σ_jj Wc[jj][j] dac[jj]  (t = 0: no recurrent term, hn = 0)
        if (t > 0) {
            float drh[RPB];
#pragma unroll
            for (int i = 0; i < RPB; ++i) drh[i] = 0.f;
#pragma unroll 2
            for (int jj = 0; jj < HC; jj += 4) {
                float w[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) w[q] = A.Wc[(int64_t)(jj + q) * HC + j];
#pragma unroll
                for (int i = 0; i < RPB; ++i) {
                    const float4 d = *reinterpret_cast<const float4*>(da + (g * RPB + i) * HC + jj);
                    drh[i] += (w[0] * d.x + w[1] * d.y) + (w[2] * d.z + w[3] * d.w);
                }
            }
#pragma unroll
            for (int i = 0; i < RPB; ++i) {
                const float dr = drh[i] * hn[i];
                dhn[i] += drh[i] * r[i];
                dar[i] = dr * r[i] * (1.f - r[i]);
                if (row0 + i >= N) dar[i] = 0.f;
            }
        } else {
#pragma unroll
            for (int i = 0; i < RPB; ++i) dar[i] = 0.f;   // r multiplies hn = 0: no gradient reaches ar
        }
        // dgx
#pragma unroll
        for (int i = 0; i < RPB; ++i) {
            const int64_t row = row0 + i;
            if (row < N) {
                float* gp = A.dgx + ((int64_t)t * N + row) * 3 * HC;
                gp[j] = dar[i];
                gp[HC + j] = daz[i];
                gp[2 * HC + j] = dac[i];
            }
        }
        if (t == 0) break;
        __syncthreads();
#pragma unroll
        for (int i = 0; i < RPB; ++i) {
            da[(g * RPB + i) * HC + j] = dar[i];
            db[(g * RPB + i) * HC + j] = daz[i];
        }
        __syncthreads();
        // dhn[k = j] += Σ_jj W_r[jj][j] dar[jj] + W_z[jj][j] daz[jj]
#pragma unroll 2
        for (int jj = 0; jj < HC; jj += 4) {
            float wr[4], wz[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                wr[q] = A.Wrz[(int64_t)(jj + q) * HC + j];
                wz[q] = A.Wrz[(int64_t)(HC + jj + q) * HC + j];
            }
#pragma unroll
            for (int i = 0; i < RPB; ++i) {
                const float4 d1 = *reinterpret_cast<const float4*>(da + (g * RPB + i) * HC + jj);
                const float4 d2 = *reinterpret_cast<const float4*>(db + (g * RPB + i) * HC + jj);
                dhn[i] += (wr[0] * d1.x + wr[1] * d1.y) + (wr[2] * d1.z + wr[3] * d1.w) +
                          (wz[0] * d2.x + wz[1] * d2.y) + (wz[2] * d2.z + wz[3] * d2.w);
            }
        }
        // hn = LN_h(h_{t-1}) · scale  ->  carry = dL/dh_{t-1}
        float gp2[RPB], xh2[RPB], e1[RPB], e2[RPB], rsh[RPB];
#pragma unroll
        for (int i = 0; i < RPB; ++i) {
            const int64_t row = row0 + i;
            const int64_t rc = row < N ? row : N - 1;
            float g2 = dhn[i];
            if (A.tscale) g2 *= A.tscale[(int64_t)t * N + rc];
            if (row >= N) g2 = 0.f;
            if (A.gh) {
                const float m = A.s_stat[((int64_t)t * N + rc) * 4 + 0];
                rsh[i] = A.s_stat[((int64_t)t * N + rc) * 4 + 1];
                const float hp = A.states[((int64_t)(t - 1) * N + rc) * HC + j];
                xh2[i] = (hp - m) * rsh[i];
                pgh += g2 * xh2[i];
                pbh += g2;
                gp2[i] = g2 * ghm;
                e1[i] = gp2[i] * xh2[i];
                e2[i] = gp2[i];
            } else {
                gp2[i] = g2;
            }
        }
        if (A.gh) {
            group_sum8<HC, RPB>(e1, red);
            group_sum8<HC, RPB>(e2, red);
        }
#pragma unroll
        for (int i = 0; i < RPB; ++i)
            carry[i] = A.gh ? rsh[i] * (gp2[i] - xh2[i] * e1[i] / (float)HC - e2[i] / (float)HC) : gp2[i];
    }
    if (A.part) {   // LayerNorm parameter partials of this workgroup, groups summed in order
        __syncthreads();
        float* pp = sm;
        pp[(g * 4 + 0) * HC + j] = pgh;
        pp[(g * 4 + 1) * HC + j] = pbh;
        pp[(g * 4 + 2) * HC + j] = pgo;
        pp[(g * 4 + 3) * HC + j] = pbo;
        __syncthreads();
        for (int x = threadIdx.x; x < 4 * HC; x += GB) {
            float s = 0.f;
            for (int gg = 0; gg < G; ++gg) s += pp[gg * 4 * HC + x];
            A.part[(int64_t)blockIdx.x * 4 * HC + x] = s;
        }
    }
}


// ---------------------------------------------------------------------------------------------------------
// Forward on the matrix cores (hc in {64, 128, 256}).  The VALU form above is LDS-bound: every FMA needs an
// h operand broadcast from LDS.  Here a workgroup (4 waves) owns MR = 32 node rows for all T steps and each
// step's recurrent products are small GEMMs on v_mfma_f32_16x16x4_f32 (exact fp32 products): [32 x hc] hn
// (A operand, LDS, float4 = four k) times W_rzᵀ / W_cᵀ (B operand: nn.Linear rows straight from L2, float4).
// Wave w owns hc/32 column tiles of the r|z product and hc/64 of the candidate product, for both 16-row
// tiles; the accumulators go to an LDS pre-activation tile and the gate math runs with one thread per
// (row, column) element, so gx loads and the saved-tensor stores are row-contiguous runs.
// Per step: LN_h (wave w: rows 8w..8w+7) | r|z MFMA -> pre | r, z, r⊙hn in place | candidate MFMA -> pre |
// h~, u = (1-z)·hn + z·h~ (+dropout) in place | LN_out rows -> h_t; a barrier between phases.  The saved
// tensors and statistics are those of k_gru_fwd, so the backward is shared.
// ---------------------------------------------------------------------------------------------------------
typedef float f4m __attribute__((ext_vector_type(4)));
constexpr int MR = 32;   // max rows per workgroup (MT = 1 or 2 16-row MFMA tiles; TAGAN_GRU_MR=16 picks one)

__device__ __forceinline__ f4m mfma16(float a, float b, f4m c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// LDS pitches (floats): 4m with m = 2 (mod 4) -> conflict-free float4 A-operand reads of lanes (c, g)
template <int HC> constexpr int gm_ph() { return HC + 8; }        // hs [MR][HC]
template <int HC> constexpr int gm_pp() { return 2 * HC + 8; }    // pre [MR][2HC]

// acc tiles of column tiles [nt0, nt0 + NQ) (both row tiles) -> pre[m][nt·16 + c]
template <int HC, int NQ, int MT>
__device__ __forceinline__ void gm_park(float* pre, const f4m (&acc)[MT][NQ], int nt0, int c, int g) {
    constexpr int PP = gm_pp<HC>();
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int q = 0; q < NQ; ++q)
#pragma unroll
            for (int e = 0; e < 4; ++e) pre[(mt * 16 + 4 * g + e) * PP + (nt0 + q) * 16 + c] = acc[mt][q][e];
}

// acc tiles -> T[m][nt·16 + c] for an LDS tile of pitch PT
template <int HC, int NQ, int MT, int PT>
__device__ __forceinline__ void gm_park_p(float* tile, const f4m (&acc)[MT][NQ], int nt0, int c, int g) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int q = 0; q < NQ; ++q)
#pragma unroll
            for (int e = 0; e < 4; ++e) tile[(mt * 16 + 4 * g + e) * PT + (nt0 + q) * 16 + c] = acc[mt][q][e];
}

// acc[mt][q] = A[32 x HC] (LDS, pitch PA) · W[rows (nt0 + q)·16 .. +15][0..HC)ᵀ
template <int HC, int NQ, int PA, int MT>
__device__ __forceinline__ void gm_product(const float* Als, const float* __restrict__ W, int nt0, int c, int g,
                                           f4m (&acc)[MT][NQ]) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int q = 0; q < NQ; ++q) acc[mt][q] = f4m{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
    for (int k0 = 0; k0 < HC; k0 += 16) {
        f4m a[MT], b[NQ];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) a[mt] = *(const f4m*)(Als + (mt * 16 + c) * PA + k0 + 4 * g);
#pragma unroll
        for (int q = 0; q < NQ; ++q) b[q] = *(const f4m*)(W + (int64_t)((nt0 + q) * 16 + c) * HC + k0 + 4 * g);
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                for (int q = 0; q < NQ; ++q) acc[mt][q] = mfma16(a[mt][e], b[q][e], acc[mt][q]);
    }
}

template <int HC, int MT>
__global__ void __launch_bounds__(256) k_gru_fwd_mfma(GruArgs A) {
    constexpr int RW = MT * 4;   // rows per wave in the row-wise phases
    TAGAN_LIVE_SEED(A);
    constexpr int PH = gm_ph<HC>(), PP = gm_pp<HC>(), NT = HC / 16, RZT = NT / 2, CT = NT / 4, PL = HC / 64;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* hs = sm;              // [MR][PH] h_{t-1}, then hn
    float* pre = hs + MR * PH;   // [MR][PP] gate pre-activations -> r⊙hn | z -> candidate pre-act | z -> u | z
    const int tid0 = threadIdx.x, w = tid0 >> 6;
    const int N = (int)A.N, T = A.T;
    const int row0 = blockIdx.x * (MT * 16);
    for (int t = 0; t < T; ++t) {
        // The thread index is re-derived per step behind an empty asm: otherwise every per-element row / column
        // / offset of the element loops is hoisted out of the step loop into live registers (4x the VGPRs).
        int tid = tid0;
        asm volatile("" : "+v"(tid));
        const int lane = tid & 63, c = lane & 15, g = lane >> 4;
        // per-step bases; row offsets stay 32-bit (the host guarantees N·3hc < 2^31)
        const float* gxt = A.gx + (int64_t)t * N * 3 * HC;
        const int64_t so = (int64_t)t * N * HC;
        float* sst = A.s_stat + (int64_t)t * N * 4;
        // uniform per-step bases + 32-bit element offsets (saddr + voffset addressing)
        float* const s_hn = A.s_hn + so;
        float* const s_r = A.s_r + so;
        float* const s_rh = A.s_rh + so;
        float* const s_z = A.s_z + so;
        float* const s_ht = A.s_ht + so;
        float* const s_u = A.s_u + so;
        float* const s_st = A.states + so;
        // ---- hn = LN_h(h_{t-1}) · tscale (wave w: rows 8w .. 8w+7; lane: features lane + 64q)
#pragma unroll 1
        for (int rr = 0; rr < RW; ++rr) {
            const int m = w * RW + rr, row = row0 + m;
            float v[PL];
            if (t == 0) {
#pragma unroll
                for (int q = 0; q < PL; ++q) v[q] = 0.f;
            } else {
                float s1 = 0.f;
#pragma unroll
                for (int q = 0; q < PL; ++q) { v[q] = hs[m * PH + lane + 64 * q]; s1 += v[q]; }
                float mean = 0.f, rs = 1.f;
                if (A.gh) {
                    mean = wave_sum(s1) / (float)HC;
                    float s2 = 0.f;
#pragma unroll
                    for (int q = 0; q < PL; ++q) s2 += (v[q] - mean) * (v[q] - mean);
                    rs = 1.f / sqrtf(wave_sum(s2) / (float)HC + A.eps_h);
#pragma unroll
                    for (int q = 0; q < PL; ++q) {
                        const int jj = lane + 64 * q;
                        v[q] = (v[q] - mean) * rs * A.gh[jj] + A.bh[jj];
                    }
                }
                const float sc = A.tscale ? A.tscale[(int64_t)t * N + (row < N ? row : N - 1)] : 1.f;
#pragma unroll
                for (int q = 0; q < PL; ++q) v[q] *= sc;
                if (lane == 0 && row < N) {
                    sst[row * 4 + 0] = mean;
                    sst[row * 4 + 1] = rs;
                }
            }
#pragma unroll
            for (int q = 0; q < PL; ++q) {
                hs[m * PH + lane + 64 * q] = v[q];
                if (row < N) s_hn[row * HC + lane + 64 * q] = v[q];
            }
        }
        __syncthreads();
        // ---- r | z pre-activations (zero at t = 0: h_{-1} = 0)
        {
            f4m acc[MT][RZT];
            if (t > 0) {
                gm_product<HC, RZT, PH, MT>(hs, A.Wrz, w * RZT, c, g, acc);
            } else {
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int q = 0; q < RZT; ++q) acc[mt][q] = f4m{0.f, 0.f, 0.f, 0.f};
            }
            gm_park<HC, RZT, MT>(pre, acc, w * RZT, c, g);
        }
        __syncthreads();
        // ---- r = σ(·), z = σ(·); pre[:, :HC] <- r ⊙ hn, pre[:, HC:] <- z
#pragma unroll 4
        for (int i = tid; i < MT * 16 * 2 * HC; i += 256) {
            const int m = i / (2 * HC), n = i % (2 * HC), row = row0 + m;
            const bool ok = row < N;
            const float x = pre[m * PP + n] + gxt[(ok ? row : N - 1) * 3 * HC + n];
            const float sg = 1.f / (1.f + expf(-x));
            if (n < HC) {
                const float v = sg * hs[m * PH + n];
                pre[m * PP + n] = v;
                if (ok) { s_r[row * HC + n] = sg; s_rh[row * HC + n] = v; }
            } else {
                pre[m * PP + n] = sg;
                if (ok) s_z[row * HC + n - HC] = sg;
            }
        }
        __syncthreads();
        // ---- candidate pre-activation -> pre[:, :HC] (after every wave has read r⊙hn)
        {
            f4m acc[MT][CT];
            if (t > 0) {
                gm_product<HC, CT, PP, MT>(pre, A.Wc, w * CT, c, g, acc);
            } else {
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int q = 0; q < CT; ++q) acc[mt][q] = f4m{0.f, 0.f, 0.f, 0.f};
            }
            __syncthreads();
            gm_park<HC, CT, MT>(pre, acc, w * CT, c, g);
        }
        __syncthreads();
        // ---- h~ = tanh(·), u = dropout((1 - z)·hn + z·h~) -> pre[:, :HC]
#pragma unroll 4
        for (int i = tid; i < MT * 16 * HC; i += 256) {
            const int m = i / HC, n = i % HC, row = row0 + m;
            const bool ok = row < N;
            const float ht = tanhf(pre[m * PP + n] + gxt[(ok ? row : N - 1) * 3 * HC + 2 * HC + n]);
            const float z = pre[m * PP + HC + n];
            float u = (1.f - z) * hs[m * PH + n] + z * ht;
            if (A.p_drop > 0.f) {
                const uint32_t key = drop_key(A.seed, (uint64_t)row * (uint64_t)T + (uint64_t)t);
                u = drop_u(key, (uint32_t)n) >= A.p_drop ? u * A.inv_keep : 0.f;
            }
            pre[m * PP + n] = u;
            if (ok) {
                s_ht[row * HC + n] = ht;
                s_u[row * HC + n] = u;
            }
        }
        __syncthreads();
        // ---- h_t = LN_out(u) (rows 8w .. 8w+7)
#pragma unroll 1
        for (int rr = 0; rr < RW; ++rr) {
            const int m = w * RW + rr, row = row0 + m;
            float v[PL];
            float s1 = 0.f;
#pragma unroll
            for (int q = 0; q < PL; ++q) { v[q] = pre[m * PP + lane + 64 * q]; s1 += v[q]; }
            float mean = 0.f, rs = 1.f;
            if (A.go) {
                mean = wave_sum(s1) / (float)HC;
                float s2 = 0.f;
#pragma unroll
                for (int q = 0; q < PL; ++q) s2 += (v[q] - mean) * (v[q] - mean);
                rs = 1.f / sqrtf(wave_sum(s2) / (float)HC + A.eps_o);
#pragma unroll
                for (int q = 0; q < PL; ++q) {
                    const int jj = lane + 64 * q;
                    v[q] = (v[q] - mean) * rs * A.go[jj] + A.bo[jj];
                }
            }
#pragma unroll
            for (int q = 0; q < PL; ++q) {
                hs[m * PH + lane + 64 * q] = v[q];
                if (row < N) s_st[row * HC + lane + 64 * q] = v[q];
            }
            if (lane == 0 && row < N) {
                sst[row * 4 + 2] = mean;
                sst[row * 4 + 3] = rs;
            }
        }
        __syncthreads();   // h_t rows complete before the next step's products
    }
}

// Backward on the matrix cores (same workgroup geometry as k_gru_fwd_mfma): per step, walking t = T-1 .. 0,
//   P1 rows (wave w: its RW rows, lane = features): LN_out backward, dropout, gate derivatives -> dac, daz, dhn0
//   P2 d(r⊙hn) = dac · W_c          (MFMA; B operand = W_c rows k, four scalar reads per k-quad, coalesced in c)
//   P3 rows: dar = (d(r⊙hn) ⊙ hn)·r(1-r), dhn0 += d(r⊙hn) ⊙ r
//   P4 dhn_rec = [dar | daz] · W_rz  (MFMA, K = 2hc)
//   P5 rows: LN_h backward of dhn0 + dhn_rec (times the time factor) -> dL/dh_{t-1}, kept in the dhn tile
// with a barrier after P1 .. P4.  dgx and the LayerNorm parameter partials as in k_gru_bwd (shared host code).
template <int HC, int NQ, int PA, int MT, int K>
__device__ __forceinline__ void gm_product_t(const float* Als, const float* __restrict__ W, int nt0, int c, int g,
                                             f4m (&acc)[MT][NQ]) {
    // acc[mt][q] = A[16·MT x K] (LDS, pitch PA) · W[0..K)[(nt0 + q)·16 .. +15]   (W row-major [K][HC])
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int q = 0; q < NQ; ++q) acc[mt][q] = f4m{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
    for (int k0 = 0; k0 < K; k0 += 16) {
        f4m a[MT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) a[mt] = *(const f4m*)(Als + (mt * 16 + c) * PA + k0 + 4 * g);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float b[NQ];
#pragma unroll
            for (int q = 0; q < NQ; ++q) b[q] = W[(int64_t)(k0 + 4 * g + e) * HC + (nt0 + q) * 16 + c];
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                for (int q = 0; q < NQ; ++q) acc[mt][q] = mfma16(a[mt][e], b[q], acc[mt][q]);
        }
    }
}

template <int HC> constexpr int gb_p1() { return HC + 8; }       // dac, d(r⊙hn) / dhn_rec park, dhn tiles
template <int HC> constexpr int gb_p2() { return 2 * HC + 8; }   // [dar | daz]

template <int HC, int MT>
__global__ void __launch_bounds__(256) k_gru_bwd_mfma(GruArgs A) {
    TAGAN_LIVE_SEED(A);
    constexpr int P1 = gb_p1<HC>(), P2 = gb_p2<HC>(), NT = HC / 16, CT = NT / 4, PL = HC / 64, RW = MT * 4;
    constexpr int RT = MT * 16;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* ta = sm;               // [RT][P1] dac
    float* tz = ta + RT * P1;     // [RT][P2] dar | daz
    float* td = tz + RT * P2;     // [RT][P1] d(r⊙hn), then dhn_rec
    float* th = td + RT * P1;     // [RT][P1] dhn partial; between steps dL/dh_t (the carry)
    const int tid0 = threadIdx.x, w = tid0 >> 6;
    const int N = (int)A.N, T = A.T;
    const int row0 = blockIdx.x * RT;
    float pgh[PL], pbh[PL], pgo[PL], pbo[PL];
#pragma unroll
    for (int q = 0; q < PL; ++q) pgh[q] = pbh[q] = pgo[q] = pbo[q] = 0.f;
    {   // carry = 0
        for (int i = tid0; i < RT * P1; i += 256) th[i] = 0.f;
    }
    __syncthreads();
    for (int t = T - 1; t >= 0; --t) {
        int tid = tid0;
        asm volatile("" : "+v"(tid));   // see k_gru_fwd_mfma
        const int lane = tid & 63, c = lane & 15, g = lane >> 4;
        const int64_t so = (int64_t)t * N * HC;
        const float* sst = A.s_stat + (int64_t)t * N * 4;
        float* dgt = A.dgx + (int64_t)t * N * 3 * HC;
        // ---- P1
#pragma unroll 1
        for (int rr = 0; rr < RW; ++rr) {
            const int m = w * RW + rr, row = row0 + m;
            const bool ok = row < N;
            const int rc = ok ? row : N - 1;
            float gh[PL], xh[PL], gq[PL];
            float c1 = 0.f, c2 = 0.f, rso = 1.f;
            const float mo = A.go ? sst[rc * 4 + 2] : 0.f;
            if (A.go) rso = sst[rc * 4 + 3];
#pragma unroll
            for (int q = 0; q < PL; ++q) {
                const int j = lane + 64 * q;
                gh[q] = (ok ? A.dstates[so + rc * HC + j] : 0.f) + th[m * P1 + j];
                if (A.go) {
                    xh[q] = (A.s_u[so + rc * HC + j] - mo) * rso;
                    if (ok) { pgo[q] += gh[q] * xh[q]; pbo[q] += gh[q]; }
                    gq[q] = gh[q] * A.go[j];
                    c1 += gq[q] * xh[q];
                    c2 += gq[q];
                } else {
                    gq[q] = gh[q];
                }
            }
            if (A.go) {
                c1 = wave_sum(c1);
                c2 = wave_sum(c2);
            }
#pragma unroll
            for (int q = 0; q < PL; ++q) {
                const int j = lane + 64 * q;
                float du = A.go ? rso * (gq[q] - xh[q] * c1 / (float)HC - c2 / (float)HC) : gq[q];
                if (A.p_drop > 0.f) {
                    const uint32_t key = drop_key(A.seed, (uint64_t)row * (uint64_t)T + (uint64_t)t);
                    du = drop_u(key, (uint32_t)j) >= A.p_drop ? du * A.inv_keep : 0.f;
                }
                const int o = rc * HC + j;
                const float hn = A.s_hn[so + o], z = A.s_z[so + o], ht = A.s_ht[so + o];
                const float dz = du * (ht - hn), dht = du * z;
                float dac = dht * (1.f - ht * ht), daz = dz * z * (1.f - z);
                if (!ok) { dac = 0.f; daz = 0.f; }
                ta[m * P1 + j] = dac;
                tz[m * P2 + HC + j] = daz;
                th[m * P1 + j] = du * (1.f - z);
                if (ok) {
                    dgt[row * 3 * HC + HC + j] = daz;
                    dgt[row * 3 * HC + 2 * HC + j] = dac;
                }
            }
        }
        if (t == 0) {   // r multiplies hn = 0: no gradient reaches ar, and nothing flows to h_{-1}
#pragma unroll 1
            for (int rr = 0; rr < RW; ++rr) {
                const int row = row0 + w * RW + rr;
                if (row < N)
#pragma unroll
                    for (int q = 0; q < PL; ++q) dgt[row * 3 * HC + lane + 64 * q] = 0.f;
            }
            break;
        }
        __syncthreads();
        // ---- P2: d(r⊙hn) = dac · W_c -> td
        {
            f4m acc[MT][CT];
            gm_product_t<HC, CT, P1, MT, HC>(ta, A.Wc, w * CT, c, g, acc);
            gm_park_p<HC, CT, MT, P1>(td, acc, w * CT, c, g);
        }
        __syncthreads();
        // ---- P3
#pragma unroll 1
        for (int rr = 0; rr < RW; ++rr) {
            const int m = w * RW + rr, row = row0 + m;
            const bool ok = row < N;
            const int rc = ok ? row : N - 1;
#pragma unroll
            for (int q = 0; q < PL; ++q) {
                const int j = lane + 64 * q;
                const float drh = td[m * P1 + j];
                const float hn = A.s_hn[so + rc * HC + j], r = A.s_r[so + rc * HC + j];
                th[m * P1 + j] += drh * r;
                const float dar = ok ? drh * hn * r * (1.f - r) : 0.f;
                tz[m * P2 + j] = dar;
                if (ok) dgt[row * 3 * HC + j] = dar;
            }
        }
        __syncthreads();
        // ---- P4: dhn_rec = [dar | daz] · W_rz -> td
        {
            f4m acc[MT][CT];
            gm_product_t<HC, CT, P2, MT, 2 * HC>(tz, A.Wrz, w * CT, c, g, acc);
            gm_park_p<HC, CT, MT, P1>(td, acc, w * CT, c, g);
        }
        __syncthreads();
        // ---- P5: LN_h backward -> carry (in th)
        const float* stp = A.states + (int64_t)(t - 1) * N * HC;
#pragma unroll 1
        for (int rr = 0; rr < RW; ++rr) {
            const int m = w * RW + rr, row = row0 + m;
            const bool ok = row < N;
            const int rc = ok ? row : N - 1;
            const float sc = A.tscale ? A.tscale[(int64_t)t * N + rc] : 1.f;
            float g2[PL], xh2[PL], gp2[PL];
            float e1 = 0.f, e2 = 0.f, rsh = 1.f;
            const float mh = A.gh ? sst[rc * 4 + 0] : 0.f;
            if (A.gh) rsh = sst[rc * 4 + 1];
#pragma unroll
            for (int q = 0; q < PL; ++q) {
                const int j = lane + 64 * q;
                g2[q] = ok ? (th[m * P1 + j] + td[m * P1 + j]) * sc : 0.f;
                if (A.gh) {
                    xh2[q] = (stp[rc * HC + j] - mh) * rsh;
                    pgh[q] += g2[q] * xh2[q];
                    pbh[q] += g2[q];
                    gp2[q] = g2[q] * A.gh[j];
                    e1 += gp2[q] * xh2[q];
                    e2 += gp2[q];
                } else {
                    gp2[q] = g2[q];
                }
            }
            if (A.gh) {
                e1 = wave_sum(e1);
                e2 = wave_sum(e2);
            }
#pragma unroll
            for (int q = 0; q < PL; ++q) {
                const int j = lane + 64 * q;
                th[m * P1 + j] = A.gh ? rsh * (gp2[q] - xh2[q] * e1 / (float)HC - e2 / (float)HC) : gp2[q];
            }
        }
        // the next step's P1 reads only this wave's rows of th; its MFMAs wait for the barrier after it
    }
    if (A.part) {   // LayerNorm parameter partials: the four waves in order
        __syncthreads();
        float* pp = sm;   // [4 waves][4][HC]
#pragma unroll
        for (int q = 0; q < PL; ++q) {
            const int j = (tid0 & 63) + 64 * q;
            pp[(w * 4 + 0) * HC + j] = pgh[q];
            pp[(w * 4 + 1) * HC + j] = pbh[q];
            pp[(w * 4 + 2) * HC + j] = pgo[q];
            pp[(w * 4 + 3) * HC + j] = pbo[q];
        }
        __syncthreads();
        for (int x = tid0; x < 4 * HC; x += 256) {
            float sum = 0.f;
            for (int ww = 0; ww < 4; ++ww) sum += pp[ww * 4 * HC + x];
            A.part[(int64_t)blockIdx.x * 4 * HC + x] = sum;
        }
    }
}

size_t gru_bwd_mfma_lds(int hc, int mt) { return (size_t)mt * 16 * (3 * (hc + 8) + (2 * hc + 8)) * sizeof(float); }

size_t gru_mfma_lds(int hc) { return (size_t)MR * ((hc + 8) + (2 * hc + 8)) * sizeof(float); }

int gru_mfma_optin(int hc) {
    static bool done[3] = {false, false, false};
    const int idx = hc == 64 ? 0 : hc == 128 ? 1 : 2;
    const size_t lds = gru_mfma_lds(hc);
    if (done[idx] || lds <= 64 * 1024) return TAGAN_OK;
    const void* k1 = hc == 64 ? reinterpret_cast<const void*>(&k_gru_fwd_mfma<64, 1>)
                   : hc == 128 ? reinterpret_cast<const void*>(&k_gru_fwd_mfma<128, 1>)
                               : reinterpret_cast<const void*>(&k_gru_fwd_mfma<256, 1>);
    const void* k2 = hc == 64 ? reinterpret_cast<const void*>(&k_gru_fwd_mfma<64, 2>)
                   : hc == 128 ? reinterpret_cast<const void*>(&k_gru_fwd_mfma<128, 2>)
                               : reinterpret_cast<const void*>(&k_gru_fwd_mfma<256, 2>);
    hipError_t e = hipFuncSetAttribute(k1, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e == hipSuccess) e = hipFuncSetAttribute(k2, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    TAGAN_REQUIRE(e == hipSuccess, TAGAN_ERR_LAUNCH, "gru_fwd_mfma: LDS opt-in");
    done[idx] = true;
    return TAGAN_OK;
}

// Rows per workgroup of the matrix-core kernels: 16 while that still leaves < 2 workgroups per CU at 32 (more
// of them in flight: C2's 10k rows 3.58 -> 3.00 ms intended forward), 32 above (halves the weight reads from
// L2).
int gru_mfma_rows(int64_t N, bool bwd = false) {
    // the backward measured faster at 16 at every size (C4: 211 vs 264 ms, profiles/r2_gru_mfma_ab.txt)
    return (bwd || N <= 32 * 512) ? 16 : 32;
}

// the VALU kernels take the other widths (hc 16 / 32)
bool gru_mfma_ok(int hc, int64_t N) {
    return (hc == 64 || hc == 128 || hc == 256) && N * 3 * hc < ((int64_t)1 << 31);   // 32-bit row offsets
}

size_t gru_lds(int hc) { return (size_t)(2 * 8 * GB + (GB / 64) * RPG) * sizeof(float); }   // 2·R·hc = 2·8·256

template <bool FWD>
int launch_gru(const GruArgs& A, hipStream_t s, unsigned nblk) {
    const size_t lds = gru_lds(A.hc);
#define TAGAN_GRU(HCV) \
    (FWD ? k_gru_fwd<HCV> : k_gru_bwd<HCV>)<<<nblk, GB, lds, s>>>(A)
    switch (A.hc) {
        case 16: TAGAN_GRU(16); break;
        case 32: TAGAN_GRU(32); break;
        case 64: TAGAN_GRU(64); break;
        case 128: TAGAN_GRU(128); break;
        case 256: TAGAN_GRU(256); break;
        default: return TAGAN_ERR_UNSUPPORTED;
    }
#undef TAGAN_GRU
    return TAGAN_OK;
}

unsigned gru_blocks(int64_t N, int hc, int rows = RPG) {
    const int R = (GB / hc) * rows;
    return (unsigned)((N + R - 1) / R);
}

}  // namespace
}  // namespace tagan

extern "C" {

int tagan_gru_supported(int32_t hc) { return (hc == 16 || hc == 32 || hc == 64 || hc == 128 || hc == 256) ? 1 : 0; }

int tagan_gru_fwd(int64_t N, int32_t T, int32_t hc, const float* gx, const float* Wrz, const float* Wc,
                  const float* ln_h_w, const float* ln_h_b, float eps_h, const float* ln_o_w, const float* ln_o_b,
                  float eps_o, const float* tscale, float p_drop, uint64_t seed, float* states, float* saved,
                  void* stream) {
    using namespace tagan;
    TAGAN_REQUIRE(tagan_gru_supported(hc), TAGAN_ERR_UNSUPPORTED, "gru: hc=%d", hc);
    TAGAN_REQUIRE(N > 0 && T > 0 && gx && Wrz && Wc && states && saved, TAGAN_ERR_ARG, "gru_fwd: bad args");
    TAGAN_REQUIRE(p_drop >= 0.f && p_drop < 1.f, TAGAN_ERR_ARG, "gru_fwd: p_drop");
    GruArgs A{};
    A.N = N; A.T = T; A.hc = hc; A.gx = gx; A.Wrz = Wrz; A.Wc = Wc; A.gh = ln_h_w; A.bh = ln_h_b; A.eps_h = eps_h;
    A.go = ln_o_w; A.bo = ln_o_b; A.eps_o = eps_o; A.tscale = tscale; A.p_drop = p_drop;
    A.inv_keep = 1.f / (1.f - p_drop); A.seed = seed; A.seed_ctr = seed_counter(); A.states = states;
    const int64_t S = (int64_t)T * N * hc;
    A.s_hn = saved; A.s_rh = saved + S; A.s_r = saved + 2 * S; A.s_z = saved + 3 * S; A.s_ht = saved + 4 * S;
    A.s_u = saved + 5 * S; A.s_stat = saved + 6 * S;
    hipStream_t s = as_stream(stream);
    if (gru_mfma_ok(hc, N)) {
        if (int rc = gru_mfma_optin(hc)) return rc;
        const int mr = gru_mfma_rows(N);
        const unsigned nb = (unsigned)((N + mr - 1) / mr);
        const size_t lds = gru_mfma_lds(hc);
#define TAGAN_GRUM(H) { if (mr == 16) k_gru_fwd_mfma<H, 1><<<nb, 256, lds, s>>>(A); \
                        else k_gru_fwd_mfma<H, 2><<<nb, 256, lds, s>>>(A); }
        if (hc == 64) TAGAN_GRUM(64) else if (hc == 128) TAGAN_GRUM(128) else TAGAN_GRUM(256)
#undef TAGAN_GRUM
        TAGAN_CHECK_LAUNCH("gru_fwd_mfma");
        return TAGAN_OK;
    }
    TAGAN_REQUIRE(launch_gru<true>(A, s, gru_blocks(N, hc)) == TAGAN_OK, TAGAN_ERR_UNSUPPORTED, "gru_fwd: hc");
    TAGAN_CHECK_LAUNCH("gru_fwd");
    return TAGAN_OK;
}

size_t tagan_gru_saved_floats(int64_t N, int32_t T, int32_t hc) { return (size_t)T * N * (6 * (size_t)hc + 4); }

size_t tagan_gru_bwd_workspace(int64_t N, int32_t hc) {
    return (size_t)tagan::gru_blocks(N, hc, tagan::RPB) * 4 * hc * sizeof(float);
}

int tagan_gru_bwd(int64_t N, int32_t T, int32_t hc, const float* Wrz, const float* Wc, const float* ln_h_w,
                  const float* ln_h_b, const float* ln_o_w, const float* ln_o_b, const float* tscale, float p_drop,
                  uint64_t seed, const float* states, const float* saved, const float* dstates, float* dgx,
                  float* dln_h_w, float* dln_h_b, float* dln_o_w, float* dln_o_b, void* workspace,
                  size_t workspace_bytes, void* stream) {
    using namespace tagan;
    TAGAN_REQUIRE(tagan_gru_supported(hc), TAGAN_ERR_UNSUPPORTED, "gru: hc=%d", hc);
    TAGAN_REQUIRE(N > 0 && T > 0 && Wrz && Wc && states && saved && dstates && dgx, TAGAN_ERR_ARG,
                  "gru_bwd: bad args");
    const bool want = ln_h_w || ln_o_w;
    TAGAN_REQUIRE(!want || (workspace && workspace_bytes >= tagan_gru_bwd_workspace(N, hc)), TAGAN_ERR_WORKSPACE,
                  "gru_bwd: workspace");
    GruArgs A{};
    A.N = N; A.T = T; A.hc = hc; A.Wrz = Wrz; A.Wc = Wc; A.gh = ln_h_w; A.bh = ln_h_b; A.go = ln_o_w; A.bo = ln_o_b;
    A.tscale = tscale; A.p_drop = p_drop; A.inv_keep = 1.f / (1.f - p_drop); A.seed = seed;
    A.seed_ctr = seed_counter(); A.states = (float*)states;
    const int64_t S = (int64_t)T * N * hc;
    float* sv = (float*)saved;
    A.s_hn = sv; A.s_rh = sv + S; A.s_r = sv + 2 * S; A.s_z = sv + 3 * S; A.s_ht = sv + 4 * S; A.s_u = sv + 5 * S;
    A.s_stat = sv + 6 * S;
    A.dstates = dstates; A.dgx = dgx; A.part = want ? (float*)workspace : nullptr;
    hipStream_t s = as_stream(stream);
    unsigned nblk;
    if (gru_mfma_ok(hc, N)) {
        int mr = gru_mfma_rows(N, true);
        if (gru_bwd_mfma_lds(hc, mr / 16) > 160 * 1024) mr = 16;
        nblk = (unsigned)((N + mr - 1) / mr);   // <= gru_blocks(N, hc, RPB): the workspace rows
        const size_t lds = gru_bwd_mfma_lds(hc, mr / 16);
#define TAGAN_GRUB(H, M) { auto kern = k_gru_bwd_mfma<H, M>; \
        if (lds > 64 * 1024) { hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), \
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
                               TAGAN_REQUIRE(e == hipSuccess, TAGAN_ERR_LAUNCH, "gru_bwd_mfma: LDS opt-in"); } \
        kern<<<nblk, 256, lds, s>>>(A); }
        if (mr == 16) {
            if (hc == 64) TAGAN_GRUB(64, 1) else if (hc == 128) TAGAN_GRUB(128, 1) else TAGAN_GRUB(256, 1)
        } else {
            if (hc == 64) TAGAN_GRUB(64, 2) else if (hc == 128) TAGAN_GRUB(128, 2) else TAGAN_GRUB(256, 2)
        }
#undef TAGAN_GRUB
        TAGAN_CHECK_LAUNCH("gru_bwd_mfma");
    } else {
        nblk = gru_blocks(N, hc, RPB);
        TAGAN_REQUIRE(launch_gru<false>(A, s, nblk) == TAGAN_OK, TAGAN_ERR_UNSUPPORTED, "gru_bwd: hc");
        TAGAN_CHECK_LAUNCH("gru_bwd");
    }
    if (want) {
        launch_colsum(A.part, (int)nblk, 2 * hc, dln_h_w, dln_h_b, hc, s, 1.f, 4 * hc);
        launch_colsum(A.part + 2 * hc, (int)nblk, 2 * hc, dln_o_w, dln_o_b, hc, s, 1.f, 4 * hc);
        TAGAN_CHECK_LAUNCH("gru_bwd_sum");
    }
    return TAGAN_OK;
}

}  // extern "C"
