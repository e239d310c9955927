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
// recurrent products are VALU dot products with the weights streamed from L1/L2 as coalesced runs: the forward
// takes them k-major (Wᵀ: at fixed k the threads j read consecutive words), the backward in nn.Linear layout
// (its transposed product reads columns, consecutive words again); row states are float4 LDS broadcasts.
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
    const float* Wrz;                 // fwd: [hc, 2hc] k-major (W_r | W_z)ᵀ; bwd: [2hc, hc] (nn.Linear layout)
    const float* Wc;                  // fwd: [hc, hc] k-major W_cᵀ; bwd: [hc, hc]
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
            // k-major weights: at fixed k the HC threads read one contiguous run (coalesced), the row states come
            // from LDS as float4 broadcasts
#pragma unroll 2
            for (int k = 0; k < HC; k += 4) {
                float a[4], b[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    a[q] = A.Wrz[(int64_t)(k + q) * 2 * HC + j];
                    b[q] = A.Wrz[(int64_t)(k + q) * 2 * HC + HC + j];
                }
#pragma unroll
                for (int i = 0; i < RPG; ++i) {
                    const float4 h = *reinterpret_cast<const float4*>(hs + (g * RPG + i) * HC + k);
                    ar[i] += (a[0] * h.x + a[1] * h.y) + (a[2] * h.z + a[3] * h.w);
                    az[i] += (b[0] * h.x + b[1] * h.y) + (b[2] * h.z + b[3] * h.w);
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
#pragma unroll 2
            for (int k = 0; k < HC; k += 4) {
                float a[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) a[q] = A.Wc[(int64_t)(k + q) * HC + j];
#pragma unroll
                for (int i = 0; i < RPG; ++i) {
                    const float4 h = *reinterpret_cast<const float4*>(rh + (g * RPG + i) * HC + k);
                    ac[i] += (a[0] * h.x + a[1] * h.y) + (a[2] * h.z + a[3] * h.w);
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
    const unsigned nblk = gru_blocks(N, hc, RPB);
    TAGAN_REQUIRE(launch_gru<false>(A, s, nblk) == TAGAN_OK, TAGAN_ERR_UNSUPPORTED, "gru_bwd: hc");
    TAGAN_CHECK_LAUNCH("gru_bwd");
    if (want) {
        launch_colsum(A.part, (int)nblk, 2 * hc, dln_h_w, dln_h_b, hc, s, 1.f, 4 * hc);
        launch_colsum(A.part + 2 * hc, (int)nblk, 2 * hc, dln_o_w, dln_o_b, hc, s, 1.f, 4 * hc);
        TAGAN_CHECK_LAUNCH("gru_bwd_sum");
    }
    return TAGAN_OK;
}

}  // extern "C"
