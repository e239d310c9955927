// Fused classification head + loss of TAGAN (model.py:377-459, classification.py:856-966) on gfx950.
//
// graph_features [B, T, H] (row 0 = the pooled snapshot means, rows 1..B-1 all zero: model.py:382-394)
//   -> attention pooling over T:  s_t = w2 · tanh(W1 x_t + b1),  a = softmax_t(s),  p = Σ_t a_t x_t
//   -> Linear(H, H) -> LayerNorm -> ReLU -> Dropout -> Linear(H, C)  = logits [B, C]
//   -> predictions (sigmoid for C = 1, softmax otherwise) and the loss: BCE-with-logits mean over the
//      B·C elements (TemporalLossModule's default, classification.py:453-456) or cross entropy over B
//      rows (model.py:439-441).
// The reference runs this as ~25 ATen launches forward and ~40 backward on [1..B, 32, 128] tensors; it is
// launch-bound, so here it is ONE workgroup per direction (1024 threads: HB/H groups of H feature threads, the
// [T, H] x [H, H] products split over the groups by step), every intermediate in LDS, the H x H weights streamed
// through LDS in coalesced chunks (all in flight at once, instead of one latency-bound row walk per thread),
// one wave per output row in the matrix-vector products, reductions in fixed order (bitwise reproducible).  Shapes: H <= 256, T <= 128,
// C <= 16, T·H <= 8192 (tagan_head_supported); larger heads keep the torch path.
#include "common.cuh"

namespace tagan {
namespace {

#ifndef TAGAN_HEAD_HB
#define TAGAN_HEAD_HB 1024
#endif
constexpr int HB = TAGAN_HEAD_HB;   // threads: NG = HB / H groups of H feature threads
constexpr int HU = 8192 / HB;   // max steps per thread in the [T, H] products (ceil(T / NG); T·H <= 8192)
constexpr int HC = 16;       // max classes
constexpr int KC = 64;       // weight rows / columns staged per LDS chunk (H > 128; the whole matrix at H <= 128):
                             // 64 (H + 1) floats next to both [T, H] tiles stay under 141 KB at T·H = 8192
// staging width: at H <= 128 the whole H x H weight fits the LDS next to the [T, H] tiles, so a product stages it in
// ONE pass (one global-load latency instead of H / KC dependent rounds)
__host__ __device__ inline int kstep(int H) { return H <= 128 ? H : KC; }
constexpr int NWV = HB / 64; // waves

struct HeadArgs {
    int B, T, H, C;
    const float* x0;         // [T, H] batch row 0 (rows >= 1 are zero)
    const float* W1; const float* b1; const float* w2;          // attention: Linear(H,H), Linear(H,1,no bias)
    const float* Wc1; const float* bc1; const float* lng; const float* lnb; float eps;
    const float* Wc2; const float* bc2;
    float p_drop, inv_keep;
    uint64_t seed;
    const uint64_t* seed_ctr;   // graph-replay seed source (tagan_set_seed_counter) or null
    const float* labels;     // BCE: [B*C] targets; CE: [B] class indices (as float); null: no loss
    int loss_kind;           // 0 none, 1 BCE, 2 CE
    float* logits;           // [B, C]
    float* preds;            // [B, C]
    float* loss;             // [1]
    float* saved;            // [B, head_saved_floats]
    // backward
    const float* g_loss; const float* g_logits; const float* g_preds;
    float* dx0;
    float* dW1; float* db1; float* dw2; float* dWc1; float* dbc1; float* dlng; float* dlnb; float* dWc2; float* dbc2;
};

__host__ __device__ inline int64_t saved_floats(int T, int H) { return (int64_t)T * H + T + 3 * H + 2; }

// sum over the whole block (16 wave sums folded in wave order)
__device__ float block_sum(float v, float* red) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NWV; ++i) s += red[i];
    return s;
}

// LDS layout (floats): xs[T*H] | zs[T*H] | wt[KC*(H+1)] | part[HB] | va[128] | vd[128] | vp, vu, vg, vh [256 each]
// | vl[16] | red[32]
struct HeadLds {
    float *xs, *zs, *wt, *part, *va, *vd, *vp, *vu, *vg, *vh, *vl, *red;
    __device__ HeadLds(float* sm, int T, int H) {
        xs = sm; zs = xs + T * H; wt = zs + T * H; part = wt + kstep(H) * (H + 1); va = part + HB; vd = va + 128;
        vp = vd + 128; vu = vp + 256; vg = vu + 256; vh = vg + 256; vl = vh + 256; red = vl + 16;
    }
};

// Global -> LDS copies move float4 quads and issue LB of them per thread before the first store (one latency per
// batch: a runtime-bounded copy loop otherwise waits on every load before the next); the loads of the last batch
// are clamped into range (always valid addresses), only the stores are guarded.  n, H and kn are multiples of 4.
constexpr int LB = 4;

// dst[i] = src ? src[i] : 0 for i < n (dst 16-byte aligned; src float4 runs when it is 16-byte aligned too)
__device__ __forceinline__ void copy_in(float* dst, const float* __restrict__ src, int n) {
    if (!src) {
        for (int e = threadIdx.x * 4; e < n; e += HB * 4)
            *reinterpret_cast<float4*>(dst + e) = make_float4(0.f, 0.f, 0.f, 0.f);
    } else if ((reinterpret_cast<uintptr_t>(src) & 15) == 0) {
        const int n4 = n / 4;
        for (int e0 = threadIdx.x; e0 < n4; e0 += LB * HB) {
            float4 r[LB];
#pragma unroll
            for (int q = 0; q < LB; ++q) r[q] = reinterpret_cast<const float4*>(src)[min(e0 + q * HB, n4 - 1)];
#pragma unroll
            for (int q = 0; q < LB; ++q)
                if (e0 + q * HB < n4) reinterpret_cast<float4*>(dst)[e0 + q * HB] = r[q];
        }
    } else {   // a saved row b >= 1 (saved_floats is not a multiple of 4)
        for (int e = threadIdx.x; e < n; e += HB) dst[e] = src[e];
    }
}

// weight chunk kc of W (nn.Linear [H, H], 16-byte aligned: tagan_head_fwd / _bwd check) -> wt[kk][jj] (row stride
// H + 1: conflict-free both ways), kk < kn: W[jj][kc + kk] (COLS: columns kc..kc+kn of every row) or W[kc + kk][jj]
// (rows kc..kc+kn); one float4 of a row per load, coalesced runs along the row
template <bool COLS>
__device__ __forceinline__ void stage_chunk(const float* __restrict__ W, float* wt, int H, int kc, int kn) {
    const int nq = H * kn / 4, kq = kn / 4, hq = H / 4;
    for (int e0 = threadIdx.x; e0 < nq; e0 += LB * HB) {
        float4 r[LB];
#pragma unroll
        for (int q = 0; q < LB; ++q) {
            const int e = min(e0 + q * HB, nq - 1);
            r[q] = COLS ? *reinterpret_cast<const float4*>(W + (int64_t)(e / kq) * H + kc + 4 * (e % kq))
                        : *reinterpret_cast<const float4*>(W + (int64_t)kc * H + 4 * e);
        }
#pragma unroll
        for (int q = 0; q < LB; ++q) {
            const int e = e0 + q * HB;
            if (e < nq) {
                // COLS: row jj = e / kq, columns 4 (e % kq) + i; else row e / hq of the chunk, columns 4 (e % hq) + i
                float* o = COLS ? wt + 4 * (e % kq) * (H + 1) + e / kq : wt + (e / hq) * (H + 1) + 4 * (e % hq);
                const int st = COLS ? H + 1 : 1;
                o[0] = r[q].x; o[st] = r[q].y; o[2 * st] = r[q].z; o[3 * st] = r[q].w;
            }
        }
    }
}

// acc[u] += Σ_{kk < kn} wt[kk][j] · V[t][kc + kk] for the thread's steps t = grp + NG·u, kk ascending (bitwise the
// sums of the scalar loop), four kk per float4 read of V (kc, kn, H are multiples of 4).  Steps past T read row
// T - 1 (their sums are never stored), so the NU reads of a kk quad carry no branch and go out together.
template <int NU>
__device__ __forceinline__ void chunk_fma(const float* wt, const float* V, int T, int H, int NG, int grp, int j,
                                          int kc, int kn, float (&acc)[NU]) {
    int row[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) row[u] = min(grp + NG * u, T - 1) * H + kc;
    for (int kk = 0; kk < kn; kk += 4) {
        const float w0 = wt[kk * (H + 1) + j], w1 = wt[(kk + 1) * (H + 1) + j];
        const float w2 = wt[(kk + 2) * (H + 1) + j], w3 = wt[(kk + 3) * (H + 1) + j];
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const float4 x = *reinterpret_cast<const float4*>(V + row[u] + kk);
            acc[u] = fmaf(w0, x.x, acc[u]);
            acc[u] = fmaf(w1, x.y, acc[u]);
            acc[u] = fmaf(w2, x.z, acc[u]);
            acc[u] = fmaf(w3, x.w, acc[u]);
        }
    }
}

// acc[u] = Σ_k V[t][k] Wc[k][j] over the weight chunks, Wc = Wᵀ (COLS: Z = V Wᵀ, the nn.Linear forward) or W
// (Z = V W, its input gradient), for the thread's steps t = grp + NG·u (thread (grp, j))
template <bool COLS, int NU>
__device__ __forceinline__ void xw_chunks(const float* __restrict__ W, const float* V, float* wt, int T, int H,
                                          int NG, bool act, int grp, int j, float (&acc)[NU]) {
#pragma unroll
    for (int u = 0; u < NU; ++u) acc[u] = 0.f;
    const int KS = kstep(H);
    for (int kc = 0; kc < H; kc += KS) {
        const int kn = min(KS, H - kc);
        __syncthreads();   // the previous chunk's reads of wt (and the writes of V) are done
        stage_chunk<COLS>(W, wt, H, kc, kn);
        __syncthreads();
        if (act) chunk_fma<NU>(wt, V, T, H, NG, grp, j, kc, kn, acc);
    }
}

// nn.CrossEntropyLoss's default ignore_index (model.py:439-441 uses the default constructor): rows labelled -100
// contribute nothing and the mean divides by the rows that remain
constexpr int CE_IGNORE = -100;

__device__ __forceinline__ int ce_count(const HeadArgs& A) {
    int n = 0;
    for (int b = 0; b < A.B; ++b) n += (int)A.labels[b] != CE_IGNORE;
    return n;
}

template <int NU>
__global__ void __launch_bounds__(HB) k_head_fwd(HeadArgs A) {
    TAGAN_LIVE_SEED(A);
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int T = A.T, H = A.H, C = A.C, tid = threadIdx.x;
    const int NG = HB / H, grp = tid / H, j = tid % H, w = tid >> 6, lane = tid & 63;
    const bool act = grp < NG;
    HeadLds L(sm, T, H);
    float lsum = 0.f;
    for (int b = 0; b < A.B; ++b) {
        float* sv = A.saved + (int64_t)b * saved_floats(T, H);
        copy_in(L.xs, b == 0 ? A.x0 : nullptr, T * H);
        // z_t = tanh(W1 x_t + b1)
        float acc[NU];
        xw_chunks<true, NU>(A.W1, L.xs, L.wt, T, H, NG, act, grp, j, acc);
        if (act) {
            const float bj = A.b1[j];
#pragma unroll
            for (int u = 0; u < NU; ++u) {
                const int t = grp + NG * u;
                if (t < T) L.zs[t * H + j] = tanhf(acc[u] + bj);
            }
        }
        __syncthreads();
        // s_t = w2 . z_t (one wave per step, fixed-order lane sums)
        for (int t = w; t < T; t += NWV) {
            float s = 0.f;
            for (int k = lane; k < H; k += 64) s += A.w2[k] * L.zs[t * H + k];
            s = wave_sum(s);
            if (lane == 0) L.va[t] = s;
        }
        __syncthreads();
        if (w == 0) {   // softmax over T
            float m = -INFINITY;
            for (int t = lane; t < T; t += 64) m = fmaxf(m, L.va[t]);
            m = lane_max<64>(m);
            float e[2], den = 0.f;
            for (int q = 0; q < 2; ++q) {
                const int t = lane + 64 * q;
                e[q] = t < T ? expf(L.va[t] - m) : 0.f;
                den += e[q];
            }
            den = wave_sum(den);
            for (int q = 0; q < 2; ++q) {
                const int t = lane + 64 * q;
                if (t < T) L.va[t] = e[q] / den;
            }
        }
        __syncthreads();
        // pooled[k] = Σ_t a_t x_t[k]
        if (tid < H) {
            float p = 0.f;
            for (int t = 0; t < T; ++t) p += L.va[t] * L.xs[t * H + tid];
            L.vp[tid] = p;
        }
        __syncthreads();
        // u = Wc1 p + bc1: one wave per output row, lanes over the row (H <= 256: one float4 per lane); the loads of
        // MR rows are issued together before their sums (one latency per batch instead of one per row)
        for (int r0 = 0; r0 * NWV < H; r0 += 4) {
            constexpr int MR = 4;
            float4 wv[MR];
            const int k = lane * 4;
#pragma unroll
            for (int r = 0; r < MR; ++r) {
                const int jo = w + (r0 + r) * NWV;
                wv[r] = (jo < H && k < H) ? *reinterpret_cast<const float4*>(A.Wc1 + (int64_t)jo * H + k)
                                          : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int r = 0; r < MR; ++r) {
                const int jo = w + (r0 + r) * NWV;
                if (jo >= H) break;
                float s = 0.f;
                if (k < H) s = (wv[r].x * L.vp[k] + wv[r].y * L.vp[k + 1]) + (wv[r].z * L.vp[k + 2] + wv[r].w * L.vp[k + 3]);
                s = wave_sum(s);
                if (lane == 0) L.vu[jo] = s + A.bc1[jo];
            }
        }
        __syncthreads();
        // LayerNorm ; ReLU ; dropout
        const float u = tid < H ? L.vu[tid] : 0.f;
        const float mean = block_sum(u, L.red) / (float)H;
        const float dv = tid < H ? u - mean : 0.f;
        const float rstd = 1.f / sqrtf(block_sum(dv * dv, L.red) / (float)H + A.eps);
        if (tid < H) {
            float n = dv * rstd * A.lng[tid] + A.lnb[tid];
            n = n > 0.f ? n : 0.f;
            if (A.p_drop > 0.f) {
                const uint32_t key = drop_key(A.seed, (uint64_t)b);
                n = drop_u(key, (uint32_t)tid) >= A.p_drop ? n * A.inv_keep : 0.f;
            }
            L.vh[tid] = n;
        }
        __syncthreads();
        // logits[c] = Wc2[c] . h2 + bc2[c]: one wave per class
        for (int c = w; c < C; c += NWV) {
            float s = 0.f;
            for (int k = lane; k < H; k += 64) s += A.Wc2[(int64_t)c * H + k] * L.vh[k];
            s = wave_sum(s);
            if (lane == 0) L.vl[c] = s + A.bc2[c];
        }
        __syncthreads();
        if (tid == 0) {
            float m = -INFINITY, den = 0.f;
            for (int c = 0; c < C; ++c) m = fmaxf(m, L.vl[c]);
            for (int c = 0; c < C; ++c) den += expf(L.vl[c] - m);
            for (int c = 0; c < C; ++c) {
                const float z = L.vl[c];
                A.logits[b * C + c] = z;
                A.preds[b * C + c] = C == 1 ? 1.f / (1.f + expf(-z)) : expf(z - m) / den;
                if (A.loss_kind == 1) {
                    const float y = A.labels[b * C + c];
                    lsum += fmaxf(z, 0.f) - z * y + log1pf(expf(-fabsf(z)));
                }
            }
            if (A.loss_kind == 2) {   // nn.CrossEntropyLoss(): ignore_index -100 rows drop out of the mean; any
                const int y = (int)A.labels[b];   // other out-of-range class poisons the loss (torch would raise)
                if (y != CE_IGNORE) lsum += (y >= 0 && y < C) ? (m + logf(den)) - L.vl[y] : NAN;
            }
        }
        // saved: z | a | pooled | u | mean, rstd | h2
        for (int i = tid; i < T * H; i += HB) sv[i] = L.zs[i];
        for (int t = tid; t < T; t += HB) sv[T * H + t] = L.va[t];
        if (tid < H) {
            sv[T * H + T + tid] = L.vp[tid];
            sv[T * H + T + H + tid] = u;
            sv[T * H + T + 2 * H + 2 + tid] = L.vh[tid];
        }
        if (tid == 0) { sv[T * H + T + 2 * H] = mean; sv[T * H + T + 2 * H + 1] = rstd; }
        __syncthreads();
    }
    if (tid == 0 && A.loss_kind && A.loss)   // CE over no counted row: 0/0 = NaN, as torch's mean reduction
        A.loss[0] = A.loss_kind == 1 ? lsum / (float)(A.B * C) : lsum / (float)ce_count(A);
}

template <int NU>
__global__ void __launch_bounds__(HB) k_head_bwd(HeadArgs A) {
    TAGAN_LIVE_SEED(A);
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int T = A.T, H = A.H, C = A.C, tid = threadIdx.x;
    const int NG = HB / H, grp = tid / H, j = tid % H, w = tid >> 6, lane = tid & 63;
    const bool act = grp < NG;
    HeadLds L(sm, T, H);
    float* vq = L.vu;    // x̂, then du
    const float gL = A.g_loss ? A.g_loss[0] : 0.f;
    for (int b = 0; b < A.B; ++b) {
        const bool first = b == 0;
        const float* sv = A.saved + (int64_t)b * saved_floats(T, H);
        copy_in(L.xs, first ? A.x0 : nullptr, T * H);
        copy_in(L.zs, sv, T * H);
        for (int t = tid; t < T; t += HB) L.va[t] = sv[T * H + t];
        if (tid < H) L.vp[tid] = sv[T * H + T + tid];
        if (tid == 0) {   // dlogits of this row
            float sgp = 0.f;
            if (A.g_preds && C > 1)
                for (int c = 0; c < C; ++c) sgp += A.g_preds[b * C + c] * A.preds[b * C + c];
            for (int c = 0; c < C; ++c) {
                const float p = A.preds[b * C + c];
                float g = A.g_logits ? A.g_logits[b * C + c] : 0.f;
                if (A.g_preds) g += C == 1 ? A.g_preds[b * C + c] * p * (1.f - p) : p * (A.g_preds[b * C + c] - sgp);
                if (A.loss_kind == 1 && A.g_loss) {
                    const float z = A.logits[b * C + c];
                    g += gL * (1.f / (1.f + expf(-z)) - A.labels[b * C + c]) / (float)(A.B * C);
                }
                if (A.loss_kind == 2 && A.g_loss && (int)A.labels[b] != CE_IGNORE)
                    g += gL * (p - (c == (int)A.labels[b] ? 1.f : 0.f)) / (float)ce_count(A);
                L.vl[c] = g;
            }
        }
        __syncthreads();
        if (tid < C) A.dbc2[tid] = (first ? 0.f : A.dbc2[tid]) + L.vl[tid];
        float du = 0.f;
        if (tid < H) {
            const float u = sv[T * H + T + H + tid], mean = sv[T * H + T + 2 * H], rstd = sv[T * H + T + 2 * H + 1];
            const float h2 = sv[T * H + T + 2 * H + 2 + tid];
            float dh = 0.f;
            for (int c = 0; c < C; ++c) {
                const int64_t o = (int64_t)c * H + tid;
                A.dWc2[o] = (first ? 0.f : A.dWc2[o]) + L.vl[c] * h2;
                dh += L.vl[c] * A.Wc2[o];
            }
            if (A.p_drop > 0.f) {
                const uint32_t key = drop_key(A.seed, (uint64_t)b);
                dh = drop_u(key, (uint32_t)tid) >= A.p_drop ? dh * A.inv_keep : 0.f;
            }
            const float xh = (u - mean) * rstd;
            const float n = xh * A.lng[tid] + A.lnb[tid];
            const float dn = n > 0.f ? dh : 0.f;
            A.dlng[tid] = (first ? 0.f : A.dlng[tid]) + dn * xh;
            A.dlnb[tid] = (first ? 0.f : A.dlnb[tid]) + dn;
            du = dn * A.lng[tid];         // g·dn, reduced below
            vq[tid] = xh;                 // keep x̂ for the LN backward
        }
        const float c1 = block_sum(tid < H ? du * vq[tid] : 0.f, L.red) / (float)H;
        const float c2 = block_sum(tid < H ? du : 0.f, L.red) / (float)H;
        if (tid < H) {
            const float rstd = sv[T * H + T + 2 * H + 1];
            du = rstd * (du - c1 * vq[tid] - c2);
            A.dbc1[tid] = (first ? 0.f : A.dbc1[tid]) + du;
        }
        __syncthreads();
        if (tid < H) vq[tid] = du;
        __syncthreads();
        // dWc1[j][k] += du_j p_k (coalesced over the flat index)
        for (int o = tid; o < H * H; o += HB) A.dWc1[o] = (first ? 0.f : A.dWc1[o]) + vq[o / H] * L.vp[o % H];
        // dpooled[k] = Σ_j du_j Wc1[j][k]: thread (grp, k) over j = grp, grp + NG, ..., then the groups in order
        if (act) {
            float g = 0.f;
#pragma unroll 32
            for (int jj = grp; jj < H; jj += NG) g += vq[jj] * A.Wc1[(int64_t)jj * H + j];
            L.part[grp * H + j] = g;
        }
        __syncthreads();
        if (tid < H) {
            float g = 0.f;
            for (int q = 0; q < NG; ++q) g += L.part[q * H + tid];
            L.vg[tid] = g;
        }
        __syncthreads();
        // da_t = dpooled . x_t ; ds = a (da - Σ a da)
        for (int t = w; t < T; t += NWV) {
            float s = 0.f;
            for (int k = lane; k < H; k += 64) s += L.vg[k] * L.xs[t * H + k];
            s = wave_sum(s);
            if (lane == 0) L.vd[t] = s;
        }
        __syncthreads();
        if (w == 0) {
            float s = 0.f;
            for (int t = lane; t < T; t += 64) s += L.va[t] * L.vd[t];
            s = wave_sum(s);
            for (int t = lane; t < T; t += 64) L.vd[t] = L.va[t] * (L.vd[t] - s);
        }
        __syncthreads();
        // dw2[j] += Σ_t ds_t z_tj ; dpre_tj = ds_t w2_j (1 - z_tj^2) (overwrites z) ; db1[j] += Σ_t dpre_tj
        if (tid < H) {
            float gw = 0.f, gb = 0.f;
            const float w2j = A.w2[tid];
            for (int t = 0; t < T; ++t) {
                const float z = L.zs[t * H + tid], ds = L.vd[t];
                gw += ds * z;
                const float dp = ds * w2j * (1.f - z * z);
                L.zs[t * H + tid] = dp;
                gb += dp;
            }
            A.dw2[tid] = (first ? 0.f : A.dw2[tid]) + gw;
            A.db1[tid] = (first ? 0.f : A.db1[tid]) + gb;
        }
        __syncthreads();
        if (first) {   // rows >= 1 have x = 0: no dW1 and no dx
            // dW1[j][k] = Σ_t dpre_tj x_tk, t ascending: one 4 x 4 block of (j, k) per thread and pass (two float4
            // LDS reads per 16 FMAs instead of two scalar reads per FMA); the stores stay scalar (dW1 is a caller
            // pointer, 4-byte alignment only), consecutive lanes on consecutive k quads
            const int H4 = H / 4;
            for (int o = tid; o < H4 * H4; o += HB) {
                const int j4 = (o / H4) * 4, k4 = (o % H4) * 4;
                float4 acc[4];
#pragma unroll
                for (int a = 0; a < 4; ++a) acc[a] = make_float4(0.f, 0.f, 0.f, 0.f);
                for (int t = 0; t < T; ++t) {
                    const float4 zv = *reinterpret_cast<const float4*>(L.zs + t * H + j4);
                    const float4 xv = *reinterpret_cast<const float4*>(L.xs + t * H + k4);
                    const float zz[4] = {zv.x, zv.y, zv.z, zv.w};
#pragma unroll
                    for (int a = 0; a < 4; ++a) {
                        acc[a].x = fmaf(zz[a], xv.x, acc[a].x);
                        acc[a].y = fmaf(zz[a], xv.y, acc[a].y);
                        acc[a].z = fmaf(zz[a], xv.z, acc[a].z);
                        acc[a].w = fmaf(zz[a], xv.w, acc[a].w);
                    }
                }
#pragma unroll
                for (int a = 0; a < 4; ++a) {
                    float* o4 = A.dW1 + (int64_t)(j4 + a) * H + k4;
                    o4[0] = acc[a].x; o4[1] = acc[a].y; o4[2] = acc[a].z; o4[3] = acc[a].w;
                }
            }
            // dx_t[k] = a_t dpooled_k + Σ_jj dpre_t,jj W1[jj][k]: W1 rows staged through LDS in chunks of KC
            float acc[NU];
            xw_chunks<false, NU>(A.W1, L.zs, L.wt, T, H, NG, act, grp, j, acc);
            if (act) {
#pragma unroll
                for (int u = 0; u < NU; ++u) {
                    const int t = grp + NG * u;
                    if (t < T) A.dx0[(int64_t)t * H + j] = L.va[t] * L.vg[j] + acc[u];
                }
            }
        }
        __syncthreads();
    }
}

size_t head_lds(int T, int H) {
    return (size_t)(2 * T * H + kstep(H) * (H + 1) + HB + 2 * 128 + 4 * 256 + 16 + 32) * sizeof(float);
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// steps per thread in the [T, H] products (ceil(T / NG)) rounded up to the kernels' template argument 1, 2, 4 or 8
int head_nu(int T, int H) {
    const int ng = HB / H, n = (T + ng - 1) / ng;
    return n <= 1 ? 1 : n <= 2 ? 2 : n <= 4 ? 4 : n <= 8 ? 8 : 16;
}

template <int NU>
int head_optin_nu() {
    static bool done = false;
    if (done) return TAGAN_OK;
    hipError_t e1 = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_head_fwd<NU>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipError_t e2 = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_head_bwd<NU>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    TAGAN_REQUIRE(e1 == hipSuccess && e2 == hipSuccess, TAGAN_ERR_LAUNCH, "head: LDS opt-in failed");
    done = true;
    return TAGAN_OK;
}

int head_lds_optin(size_t bytes, int nu) {
    if (bytes <= 64 * 1024) return TAGAN_OK;
    return nu == 1 ? head_optin_nu<1>() : nu == 2 ? head_optin_nu<2>() : nu == 4 ? head_optin_nu<4>()
           : nu == 8 ? head_optin_nu<8>() : head_optin_nu<HU>();
}

#define TAGAN_HEAD_LAUNCH(KERN, NU, LDS, STREAM, ARGS)                                       \
    do {                                                                                  \
        if ((NU) == 1) KERN<1><<<1, HB, LDS, STREAM>>>(ARGS);                             \
        else if ((NU) == 2) KERN<2><<<1, HB, LDS, STREAM>>>(ARGS);                        \
        else if ((NU) == 4) KERN<4><<<1, HB, LDS, STREAM>>>(ARGS);                        \
        else if ((NU) == 8) KERN<8><<<1, HB, LDS, STREAM>>>(ARGS);                        \
        else KERN<HU><<<1, HB, LDS, STREAM>>>(ARGS);                                      \
    } while (0)

}  // namespace
}  // namespace tagan

extern "C" {

int tagan_head_supported(int32_t T, int32_t H, int32_t C) {
    return (H >= 4 && H <= 256 && H % 4 == 0 && T >= 1 && T <= 128 && C >= 1 && C <= tagan::HC &&
            T * H <= 8192 && (T + tagan::HB / H - 1) / (tagan::HB / H) <= tagan::HU) ? 1 : 0;
}

size_t tagan_head_saved_floats(int32_t B, int32_t T, int32_t H) {
    return (size_t)B * (size_t)tagan::saved_floats(T, H);
}

int tagan_head_fwd(int32_t B, int32_t T, int32_t H, int32_t C, const float* x0, const float* W1, const float* b1,
                   const float* w2, const float* Wc1, const float* bc1, const float* ln_w, const float* ln_b,
                   float eps, const float* Wc2, const float* bc2, float p_drop, uint64_t seed, const float* labels,
                   int loss_kind, float* logits, float* preds, float* loss, float* saved, void* stream) {
    using namespace tagan;
    TAGAN_REQUIRE(tagan_head_supported(T, H, C), TAGAN_ERR_UNSUPPORTED, "head: T=%d H=%d C=%d", T, H, C);
    TAGAN_REQUIRE(B >= 1 && x0 && W1 && b1 && w2 && Wc1 && bc1 && ln_w && ln_b && Wc2 && bc2 && logits && preds &&
                  saved, TAGAN_ERR_ARG, "head_fwd: bad args");
    TAGAN_REQUIRE(loss_kind >= 0 && loss_kind <= 2 && (loss_kind == 0 || (labels && loss)), TAGAN_ERR_ARG,
                  "head_fwd: loss_kind %d", loss_kind);
    TAGAN_REQUIRE(p_drop >= 0.f && p_drop < 1.f, TAGAN_ERR_ARG, "head_fwd: p_drop");
    TAGAN_REQUIRE(aligned16(W1) && aligned16(Wc1) && aligned16(x0), TAGAN_ERR_ARG,
                  "head_fwd: W1, Wc1 and x0 must be 16-byte aligned");
    HeadArgs A{};
    A.B = B; A.T = T; A.H = H; A.C = C; A.x0 = x0; A.W1 = W1; A.b1 = b1; A.w2 = w2; A.Wc1 = Wc1; A.bc1 = bc1;
    A.lng = ln_w; A.lnb = ln_b; A.eps = eps; A.Wc2 = Wc2; A.bc2 = bc2; A.p_drop = p_drop;
    A.inv_keep = 1.f / (1.f - p_drop); A.seed = seed; A.seed_ctr = seed_counter(); A.labels = labels; A.loss_kind = loss_kind;
    A.logits = logits; A.preds = preds; A.loss = loss; A.saved = saved;
    const int nu = head_nu(T, H);
    if (int rc = head_lds_optin(head_lds(T, H), nu)) return rc;
    TAGAN_HEAD_LAUNCH(k_head_fwd, nu, head_lds(T, H), as_stream(stream), A);
    TAGAN_CHECK_LAUNCH("head_fwd");
    return TAGAN_OK;
}

int tagan_head_bwd(int32_t B, int32_t T, int32_t H, int32_t C, const float* x0, const float* W1, const float* w2,
                   const float* Wc1, const float* ln_w, const float* ln_b, const float* Wc2, float p_drop,
                   uint64_t seed, const float* labels, int loss_kind, const float* logits, const float* preds,
                   const float* saved, const float* g_loss, const float* g_logits, const float* g_preds,
                   float* dx0, float* dW1, float* db1, float* dw2, float* dWc1, float* dbc1, float* dln_w,
                   float* dln_b, float* dWc2, float* dbc2, void* stream) {
    using namespace tagan;
    TAGAN_REQUIRE(tagan_head_supported(T, H, C), TAGAN_ERR_UNSUPPORTED, "head: T=%d H=%d C=%d", T, H, C);
    TAGAN_REQUIRE(B >= 1 && x0 && W1 && w2 && Wc1 && ln_w && ln_b && Wc2 && logits && preds && saved && dx0 && dW1 &&
                  db1 && dw2 && dWc1 && dbc1 && dln_w && dln_b && dWc2 && dbc2, TAGAN_ERR_ARG, "head_bwd: bad args");
    TAGAN_REQUIRE(loss_kind >= 0 && loss_kind <= 2 && (loss_kind == 0 || labels), TAGAN_ERR_ARG,
                  "head_bwd: loss_kind %d", loss_kind);
    TAGAN_REQUIRE(aligned16(W1) && aligned16(Wc1) && aligned16(x0), TAGAN_ERR_ARG,
                  "head_bwd: W1, Wc1 and x0 must be 16-byte aligned");
    HeadArgs A{};
    A.B = B; A.T = T; A.H = H; A.C = C; A.x0 = x0; A.W1 = W1; A.w2 = w2; A.Wc1 = Wc1; A.lng = ln_w; A.lnb = ln_b;
    A.Wc2 = Wc2; A.p_drop = p_drop; A.inv_keep = 1.f / (1.f - p_drop); A.seed = seed; A.seed_ctr = seed_counter(); A.labels = labels;
    A.loss_kind = loss_kind; A.logits = (float*)logits; A.preds = (float*)preds; A.saved = (float*)saved;
    A.g_loss = g_loss; A.g_logits = g_logits; A.g_preds = g_preds; A.dx0 = dx0; A.dW1 = dW1; A.db1 = db1;
    A.dw2 = dw2; A.dWc1 = dWc1; A.dbc1 = dbc1; A.dlng = dln_w; A.dlnb = dln_b; A.dWc2 = dWc2; A.dbc2 = dbc2;
    const int nu = head_nu(T, H);
    if (int rc = head_lds_optin(head_lds(T, H), nu)) return rc;
    TAGAN_HEAD_LAUNCH(k_head_bwd, nu, head_lds(T, H), as_stream(stream), A);
    TAGAN_CHECK_LAUNCH("head_bwd");
    return TAGAN_OK;
}

}  // extern "C"
