// Fused classification head + loss of TAGAN (model.py:377-459, classification.py:856-966) on gfx950.
//
// graph_features [B, T, H] (row 0 = the pooled snapshot means, rows 1..B-1 all zero: model.py:382-394)
//   -> attention pooling over T:  s_t = w2 · tanh(W1 x_t + b1),  a = softmax_t(s),  p = Σ_t a_t x_t
//   -> Linear(H, H) -> LayerNorm -> ReLU -> Dropout -> Linear(H, C)  = logits [B, C]
//   -> predictions (sigmoid for C = 1, softmax otherwise) and the loss: BCE-with-logits mean over the
//      B·C elements (TemporalLossModule's default, classification.py:453-456) or cross entropy over B
//      rows (model.py:439-441).
// The reference runs this as ~25 ATen launches forward and ~40 backward on [1..B, 32, 128] tensors; it is
// launch-bound, so here it is ONE workgroup (256 threads, thread j <-> feature j) per direction, every
// intermediate in LDS, reductions in fixed order (bitwise reproducible).  Shapes: H <= 256, T <= 128,
// C <= 16, T·H <= 8192 (tagan_head_supported); larger heads keep the torch path.
#include "common.cuh"

namespace tagan {
namespace {

constexpr int HB = 256;      // threads
constexpr int HT = 32;       // time-step tile held in registers
constexpr int HC = 16;       // max classes

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

__device__ float block_sum(float v, float* red) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    return (red[0] + red[1]) + (red[2] + red[3]);
}

// LDS: xs[T*H] | zs[T*H] | vec[4*256] (a/da, pooled/dp, u/du, misc) | red[8]
__global__ void __launch_bounds__(HB) k_head_fwd(HeadArgs A) {
    TAGAN_LIVE_SEED(A);
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int T = A.T, H = A.H, C = A.C, j = threadIdx.x;
    float* xs = sm;
    float* zs = xs + T * H;
    float* va = zs + T * H;          // a [T]
    float* vp = va + 256;            // pooled [H]
    float* vh = vp + 256;            // h2 [H]
    float* vl = vh + 256;            // logits of this row [C]
    float* red = vl + 256;
    float lsum = 0.f;
    for (int b = 0; b < A.B; ++b) {
        float* sv = A.saved + (int64_t)b * saved_floats(T, H);
        for (int i = j; i < T * H; i += HB) xs[i] = b == 0 ? A.x0[i] : 0.f;
        __syncthreads();
        // z_t = tanh(W1 x_t + b1): thread j, a tile of HT steps in registers, W1 row j streamed as float4
        if (j < H) {
            for (int t0 = 0; t0 < T; t0 += HT) {
                float acc[HT];
#pragma unroll
                for (int u = 0; u < HT; ++u) acc[u] = 0.f;
                for (int k = 0; k < H; k += 4) {
                    const float4 w = *reinterpret_cast<const float4*>(A.W1 + (int64_t)j * H + k);
#pragma unroll
                    for (int u = 0; u < HT; ++u) {
                        if (t0 + u < T) {
                            const float4 x = *reinterpret_cast<const float4*>(xs + (t0 + u) * H + k);
                            acc[u] += (w.x * x.x + w.y * x.y) + (w.z * x.z + w.w * x.w);
                        }
                    }
                }
                const float bj = A.b1[j];
#pragma unroll
                for (int u = 0; u < HT; ++u)
                    if (t0 + u < T) zs[(t0 + u) * H + j] = tanhf(acc[u] + bj);
            }
        }
        __syncthreads();
        // s_t = w2 . z_t (one wave per step, fixed-order lane sums)
        const int w = j >> 6, lane = j & 63;
        for (int t = w; t < T; t += HB / 64) {
            float s = 0.f;
            for (int k = lane; k < H; k += 64) s += A.w2[k] * zs[t * H + k];
            s = wave_sum(s);
            if (lane == 0) va[t] = s;
        }
        __syncthreads();
        if (w == 0) {   // softmax over T
            float m = -INFINITY;
            for (int t = lane; t < T; t += 64) m = fmaxf(m, va[t]);
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
            float e[2], den = 0.f;
            for (int q = 0; q < 2; ++q) {
                const int t = lane + 64 * q;
                e[q] = t < T ? expf(va[t] - m) : 0.f;
                den += e[q];
            }
            den = wave_sum(den);
            for (int q = 0; q < 2; ++q) {
                const int t = lane + 64 * q;
                if (t < T) va[t] = e[q] / den;
            }
        }
        __syncthreads();
        // pooled[k] = Σ_t a_t x_t[k]
        if (j < H) {
            float p = 0.f;
            for (int t = 0; t < T; ++t) p += va[t] * xs[t * H + j];
            vp[j] = p;
        }
        __syncthreads();
        // u = Wc1 p + bc1 ; LayerNorm ; ReLU ; dropout
        float u = 0.f;
        if (j < H) {
            u = A.bc1[j];
            for (int k = 0; k < H; k += 4) {
                const float4 wv = *reinterpret_cast<const float4*>(A.Wc1 + (int64_t)j * H + k);
                u += (wv.x * vp[k] + wv.y * vp[k + 1]) + (wv.z * vp[k + 2] + wv.w * vp[k + 3]);
            }
        }
        const float mean = block_sum(j < H ? u : 0.f, red) / (float)H;
        const float dv = j < H ? u - mean : 0.f;
        const float rstd = 1.f / sqrtf(block_sum(dv * dv, red) / (float)H + A.eps);
        if (j < H) {
            float n = dv * rstd * A.lng[j] + A.lnb[j];
            n = n > 0.f ? n : 0.f;
            if (A.p_drop > 0.f) {
                const uint32_t key = drop_key(A.seed, (uint64_t)b);
                n = drop_u(key, (uint32_t)j) >= A.p_drop ? n * A.inv_keep : 0.f;
            }
            vh[j] = n;
        }
        __syncthreads();
        // logits[c] = Wc2[c] . h2 + bc2[c]
        for (int c = 0; c < C; ++c) {
            const float v = block_sum(j < H ? A.Wc2[(int64_t)c * H + j] * vh[j] : 0.f, red);
            if (j == 0) vl[c] = v + A.bc2[c];
        }
        __syncthreads();
        if (j == 0) {
            float m = -INFINITY, den = 0.f;
            for (int c = 0; c < C; ++c) m = fmaxf(m, vl[c]);
            for (int c = 0; c < C; ++c) den += expf(vl[c] - m);
            for (int c = 0; c < C; ++c) {
                const float z = vl[c];
                A.logits[b * C + c] = z;
                A.preds[b * C + c] = C == 1 ? 1.f / (1.f + expf(-z)) : expf(z - m) / den;
                if (A.loss_kind == 1) {
                    const float y = A.labels[b * C + c];
                    lsum += fmaxf(z, 0.f) - z * y + log1pf(expf(-fabsf(z)));
                }
            }
            if (A.loss_kind == 2) {   // an out-of-range class index poisons the loss (torch would raise)
                const int y = (int)A.labels[b];
                lsum += (y >= 0 && y < C) ? (m + logf(den)) - vl[y] : NAN;
            }
        }
        // saved: z | a | pooled | u | mean, rstd | h2
        for (int i = j; i < T * H; i += HB) sv[i] = zs[i];
        for (int t = j; t < T; t += HB) sv[T * H + t] = va[t];
        if (j < H) {
            sv[T * H + T + j] = vp[j];
            sv[T * H + T + H + j] = u;
            sv[T * H + T + 2 * H + 2 + j] = vh[j];
        }
        if (j == 0) { sv[T * H + T + 2 * H] = mean; sv[T * H + T + 2 * H + 1] = rstd; }
        __syncthreads();
    }
    if (j == 0 && A.loss_kind && A.loss)
        A.loss[0] = A.loss_kind == 1 ? lsum / (float)(A.B * C) : lsum / (float)A.B;
}

__global__ void __launch_bounds__(HB) k_head_bwd(HeadArgs A) {
    TAGAN_LIVE_SEED(A);
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int T = A.T, H = A.H, C = A.C, j = threadIdx.x;
    const int w = j >> 6, lane = j & 63;
    float* xs = sm;
    float* zs = xs + T * H;          // z, then dpre
    float* va = zs + T * H;          // a [T]
    float* vd = va + 256;            // da, then ds [T]
    float* vp = vd + 256;            // pooled [H]
    float* vq = vp + 256;            // du [H]
    float* vg = vq + 256;            // dpooled [H]
    float* vl = vg + 256;            // dlogits [C]
    float* red = vl + 256;
    const float gL = A.g_loss ? A.g_loss[0] : 0.f;
    for (int b = 0; b < A.B; ++b) {
        const bool first = b == 0;
        const float* sv = A.saved + (int64_t)b * saved_floats(T, H);
        for (int i = j; i < T * H; i += HB) { xs[i] = first ? A.x0[i] : 0.f; zs[i] = sv[i]; }
        for (int t = j; t < T; t += HB) va[t] = sv[T * H + t];
        if (j < H) vp[j] = sv[T * H + T + j];
        if (j == 0) {   // dlogits of this row
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
                if (A.loss_kind == 2 && A.g_loss)
                    g += gL * (p - (c == (int)A.labels[b] ? 1.f : 0.f)) / (float)A.B;
                vl[c] = g;
            }
        }
        __syncthreads();
        if (j < C) A.dbc2[j] = (first ? 0.f : A.dbc2[j]) + vl[j];
        float du = 0.f;
        if (j < H) {
            const float u = sv[T * H + T + H + j], mean = sv[T * H + T + 2 * H], rstd = sv[T * H + T + 2 * H + 1];
            const float h2 = sv[T * H + T + 2 * H + 2 + j];
            float dh = 0.f;
            for (int c = 0; c < C; ++c) {
                const int64_t o = (int64_t)c * H + j;
                A.dWc2[o] = (first ? 0.f : A.dWc2[o]) + vl[c] * h2;
                dh += vl[c] * A.Wc2[o];
            }
            if (A.p_drop > 0.f) {
                const uint32_t key = drop_key(A.seed, (uint64_t)b);
                dh = drop_u(key, (uint32_t)j) >= A.p_drop ? dh * A.inv_keep : 0.f;
            }
            const float xh = (u - mean) * rstd;
            const float n = xh * A.lng[j] + A.lnb[j];
            const float dn = n > 0.f ? dh : 0.f;
            A.dlng[j] = (first ? 0.f : A.dlng[j]) + dn * xh;
            A.dlnb[j] = (first ? 0.f : A.dlnb[j]) + dn;
            du = dn * A.lng[j];           // g·dn, reduced below
            vq[j] = xh;                   // keep x̂ for the LN backward
        }
        const float c1 = block_sum(j < H ? du * vq[j] : 0.f, red) / (float)H;
        const float c2 = block_sum(j < H ? du : 0.f, red) / (float)H;
        if (j < H) {
            const float rstd = sv[T * H + T + 2 * H + 1];
            du = rstd * (du - c1 * vq[j] - c2);
            A.dbc1[j] = (first ? 0.f : A.dbc1[j]) + du;
        }
        __syncthreads();
        if (j < H) vq[j] = du;
        __syncthreads();
        if (j < H) {
            // dWc1[j][k] += du_j p_k ; dpooled[k] = Σ_j du_j Wc1[j][k]
            for (int k = 0; k < H; ++k) {
                const int64_t o = (int64_t)j * H + k;
                A.dWc1[o] = (first ? 0.f : A.dWc1[o]) + vq[j] * vp[k];
            }
            float g = 0.f;
            for (int jj = 0; jj < H; ++jj) g += vq[jj] * A.Wc1[(int64_t)jj * H + j];
            vg[j] = g;
        }
        __syncthreads();
        // da_t = dpooled . x_t ; ds = a (da - Σ a da)
        for (int t = w; t < T; t += HB / 64) {
            float s = 0.f;
            for (int k = lane; k < H; k += 64) s += vg[k] * xs[t * H + k];
            s = wave_sum(s);
            if (lane == 0) vd[t] = s;
        }
        __syncthreads();
        if (w == 0) {
            float s = 0.f;
            for (int t = lane; t < T; t += 64) s += va[t] * vd[t];
            s = wave_sum(s);
            for (int t = lane; t < T; t += 64) vd[t] = va[t] * (vd[t] - s);
        }
        __syncthreads();
        // dw2[j] += Σ_t ds_t z_tj ; dpre_tj = ds_t w2_j (1 - z_tj^2) (overwrites z) ; db1[j] += Σ_t dpre_tj
        if (j < H) {
            float gw = 0.f, gb = 0.f;
            const float w2j = A.w2[j];
            for (int t = 0; t < T; ++t) {
                const float z = zs[t * H + j], ds = vd[t];
                gw += ds * z;
                const float dp = ds * w2j * (1.f - z * z);
                zs[t * H + j] = dp;
                gb += dp;
            }
            A.dw2[j] = (first ? 0.f : A.dw2[j]) + gw;
            A.db1[j] = (first ? 0.f : A.db1[j]) + gb;
        }
        __syncthreads();
        if (first) {   // rows >= 1 have x = 0: no dW1 and no dx
            if (j < H) {
                // dW1[j][k] = Σ_t dpre_tj x_tk
                for (int k = 0; k < H; k += 4) {
                    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
                    for (int t = 0; t < T; ++t) {
                        const float dp = zs[t * H + j];
                        const float4 x = *reinterpret_cast<const float4*>(xs + t * H + k);
                        acc.x += dp * x.x; acc.y += dp * x.y; acc.z += dp * x.z; acc.w += dp * x.w;
                    }
                    *reinterpret_cast<float4*>(A.dW1 + (int64_t)j * H + k) = acc;
                }
                // dx_t[k=j] = a_t dpooled_j + Σ_jj dpre_t,jj W1[jj][j]
                for (int t0 = 0; t0 < T; t0 += HT) {
                    float acc[HT];
#pragma unroll
                    for (int u = 0; u < HT; ++u) acc[u] = 0.f;
                    for (int jj = 0; jj < H; ++jj) {
                        const float wv = A.W1[(int64_t)jj * H + j];
#pragma unroll
                        for (int u = 0; u < HT; ++u)
                            if (t0 + u < T) acc[u] += zs[(t0 + u) * H + jj] * wv;
                    }
#pragma unroll
                    for (int u = 0; u < HT; ++u)
                        if (t0 + u < T) A.dx0[(int64_t)(t0 + u) * H + j] = va[t0 + u] * vg[j] + acc[u];
                }
            }
        }
        __syncthreads();
    }
}

size_t head_lds(int T, int H) { return (size_t)(2 * T * H + 6 * 256 + 8) * sizeof(float); }

}  // namespace
}  // namespace tagan

extern "C" {

int tagan_head_supported(int32_t T, int32_t H, int32_t C) {
    return (H >= 4 && H <= tagan::HB && H % 4 == 0 && T >= 1 && T <= 128 && C >= 1 && C <= tagan::HC &&
            T * H <= 8192) ? 1 : 0;
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
    HeadArgs A{};
    A.B = B; A.T = T; A.H = H; A.C = C; A.x0 = x0; A.W1 = W1; A.b1 = b1; A.w2 = w2; A.Wc1 = Wc1; A.bc1 = bc1;
    A.lng = ln_w; A.lnb = ln_b; A.eps = eps; A.Wc2 = Wc2; A.bc2 = bc2; A.p_drop = p_drop;
    A.inv_keep = 1.f / (1.f - p_drop); A.seed = seed; A.seed_ctr = seed_counter(); A.labels = labels; A.loss_kind = loss_kind;
    A.logits = logits; A.preds = preds; A.loss = loss; A.saved = saved;
    k_head_fwd<<<1, HB, head_lds(T, H), as_stream(stream)>>>(A);
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
    HeadArgs A{};
    A.B = B; A.T = T; A.H = H; A.C = C; A.x0 = x0; A.W1 = W1; A.w2 = w2; A.Wc1 = Wc1; A.lng = ln_w; A.lnb = ln_b;
    A.Wc2 = Wc2; A.p_drop = p_drop; A.inv_keep = 1.f / (1.f - p_drop); A.seed = seed; A.seed_ctr = seed_counter(); A.labels = labels;
    A.loss_kind = loss_kind; A.logits = (float*)logits; A.preds = (float*)preds; A.saved = (float*)saved;
    A.g_loss = g_loss; A.g_logits = g_logits; A.g_preds = g_preds; A.dx0 = dx0; A.dW1 = dW1; A.db1 = db1;
    A.dw2 = dw2; A.dWc1 = dWc1; A.dbc1 = dbc1; A.dlng = dln_w; A.dlnb = dln_b; A.dWc2 = dWc2; A.dbc2 = dbc2;
    k_head_bwd<<<1, HB, head_lds(T, H), as_stream(stream)>>>(A);
    TAGAN_CHECK_LAUNCH("head_bwd");
    return TAGAN_OK;
}

}  // extern "C"
