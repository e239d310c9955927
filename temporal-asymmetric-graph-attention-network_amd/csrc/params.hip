// Projection-parameter packing for the attention blocks (fused.py::attention_block).
//
// The reference keeps q_linear / k_linear / v_linear as three nn.Linear modules
// (geometric_attention.py:263-266, temporal_attention.py:356-359); the fused block multiplies by their
// concatenation.  Concatenating per step took 3-4 small torch launches per block (weight cat, bias cat, the
// augmented [W | b | 0] cat and its zero pad) and the backward 2-4 slice copies; here one launch packs the six
// tensors into the layout the QKV GEMM reads, and one launch unpacks the packed gradient into the six
// parameter gradients.  Pure copies: bit-exact.
#include "common.cuh"

namespace tagan {
namespace {

constexpr int BLK = 256;

// one workgroup per packed row r < 3H (blockIdx.x), its threads over the row's ld columns (bias column / zero pad
// included): no per-element index divisions
__global__ void __launch_bounds__(BLK) k_qkv_pack(int64_t H, const float* __restrict__ wq, const float* __restrict__ wk,
                                                  const float* __restrict__ wv, const float* __restrict__ bq,
                                                  const float* __restrict__ bk, const float* __restrict__ bv,
                                                  float* __restrict__ w, int64_t ld, int bias_col,
                                                  float* __restrict__ b) {
    const int r = blockIdx.x, part = r / (int)H, rr = r - part * (int)H;
    const float* src = part == 0 ? wq : part == 1 ? wk : wv;
    const float* bs = part == 0 ? bq : part == 1 ? bk : bv;
    for (int c = threadIdx.x; c < (int)ld; c += BLK) {
        float val = 0.f;
        if (c < H) val = src[(int64_t)rr * H + c];
        else if (c == H && bias_col) val = bs[rr];
        if (c < H || bias_col) w[(int64_t)r * ld + c] = val;
    }
    if (b && threadIdx.x == 0) b[r] = bs[rr];
}

// dW rows r < 3H (row stride ld_dw) -> dwq | dwk | dwv [H, H]; db[r * db_stride] -> dbq | dbk | dbv [H]; one
// workgroup per row
__global__ void __launch_bounds__(BLK) k_qkv_unpack(int64_t H, const float* __restrict__ dw, int64_t ld_dw,
                                                    const float* __restrict__ db, int64_t db_stride,
                                                    float* __restrict__ dwq, float* __restrict__ dwk,
                                                    float* __restrict__ dwv, float* __restrict__ dbq,
                                                    float* __restrict__ dbk, float* __restrict__ dbv) {
    const int r = blockIdx.x, part = r / (int)H, rr = r - part * (int)H;
    float* dst = part == 0 ? dwq : part == 1 ? dwk : dwv;
    if (dw && dst)
        for (int c = threadIdx.x; c < (int)H; c += BLK) dst[(int64_t)rr * H + c] = dw[(int64_t)r * ld_dw + c];
    float* dstb = part == 0 ? dbq : part == 1 ? dbk : dbv;
    if (db && dstb && threadIdx.x == 0) dstb[rr] = db[(int64_t)r * db_stride];
}

// Temporal bias table (temporal_attention.py:732-790, the additive terms of :1010-1027): tab[h][d], d = i - j + T - 1,
// = R[clamp(δ + m, 0, 2m)][h] + K[δ + W][h]·[|δ| <= W] with δ = d - (T - 1) -- the gathers the layer used to run as
// two one-hot GEMMs, an add and a transpose copy (forward) and two GEMMs (backward).  Forward: the same fp32 add as
// before (bitwise).  Backward: dK[k][h] = g[h][k - W + T - 1] (one diagonal each), dR[k][h] = Σ over the diagonals
// clamped onto k, in ascending d (deterministic).
__global__ void __launch_bounds__(BLK) k_bias_table_fwd(int T, int heads, const float* __restrict__ K, int W,
                                                        const float* __restrict__ R, int m, float* __restrict__ tab) {
    const int D = 2 * T - 1;
    for (int i = blockIdx.x * BLK + threadIdx.x; i < heads * D; i += gridDim.x * BLK) {
        const int h = i / D, d = i % D, dl = d - (T - 1);
        const float kv = (dl >= -W && dl <= W) ? K[(dl + W) * heads + h] : 0.f;
        tab[i] = R ? R[min(max(dl + m, 0), 2 * m) * heads + h] + kv : kv;
    }
}

__global__ void __launch_bounds__(BLK) k_bias_table_bwd(int T, int heads, const float* __restrict__ g, int W, int m,
                                                        float* __restrict__ dK, float* __restrict__ dR) {
    const int D = 2 * T - 1, nk = (2 * W + 1) * heads, nr = dR ? (2 * m + 1) * heads : 0;
    for (int i = blockIdx.x * BLK + threadIdx.x; i < nk + nr; i += gridDim.x * BLK) {
        if (i < nk) {
            const int k = i / heads, h = i % heads, d = k - W + T - 1;
            if (dK) dK[i] = (d >= 0 && d < D) ? g[h * D + d] : 0.f;
        } else {
            const int j = i - nk, k = j / heads, h = j % heads;
            float acc = 0.f;
            for (int d = 0; d < D; ++d)
                if (min(max(d - (T - 1) + m, 0), 2 * m) == k) acc += g[h * D + d];
            dR[j] = acc;
        }
    }
}

}  // namespace
}  // namespace tagan

extern "C" {

int tagan_qkv_pack(int64_t H, const float* wq, const float* wk, const float* wv, const float* bq, const float* bk,
                   const float* bv, float* w, int64_t ld_w, int32_t bias_col, float* b, void* stream) {
    using namespace tagan;
    TAGAN_REQUIRE(H > 0 && wq && wk && wv && w && ld_w >= H + (bias_col ? 1 : 0), TAGAN_ERR_ARG,
                  "qkv_pack: bad argument (H=%lld ld=%lld)", (long long)H, (long long)ld_w);
    TAGAN_REQUIRE(!(bias_col || b) || (bq && bk && bv), TAGAN_ERR_ARG, "qkv_pack: null bias");
    TAGAN_REQUIRE(3 * H <= (1 << 30) && ld_w <= (1 << 30), TAGAN_ERR_ARG, "qkv_pack: H=%lld too large", (long long)H);
    k_qkv_pack<<<(unsigned)(3 * H), BLK, 0, as_stream(stream)>>>(H, wq, wk, wv, bq, bk, bv, w, ld_w, bias_col, b);
    TAGAN_CHECK_LAUNCH("qkv_pack");
    return TAGAN_OK;
}

int tagan_qkv_unpack(int64_t H, const float* dw, int64_t ld_dw, const float* db, int64_t db_stride, float* dwq,
                     float* dwk, float* dwv, float* dbq, float* dbk, float* dbv, void* stream) {
    using namespace tagan;
    TAGAN_REQUIRE(H > 0 && (!dw || ld_dw >= H) && (!db || db_stride >= 1), TAGAN_ERR_ARG, "qkv_unpack: bad argument");
    TAGAN_REQUIRE(3 * H <= (1 << 30), TAGAN_ERR_ARG, "qkv_unpack: H=%lld too large", (long long)H);
    k_qkv_unpack<<<(unsigned)(3 * H), BLK, 0, as_stream(stream)>>>(H, dw, ld_dw, db, db_stride, dwq, dwk, dwv, dbq, dbk,
                                                                 dbv);
    TAGAN_CHECK_LAUNCH("qkv_unpack");
    return TAGAN_OK;
}

int tagan_temporal_bias_table(int32_t T, int32_t heads, const float* K, int32_t W, const float* R, int32_t m,
                              float* tab, void* stream) {
    using namespace tagan;
    TAGAN_REQUIRE(T > 0 && heads > 0 && W >= 0 && m >= 0 && K && tab, TAGAN_ERR_ARG, "temporal_bias_table: bad args");
    const int n = heads * (2 * T - 1);
    k_bias_table_fwd<<<(unsigned)((n + BLK - 1) / BLK), BLK, 0, as_stream(stream)>>>(T, heads, K, W, R, m, tab);
    TAGAN_CHECK_LAUNCH("temporal_bias_table");
    return TAGAN_OK;
}

int tagan_temporal_bias_table_bwd(int32_t T, int32_t heads, const float* g, int32_t W, int32_t m, float* dK,
                                  float* dR, void* stream) {
    using namespace tagan;
    TAGAN_REQUIRE(T > 0 && heads > 0 && W >= 0 && m >= 0 && g && (dK || dR), TAGAN_ERR_ARG,
                  "temporal_bias_table_bwd: bad args");
    const int n = (2 * W + 1) * heads + (dR ? (2 * m + 1) * heads : 0);
    k_bias_table_bwd<<<(unsigned)((n + BLK - 1) / BLK), BLK, 0, as_stream(stream)>>>(T, heads, g, W, m, dK, dR);
    TAGAN_CHECK_LAUNCH("temporal_bias_table_bwd");
    return TAGAN_OK;
}

}  // extern "C"
