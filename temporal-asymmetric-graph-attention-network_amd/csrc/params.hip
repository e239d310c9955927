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

// one thread per element of the packed [3H, ld] matrix (bias column / zero pad included)
__global__ void __launch_bounds__(BLK) k_qkv_pack(int64_t H, const float* __restrict__ wq, const float* __restrict__ wk,
                                                  const float* __restrict__ wv, const float* __restrict__ bq,
                                                  const float* __restrict__ bk, const float* __restrict__ bv,
                                                  float* __restrict__ w, int64_t ld, int bias_col,
                                                  float* __restrict__ b) {
    const int64_t n = 3 * H * ld;
    for (int64_t t = blockIdx.x * (int64_t)BLK + threadIdx.x; t < n; t += (int64_t)gridDim.x * BLK) {
        const int64_t r = t / ld, c = t - r * ld;
        const int64_t part = r / H, rr = r - part * H;
        const float* src = part == 0 ? wq : part == 1 ? wk : wv;
        const float* bs = part == 0 ? bq : part == 1 ? bk : bv;
        float val = 0.f;
        if (c < H) val = src[rr * H + c];
        else if (c == H && bias_col) val = bs[rr];
        if (c < H || bias_col) w[t] = val;
        if (b && c == 0) b[r] = bs[rr];
    }
}

// dW rows r < 3H (row stride ld_dw) -> dwq | dwk | dwv [H, H]; db[r * db_stride] -> dbq | dbk | dbv [H]
__global__ void __launch_bounds__(BLK) k_qkv_unpack(int64_t H, const float* __restrict__ dw, int64_t ld_dw,
                                                    const float* __restrict__ db, int64_t db_stride,
                                                    float* __restrict__ dwq, float* __restrict__ dwk,
                                                    float* __restrict__ dwv, float* __restrict__ dbq,
                                                    float* __restrict__ dbk, float* __restrict__ dbv) {
    const int64_t n = 3 * H * (H + 1);
    for (int64_t t = blockIdx.x * (int64_t)BLK + threadIdx.x; t < n; t += (int64_t)gridDim.x * BLK) {
        const int64_t r = t / (H + 1), c = t - r * (H + 1);
        const int64_t part = r / H, rr = r - part * H;
        if (c < H) {
            float* dst = part == 0 ? dwq : part == 1 ? dwk : dwv;
            if (dw && dst) dst[rr * H + c] = dw[r * ld_dw + c];
        } else {
            float* dst = part == 0 ? dbq : part == 1 ? dbk : dbv;
            if (db && dst) dst[rr] = db[r * db_stride];
        }
    }
}

int grid_for(int64_t n) {
    const int64_t g = (n + BLK - 1) / BLK;
    return (int)std::min<int64_t>(std::max<int64_t>(g, 1), 2048);
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
    k_qkv_pack<<<grid_for(3 * H * ld_w), BLK, 0, as_stream(stream)>>>(H, wq, wk, wv, bq, bk, bv, w, ld_w, bias_col, b);
    TAGAN_CHECK_LAUNCH("qkv_pack");
    return TAGAN_OK;
}

int tagan_qkv_unpack(int64_t H, const float* dw, int64_t ld_dw, const float* db, int64_t db_stride, float* dwq,
                     float* dwk, float* dwv, float* dbq, float* dbk, float* dbv, void* stream) {
    using namespace tagan;
    TAGAN_REQUIRE(H > 0 && (!dw || ld_dw >= H) && (!db || db_stride >= 1), TAGAN_ERR_ARG, "qkv_unpack: bad argument");
    k_qkv_unpack<<<grid_for(3 * H * (H + 1)), BLK, 0, as_stream(stream)>>>(H, dw, ld_dw, db, db_stride, dwq, dwk, dwv,
                                                                          dbq, dbk, dbv);
    TAGAN_CHECK_LAUNCH("qkv_unpack");
    return TAGAN_OK;
}

}  // extern "C"
