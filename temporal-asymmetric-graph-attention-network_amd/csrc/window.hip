// Windowed aggregation over T of TemporalSkipConnection (temporal_propagation.py:846-946; TemporalPropagation's
// intended compute), time-major and in place of the reference's per-step Python loop:
//   out[t, n, :] = agg_{t' in [t-w, t+w] ∩ [0, T)} x[t', n, :]
// agg = mean (over the in-range steps: avg_pool1d count_include_pad=False), sum, or max (first maximum in
// window order wins, as max_pool1d's index).  One thread per (t, n, 4 features), float4 loads of the 2w+1
// rows; backward scatters by the transpose of the same windows (gather form: dx[t'] = Σ_t∈win(t') w_t·dy[t],
// no atomics), max by recomputing each window's winner.  HBM-bound: (2w+1) reads + 1 write per element,
// mostly L2 hits for neighbouring t.
#include "common.cuh"

namespace tagan {
namespace {

constexpr int WB = 256;

enum { AGG_MEAN = 0, AGG_MAX = 1, AGG_SUM = 2 };

template <int MODE>
__global__ void __launch_bounds__(WB) k_window_fwd(int T, int64_t N, int H4, int w, const float4* __restrict__ x,
                                                   float4* __restrict__ out) {
    const int64_t total = (int64_t)T * N * H4;
    for (int64_t i = blockIdx.x * (int64_t)WB + threadIdx.x; i < total; i += (int64_t)gridDim.x * WB) {
        const int64_t rowc = i % (N * H4);      // (n, c4) within a step
        const int t = (int)(i / (N * H4));
        const int t0 = max(0, t - w), t1 = min(T - 1, t + w);
        float4 acc = x[(int64_t)t0 * N * H4 + rowc];
        for (int tp = t0 + 1; tp <= t1; ++tp) {
            const float4 v = x[(int64_t)tp * N * H4 + rowc];
            if (MODE == AGG_MAX) {
                acc.x = (v.x > acc.x || v.x != v.x) ? v.x : acc.x;
                acc.y = (v.y > acc.y || v.y != v.y) ? v.y : acc.y;
                acc.z = (v.z > acc.z || v.z != v.z) ? v.z : acc.z;
                acc.w = (v.w > acc.w || v.w != v.w) ? v.w : acc.w;
            } else {
                acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
            }
        }
        if (MODE == AGG_MEAN) {
            const float s = 1.f / (float)(t1 - t0 + 1);
            acc.x *= s; acc.y *= s; acc.z *= s; acc.w *= s;
        }
        out[i] = acc;
    }
}

// winner index of one component of the window around t (first maximum in window order)
__device__ __forceinline__ int win_arg(const float* x, int64_t stride, int64_t off, int t0, int t1) {
    int best = t0;
    float bv = x[(int64_t)t0 * stride + off];
    for (int tp = t0 + 1; tp <= t1; ++tp) {
        const float v = x[(int64_t)tp * stride + off];
        if (v > bv || v != v) { bv = v; best = tp; }
    }
    return best;
}

template <int MODE>
__global__ void __launch_bounds__(WB) k_window_bwd(int T, int64_t N, int H4, int w, const float* __restrict__ x,
                                                   const float4* __restrict__ dy, float4* __restrict__ dx) {
    const int64_t total = (int64_t)T * N * H4;
    const int64_t stride = N * H4 * 4;
    for (int64_t i = blockIdx.x * (int64_t)WB + threadIdx.x; i < total; i += (int64_t)gridDim.x * WB) {
        const int64_t rowc = i % (N * H4);
        const int tp = (int)(i / (N * H4));     // the input step receiving gradient
        const int ta = max(0, tp - w), tb = min(T - 1, tp + w);   // outputs whose window contains tp
        float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int t = ta; t <= tb; ++t) {
            const float4 d = dy[(int64_t)t * N * H4 + rowc];
            if (MODE == AGG_MAX) {
                const int t0 = max(0, t - w), t1 = min(T - 1, t + w);
                const int64_t off = rowc * 4;
                if (win_arg(x, stride, off + 0, t0, t1) == tp) g.x += d.x;
                if (win_arg(x, stride, off + 1, t0, t1) == tp) g.y += d.y;
                if (win_arg(x, stride, off + 2, t0, t1) == tp) g.z += d.z;
                if (win_arg(x, stride, off + 3, t0, t1) == tp) g.w += d.w;
            } else {
                const float s = MODE == AGG_MEAN ? 1.f / (float)(min(T - 1, t + w) - max(0, t - w) + 1) : 1.f;
                g.x += d.x * s; g.y += d.y * s; g.z += d.z * s; g.w += d.w * s;
            }
        }
        dx[i] = g;
    }
}

unsigned wgrid(int64_t total) {
    const int64_t b = (total + WB - 1) / WB;
    return (unsigned)(b < 8192 ? b : 8192);
}

}  // namespace
}  // namespace tagan

extern "C" {

int tagan_window_fwd(int mode, int32_t T, int64_t N, int32_t H, int32_t w, const float* x, float* out, void* stream) {
    using namespace tagan;
    TAGAN_REQUIRE(mode >= 0 && mode <= 2, TAGAN_ERR_UNSUPPORTED, "window: mode %d", mode);
    TAGAN_REQUIRE(T > 0 && N > 0 && H > 0 && H % 4 == 0 && w >= 0 && x && out, TAGAN_ERR_ARG, "window_fwd: bad args");
    const int64_t total = (int64_t)T * N * (H / 4);
    hipStream_t s = as_stream(stream);
    const float4* xv = reinterpret_cast<const float4*>(x);
    float4* ov = reinterpret_cast<float4*>(out);
    if (mode == AGG_MEAN) k_window_fwd<AGG_MEAN><<<wgrid(total), WB, 0, s>>>(T, N, H / 4, w, xv, ov);
    else if (mode == AGG_MAX) k_window_fwd<AGG_MAX><<<wgrid(total), WB, 0, s>>>(T, N, H / 4, w, xv, ov);
    else k_window_fwd<AGG_SUM><<<wgrid(total), WB, 0, s>>>(T, N, H / 4, w, xv, ov);
    TAGAN_CHECK_LAUNCH("window_fwd");
    return TAGAN_OK;
}

int tagan_window_bwd(int mode, int32_t T, int64_t N, int32_t H, int32_t w, const float* x, const float* dy, float* dx,
                     void* stream) {
    using namespace tagan;
    TAGAN_REQUIRE(mode >= 0 && mode <= 2, TAGAN_ERR_UNSUPPORTED, "window: mode %d", mode);
    TAGAN_REQUIRE(T > 0 && N > 0 && H > 0 && H % 4 == 0 && w >= 0 && dy && dx && (mode != AGG_MAX || x), TAGAN_ERR_ARG,
                  "window_bwd: bad args");
    const int64_t total = (int64_t)T * N * (H / 4);
    hipStream_t s = as_stream(stream);
    const float4* dv = reinterpret_cast<const float4*>(dy);
    float4* ov = reinterpret_cast<float4*>(dx);
    if (mode == AGG_MEAN) k_window_bwd<AGG_MEAN><<<wgrid(total), WB, 0, s>>>(T, N, H / 4, w, x, dv, ov);
    else if (mode == AGG_MAX) k_window_bwd<AGG_MAX><<<wgrid(total), WB, 0, s>>>(T, N, H / 4, w, x, dv, ov);
    else k_window_bwd<AGG_SUM><<<wgrid(total), WB, 0, s>>>(T, N, H / 4, w, x, dv, ov);
    TAGAN_CHECK_LAUNCH("window_bwd");
    return TAGAN_OK;
}

}  // extern "C"
