// Graph-feature pooling of model.py:377-427 on the time-major temporal output.
//
// The reference holds the temporal output node-major [N, T, H] and takes
//   gf[t] = mean(out.view(T, -1, H)[t]) = mean of node-major flat rows [t*N, (t+1)*N)
// (flat row f = n*T + t'), which mixes nodes and steps.  Here the output is time-major
// [T, N, H]; flat row f lives at time-major row (f % T)*N + f / T.  HBM-bound gather:
// a group of H/4 lanes (float4) owns one row; block (t, s) sums slice s of chunk t
// into a partial, and the ordered column sum (k_colsum_parts) folds the slices —
// deterministic.  Backward broadcasts g[t]/N back to the rows of chunk t.
#include "common.cuh"

namespace tagan {
namespace {

constexpr int BLK = 256;
constexpr int SLICES = 16;   // partial slices per chunk (T * 16 blocks: >= 512 at T = 32)

__global__ void __launch_bounds__(BLK) k_pool_fwd(const float* __restrict__ x, int T, int64_t N, int H,
                                                  int64_t ld_row, int64_t ld_t, float* __restrict__ part) {
    __shared__ float red[4 * BLK];   // rpb * H = 4 * BLK floats
    const int t = blockIdx.x / SLICES, sl = blockIdx.x % SLICES;
    const int lpr = H / 4, rpb = BLK / lpr;          // lanes per row, rows per block-iteration
    const int lane = threadIdx.x % lpr, rsub = threadIdx.x / lpr;
    const int64_t f_beg = (int64_t)t * N, per = (N + SLICES - 1) / SLICES;
    const int64_t a = f_beg + sl * per, b = f_beg + min<int64_t>(N, (int64_t)(sl + 1) * per);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t f = a + rsub; f < b; f += rpb) {
        const int64_t tp = f % T, n = f / T;
        const float4 v = *(const float4*)(x + tp * ld_t + n * ld_row + lane * 4);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    // fixed-order block reduction over the rpb row groups
    float* r = red;
    *(float4*)(r + (size_t)rsub * H + lane * 4) = acc;
    __syncthreads();
    for (int c = threadIdx.x; c < H; c += BLK) {
        float s = 0.f;
        for (int k = 0; k < rpb; ++k) s += r[(size_t)k * H + c];
        part[((int64_t)sl * T + t) * H + c] = s;
    }
}

__global__ void __launch_bounds__(BLK) k_pool_bwd(const float* __restrict__ g, int T, int64_t N, int H,
                                                  float inv_n, float* __restrict__ dx, int64_t ld_row,
                                                  int64_t ld_t) {
    const int lpr = H / 4;
    const int64_t rows = (int64_t)T * N;
    for (int64_t i = blockIdx.x * (int64_t)BLK + threadIdx.x; i < rows * lpr; i += (int64_t)gridDim.x * BLK) {
        const int64_t row = i / lpr;            // time-major row = t'*N + n
        const int c = (int)(i % lpr) * 4;
        const int64_t tp = row / N, n = row % N;
        const int64_t chunk = (n * T + tp) / N;
        const float4 v = *(const float4*)(g + chunk * H + c);
        *(float4*)(dx + tp * ld_t + n * ld_row + c) = make_float4(v.x * inv_n, v.y * inv_n, v.z * inv_n, v.w * inv_n);
    }
}

}  // namespace
}  // namespace tagan

extern "C" {

size_t tagan_pool_workspace(int32_t T, int32_t H) { return (size_t)tagan::SLICES * T * H * sizeof(float); }

int tagan_pool_fwd(int dtype, int32_t T, int64_t N, int32_t H, const float* x, int64_t ld_row, int64_t ld_t,
                   float* out, void* workspace, size_t workspace_bytes, void* stream) {
    using namespace tagan;
    TAGAN_REQUIRE(dtype == TAGAN_F32, TAGAN_ERR_UNSUPPORTED, "pool: dtype %d", dtype);
    TAGAN_REQUIRE(T > 0 && N > 0 && H % 4 == 0 && H >= 4 && H <= 1024 && BLK % (H / 4) == 0,
                  TAGAN_ERR_UNSUPPORTED, "pool: H=%d unsupported", H);
    TAGAN_REQUIRE(x && out && ld_row % 4 == 0 && ld_t % 4 == 0, TAGAN_ERR_ARG, "pool: bad args");
    TAGAN_REQUIRE(workspace && workspace_bytes >= tagan_pool_workspace(T, H), TAGAN_ERR_WORKSPACE, "pool: ws");
    hipStream_t s = as_stream(stream);
    float* part = (float*)workspace;
    k_pool_fwd<<<T * SLICES, BLK, 0, s>>>(x, T, N, H, ld_row, ld_t, part);
    TAGAN_CHECK_LAUNCH("pool_fwd");
    // ordered sum over slices, times the 1/N of the mean
    launch_colsum(part, SLICES, T * H, out, nullptr, T * H, s, 1.f / (float)N);
    TAGAN_CHECK_LAUNCH("pool_fwd_sum");
    return TAGAN_OK;
}

int tagan_pool_bwd(int dtype, int32_t T, int64_t N, int32_t H, const float* g, float* dx, int64_t ld_row,
                   int64_t ld_t, void* stream) {
    using namespace tagan;
    TAGAN_REQUIRE(dtype == TAGAN_F32, TAGAN_ERR_UNSUPPORTED, "pool: dtype %d", dtype);
    TAGAN_REQUIRE(T > 0 && N > 0 && H % 4 == 0 && g && dx, TAGAN_ERR_ARG, "pool_bwd: bad args");
    const int64_t work = (int64_t)T * N * (H / 4);
    const int grid = (int)std::min<int64_t>((work + BLK - 1) / BLK, 256 * 64);
    k_pool_bwd<<<grid, BLK, 0, as_stream(stream)>>>(g, T, N, H, 1.f / (float)N, dx, ld_row, ld_t);
    TAGAN_CHECK_LAUNCH("pool_bwd");
    return TAGAN_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------- column sums
// Bias gradients of the projections: out[c] = sum_r x[r][c] for a tall [M, N] matrix.  Stage 1:
// block b sums a contiguous row range with float4 lanes (N/4 lanes per row, several rows per
// block iteration) into part[b][N]; stage 2 = the ordered column sum (k_colsum_parts).
namespace tagan {
namespace {

constexpr int CS_BLOCKS = 1024;

template <typename S>
__global__ void __launch_bounds__(BLK) k_colsum_rows(const void* __restrict__ x, int64_t M, int N, int64_t ld,
                                                     float* __restrict__ part) {
    __shared__ float red[4 * BLK];
    const int lpr = N / 4, rpb = BLK / lpr;
    const int lane = threadIdx.x % lpr, rsub = threadIdx.x / lpr;
    const int64_t per = (M + gridDim.x - 1) / gridDim.x;
    const int64_t a = blockIdx.x * per, b = min<int64_t>(M, a + per);
    float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0, s2 = s0, s3 = s0;
    if (rsub < rpb) {
        int64_t r = a + rsub;
        for (; r + 3 * rpb < b; r += 4 * rpb) {        // four rows in flight per thread
            const float4 v0 = Io<S>::ld(x, r * ld + lane * 4);
            const float4 v1 = Io<S>::ld(x, (r + rpb) * ld + lane * 4);
            const float4 v2 = Io<S>::ld(x, (r + 2 * rpb) * ld + lane * 4);
            const float4 v3 = Io<S>::ld(x, (r + 3 * rpb) * ld + lane * 4);
            s0.x += v0.x; s0.y += v0.y; s0.z += v0.z; s0.w += v0.w;
            s1.x += v1.x; s1.y += v1.y; s1.z += v1.z; s1.w += v1.w;
            s2.x += v2.x; s2.y += v2.y; s2.z += v2.z; s2.w += v2.w;
            s3.x += v3.x; s3.y += v3.y; s3.z += v3.z; s3.w += v3.w;
        }
        for (; r < b; r += rpb) {
            const float4 v = Io<S>::ld(x, r * ld + lane * 4);
            s0.x += v.x; s0.y += v.y; s0.z += v.z; s0.w += v.w;
        }
        const float4 acc = make_float4((s0.x + s1.x) + (s2.x + s3.x), (s0.y + s1.y) + (s2.y + s3.y),
                                       (s0.z + s1.z) + (s2.z + s3.z), (s0.w + s1.w) + (s2.w + s3.w));
        *(float4*)(red + (size_t)rsub * N + lane * 4) = acc;
    }
    __syncthreads();
    for (int c = threadIdx.x; c < N; c += BLK) {
        float s = 0.f;
        for (int k = 0; k < rpb; ++k) s += red[(size_t)k * N + c];
        part[(int64_t)blockIdx.x * N + c] = s;
    }
}

}  // namespace
}  // namespace tagan

extern "C" {

size_t tagan_colsum_workspace(int64_t M, int32_t N) {
    (void)M;
    return (size_t)tagan::CS_BLOCKS * N * sizeof(float);
}

int tagan_colsum(int dtype, int64_t M, int32_t N, const void* x, int64_t ld, float* out, void* workspace,
                 size_t workspace_bytes, void* stream) {
    using namespace tagan;
    TAGAN_REQUIRE(dtype == TAGAN_F32 || dtype == TAGAN_BF16, TAGAN_ERR_UNSUPPORTED, "colsum: dtype %d", dtype);
    TAGAN_REQUIRE(M > 0 && N % 4 == 0 && N >= 4 && N / 4 <= BLK && ld % 4 == 0 && ld >= N && x && out,
                  TAGAN_ERR_ARG, "colsum: bad args (N=%d)", N);
    TAGAN_REQUIRE(workspace && workspace_bytes >= tagan_colsum_workspace(M, N), TAGAN_ERR_WORKSPACE, "colsum: ws");
    const int nblk = (int)std::min<int64_t>(CS_BLOCKS, (M + 63) / 64);
    hipStream_t s = as_stream(stream);
    if (dtype == TAGAN_BF16) k_colsum_rows<bf16s><<<nblk, BLK, 0, s>>>(x, M, N, ld, (float*)workspace);
    else k_colsum_rows<float><<<nblk, BLK, 0, s>>>(x, M, N, ld, (float*)workspace);
    TAGAN_CHECK_LAUNCH("colsum_rows");
    launch_colsum((float*)workspace, nblk, N, out, nullptr, N, s);
    TAGAN_CHECK_LAUNCH("colsum_parts");
    return TAGAN_OK;
}

}  // extern "C"
