// Graph-feature pooling of model.py:377-427 on the time-major temporal output.
//
// The reference holds the temporal output node-major [N, T, H] and takes
//   gf[t] = mean(out.view(T, -1, H)[t]) = mean of node-major flat rows [t*N, (t+1)*N)
// (flat row f = n*T + t'), which mixes nodes and steps.  Here the output is time-major
// [T, N, H]; flat row f lives at time-major row (f % T)*N + f / T.  HBM-bound gather:
// a group of H/4 lanes (float4) owns one row, 4 row loads in flight per lane; block (t, s) sums slice s of chunk t
// into a partial, and the ordered column sum (k_colsum_parts) folds the slices —
// deterministic.  Backward broadcasts g[t]/N back to the rows of chunk t.
#include "common.cuh"

namespace tagan {
namespace {

constexpr int BLK = 256;
constexpr int SLICES = 64;   // partial slices per chunk (T * 64 blocks: 2048 at T = 32, 8 waves per CU)
constexpr int PU = 4;        // independent row loads in flight per thread

// IDX = int32_t whenever T * N * H fits (every config here): the flat-row -> (step, node) split is a
// 32-bit divide instead of a ~40-instruction 64-bit one per row.
template <typename IDX>
__global__ void __launch_bounds__(BLK) k_pool_fwd(const float* __restrict__ x, int T, int64_t N, int H,
                                                  int64_t ld_row, int64_t ld_t, float* __restrict__ part) {
    __shared__ float red[4 * BLK];   // rpb * H = 4 * BLK floats
    const int t = blockIdx.x / SLICES, sl = blockIdx.x % SLICES;
    const int lpr = H / 4, rpb = BLK / lpr;          // lanes per row, rows per block-iteration
    const int lane = threadIdx.x % lpr, rsub = threadIdx.x / lpr;
    const IDX n_ = (IDX)N, t_ = (IDX)T;
    const IDX f_beg = (IDX)t * n_, per = (n_ + SLICES - 1) / SLICES;
    const IDX a = f_beg + (IDX)sl * per, b = f_beg + ((IDX)(sl + 1) * per < n_ ? (IDX)(sl + 1) * per : n_);
    float4 acc[PU];
#pragma unroll
    for (int u = 0; u < PU; ++u) acc[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    IDX f = a + rsub;
    for (; f + (PU - 1) * rpb < b; f += PU * rpb) {
        float4 v[PU];
#pragma unroll
        for (int u = 0; u < PU; ++u) {
            const IDX ff = f + u * rpb, tp = ff % t_, n = ff / t_;
            v[u] = *(const float4*)(x + (int64_t)tp * ld_t + (int64_t)n * ld_row + lane * 4);
        }
#pragma unroll
        for (int u = 0; u < PU; ++u) {
            acc[u].x += v[u].x; acc[u].y += v[u].y; acc[u].z += v[u].z; acc[u].w += v[u].w;
        }
    }
#pragma unroll
    for (int u = 0; u < PU - 1; ++u) {               // tail: fewer than PU rows left for this thread
        const IDX ff = f + u * rpb;
        if (ff < b) {
            const IDX tp = ff % t_, n = ff / t_;
            const float4 v = *(const float4*)(x + (int64_t)tp * ld_t + (int64_t)n * ld_row + lane * 4);
            acc[u].x += v.x; acc[u].y += v.y; acc[u].z += v.z; acc[u].w += v.w;
        }
    }
    float4 tot = acc[0];
#pragma unroll
    for (int u = 1; u < PU; ++u) { tot.x += acc[u].x; tot.y += acc[u].y; tot.z += acc[u].z; tot.w += acc[u].w; }
    // fixed-order block reduction over the rpb row groups
    float* r = red;
    *(float4*)(r + (size_t)rsub * H + lane * 4) = tot;
    __syncthreads();
    for (int c = threadIdx.x; c < H; c += BLK) {
        float s = 0.f;
        for (int k = 0; k < rpb; ++k) s += r[(size_t)k * H + c];
        part[((int64_t)sl * T + t) * H + c] = s;
    }
}

template <typename IDX>
__global__ void __launch_bounds__(BLK) k_pool_bwd(const float* __restrict__ g, int T, int64_t N, int H,
                                                  float inv_n, float* __restrict__ dx, int64_t ld_row,
                                                  int64_t ld_t) {
    const IDX lpr = H / 4, n_ = (IDX)N, t_ = (IDX)T;
    const IDX total = t_ * n_ * lpr;
    for (IDX i = blockIdx.x * (IDX)BLK + threadIdx.x; i < total; i += (IDX)gridDim.x * BLK) {
        const IDX row = i / lpr;                // time-major row = t'*N + n
        const int c = (int)(i - row * lpr) * 4;
        const IDX tp = row / n_, n = row - tp * n_;
        const IDX chunk = (n * t_ + tp) / n_;
        const float4 v = *(const float4*)(g + (int64_t)chunk * H + c);
        *(float4*)(dx + (int64_t)tp * ld_t + (int64_t)n * ld_row + c) =
            make_float4(v.x * inv_n, v.y * inv_n, v.z * inv_n, v.w * inv_n);
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
    if ((int64_t)T * N * H < ((int64_t)1 << 31)) k_pool_fwd<int32_t><<<T * SLICES, BLK, 0, s>>>(x, T, N, H, ld_row, ld_t, part);
    else k_pool_fwd<int64_t><<<T * SLICES, BLK, 0, s>>>(x, T, N, H, ld_row, ld_t, part);
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
    if ((int64_t)T * N * H < ((int64_t)1 << 31))
        k_pool_bwd<int32_t><<<grid, BLK, 0, as_stream(stream)>>>(g, T, N, H, 1.f / (float)N, dx, ld_row, ld_t);
    else k_pool_bwd<int64_t><<<grid, BLK, 0, as_stream(stream)>>>(g, T, N, H, 1.f / (float)N, dx, ld_row, ld_t);
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
