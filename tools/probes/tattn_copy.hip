// Probe: the temporal kernels' HBM access pattern with no compute.  Same wave -> (row, head) map as
// k_tattn_fwd_v4 / k_tattn_bwd_v4 (XCD-aware, persistent over rows), same lane -> (step, 4 features) loads of the
// time-major [T, N, 3H] projection; "fwd" reads Q, K, V and writes one [T, N, H] tensor, "bwd" reads Q, K, V, dO
// and writes three.  Prints GB/s of the algorithmic bytes: the bandwidth this layout allows the real kernels.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int TT, int MODE>
__global__ void __launch_bounds__(64) k_copy(long rows, int T, int heads, int d, long s_row, long s_t,
                                             const float* qkv, const float* dout, float* o1, float* o2, float* o3,
                                             int xcd, long do_row = -1, long do_t = -1) {
    if (do_row < 0) { do_row = heads * d; do_t = rows * heads * d; }
    const int lane = threadIdx.x, c = lane & 15, g = lane >> 4;
    const int b = blockIdx.x, nb = gridDim.x;
    int h; long rg;
    if (xcd && nb % (8 * heads) == 0) { const int y = b >> 3; h = y % heads; rg = (long)(y / heads) * 8 + (b & 7); }
    else { h = b % heads; rg = b / heads; }
    const long G = nb / heads;
    const int H = heads * d;
    for (long r = rg; r < rows; r += G) {
        float4 q[TT], k[TT], v[TT], dd[TT];
#pragma unroll
        for (int t = 0; t < TT; ++t) {
            const int i = t * 16 + c;
            const long off = r * s_row + (long)i * s_t + h * d + 4 * g;
            if (i < T) {
                q[t] = *(const float4*)(qkv + off);
                k[t] = *(const float4*)(qkv + off + H);
                v[t] = *(const float4*)(qkv + off + 2 * H);
                if (MODE) dd[t] = *(const float4*)(dout + r * do_row + (long)i * do_t + h * d + 4 * g);
            }
        }
#pragma unroll
        for (int t = 0; t < TT; ++t) {
            const int i = t * 16 + c;
            if (i >= T) continue;
            const long oo = r * do_row + (long)i * do_t + h * d + 4 * g;
            float4 a = make_float4(q[t].x + k[t].x + v[t].x, q[t].y + k[t].y + v[t].y, q[t].z + k[t].z + v[t].z,
                                   q[t].w + k[t].w + v[t].w);
            if (!MODE) { *(float4*)(o1 + oo) = a; continue; }
            const long od = r * s_row + (long)i * s_t + h * d + 4 * g;
            *(float4*)(o1 + od) = make_float4(a.x + dd[t].x, a.y, a.z, a.w);
            *(float4*)(o2 + od + H) = make_float4(a.x, a.y + dd[t].y, a.z, a.w);
            *(float4*)(o3 + od + 2 * H) = make_float4(a.x, a.y, a.z + dd[t].z, a.w);
        }
    }
}

// the same traffic with two heads per wave at d = 16: 8 lanes cover one step's 128-B two-head segment (one full
// line), 8 steps per instruction
template <int TT, int MODE>
__global__ void __launch_bounds__(64) k_copy2(long rows, int T, int heads, int d, long s_row, long s_t,
                                              const float* qkv, const float* dout, float* o1, float* o2, float* o3) {
    const int lane = threadIdx.x, sl = lane >> 3, g = lane & 7;
    const int b = blockIdx.x, nb = gridDim.x, hp = heads / 2;
    int h; long rg;
    { const int y = b >> 3; h = y % hp; rg = (long)(y / hp) * 8 + (b & 7); }
    const long G = nb / hp;
    const int H = heads * d;
    for (long r = rg; r < rows; r += G) {
        float4 q[2 * TT], k[2 * TT], v[2 * TT], dd[2 * TT];
#pragma unroll
        for (int t = 0; t < 2 * TT; ++t) {
            const int i = t * 8 + sl;
            const long off = r * s_row + (long)i * s_t + h * 2 * d + 4 * g;
            if (i < T) {
                q[t] = *(const float4*)(qkv + off);
                k[t] = *(const float4*)(qkv + off + H);
                v[t] = *(const float4*)(qkv + off + 2 * H);
                if (MODE) dd[t] = *(const float4*)(dout + r * H + (long)i * rows * H + h * 2 * d + 4 * g);
            }
        }
#pragma unroll
        for (int t = 0; t < 2 * TT; ++t) {
            const int i = t * 8 + sl;
            if (i >= T) continue;
            const long oo = r * H + (long)i * rows * H + h * 2 * d + 4 * g;
            float4 a = make_float4(q[t].x + k[t].x + v[t].x, q[t].y + k[t].y + v[t].y, q[t].z + k[t].z + v[t].z,
                                   q[t].w + k[t].w + v[t].w);
            if (!MODE) { *(float4*)(o1 + oo) = a; continue; }
            const long od = r * s_row + (long)i * s_t + h * 2 * d + 4 * g;
            *(float4*)(o1 + od) = make_float4(a.x + dd[t].x, a.y, a.z, a.w);
            *(float4*)(o2 + od + H) = make_float4(a.x, a.y + dd[t].y, a.z, a.w);
            *(float4*)(o3 + od + 2 * H) = make_float4(a.x, a.y, a.z + dd[t].z, a.w);
        }
    }
}

// whole-row slabs: one 256-thread workgroup per node row streams the row's [T, 3H] Q|K|V (and [T, H] dO) as flat
// float4 runs (1.5 KB contiguous per step), writes [T, H] (fwd) or [T, 3H] (bwd)
template <int MODE>
__global__ void __launch_bounds__(256) k_copy_row(long rows, int T, int H, long s_row, long s_t, const float* qkv,
                                                  const float* dout, float* o1, float* o3) {
    const int H4 = H / 4;
    for (long r = blockIdx.x; r < rows; r += gridDim.x) {
        if (!MODE) {
            for (int e = threadIdx.x; e < T * H4; e += 256) {
                const int t = e / H4, c4 = e % H4;
                const long off = r * s_row + (long)t * s_t + 4 * c4;
                const float4 q = *(const float4*)(qkv + off), k = *(const float4*)(qkv + off + H),
                             v = *(const float4*)(qkv + off + 2 * H);
                *(float4*)(o1 + r * H + (long)t * rows * H + 4 * c4) =
                    make_float4(q.x + k.x + v.x, q.y + k.y + v.y, q.z + k.z + v.z, q.w + k.w + v.w);
            }
        } else {
            for (int e = threadIdx.x; e < T * H4; e += 256) {
                const int t = e / H4, c4 = e % H4;
                const long off = r * s_row + (long)t * s_t + 4 * c4;
                const float4 q = *(const float4*)(qkv + off), k = *(const float4*)(qkv + off + H),
                             v = *(const float4*)(qkv + off + 2 * H);
                const float4 dd = *(const float4*)(dout + r * H + (long)t * rows * H + 4 * c4);
                *(float4*)(o3 + off) = make_float4(q.x + dd.x, q.y, q.z, q.w);
                *(float4*)(o3 + off + H) = make_float4(k.x, k.y + dd.y, k.z, k.w);
                *(float4*)(o3 + off + 2 * H) = make_float4(v.x, v.y, v.z + dd.z, v.w);
            }
        }
    }
}

int main(int argc, char** argv) {
    const long N = argc > 1 ? atol(argv[1]) : 10000;
    const int T = argc > 2 ? atoi(argv[2]) : 32, H = argc > 3 ? atoi(argv[3]) : 128, heads = argc > 4 ? atoi(argv[4]) : 8;
    const int d = H / heads;
    const size_t nqkv = (size_t)T * N * 3 * H, nh = (size_t)T * N * H;
    float *qkv, *dout, *o, *dq;
    CK(hipMalloc(&qkv, nqkv * 4)); CK(hipMalloc(&dout, nh * 4)); CK(hipMalloc(&o, nh * 4)); CK(hipMalloc(&dq, nqkv * 4));
    CK(hipMemset(qkv, 0, nqkv * 4)); CK(hipMemset(dout, 0, nh * 4));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const double unit = (double)N * T * H * 4;
    for (int G : {256, 1024, 4096}) {
        for (int xcd = 0; xcd < 2; ++xcd) {
            for (int mode = 0; mode < 2; ++mode) {
                const int grid = (int)std::min<long>(N, G) / 8 * 8 * heads;
                auto go = [&] {
                    if (mode == 0) {
                        if (T <= 16) k_copy<1, 0><<<grid, 64>>>(N, T, heads, d, 3 * H, N * 3 * H, qkv, dout, o, o, o, xcd);
                        else k_copy<2, 0><<<grid, 64>>>(N, T, heads, d, 3 * H, N * 3 * H, qkv, dout, o, o, o, xcd);
                    } else {
                        if (T <= 16) k_copy<1, 1><<<grid, 64>>>(N, T, heads, d, 3 * H, N * 3 * H, qkv, dout, dq, dq, dq, xcd);
                        else k_copy<2, 1><<<grid, 64>>>(N, T, heads, d, 3 * H, N * 3 * H, qkv, dout, dq, dq, dq, xcd);
                    }
                };
                for (int i = 0; i < 3; ++i) go();
                CK(hipEventRecord(e0));
                const int reps = 20;
                for (int i = 0; i < reps; ++i) go();
                CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
                float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
                const double bytes = mode == 0 ? 4 * unit : 7 * unit;
                printf("N=%ld T=%d H=%d heads=%d groups=%d xcd=%d %s: %.1f us  %.0f GB/s\n", N, T, H, heads, G, xcd,
                       mode ? "bwd(4r+3w)" : "fwd(3r+1w)", ms * 1e3, bytes / ms / 1e6);
            }
        }
    }
    for (int G : {2048, 8192}) {
        for (int mode = 0; mode < 2; ++mode) {
            const int grid = (int)std::min<long>(N, G);
            auto go = [&] {
                if (mode == 0) k_copy_row<0><<<grid, 256>>>(N, T, H, 3 * H, N * 3 * H, qkv, dout, o, o);
                else k_copy_row<1><<<grid, 256>>>(N, T, H, 3 * H, N * 3 * H, qkv, dout, dq, dq);
            };
            for (int i = 0; i < 3; ++i) go();
            CK(hipEventRecord(e0));
            const int reps = 20;
            for (int i = 0; i < reps; ++i) go();
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
            const double bytes = mode == 0 ? 4 * unit : 7 * unit;
            printf("ROW N=%ld T=%d blocks=%d %s: %.1f us  %.0f GB/s\n", N, T, G, mode ? "bwd(4r+3w)" : "fwd(3r+1w)",
                   ms * 1e3, bytes / ms / 1e6);
        }
    }
    if (d == 16) {
        for (int G : {1024, 4096}) {
            for (int mode = 0; mode < 2; ++mode) {
                const int grid = (int)std::min<long>(N, G) / 8 * 8 * (heads / 2);
                auto go = [&] {
                    if (mode == 0) k_copy2<2, 0><<<grid, 64>>>(N, T, heads, d, 3 * H, N * 3 * H, qkv, dout, o, o, o);
                    else k_copy2<2, 1><<<grid, 64>>>(N, T, heads, d, 3 * H, N * 3 * H, qkv, dout, dq, dq, dq);
                };
                for (int i = 0; i < 3; ++i) go();
                CK(hipEventRecord(e0));
                const int reps = 20;
                for (int i = 0; i < reps; ++i) go();
                CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
                float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
                const double bytes = mode == 0 ? 4 * unit : 7 * unit;
                printf("PAIR N=%ld T=%d groups=%d %s: %.1f us  %.0f GB/s\n", N, T, G, mode ? "bwd(4r+3w)" : "fwd(3r+1w)",
                       ms * 1e3, bytes / ms / 1e6);
            }
        }
    }
    // node-major layouts: [N, T, 3H] projection (s_row = T*3H, s_t = 3H); dO / O time-major (nm=1) or node-major (nm=2)
    for (int nm = 1; nm <= 2; ++nm) {
        for (int G : {1024, 4096}) {
            for (int mode = 0; mode < 2; ++mode) {
                const int grid = (int)std::min<long>(N, G) / 8 * 8 * heads;
                const long dr = nm == 2 ? (long)T * H : H, dt = nm == 2 ? H : N * H;
                auto go = [&] {
                    if (mode == 0) k_copy<2, 0><<<grid, 64>>>(N, T, heads, d, (long)T * 3 * H, 3 * H, qkv, dout, o, o, o, 1, dr, dt);
                    else k_copy<2, 1><<<grid, 64>>>(N, T, heads, d, (long)T * 3 * H, 3 * H, qkv, dout, dq, dq, dq, 1, dr, dt);
                };
                for (int i = 0; i < 3; ++i) go();
                CK(hipEventRecord(e0));
                const int reps = 20;
                for (int i = 0; i < reps; ++i) go();
                CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
                float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
                const double bytes = mode == 0 ? 4 * unit : 7 * unit;
                printf("NODEMAJOR%s N=%ld T=%d groups=%d %s: %.1f us  %.0f GB/s\n", nm == 2 ? "-all" : "-qkv", N, T, G,
                       mode ? "bwd(4r+3w)" : "fwd(3r+1w)", ms * 1e3, bytes / ms / 1e6);
            }
        }
    }
    return 0;
}
