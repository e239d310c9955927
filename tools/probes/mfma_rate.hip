// f32 MFMA issue-rate probe: 32x32x2 f32, 4 accumulators per wave, operands in registers (mode 0) or B from
// LDS by ds_read_b128 every 4 k-steps (mode 1, the proj_gemm.hip inner loop).  Prints TF/s per config.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f16v __attribute__((ext_vector_type(16)));
template <int MODE>
__global__ void k(float* out, int iters) {
    __shared__ float lds[128 * 132];
    const int lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 128 * 132; i += blockDim.x) lds[i] = (float)(i & 7);
    __syncthreads();
    f16v acc[4];
    for (int c = 0; c < 4; ++c) for (int i = 0; i < 16; ++i) acc[c][i] = 0.f;
    float a[64];
    for (int j = 0; j < 64; ++j) a[j] = (float)(lane + j);
    const float* bp = lds + (lane & 31) * 132 + 64 * (lane >> 5);
    for (int it = 0; it < iters; ++it) {
        asm volatile("" ::: "memory");   // LDS re-read every iteration (as per panel in proj_gemm)
#pragma unroll
        for (int s4 = 0; s4 < 16; ++s4) {
            float b[4][4];
            if (MODE == 1) {
#pragma unroll
                for (int cb = 0; cb < 4; ++cb) {
                    float4 v = *(const float4*)(bp + cb * 32 * 132 + 4 * s4);
                    b[cb][0] = v.x; b[cb][1] = v.y; b[cb][2] = v.z; b[cb][3] = v.w;
                }
            } else {
#pragma unroll
                for (int cb = 0; cb < 4; ++cb) for (int j = 0; j < 4; ++j) b[cb][j] = a[(s4 * 4 + j + cb) & 63];
            }
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int cb = 0; cb < 4; ++cb)
                    acc[cb] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[4 * s4 + j], b[cb][j], acc[cb], 0, 0, 0);
        }
    }
    float t = 0.f;
    for (int c = 0; c < 4; ++c) for (int i = 0; i < 16; ++i) t += acc[c][i];
    if (t == 1.2345f) out[0] = t;
}
int main() {
    float* d;
    hipMalloc(&d, 4);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int iters = 200;
    for (int mode = 0; mode < 2; ++mode)
        for (int waves = 4; waves <= 8; waves += 4)
            for (int wgpc = 1; wgpc <= 2; ++wgpc) {
                hipEvent_t e0, e1;
                hipEventCreate(&e0); hipEventCreate(&e1);
                dim3 g(cus * wgpc), b(64 * waves);
                auto launch = [&] { if (mode) k<1><<<g, b>>>(d, iters); else k<0><<<g, b>>>(d, iters); };
                launch();
                hipDeviceSynchronize();
                hipEventRecord(e0);
                for (int r = 0; r < 5; ++r) launch();
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms; hipEventElapsedTime(&ms, e0, e1);
                double flop = 5.0 * g.x * waves * (double)iters * 256 * 4096;
                printf("mode %d (%s) waves/WG %d WG/CU %d: %.1f TF/s\n", mode, mode ? "B from LDS" : "regs", waves,
                       wgpc, flop / (ms * 1e-3) / 1e12);
            }
    return 0;
}
