// Probe: sustained v_mfma_f32_32x32x2_f32 rate with register operands (4 accumulators per wave).
//   hipcc -O3 --offload-arch=gfx950 mfma_f32_rate.hip -o /tmp/mfma_rate && /tmp/mfma_rate
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void __launch_bounds__(256) k(float* out, int iters, float s) {
    f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    float a = threadIdx.x * 1e-3f, b = s;
    for (int i = 0; i < iters; ++i) {
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b, a, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, a, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_32x32x2f32(b, b, c3, 0, 0, 0);
        a += 1e-7f;
    }
    float t = 0.f;
    for (int g = 0; g < 16; ++g) t += c0[g] + c1[g] + c2[g] + c3[g];
    out[blockIdx.x * 256 + threadIdx.x] = t;
}

int main() {
    float* out;
    hipMalloc(&out, 4096 * 256 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int blocks : {256, 512, 1024, 2048}) {
        const int iters = 4096;
        k<<<blocks, 256>>>(out, 16, 1.f);
        hipEventRecord(e0);
        k<<<blocks, 256>>>(out, iters, 1.f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double fl = 2.0 * 32 * 32 * 2 * 4.0 * iters * (blocks * 4.0);
        printf("blocks %d (waves/SIMD %.1f): %.3f ms  %.1f TF/s\n", blocks, blocks * 4.0 / 1024, ms, fl / ms / 1e9);
    }
    return 0;
}
