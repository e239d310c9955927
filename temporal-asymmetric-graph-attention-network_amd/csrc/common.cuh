// Shared device/host helpers for libtagan_hip.so (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <math.h>

#include "../../include/tagan_hip.h"

namespace tagan {

// ---------------------------------------------------------------- error plumbing
void set_error(const char* fmt, ...);

#define TAGAN_REQUIRE(cond, code, ...)          \
    do {                                         \
        if (!(cond)) {                           \
            ::tagan::set_error(__VA_ARGS__);     \
            return (code);                       \
        }                                        \
    } while (0)

#define TAGAN_CHECK_LAUNCH(what)                                                       \
    do {                                                                               \
        hipError_t e_ = hipGetLastError();                                             \
        if (e_ != hipSuccess) {                                                        \
            ::tagan::set_error("%s: launch failed: %s", what, hipGetErrorString(e_));  \
            return TAGAN_ERR_LAUNCH;                                                   \
        }                                                                              \
    } while (0)

#define TAGAN_CHECK_HIP(call, what)                                                    \
    do {                                                                               \
        hipError_t e_ = (call);                                                        \
        if (e_ != hipSuccess) {                                                        \
            ::tagan::set_error("%s: %s", what, hipGetErrorString(e_));                 \
            return TAGAN_ERR_LAUNCH;                                                   \
        }                                                                              \
    } while (0)

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

static inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// ---------------------------------------------------------------- device helpers
constexpr int WAVE = 64;

// splitmix64 finaliser: counter-based uniform in [0,1) shared by every dropout mask.
__host__ __device__ __forceinline__ float uniform01(uint64_t seed, uint64_t index) {
    uint64_t z = seed + 0x9E3779B97F4A7C15ull * (index + 1ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (float)(uint32_t)(z >> 40) * (1.0f / 16777216.0f);
}

// XOR-butterfly sum over aligned groups of G lanes (G power of two <= 64).
template <int G>
__device__ __forceinline__ float group_sum(float x) {
#pragma unroll
    for (int o = 1; o < G; o <<= 1) x += __shfl_xor(x, o, 64);
    return x;
}

__device__ __forceinline__ float wave_sum(float x) { return group_sum<64>(x); }

// Bijective XCD-aware remap (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): blocks dealt round-robin to the 8 XCDs get contiguous logical ids,
// so each XCD walks a contiguous range of rows (one snapshot's K/V stay L2/MALL hot).
__device__ __forceinline__ int64_t xcd_remap(int64_t bid, int64_t nblk) {
    const int64_t q = nblk / 8, r = nblk % 8;
    const int64_t x = bid % 8, k = bid / 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
}

}  // namespace tagan
