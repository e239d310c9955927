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

// ---------------------------------------------------------------- bounds-check debug build
// `make debug` (= EXTRA=-DTAGAN_DEBUG into build_debug/ and libtagan_hip_debug.so; never the shipped library)
// compiles the device checks TAGAN_DBAD(cond, a, b) in: a failing check records (line, a, b) in this translation
// unit's device word, prints the first failure, and evaluates to true so the caller SKIPS the access it guards (no
// out-of-bounds access, no trap: a check must not take the GPU down).  Every TAGAN_CHECK_LAUNCH then synchronises
// the device and turns a recorded failure into TAGAN_ERR_LAUNCH with the file / line / values in tagan_last_error().
// The per-launch synchronisation makes the debug build eager-only (no HIP-graph capture).  In the default build the
// checks compile to `false` and cost nothing.
#ifdef TAGAN_DEBUG
static __device__ unsigned int g_tagan_dbg[4];   // per translation unit: {failures, line, a, b}
__device__ __noinline__ static bool tagan_dbg_record(const char* file, int line, long long a, long long b) {
    if (atomicAdd(&g_tagan_dbg[0], 1u) == 0u) {
        g_tagan_dbg[1] = (unsigned)line;
        g_tagan_dbg[2] = (unsigned)a;
        g_tagan_dbg[3] = (unsigned)b;
        printf("TAGAN_DEBUG %s:%d: check failed (a=%lld b=%lld)\n", file, line, a, b);
    }
    return true;
}
#define TAGAN_DBAD(cond, a, b) (!(cond) && tagan_dbg_record(__FILE__, __LINE__, (long long)(a), (long long)(b)))
static inline int tagan_dbg_poll(const char* what) {
    unsigned int h[4] = {0, 0, 0, 0};
    if (hipDeviceSynchronize() != hipSuccess) {
        ::tagan::set_error("%s: device error (debug build)", what);
        return TAGAN_ERR_LAUNCH;
    }
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_tagan_dbg), sizeof(h)) != hipSuccess) return TAGAN_OK;
    if (h[0] == 0) return TAGAN_OK;
    const unsigned int z[4] = {0, 0, 0, 0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_tagan_dbg), z, sizeof(z));
    ::tagan::set_error("%s: TAGAN_DEBUG check failed %u time(s), first at line %u of the kernel source (a=%d b=%d)",
                       what, h[0], h[1], (int)h[2], (int)h[3]);
    return TAGAN_ERR_LAUNCH;
}
#define TAGAN_DBG_POLL(what)                     \
    do {                                         \
        const int d_ = ::tagan::tagan_dbg_poll(what);     \
        if (d_ != TAGAN_OK) return d_;           \
    } while (0)
#else
#define TAGAN_DBAD(cond, a, b) false
#define TAGAN_DBG_POLL(what) \
    do {                     \
    } while (0)
#endif

#define TAGAN_CHECK_LAUNCH(what)                                                       \
    do {                                                                               \
        hipError_t e_ = hipGetLastError();                                             \
        if (e_ != hipSuccess) {                                                        \
            ::tagan::set_error("%s: launch failed: %s", what, hipGetErrorString(e_));  \
            return TAGAN_ERR_LAUNCH;                                                   \
        }                                                                              \
        TAGAN_DBG_POLL(what);                                                          \
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

// ---------------------------------------------------------------- lane reductions without the LDS crossbar
// __shfl_xor lowers to ds_bpermute_b32: an LDS-pipe round trip (~100 cycles) per butterfly step, serialised by the
// reduction's dependency chain and waited for with s_waitcnt lgkmcnt(0) each time.  Here the steps inside a 16-lane
// row are DPP moves (quad_perm xor 1 / xor 2; row_half_mirror pairs the same quads as xor 4, row_mirror the same
// octets as xor 8) and the steps across rows are v_permlane16_swap / v_permlane32_swap (gfx950 VALU): the same
// pairwise association as the xor butterfly, so every lane ends with the bitwise-same value the shuffle form gave.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}
// the value of lane l ^ 16 / l ^ 32 (both results of the swap pair, own row first for the even rows)
__device__ __forceinline__ void swap16(float x, float& a, float& b) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
}
__device__ __forceinline__ void swap32(float x, float& a, float& b) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
}
// x combined over the aligned group of G lanes (G = 1, 2, 4, ..., 64) with op (sum / max); G is a compile-time power
// of two.  lo_steps = false skips the inside-row steps (the caller's group is the lanes l, l ^ 16, l ^ 32, l ^ 48).
template <int G, bool LO = true, class Op>
__device__ __forceinline__ float lane_reduce(float x, Op op) {
    if constexpr (LO && G >= 2) x = op(x, dpp_mov<0xB1>(x));    // quad_perm [1,0,3,2]
    if constexpr (LO && G >= 4) x = op(x, dpp_mov<0x4E>(x));    // quad_perm [2,3,0,1]
    if constexpr (LO && G >= 8) x = op(x, dpp_mov<0x141>(x));   // row_half_mirror
    if constexpr (LO && G >= 16) x = op(x, dpp_mov<0x140>(x));  // row_mirror
    if constexpr (G >= 32) {
        float a, b;
        swap16(x, a, b);
        x = op(a, b);
    }
    if constexpr (G >= 64) {
        float a, b;
        swap32(x, a, b);
        x = op(a, b);
    }
    return x;
}
struct OpAdd {
    __device__ __forceinline__ float operator()(float a, float b) const { return a + b; }
};
struct OpMax {
    __device__ __forceinline__ float operator()(float a, float b) const { return fmaxf(a, b); }
};
template <int G>
__device__ __forceinline__ float lane_sum(float x) { return lane_reduce<G>(x, OpAdd()); }
template <int G>
__device__ __forceinline__ float lane_max(float x) { return lane_reduce<G>(x, OpMax()); }
// over the lanes l, l ^ 16, l ^ 32, l ^ 48 (same lane index inside each row): two swaps
__device__ __forceinline__ float rows_sum(float x) { return lane_reduce<64, false>(x, OpAdd()); }
__device__ __forceinline__ float rows_max(float x) { return lane_reduce<64, false>(x, OpMax()); }

// Dropout masks: counter-based, two-level.  A 32-bit key per (seed, stream) is mixed once
// (per lane / per row, amortised), then each element costs one lowbias32 round
// (2 integer multiplies) on (counter ^ key).  Streams / counters per kernel are
// documented in include/tagan_hip.h.  lowbias32: C. Wellons' 2-multiply integer hash.
__host__ __device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

__host__ __device__ __forceinline__ uint32_t drop_key(uint64_t seed, uint64_t stream) {
    uint32_t k = lowbias32((uint32_t)seed ^ 0x9E3779B9u);
    k = lowbias32(k ^ (uint32_t)(seed >> 32));
    k = lowbias32(k ^ (uint32_t)stream);
    return lowbias32(k ^ (uint32_t)(stream >> 32));
}

// Graph-replay seed source.  When the host registered a device counter (tagan_set_seed_counter), every kernel
// that draws a dropout mask mixes the counter's CURRENT value into its seed when it starts (TAGAN_LIVE_SEED), so
// a captured HIP graph whose first node advances the counter (tagan_seed_counter_step) draws fresh masks on
// every replay.  Null (the default) = the seed as passed: eager calls are unchanged.
const uint64_t* seed_counter();
#define TAGAN_LIVE_SEED(A)                                                          \
    do {                                                                            \
        if ((A).seed_ctr) (A).seed ^= *(A).seed_ctr * 0x9E3779B97F4A7C15ull;        \
    } while (0)

// uniform in [0,1) with 24-bit resolution
__host__ __device__ __forceinline__ float drop_u(uint32_t key, uint32_t counter) {
    return (float)(lowbias32(counter ^ key) >> 8) * (1.0f / 16777216.0f);
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

// ---------------------------------------------------------------- storage types
// Activations are stored fp32 (TAGAN_F32) or bf16 (TAGAN_BF16); math is always fp32.
// Io<S>::ld / st move 4 consecutive elements (element index i, a multiple of 4) as a float4.
struct bf16s {};   // tag for bf16 storage


// two fp32 -> two bf16 packed low | high with the hardware conversion (v_cvt_pk_bf16_f32: round to nearest even,
// the same bits as f2bf_bits for every non-NaN value, a NaN stays a NaN) -- one instruction per pair instead of the
// integer sequence's six per value
typedef float cm_f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 cm_bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t f2bf2(float a, float b) {
    const cm_f32x2 v = {a, b};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, cm_bf16x2));
}

template <typename S>
struct Io;

template <>
struct Io<float> {
    static constexpr int bytes = 4;
    __device__ static __forceinline__ float4 ld(const void* p, int64_t i) {
        return *(const float4*)((const float*)p + i);
    }
    __device__ static __forceinline__ void st(void* p, int64_t i, float4 v) { *(float4*)((float*)p + i) = v; }
    __device__ static __forceinline__ float ld1(const void* p, int64_t i) { return ((const float*)p)[i]; }
};

template <>
struct Io<bf16s> {
    static constexpr int bytes = 2;
    __device__ static __forceinline__ float4 ld(const void* p, int64_t i) {
        const uint2 u = *(const uint2*)((const uint16_t*)p + i);
        return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                           __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
    }
    __device__ static __forceinline__ void st(void* p, int64_t i, float4 v) {
        uint2 u;
        u.x = f2bf2(v.x, v.y);
        u.y = f2bf2(v.z, v.w);
        *(uint2*)((uint16_t*)p + i) = u;
    }
    __device__ static __forceinline__ float ld1(const void* p, int64_t i) {
        return __uint_as_float((uint32_t)((const uint16_t*)p)[i] << 16);
    }
};

// Deterministic column sums of a [nblk, n] (row stride ld) partials table (per-block dγ/dβ, bias-table
// grads): one 1024-thread block per CS_CW = 16 columns (a wave-instruction reads 4 rows x 64 B), so a
// 256-column table spreads over 16 CUs instead of 4; lane (w, rsub) sums rows w*4+rsub, +64, ... with
// four independent accumulators (loads in flight), then one fixed-order LDS pass per column.
// Column x < split goes to out0[x], the rest to out1[x - split] (either may be null), times ``scale``.
constexpr int COLSUM_BLK = 1024;
constexpr int CS_CW = 16;
namespace {
__global__ void __launch_bounds__(COLSUM_BLK) k_colsum_parts(const float* __restrict__ part, int nblk, int n,
                                                            float* __restrict__ out0, float* __restrict__ out1,
                                                            int split, float scale, int64_t ld) {
    constexpr int RPI = WAVE / CS_CW;                 // rows per wave-instruction
    constexpr int NR = (COLSUM_BLK / WAVE) * RPI;     // row lanes per block
    __shared__ float red[NR][CS_CW];
    const int lane = threadIdx.x & (WAVE - 1), w = threadIdx.x >> 6;
    const int col = lane % CS_CW, r0 = w * RPI + lane / CS_CW;
    const int x = blockIdx.x * CS_CW + col;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    if (x < n) {
        int b = r0;
        for (; b + 3 * NR < nblk; b += 4 * NR) {
            s0 += part[(int64_t)b * ld + x];
            s1 += part[(int64_t)(b + NR) * ld + x];
            s2 += part[(int64_t)(b + 2 * NR) * ld + x];
            s3 += part[(int64_t)(b + 3 * NR) * ld + x];
        }
        for (; b < nblk; b += NR) s0 += part[(int64_t)b * ld + x];
    }
    red[r0][col] = (s0 + s1) + (s2 + s3);
    __syncthreads();
    if (threadIdx.x < CS_CW) {
        const int xo = blockIdx.x * CS_CW + threadIdx.x;
        float v = 0.f;
        for (int r = 0; r < NR; ++r) v += red[r][threadIdx.x];
        if (xo < n) {
            if (scale != 1.f) v *= scale;
            if (xo < split) { if (out0) out0[xo] = v; }
            else if (out1) out1[xo - split] = v;
        }
    }
}

}  // namespace

// ld = row stride of the partials table (default n)
static inline void launch_colsum(const float* part, int nblk, int n, float* out0, float* out1, int split,
                                 hipStream_t s, float scale = 1.f, int64_t ld = -1) {
    k_colsum_parts<<<(n + CS_CW - 1) / CS_CW, COLSUM_BLK, 0, s>>>(part, nblk, n, out0, out1, split, scale,
                                                                ld < 0 ? n : ld);
}

}  // namespace tagan
