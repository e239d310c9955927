// Deterministic device exclusive scans (no decoupled look-back, no memset nodes): reduce-then-scan over
// fixed tiles, so a captured HIP graph replays them with nothing but kernel nodes and every result is
// bitwise identical run to run.  Used by the CSR builder and the chunk work lists (csr_build.hip).
#pragma once
#include "common.cuh"

namespace tagan {
namespace scan {

constexpr int NT = 1024;            // threads per scan block
constexpr int IPT = 8;              // items per thread
constexpr int TILE = NT * IPT;      // items per block

__device__ __forceinline__ int32_t shfl_up(int32_t x, int o) { return __shfl_up(x, o, WAVE); }
__device__ __forceinline__ int64_t shfl_up(int64_t x, int o) { return __shfl_up(x, o, WAVE); }

struct Plus {
    template <typename T>
    __host__ __device__ T operator()(const T& a, const T& b) const { return a + b; }
};

// wave-level inclusive scan (wave64, shuffles)
template <typename T, typename Op>
__device__ __forceinline__ T wave_incl(T x, Op op) {
    const int lane = threadIdx.x & (WAVE - 1);
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) {
        const T y = shfl_up(x, o);
        if (lane >= o) x = op(y, x);
    }
    return x;
}

// Block-wide exclusive scan of one value per thread (NTH threads); returns the prefix, *total = block sum.
// sm must hold NTH / 64 + 1 elements; ends with a barrier (sm reusable afterwards).
template <int NTH, typename T, typename Op>
__device__ __forceinline__ T block_excl(T x, T zero, Op op, T* sm, T* total) {
    constexpr int NW = NTH / WAVE;
    const int lane = threadIdx.x & (WAVE - 1), w = threadIdx.x >> 6;
    const T inc = wave_incl(x, op);
    if (lane == WAVE - 1) sm[w] = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
        T run = zero;
        for (int i = 0; i < NW; ++i) {
            const T c = sm[i];
            sm[i] = run;
            run = op(run, c);
        }
        sm[NW] = run;
    }
    __syncthreads();
    const T base = sm[w];
    const T up = shfl_up(inc, 1);   // every lane takes part (a shuffle from an inactive lane reads garbage)
    *total = sm[NW];
    __syncthreads();
    return op(base, lane == 0 ? zero : up);
}

// per-block reduction of tile blk of in[0..n)
template <typename T, typename Op>
__global__ void __launch_bounds__(NT) k_tile_reduce(const T* __restrict__ in, int64_t n, T zero, Op op,
                                                    T* __restrict__ part) {
    __shared__ T sm[NT / WAVE + 1];
    const int64_t base = (int64_t)blockIdx.x * TILE + (int64_t)threadIdx.x * IPT;
    T acc = zero;
#pragma unroll
    for (int k = 0; k < IPT; ++k)
        if (base + k < n) acc = op(acc, in[base + k]);
    T tot;
    (void)block_excl<NT>(acc, zero, op, sm, &tot);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// exclusive scan of part[0..nb) in place by ONE block, in fixed order; part[nb] = total
template <typename T, typename Op>
__global__ void __launch_bounds__(NT) k_scan_parts(T* __restrict__ part, int64_t nb, T zero, Op op) {
    __shared__ T sm[NT / WAVE + 1];
    T carry = zero;
    for (int64_t t0 = 0; t0 < nb; t0 += NT) {
        const int64_t i = t0 + threadIdx.x;
        const T x = i < nb ? part[i] : zero;
        T tot;
        const T ex = block_excl<NT>(x, zero, op, sm, &tot);
        if (i < nb) part[i] = op(carry, ex);
        carry = op(carry, tot);
    }
    if (threadIdx.x == 0) part[nb] = carry;
}

// out[i] = part[blk] + exclusive prefix of in within tile blk; out may alias in.  With total != null the last
// block also writes the grand total (part[nblk]) to *total and, if out_n, to out[n] (the "ptr[n]" slot).
template <typename T, typename Op>
__global__ void __launch_bounds__(NT) k_tile_scan(const T* in, int64_t n, T zero, Op op, const T* __restrict__ part,
                                                  T* out, bool out_n) {
    __shared__ T sm[NT / WAVE + 1];
    const int64_t base = (int64_t)blockIdx.x * TILE + (int64_t)threadIdx.x * IPT;
    T v[IPT];
    T acc = zero;
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
        v[k] = base + k < n ? in[base + k] : zero;
        acc = op(acc, v[k]);
    }
    T tot;
    T run = op(part[blockIdx.x], block_excl<NT>(acc, zero, op, sm, &tot));
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
        if (base + k < n) out[base + k] = run;
        run = op(run, v[k]);
    }
    if (out_n && blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) out[n] = part[gridDim.x];
}

inline int64_t tiles(int64_t n) { return n <= 0 ? 1 : (n + TILE - 1) / TILE; }

// workspace elements of T for scanning n items
inline int64_t parts_len(int64_t n) { return tiles(n) + 1; }

// out[0..n) = exclusive scan of in (out may alias in); out[n] = total when out_n.  part: parts_len(n) items.
// one block, one tile (n <= TILE): the whole scan in one launch
template <typename T, typename Op>
__global__ void __launch_bounds__(NT) k_scan_one(const T* in, int64_t n, T zero, Op op, T* out, bool out_n) {
    __shared__ T sm[NT / WAVE + 1];
    const int64_t base = (int64_t)threadIdx.x * IPT;
    T v[IPT];
    T acc = zero;
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
        v[k] = base + k < n ? in[base + k] : zero;
        acc = op(acc, v[k]);
    }
    T tot;
    T run = block_excl<NT>(acc, zero, op, sm, &tot);
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
        if (base + k < n) out[base + k] = run;
        run = op(run, v[k]);
    }
    if (out_n && threadIdx.x == 0) out[n] = tot;
}

template <typename T, typename Op>
inline void exclusive(const T* in, T* out, int64_t n, T zero, Op op, T* part, bool out_n, hipStream_t s) {
    const int64_t nb = tiles(n);
    if (nb == 1) {
        k_scan_one<T, Op><<<1, NT, 0, s>>>(in, n, zero, op, out, out_n);
        return;
    }
    k_tile_reduce<T, Op><<<(unsigned)nb, NT, 0, s>>>(in, n, zero, op, part);
    k_scan_parts<T, Op><<<1, NT, 0, s>>>(part, nb, zero, op);
    k_tile_scan<T, Op><<<(unsigned)nb, NT, 0, s>>>(in, n, zero, op, part, out, out_n);
}

}  // namespace scan
}  // namespace tagan
