// Snapshot CSR/CSC builder: the sparse form of graph_attention.py:96-105
//   adj = zeros(N,N); adj[edge_index[0], edge_index[1]] = 1; adj += eye(N)
// for a block-diagonal batch of snapshots.  Integer/byte work: HBM-bound, no MFMA, no library sort.
//
// Bucketed counting sort, every bucket finished in LDS:
//   rows are grouped into BUCKETS of 2^SB consecutive global node ids (SB set so a bucket holds ~2k entries),
//   buckets into COARSE BINS of 2^SC buckets (SC set so one snapshot spans <= ~256 bins: every partition pass
//   keeps at most a few hundred write frontiers per block, so its scattered 4-B stores merge into whole lines
//   in L2 instead of costing a read-modify-write each);
//   1. count   : one pass over the raw edges, per-block LDS histograms of src AND dst buckets per snapshot
//                (one atomic per non-empty bin), index validation;
//   2. scan    : bucket capacities (raw edges + the bucket's self-loops) -> bucket regions;
//   3. part    : second pass over the raw edges into the coarse bins, 32-bit keys
//                (bucket-in-bin << SB+LB | row-in-bucket << LB | local dst);
//   4. refine  : one workgroup per coarse bin moves its keys into the bucket regions (skipped when SC = 0);
//   5. finish  : one workgroup per bucket loads its keys (+ its rows' self-loops) into LDS, radix-sorts them
//                (stable LSD, 8-bit digits, wave-ballot ranks, up to 8 keys per thread per round), drops
//                duplicates, counts entries per row;
//   6. scan    : unique counts per bucket -> CSR offsets;  place: col, rowptr, and each entry's local src;
//   7. CSC     : steps 3-5 again over the final CSR entries keyed by dst, carrying the CSR position
//                (key = column-in-bucket << LB | local src, value = CSR position); the finish sorts the pairs
//                (src ascending within a column = CSR order) and writes csc_ptr, csc_row, csc_eid and the
//                CSR -> CSC position map in the same pass.
// Buckets too large for the small LDS finish (power-law hubs) go on a device-side list that a persistent
// 1024-thread kernel with 128 KB of LDS works through; beyond that, the same sort runs in global memory.
// Every result is bitwise deterministic (a bucket is sorted on its full key); the launches are kernel nodes
// only -- no library sort (rocPRIM's onesweep faulted on HIP-graph replay with eager kernels in between,
// DESIGN.md §6), no memset nodes, no host synchronisation.
#include <algorithm>

#include "common.cuh"
#include "scan.cuh"

namespace tagan {
namespace {

constexpr int BLK = 256;           // generic grid-stride kernels
constexpr int PNT = 1024;          // partition (count / part) blocks
constexpr int LDS_BINS = 16384;    // LDS histogram bins per count block and direction
constexpr int PART_BINS = 2048;    // LDS bins of the partition passes (more: global atomics)
constexpr int RNT = 1024;          // refine blocks (one per coarse bin)
#ifndef TAGAN_CSR_FNT
#define TAGAN_CSR_FNT 256
#endif
constexpr int FNT = TAGAN_CSR_FNT;  // small-bucket finish workgroups (4 waves)
#ifndef TAGAN_CSR_TARGET
#define TAGAN_CSR_TARGET 2048
#endif
constexpr int CAP_S = TAGAN_CSR_TARGET * 5 / 4;   // keys per small CSR finish (LDS)
constexpr int CAP_C = TAGAN_CSR_TARGET;           // (key, CSR position) pairs per small CSC finish
#ifndef TAGAN_CSR_BNT
#define TAGAN_CSR_BNT 512
#endif
constexpr int BNT = TAGAN_CSR_BNT;   // big-bucket finish workgroups (8 waves)
#ifndef TAGAN_CSR_BIG_LDS_KB
#define TAGAN_CSR_BIG_LDS_KB 140
#endif
constexpr int BIG_LDS = TAGAN_CSR_BIG_LDS_KB * 1024;   // dynamic LDS of the big-bucket kernels (2 key buffers / 2 + 2 pair buffers)
constexpr int BIG_WG = 256;        // persistent workgroups of the big-bucket kernels (one per CU)
constexpr int RB = 8;              // radix digit bits
constexpr int RBINS = 1 << RB;
constexpr int TARGET = TAGAN_CSR_TARGET;   // average entries per bucket
constexpr int SB_MAX = 8;          // at most 256 rows per bucket
constexpr int SC_MAX = 8;          // at most 256 buckets per coarse bin
constexpr int COARSE_PER_SNAPSHOT = 192;

// Graph of edge e: binary search in edge_ptr[0..G] (G small; edge_ptr in L2/scalar cache).
__device__ __forceinline__ int find_graph(const int64_t* __restrict__ ptr, int G, int64_t e) {
    int lo = 0, hi = G - 1;
    while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if (ptr[mid] <= e) lo = mid; else hi = mid - 1;
    }
    return lo;
}

__device__ __forceinline__ int64_t node_base(const int64_t* __restrict__ node_ptr, int G, int64_t n) {
    return node_ptr[find_graph(node_ptr, G, n)];
}

// node_base over the rows [r0, r0 + n) of one bucket: one search for the bucket's first row, another only for rows
// past the end of that snapshot (a bucket straddles at most a few snapshots)
struct BucketBase {
    int64_t base0, end0;
    const int64_t* node_ptr;
    int G;
    __device__ BucketBase(const int64_t* __restrict__ np, int g, int64_t r0) : node_ptr(np), G(g) {
        const int s = find_graph(np, g, r0);
        base0 = np[s];
        end0 = np[s + 1];
    }
    __device__ int64_t operator()(int64_t v) const { return v < end0 ? base0 : node_base(node_ptr, G, v); }
};

struct Geo {
    int64_t N, E, NL;
    int G, LB, SB, SC;
    int64_t NB, NCB;     // buckets, coarse bins (the same geometry for CSR rows and CSC columns)
    int64_t CHn;         // raw edges per count block (>> the buckets one snapshot spans: few flush atomics)
    int64_t CH, CHc;     // raw edges / CSR entries per partition block
};

int bits_for(int64_t x) {   // bits to hold values 0..x
    int b = 0;
    while (b < 62 && ((int64_t)1 << b) <= x) ++b;
    return b;
}

Geo geometry(int64_t E, int64_t N, int G, int64_t NL) {
    Geo g{};
    g.N = N; g.E = E; g.G = G; g.NL = NL;
    g.LB = bits_for(NL - 1);
    const double per_node = (double)(E + N) / (double)N;
    int sb = 0;
    while (sb < SB_MAX && (double)((int64_t)1 << (sb + 1)) * per_node <= TARGET) ++sb;
    if (sb + g.LB > 31) sb = 31 - g.LB;
    if (sb < 0) sb = 0;
    g.SB = sb;
    g.NB = (N + ((int64_t)1 << sb) - 1) >> sb;
    const int64_t per_snap = (NL >> sb) + 2;   // buckets one snapshot spans
    int sc = 0;
    while (sc < SC_MAX && (per_snap >> sc) > COARSE_PER_SNAPSHOT && sc + 1 + sb + g.LB <= 32) ++sc;
    g.SC = sc;
    g.NCB = (g.NB + ((int64_t)1 << sc) - 1) >> sc;
    // partition blocks: 64k edges each at scale, smaller (down to 4k) so a small batch still fills the 256 CUs
    int64_t ch = 4096;
    while (ch < 65536 && ch * 1024 < E + N) ch <<= 1;
    int64_t chn = ch;
    while (chn < 16 * per_snap && chn < ((int64_t)1 << 20)) chn <<= 1;
    g.CHn = chn;
    g.CH = ch;
    g.CHc = ch;
    return g;
}

__device__ __forceinline__ int64_t bucket_rows(int64_t b, int sb, int64_t N) {
    const int64_t r0 = b << sb;
    return min(N, r0 + ((int64_t)1 << sb)) - r0;
}

// Global -> LDS copy of n items with PER loads in flight per thread (a plain strided loop waits for each load before
// its LDS store, so a bucket's ~8 loads per thread ran back to back: the finish kernels' serial latency chain)
template <int NTH, int PER, typename T>
__device__ __forceinline__ void gload_lds(T* dst, const T* __restrict__ src, int n) {
    for (int base = 0; base < n; base += NTH * PER) {
        T r[PER];
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int i = base + u * NTH + (int)threadIdx.x;
            if (i < n) r[u] = src[i];
        }
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int i = base + u * NTH + (int)threadIdx.x;
            if (i < n) dst[i] = r[u];
        }
    }
}
template <int NTH, int PER>
__device__ __forceinline__ void gload_lds2(uint32_t* dk, const uint32_t* __restrict__ sk, int32_t* dv,
                                           const int32_t* __restrict__ sv, int n) {
    for (int base = 0; base < n; base += NTH * PER) {
        uint32_t rk[PER];
        int32_t rv[PER];
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int i = base + u * NTH + (int)threadIdx.x;
            if (i < n) {
                rk[u] = sk[i];
                rv[u] = sv[i];
            }
        }
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int i = base + u * NTH + (int)threadIdx.x;
            if (i < n) {
                dk[i] = rk[u];
                dv[i] = rv[u];
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------- LDS radix sort
// Stable LSD radix sort of n 32-bit keys over bits [0, nbits) (+ int32 values), NTH threads, ping-pong between
// (ka, va) and (kb, vb) -- LDS or global (the big-bucket fallback).  Per pass and per round of NTH*IPT keys
// (key i = r0 + k*NTH + tid: item slot k, wave w, lane): a lane's rank among the lanes of its wave with the same
// digit comes from RB ballots; the per-(slot, wave) digit counts are prefixed in (slot, wave) order -> stable.
// A single-round sort takes the digit offsets from that table; larger ones pre-count the pass's digits.
// Returns the parity of the buffer holding the result (0 = a, 1 = b).
// LDS: sh_base, sh_tot: RBINS ints each; sh_wc: IPT * (NTH/64) * RBINS ints; sh_sm: NTH/64 + 1 ints.
template <int NTH, int IPT, bool VAL>
__device__ int block_radix_sort(uint32_t* ka, uint32_t* kb, int32_t* va, int32_t* vb, int n, int nbits,
                                int* sh_base, int* sh_tot, int* sh_wc, int32_t* sh_sm) {
    constexpr int NW = NTH / WAVE;
    constexpr int RND = NTH * IPT;
    constexpr int SLOTS = IPT * NW;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & (WAVE - 1);
    const uint64_t below = lane ? (~0ull >> (WAVE - lane)) : 0ull;
    const bool multi = n > RND;
    int par = 0;
    for (int sh = 0; sh < nbits; sh += RB) {
        const int dbits = min(RB, nbits - sh);
        if (multi) {   // digit offsets of the whole pass
            for (int i = tid; i < RBINS; i += NTH) sh_tot[i] = 0;
            __syncthreads();
            for (int i = tid; i < n; i += NTH) atomicAdd(&sh_tot[(ka[i] >> sh) & (RBINS - 1)], 1);
            __syncthreads();
            int32_t tot;
            int x = 0;
            if (tid < RBINS) x = sh_tot[tid];
            const int32_t ex = scan::block_excl<NTH>((int32_t)x, (int32_t)0, scan::Plus(), sh_sm, &tot);
            if (tid < RBINS) sh_base[tid] = ex;
            __syncthreads();
        }
        for (int r0 = 0; r0 < n; r0 += RND) {
            for (int i = tid; i < SLOTS * RBINS; i += NTH) sh_wc[i] = 0;
            __syncthreads();
            uint32_t key[IPT];
            int32_t val[IPT];
            int dig[IPT], rank[IPT];
#pragma unroll
            for (int k = 0; k < IPT; ++k) {
                const int i = r0 + k * NTH + tid;
                const bool ok = i < n;
                key[k] = ok ? ka[i] : 0u;
                val[k] = 0;
                if (VAL && ok) val[k] = va[i];
                const int d = (int)((key[k] >> sh) & (RBINS - 1));
                uint64_t peers = __ballot(ok);
                for (int b = 0; b < dbits; ++b) {
                    const bool bit = (d >> b) & 1;
                    const uint64_t m = __ballot(bit);
                    peers &= bit ? m : ~m;
                }
                dig[k] = ok ? d : -1;
                rank[k] = __popcll(peers & below);
                if (ok && rank[k] == 0) sh_wc[(k * NW + w) * RBINS + d] = __popcll(peers);
            }
            __syncthreads();
            int x = 0;
            for (int dd = tid; dd < RBINS; dd += NTH) {   // per digit: offsets of the (slot, wave) groups in order
                int run = 0;
                for (int s = 0; s < SLOTS; ++s) {
                    const int c = sh_wc[s * RBINS + dd];
                    sh_wc[s * RBINS + dd] = run;
                    run += c;
                }
                sh_tot[dd] = run;
                x = run;
            }
            if (!multi) {   // one round: the digit offsets are the scan of this round's totals
                int32_t tot;
                const int32_t ex = scan::block_excl<NTH>((int32_t)(tid < RBINS ? x : 0), (int32_t)0, scan::Plus(),
                                                         sh_sm, &tot);
                if (tid < RBINS) sh_base[tid] = ex;
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < IPT; ++k) {
                if (dig[k] >= 0) {
                    const int p = sh_base[dig[k]] + sh_wc[(k * NW + w) * RBINS + dig[k]] + rank[k];
                    kb[p] = key[k];
                    if (VAL) vb[p] = val[k];
                }
            }
            __syncthreads();
            if (multi) {
                for (int dd = tid; dd < RBINS; dd += NTH) sh_base[dd] += sh_tot[dd];
                __syncthreads();
            }
        }
        uint32_t* tk = ka; ka = kb; kb = tk;
        int32_t* tv = va; va = vb; vb = tv;
        par ^= 1;
    }
    return par;
}

// --------------------------------------------------------------------------------------------- the kernels
__global__ void __launch_bounds__(BLK) k_init(Geo g, int32_t* __restrict__ cap_src, int32_t* __restrict__ fill_src,
                                              int32_t* __restrict__ cap_dst, int32_t* __restrict__ fill_dst,
                                              int32_t* __restrict__ fillc_src, int32_t* __restrict__ fillc_dst,
                                              int32_t* __restrict__ nbig, int32_t* __restrict__ err) {
    for (int64_t b = blockIdx.x * (int64_t)BLK + threadIdx.x; b < g.NB; b += (int64_t)gridDim.x * BLK) {
        const int32_t rows = (int32_t)bucket_rows(b, g.SB, g.N);
        cap_src[b] = rows;
        cap_dst[b] = rows;
        fill_src[b] = 0;
        fill_dst[b] = 0;
        if (b < g.NCB) { fillc_src[b] = 0; fillc_dst[b] = 0; }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) { nbig[0] = 0; nbig[1] = 0; *err = 0; }
}

__device__ __forceinline__ bool valid_edge(int64_t s, int64_t d, int64_t base, int64_t n, int64_t& gs,
                                           int64_t& dl) {
    s += (s < 0) ? n : 0;
    d += (d < 0) ? n : 0;
    if (s < 0 || s >= n || d < 0 || d >= n) return false;
    gs = base + s;
    dl = d;
    return true;
}

constexpr int UNR = 4;   // loads in flight per lane in the streaming passes

// LDS-staged tile partition.  Each tile of NTH * IPT items (bins bin[k] in [0, NB), -1: no item) is counted per bin
// with one LDS atomic per item, the per-bin counts are scanned, the items are placed in LDS grouped by bin together
// with their global position (sh_base[bin] + slot; sh_base advances by the tile's counts), and the tile is written
// out from LDS in that order: consecutive lanes store consecutive addresses of one bin's run, so a wave touches a few
// cache lines instead of one per lane.  The order inside a bin is unspecified -- every consumer sorts its bucket on
// the full key.  The loader fetches item i's raw values one tile ahead (issued before this tile's scan and write-out,
// so the loads overlap them) and decodes them into (bin, key, value).
// LDS: tcnt, tstart, gpos: NB ints each (tcnt zero on entry and exit); stk / stv / stp: NTH * IPT each; sm: NTH/64+1.
// GRES: no per-block bases -- each tile reserves its run of every non-empty bin with one global atomic
// (res.start[(res.b0 + bin) << res.sc] + atomicAdd(&res.fill[res.b0 + bin], count)), so the caller needs no histogram
// pre-pass over its chunk (a second read of the raw input).
struct TileRes {
    const int32_t* start;
    int32_t* fill;
    int64_t b0;
    int sc;
};

template <int NTH, int IPT, int NB, bool VAL, bool GRES = false, typename Loader>
__device__ void tile_partition(int64_t a, int64_t z, const Loader& ld, int* sh_base, int* tcnt, int* tstart, int* gpos,
                               uint32_t* stk, int32_t* stv, int* stp, int32_t* sm, uint32_t* __restrict__ out_k,
                               int32_t* __restrict__ out_v, TileRes res = TileRes{}) {
    using Raw = typename Loader::Raw;
    constexpr int TILE = NTH * IPT;
    const int tid = threadIdx.x;
    Raw cur[IPT];
#pragma unroll
    for (int k = 0; k < IPT; ++k) cur[k] = ld.fetch(a + k * NTH + tid, z);
    for (int64_t t0 = a; t0 < z; t0 += TILE) {
        int bin[IPT], slot[IPT];
        uint32_t key[IPT];
        int32_t val[IPT];
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
            ld.decode(cur[k], t0 + k * NTH + tid, z, bin[k], key[k], val[k]);
            slot[k] = bin[k] >= 0 ? atomicAdd(&tcnt[bin[k]], 1) : 0;
        }
#pragma unroll
        for (int k = 0; k < IPT; ++k) cur[k] = ld.fetch(t0 + TILE + k * NTH + tid, z);   // next tile, in flight
        __syncthreads();
        const int c = tid < NB ? tcnt[tid] : 0;
        int32_t tot;
        const int32_t ex = scan::block_excl<NTH>((int32_t)c, (int32_t)0, scan::Plus(), sm, &tot);
        if (tid < NB) {
            tstart[tid] = ex;
            if (GRES) {
                gpos[tid] = c ? res.start[(res.b0 + tid) << res.sc] + atomicAdd(&res.fill[res.b0 + tid], c) : 0;
            } else {
                gpos[tid] = sh_base[tid];
                sh_base[tid] += c;
            }
            tcnt[tid] = 0;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
            if (bin[k] >= 0) {
                const int l = tstart[bin[k]] + slot[k];
                stk[l] = key[k];
                if (VAL) stv[l] = val[k];
                stp[l] = gpos[bin[k]] + slot[k];
            }
        }
        __syncthreads();
        for (int t = tid; t < tot; t += NTH) {
            const int p = stp[t];
            out_k[p] = stk[t];
            if (VAL) out_v[p] = stv[t];
        }
        __syncthreads();
    }
}

constexpr int PNB = 256;   // bins of the staged partition passes (coarse bins per snapshot, buckets per coarse bin)
constexpr int PIPT = 4;    // items per thread per tile in the partition passes
constexpr int PTILE = PNT * PIPT;
#ifndef TAGAN_CSR_TILE_RES
#define TAGAN_CSR_TILE_RES 1   // staged partition passes reserve per tile (one read of the input, no block pre-pass)
#endif

// bins of shift `sh` spanned by the nodes [v0, v1) of one snapshot
struct Span {
    int64_t b0;
    int nb;
    bool lds;
};

__device__ __forceinline__ Span span_of(int64_t v0, int64_t v1, int sh, int maxbins = LDS_BINS) {
    Span s;
    s.b0 = v0 >> sh;
    const int64_t b1 = v1 > v0 ? ((v1 - 1) >> sh) + 1 : s.b0;
    s.lds = b1 - s.b0 <= maxbins;
    s.nb = s.lds ? (int)(b1 - s.b0) : 0;
    return s;
}

// raw edge e -> (coarse src bin, key = (bucket-in-bin << SB | row-in-bucket) << LB | local dst)
struct EdgeLoader {
    struct Raw { int64_t s, d; };
    const int64_t* ei;
    int64_t ld, base, n, b0;
    int shc, SB, LB;
    uint32_t rmask, fmask;
    __device__ Raw fetch(int64_t e, int64_t z) const {
        Raw r{-1, -1};
        if (e < z) { r.s = ei[e]; r.d = ei[ld + e]; }
        return r;
    }
    __device__ void decode(const Raw& r, int64_t e, int64_t z, int& bin, uint32_t& key, int32_t& val) const {
        int64_t gs, dl;
        bin = -1;
        key = 0u;
        val = 0;
        if (e < z && valid_edge(r.s, r.d, base, n, gs, dl)) {
            bin = (int)((gs >> shc) - b0);
            key = ((((uint32_t)(gs >> SB) & fmask) << SB | ((uint32_t)gs & rmask)) << LB) | (uint32_t)dl;
        }
    }
};

// CSR entry e -> (coarse dst bin, key = (bucket-in-bin << SB | column-in-bucket) << LB | local src, value = e)
struct CsrEntryLoader {
    struct Raw { int32_t d, sl; };
    const int32_t* col;
    const int32_t* sloc;
    int64_t b0;
    int shc, SB, LB;
    uint32_t cmask, fmask;
    __device__ Raw fetch(int64_t e, int64_t z) const {
        Raw r{0, 0};
        if (e < z) { r.d = col[e]; r.sl = sloc[e]; }
        return r;
    }
    __device__ void decode(const Raw& r, int64_t e, int64_t z, int& bin, uint32_t& key, int32_t& val) const {
        bin = e < z ? (int)((r.d >> shc) - b0) : -1;
        key = ((((uint32_t)(r.d >> SB) & fmask) << SB | ((uint32_t)r.d & cmask)) << LB) | (uint32_t)r.sl;
        val = (int32_t)e;
    }
};

// staged key (value) i of a coarse bin -> (bucket-in-bin, key without those bits, value)
template <bool VAL>
struct StageLoader {
    struct Raw { uint32_t k; int32_t v; };
    const uint32_t* skey;
    const int32_t* sval;
    int kb;
    uint32_t kmask;
    __device__ Raw fetch(int64_t i, int64_t z) const {
        Raw r{0u, 0};
        if (i < z) { r.k = skey[i]; if (VAL) r.v = sval[i]; }
        return r;
    }
    __device__ void decode(const Raw& r, int64_t i, int64_t z, int& bin, uint32_t& key, int32_t& val) const {
        bin = i < z ? (int)(r.k >> kb) : -1;
        key = r.k & kmask;
        val = r.v;
    }
};

// 1. bucket histograms of the raw edges (src and dst), index validation; snapshot by snapshot inside the block
__global__ void __launch_bounds__(PNT) k_count(Geo g, const int64_t* __restrict__ ei, int64_t ld,
                                               const int64_t* __restrict__ edge_ptr,
                                               const int64_t* __restrict__ node_ptr, int32_t* __restrict__ cap_src,
                                               int32_t* __restrict__ cap_dst, int32_t* __restrict__ err) {
    __shared__ int hs[LDS_BINS], hd[LDS_BINS];
    __shared__ int bad;
    const int64_t e0 = blockIdx.x * g.CHn, e1 = min(g.E, e0 + g.CHn);
    const int g0 = find_graph(edge_ptr, g.G, e0), g1 = find_graph(edge_ptr, g.G, e1 - 1);
    if (threadIdx.x == 0) bad = 0;
    bool my_bad = false;
    for (int gg = g0; gg <= g1; ++gg) {
        const int64_t base = node_ptr[gg], n = node_ptr[gg + 1] - base;
        const int64_t a = max(e0, edge_ptr[gg]), z = min(e1, edge_ptr[gg + 1]);
        const Span sp = span_of(base, base + n, g.SB);
        for (int i = threadIdx.x; i < sp.nb; i += PNT) { hs[i] = 0; hd[i] = 0; }
        __syncthreads();
        for (int64_t e4 = a + threadIdx.x; e4 < z; e4 += UNR * PNT) {   // UNR edges' loads in flight per lane
            int64_t sv[UNR], dv[UNR];
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                const int64_t e = e4 + u * PNT;
                sv[u] = e < z ? ei[e] : 0;
                dv[u] = e < z ? ei[ld + e] : 0;
            }
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                if (e4 + u * PNT >= z) break;
                int64_t gs, dl;
                if (!valid_edge(sv[u], dv[u], base, n, gs, dl)) { my_bad = true; continue; }
                const int64_t bs = gs >> g.SB, bd = (base + dl) >> g.SB;
                if (sp.lds) { atomicAdd(&hs[bs - sp.b0], 1); atomicAdd(&hd[bd - sp.b0], 1); }
                else { atomicAdd(&cap_src[bs], 1); atomicAdd(&cap_dst[bd], 1); }
            }
        }
        __syncthreads();
        for (int i = threadIdx.x; i < sp.nb; i += PNT) {
            if (hs[i]) atomicAdd(&cap_src[sp.b0 + i], hs[i]);
            if (hd[i]) atomicAdd(&cap_dst[sp.b0 + i], hd[i]);
        }
        __syncthreads();
    }
    if (my_bad) bad = 1;
    __syncthreads();
    if (threadIdx.x == 0 && bad) atomicOr(err, 1);
}

// 3. raw edges -> coarse src bins (SC > 0: staging layout) or straight into the buckets (SC = 0)
__global__ void __launch_bounds__(PNT) k_part_edges(Geo g, const int64_t* __restrict__ ei, int64_t ld_,
                                                    const int64_t* __restrict__ edge_ptr,
                                                    const int64_t* __restrict__ node_ptr,
                                                    const int32_t* __restrict__ bstart, int32_t* __restrict__ fill,
                                                    uint32_t* __restrict__ out) {
    __shared__ int h[PART_BINS];
    __shared__ int tcnt[PNB], tstart[PNB], gpos[PNB];
    __shared__ uint32_t stk[PTILE];
    __shared__ int stp[PTILE];
    __shared__ int32_t sm[PNT / WAVE + 1];
    for (int i = threadIdx.x; i < PNB; i += PNT) tcnt[i] = 0;
    const int64_t e0 = blockIdx.x * g.CH, e1 = min(g.E, e0 + g.CH);
    const int g0 = find_graph(edge_ptr, g.G, e0), g1 = find_graph(edge_ptr, g.G, e1 - 1);
    const int shc = g.SB + g.SC;                       // node id -> coarse bin
    const uint32_t rmask = (1u << g.SB) - 1u, fmask = (1u << g.SC) - 1u;
    for (int gg = g0; gg <= g1; ++gg) {
        const int64_t base = node_ptr[gg], n = node_ptr[gg + 1] - base;
        const int64_t a = max(e0, edge_ptr[gg]), z = min(e1, edge_ptr[gg + 1]);
        const Span sp = span_of(base, base + n, shc, PART_BINS);
        const bool staged = sp.lds && sp.nb <= PNB;
        if (sp.lds && !(TAGAN_CSR_TILE_RES && staged)) {
            for (int i = threadIdx.x; i < sp.nb; i += PNT) h[i] = 0;
            __syncthreads();
            for (int64_t e4 = a + threadIdx.x; e4 < z; e4 += UNR * PNT) {
                int64_t sv[UNR], dv[UNR];
#pragma unroll
                for (int u = 0; u < UNR; ++u) {
                    const int64_t e = e4 + u * PNT;
                    sv[u] = e < z ? ei[e] : 0;
                    dv[u] = e < z ? ei[ld_ + e] : 0;
                }
#pragma unroll
                for (int u = 0; u < UNR; ++u) {
                    int64_t gs, dl;
                    if (e4 + u * PNT < z && valid_edge(sv[u], dv[u], base, n, gs, dl))
                        atomicAdd(&h[(gs >> shc) - sp.b0], 1);
                }
            }
            __syncthreads();
            for (int i = threadIdx.x; i < sp.nb; i += PNT) {   // one reservation per non-empty bin
                const int c = h[i];
                const int64_t bin = sp.b0 + i;
                if (c) h[i] = bstart[bin << g.SC] + atomicAdd(&fill[bin], c);
            }
            __syncthreads();
        }
        if (staged) {   // LDS-staged scatter
            const EdgeLoader ld{ei, ld_, base, n, sp.b0, shc, g.SB, g.LB, rmask, fmask};
            tile_partition<PNT, PIPT, PNB, false, TAGAN_CSR_TILE_RES>(a, z, ld, h, tcnt, tstart, gpos, stk, nullptr, stp,
                                                                      sm, out, nullptr,
                                                                      TileRes{bstart, fill, sp.b0, g.SC});
        } else {
            for (int64_t e4 = a + threadIdx.x; e4 < z; e4 += UNR * PNT) {
                int64_t sv[UNR], dv[UNR];
#pragma unroll
                for (int u = 0; u < UNR; ++u) {
                    const int64_t e = e4 + u * PNT;
                    sv[u] = e < z ? ei[e] : 0;
                    dv[u] = e < z ? ei[ld_ + e] : 0;
                }
#pragma unroll
                for (int u = 0; u < UNR; ++u) {
                    if (e4 + u * PNT >= z) break;
                    int64_t gs, dl;
                    if (!valid_edge(sv[u], dv[u], base, n, gs, dl)) continue;
                    const int64_t bin = gs >> shc;
                    const int pos = sp.lds ? atomicAdd(&h[bin - sp.b0], 1)
                                           : bstart[bin << g.SC] + atomicAdd(&fill[bin], 1);
                    out[pos] = ((((uint32_t)(gs >> g.SB) & fmask) << g.SB | ((uint32_t)gs & rmask)) << g.LB) |
                               (uint32_t)dl;
                }
            }
        }
        __syncthreads();
    }
}

// 4. one workgroup per coarse bin: its staged keys (bucket-in-bin in the bits above SB + LB) -> bucket regions
// (LDS-staged tiles from each bucket's region start); fill[] = the keys each bucket received
template <bool VAL>
__global__ void __launch_bounds__(RNT) k_refine(Geo g, const int32_t* __restrict__ bstart,
                                                const int32_t* __restrict__ fillc, const uint32_t* __restrict__ skey,
                                                const int32_t* __restrict__ sval, int32_t* __restrict__ fill,
                                                uint32_t* __restrict__ key, int32_t* __restrict__ val) {
    constexpr int TILE = RNT * PIPT;
    __shared__ int base[PNB], tcnt[PNB], tstart[PNB], gpos[PNB];
    __shared__ uint32_t stk[TILE];
    __shared__ int32_t stv[VAL ? TILE : 1];
    __shared__ int stp[TILE];
    __shared__ int32_t sm[RNT / WAVE + 1];
    const int64_t c = blockIdx.x;
    const int64_t f0 = c << g.SC;
    const int nf = (int)(min(g.NB, f0 + ((int64_t)1 << g.SC)) - f0);
    const int32_t s0 = bstart[f0], cnt = fillc[c];
    const int kb = g.SB + g.LB;
    const uint32_t kmask = (uint32_t)(((uint64_t)1 << kb) - 1);
    for (int i = threadIdx.x; i < PNB; i += RNT) {
        base[i] = i < nf ? bstart[f0 + i] : 0;
        tcnt[i] = 0;
    }
    __syncthreads();
    const StageLoader<VAL> ld{skey + s0, sval ? sval + s0 : nullptr, kb, kmask};
    tile_partition<RNT, PIPT, PNB, VAL>(0, cnt, ld, base, tcnt, tstart, gpos, stk, stv, stp, sm, key, val);
    for (int i = threadIdx.x; i < nf; i += RNT) fill[f0 + i] = base[i] - bstart[f0 + i];
}

// 5. bucket finish.  The bucket's keys (row-in-bucket << LB | low) are counting-sorted by row in LDS (one LDS
// atomic per key: the order inside a row is free, the row sort below is on the full key), then every row is sorted
// on its own.  A row of <= 64 entries is RANK-sorted: each entry counts the entries of its row that precede it in
// (key, index) order -- a few independent LDS reads per entry, no shuffle network, no dependent chains.  A longer row
// (a power-law hub) goes through a per-wave LDS bitmap over the local ids when LB <= BM_LB -- set the bits, prefix
// the words' popcounts, and each entry's rank is the number of distinct ids below it: sorted AND deduplicated in
// O(entries + 2^LB / 32), the payload carried along.  A bucket with a long row and a wider local-id
// range takes the stable LSD radix sort of the whole bucket instead.  CSR rows are deduplicated on emission (the
// adjacency is a set: an entry is kept when it differs from its sorted predecessor); CSC columns carry each entry's
// CSR position.
constexpr int BM_LB = 14;                      // bitmap path for local ids < 2^14 (C1, C2)
constexpr int BMW = (1 << BM_LB) / 32;         // bitmap words per wave
constexpr int SHORT_ROW = WAVE;                // rank-sorted rows: at most this many entries

// LDS (or global) scratch of one bucket finish (rows = 2^SB_MAX at most)
struct SegLds {
    int* rc;        // entries per row (2^SB_MAX)
    int* ro;        // row start in the row-sorted buffer
    uint32_t* bm;   // NW * BMW bitmap words (null: no bitmap path); may alias rank
    uint16_t* pw;   // NW * BMW per-word prefixes of the bitmaps
    int* rank;      // [m] slot of each key within its row (LDS, or global scratch in the big kernels)
    int* wc;        // the LSD fallback's count table: NTH/64 * RBINS ints (may alias rank)
    int* flag;      // fallback request
};

// hub rows of a big bucket, one at a time with the whole block: bitmap over the local ids, block scan of the words'
// popcounts, rank = distinct ids below (the per-wave form below, spread over NTH threads)
template <int NTH, bool VAL, bool DEDUP>
__device__ void hub_rows_block(const Geo& g, int nrows, uint32_t* K, const uint32_t* K2, int32_t* V, const int32_t* V2,
                               SegLds L, int32_t* sh_sm) {
    const int tid = threadIdx.x;
    const uint32_t lmask = (uint32_t)(((uint64_t)1 << g.LB) - 1);
    const int nw = (int)((lmask >> 5) + 1);
    uint32_t* bm = L.bm;
    uint16_t* pw = L.pw;
    for (int j = 0; j < nrows; ++j) {
        const int n = L.rc[j];
        if (n <= SHORT_ROW) continue;
        const int base = L.ro[j];
        for (int i = tid; i < nw; i += NTH) bm[i] = 0u;
        __syncthreads();
        for (int i = tid; i < n; i += NTH) {
            const uint32_t lo = K2[base + i] & lmask;
            atomicOr(&bm[lo >> 5], 1u << (lo & 31));
        }
        __syncthreads();
        const int per = (nw + NTH - 1) / NTH, w0 = tid * per, w1 = min(nw, w0 + per);
        int cnt = 0;
        for (int q = w0; q < w1; ++q) cnt += __popc(bm[q]);
        int32_t tot;
        int run = scan::block_excl<NTH>((int32_t)cnt, (int32_t)0, scan::Plus(), sh_sm, &tot);
        for (int q = w0; q < w1; ++q) {
            pw[q] = (uint16_t)run;
            run += __popc(bm[q]);
        }
        __syncthreads();
        for (int i = tid; i < n; i += NTH) {
            const uint32_t k = K2[base + i], lo = k & lmask;
            const int r = pw[lo >> 5] + __popc(bm[lo >> 5] & ((1u << (lo & 31)) - 1u));
            K[base + r] = k;
            if (VAL) V[base + r] = V2[base + i];
        }
        if (DEDUP && tot < n) {
            __syncthreads();
            const uint32_t last = K[base + tot - 1];
            for (int i = tot + tid; i < n; i += NTH) K[base + i] = last;
        }
        __syncthreads();
    }
}

// Sorts the bucket K[0..m) (V) by its full key into row order, in place: rows at L.ro[j] with L.rc[j] entries,
// K2 (V2) the row-grouped staging copy.  DEDUP (CSR): duplicate keys are left next to their first copy (a hub row
// produced by the bitmap repeats its largest key over the tail), dropped on emission.  Returns false -- K and V
// untouched -- when the bucket needs the LSD fallback (a long row and LB > BM_LB, or no bitmap space).
template <int NTH, bool VAL, bool DEDUP>
__device__ bool seg_sort(const Geo& g, int nrows, uint32_t* K, uint32_t* K2, int32_t* V, int32_t* V2, int m,
                         SegLds L, int32_t* sh_sm) {
    constexpr int NW = NTH / WAVE;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & (WAVE - 1);
    const uint32_t lmask = (uint32_t)(((uint64_t)1 << g.LB) - 1);
    const bool bitmap_ok = L.bm != nullptr && g.LB <= BM_LB;
    for (int j = tid; j < (1 << SB_MAX); j += NTH) L.rc[j] = 0;
    if (tid == 0) *L.flag = 0;
    __syncthreads();
    for (int i = tid; i < m; i += NTH) L.rank[i] = atomicAdd(&L.rc[K[i] >> g.LB], 1);
    __syncthreads();
    {   // row starts: one block scan over the (<= 256) rows; a long row without the bitmap path -> fallback
        const int x = tid < nrows ? L.rc[tid] : 0;
        int32_t tot;
        const int32_t ex = scan::block_excl<NTH>((int32_t)x, (int32_t)0, scan::Plus(), sh_sm, &tot);
        if (tid < nrows) L.ro[tid] = ex;
        if (x > SHORT_ROW && !bitmap_ok) *L.flag = 1;
    }
    __syncthreads();
    if (*L.flag) return false;
    for (int i = tid; i < m; i += NTH) {
        const uint32_t k = K[i];
        const int p = L.ro[k >> g.LB] + L.rank[i];
        K2[p] = k;
        if (VAL) V2[p] = V[i];
    }
    __syncthreads();
    for (int i = tid; i < m; i += NTH) {   // short rows: rank of (key, index) within the row
        const uint32_t x = K2[i];
        const int j = (int)(x >> g.LB), n = L.rc[j];
        if (n > SHORT_ROW) continue;
        const int s = L.ro[j];
        int p = 0;
        const uint64_t me = ((uint64_t)x << 32) | (uint32_t)i;
        for (int t = s; t < s + n; ++t) p += (((uint64_t)K2[t] << 32) | (uint32_t)t) < me ? 1 : 0;
        K[s + p] = x;
        if (VAL) V[s + p] = V2[i];
    }
    if constexpr (NTH >= BNT) {   // big buckets: the whole block ranks one hub row at a time
        hub_rows_block<NTH, VAL, DEDUP>(g, nrows, K, K2, V, V2, L, sh_sm);
        __syncthreads();
        return true;
    }
    for (int j = w; j < nrows; j += NW) {   // hub rows: one wave each, ranked through a bitmap over the local ids
        const int n = L.rc[j], base = L.ro[j];
        if (n <= SHORT_ROW) continue;
        uint32_t* bm = L.bm + w * BMW;
        uint16_t* pw = L.pw + w * BMW;
        const int nw = (int)((lmask >> 5) + 1);
        for (int i = lane; i < nw; i += WAVE) bm[i] = 0u;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        for (int i = lane; i < n; i += WAVE) {
            const uint32_t lo = K2[base + i] & lmask;
            atomicOr(&bm[lo >> 5], 1u << (lo & 31));
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
        __builtin_amdgcn_wave_barrier();
        const int per = (nw + WAVE - 1) / WAVE, w0 = lane * per, w1 = min(nw, w0 + per);
        int cnt = 0;
        for (int q = w0; q < w1; ++q) cnt += __popc(bm[q]);
        const int inc = scan::wave_incl((int32_t)cnt, scan::Plus());
        const int tot = __shfl(inc, WAVE - 1, WAVE);
        int run = inc - cnt;
        for (int q = w0; q < w1; ++q) {   // distinct ids below each word
            pw[q] = (uint16_t)run;
            run += __popc(bm[q]);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
        __builtin_amdgcn_wave_barrier();
        for (int i = lane; i < n; i += WAVE) {   // rank = distinct ids below; duplicates share (and rewrite) a slot
            const uint32_t k = K2[base + i], lo = k & lmask;
            const int r = pw[lo >> 5] + __popc(bm[lo >> 5] & ((1u << (lo & 31)) - 1u));
            K[base + r] = k;
            if (VAL) V[base + r] = V2[base + i];
        }
        if (DEDUP && tot < n) {   // the duplicates' slots repeat the row's largest key
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
            __builtin_amdgcn_wave_barrier();
            const uint32_t last = K[base + tot - 1];
            for (int i = tot + lane; i < n; i += WAVE) K[base + i] = last;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    return true;
}

// CSR: the sorted bucket S[0..m) -> its unique keys (compacted through C, then out coalesced), the in-bucket row
// prefix into rowptr (a row starts where the row bits change: every row holds at least its self-loop), unique count
template <int NTH>
__device__ void csr_emit(const Geo& g, int64_t b, const uint32_t* S, uint32_t* C, int m, int32_t* sh_sm, int32_t off,
                         uint32_t* __restrict__ keys, int32_t* __restrict__ rowptr, int32_t* __restrict__ ucnt) {
    constexpr int EI = 8;
    const int tid = threadIdx.x;
    int32_t carry = 0;
    for (int t0 = 0; t0 < m; t0 += NTH * EI) {
        const int q0 = t0 + tid * EI;
        uint32_t v[EI];
        uint32_t prev = q0 > 0 && q0 < m ? S[q0 - 1] : 0u;
        int c = 0;
        unsigned keep = 0, first = 0;
#pragma unroll
        for (int k = 0; k < EI; ++k) {
            const int q = q0 + k;
            v[k] = q < m ? S[q] : 0u;
            if (q < m) {
                const bool kp = q == 0 || v[k] != prev;
                keep |= (unsigned)kp << k;
                first |= (unsigned)(q == 0 || (v[k] >> g.LB) != (prev >> g.LB)) << k;
                c += kp ? 1 : 0;
            }
            prev = v[k];
        }
        int32_t tot;
        int32_t p = carry + scan::block_excl<NTH>((int32_t)c, (int32_t)0, scan::Plus(), sh_sm, &tot);
#pragma unroll
        for (int k = 0; k < EI; ++k) {
            if ((keep >> k) & 1) {
                if ((first >> k) & 1) rowptr[(b << g.SB) + (v[k] >> g.LB)] = p;
                C[p++] = v[k];
            }
        }
        carry += tot;
    }
    __syncthreads();
    for (int i = tid; i < carry; i += NTH) keys[off + i] = C[i];
    if (tid == 0) ucnt[b] = carry;
    __syncthreads();
}

// CSC: csc_row / csc_eid / csc_ptr of the bucket's columns and the CSR -> CSC position map
template <int NTH>
__device__ void csc_emit(const Geo& g, int64_t b, int nrows, const uint32_t* S, const int32_t* SV, int m, SegLds L,
                         const int32_t* colbase, int32_t o, int32_t* __restrict__ csc_ptr,
                         int32_t* __restrict__ csc_row, int32_t* __restrict__ csc_eid, int32_t* __restrict__ cpos) {
    const int tid = threadIdx.x;
    const uint32_t lmask = (uint32_t)(((uint64_t)1 << g.LB) - 1);
    if (tid < nrows) csc_ptr[(b << g.SB) + tid] = o + L.ro[tid];
    for (int q = tid; q < m; q += NTH) {
        const uint32_t k = S[q];
        const int32_t e = SV[q];
        csc_row[o + q] = colbase[k >> g.LB] + (int32_t)(k & lmask);
        csc_eid[o + q] = e;
        if (cpos) cpos[e] = o + q;
    }
}

// the LSD fallback of a CSR bucket (K holds its m raw keys + self-loops): sort, dedupe, emit
template <int NTH>
__device__ void csr_lsd(const Geo& g, int64_t b, int nrows, uint32_t* A, uint32_t* B, int m, int32_t off,
                        uint32_t* __restrict__ keys, int32_t* __restrict__ rowptr, int32_t* __restrict__ ucnt,
                        int* sh_base, int* sh_tot, int* sh_wc, int* sh_rc, int32_t* sh_sm) {
    const int tid = threadIdx.x;
    for (int j = tid; j < nrows; j += NTH) sh_rc[j] = 0;
    __syncthreads();
    const uint32_t* R = block_radix_sort<NTH, 1, false>(A, B, nullptr, nullptr, m, g.SB + g.LB, sh_base, sh_tot,
                                                        sh_wc, sh_sm) ? B : A;
    int32_t run = 0;
    for (int t0 = 0; t0 < m; t0 += NTH) {
        const int i = t0 + tid;
        const uint32_t k = i < m ? R[i] : 0u;
        const bool first = i < m && (i == 0 || R[i - 1] != k);
        int32_t tot;
        const int32_t pos = run + scan::block_excl<NTH>((int32_t)(first ? 1 : 0), (int32_t)0, scan::Plus(), sh_sm, &tot);
        if (first) {
            keys[off + pos] = k;
            atomicAdd(&sh_rc[k >> g.LB], 1);
        }
        run += tot;
        __syncthreads();
    }
    const int x = tid < nrows ? sh_rc[tid] : 0;
    int32_t tot;
    const int32_t ex = scan::block_excl<NTH>((int32_t)x, (int32_t)0, scan::Plus(), sh_sm, &tot);
    if (tid < nrows) rowptr[(b << g.SB) + tid] = ex;
    if (tid == 0) ucnt[b] = run;
    __syncthreads();
}

// the LSD fallback of a CSC bucket (K, V its pairs): sort by (column, local src), emit
template <int NTH>
__device__ void csc_lsd(const Geo& g, int64_t b, int nrows, uint32_t* K, uint32_t* K2, int32_t* V, int32_t* V2, int m,
                        int32_t o, const int32_t* colbase, int32_t* __restrict__ csc_ptr, int32_t* __restrict__ csc_row,
                        int32_t* __restrict__ csc_eid, int32_t* __restrict__ cpos, int* sh_base, int* sh_tot,
                        int* sh_wc, int* sh_rc, int32_t* sh_sm) {
    const int tid = threadIdx.x;
    for (int j = tid; j < nrows; j += NTH) sh_rc[j] = 0;
    __syncthreads();
    const int par = block_radix_sort<NTH, 1, true>(K, K2, V, V2, m, g.SB + g.LB, sh_base, sh_tot, sh_wc, sh_sm);
    const uint32_t* RK = par ? K2 : K;
    const int32_t* RV = par ? V2 : V;
    const uint32_t lmask = (uint32_t)(((uint64_t)1 << g.LB) - 1);
    for (int i = tid; i < m; i += NTH) {
        const uint32_t k = RK[i];
        const int j = (int)(k >> g.LB);
        const int32_t e = RV[i];
        csc_row[o + i] = colbase[j] + (int32_t)(k & lmask);
        csc_eid[o + i] = e;
        if (cpos) cpos[e] = o + i;
        atomicAdd(&sh_rc[j], 1);
    }
    __syncthreads();
    const int x = tid < nrows ? sh_rc[tid] : 0;
    int32_t tot;
    const int32_t ex = scan::block_excl<NTH>((int32_t)x, (int32_t)0, scan::Plus(), sh_sm, &tot);
    if (tid < nrows) csc_ptr[(b << g.SB) + tid] = o + ex;
    __syncthreads();
}

// one CSR bucket: load its raw keys (+ self-loops) into A, sort in place (B staging), emit (or the LSD fallback)
template <int NTH>
__device__ void csr_bucket(const Geo& g, int64_t b, uint32_t* A, uint32_t* B, bool global_bufs, int c, int32_t off,
                           const int64_t* __restrict__ node_ptr, uint32_t* __restrict__ keys,
                           int32_t* __restrict__ rowptr, int32_t* __restrict__ ucnt, SegLds L, int* sh_base,
                           int* sh_tot, int32_t* sh_sm) {
    const int tid = threadIdx.x;
    const int64_t r0 = b << g.SB;
    const int nv = (int)bucket_rows(b, g.SB, g.N);
    if (!global_bufs) gload_lds<NTH, NTH >= BNT ? 4 : 8>(A, keys + off, c);
    const BucketBase nbase(node_ptr, g.G, r0);
    for (int j = tid; j < nv; j += NTH) {     // the bucket's self-loops ("+ eye")
        const int64_t v = r0 + j;
        A[c + j] = ((uint32_t)j << g.LB) | (uint32_t)(v - nbase(v));
    }
    __syncthreads();
    const int m = c + nv;
    if (seg_sort<NTH, false, true>(g, nv, A, B, nullptr, nullptr, m, L, sh_sm))
        csr_emit<NTH>(g, b, A, B, m, sh_sm, off, keys, rowptr, ucnt);
    else
        csr_lsd<NTH>(g, b, nv, A, B, m, off, keys, rowptr, ucnt, sh_base, sh_tot, L.wc, L.rc, sh_sm);
}

// the buckets too large for the small finish kernels (CSR: raw keys + self-loops > CAP_S; CSC: pairs > CAP_C), listed
// before the finish so the big-bucket kernel's workgroups take them straight from the list (the list order is
// irrelevant: every bucket's output depends on the bucket alone).  Running that kernel on a side stream beside the
// small-bucket one was measured slower in the step (profiles/r4k_csr_side_ab.txt) and removed.
template <bool CSC>
__global__ void __launch_bounds__(BLK) k_big_list(Geo g, const int32_t* __restrict__ fill, int32_t* __restrict__ big,
                                                  int32_t* __restrict__ nbig) {
    for (int64_t b = blockIdx.x * (int64_t)BLK + threadIdx.x; b < g.NB; b += (int64_t)gridDim.x * BLK) {
        const bool is_big = CSC ? fill[b] > CAP_C : fill[b] + (int)bucket_rows(b, g.SB, g.N) > CAP_S;
        if (is_big) big[atomicAdd(nbig + (CSC ? 1 : 0), 1)] = (int32_t)b;
    }
}

__global__ void __launch_bounds__(FNT) k_csr_finish(Geo g, const int32_t* __restrict__ bstart,
                                                    const int32_t* __restrict__ fill_src,
                                                    const int64_t* __restrict__ node_ptr, uint32_t* __restrict__ keys,
                                                    int32_t* __restrict__ rowptr, int32_t* __restrict__ ucnt,
                                                    int32_t* __restrict__ big, int32_t* __restrict__ nbig) {
    constexpr int RK = CAP_S > (FNT / WAVE) * BMW * 3 / 2 ? CAP_S : (FNT / WAVE) * BMW * 3 / 2;
    static_assert(RK >= (FNT / WAVE) * RBINS, "the LSD count table aliases the rank array");
    __shared__ uint32_t A[CAP_S], Bk[CAP_S];
    __shared__ int rc[1 << SB_MAX], ro[1 << SB_MAX], flag;
    __shared__ int rk[RK];   // row slots, then the per-wave bitmaps / the LSD count table
    __shared__ int base[RBINS], tot[RBINS];
    __shared__ int32_t sm[FNT / WAVE + 1];
    const int64_t b = blockIdx.x;
    const int c = fill_src[b];
    if (c + (int)bucket_rows(b, g.SB, g.N) > CAP_S) return;   // listed by k_big_list, finished by k_csr_finish_big
    const SegLds L{rc, ro, (uint32_t*)rk, (uint16_t*)(rk + (FNT / WAVE) * BMW), rk, rk, &flag};
    csr_bucket<FNT>(g, b, A, Bk, false, c, bstart[b], node_ptr, keys, rowptr, ucnt, L, base, tot, sm);
}

__global__ void __launch_bounds__(BNT) k_csr_finish_big(Geo g, const int32_t* __restrict__ bstart,
                                                        const int32_t* __restrict__ fill_src,
                                                        const int64_t* __restrict__ node_ptr,
                                                        uint32_t* __restrict__ keys, uint32_t* __restrict__ scratch,
                                                        int32_t* __restrict__ rank_g,
                                                        int32_t* __restrict__ rowptr, int32_t* __restrict__ ucnt,
                                                        const int32_t* __restrict__ big,
                                                        const int32_t* __restrict__ nbig) {
    extern __shared__ __attribute__((aligned(16))) uint32_t dyn[];
    __shared__ int rc[1 << SB_MAX], ro[1 << SB_MAX], flag;
    __shared__ uint32_t bm[BMW];   // one bitmap: the block ranks hub rows together
    __shared__ uint16_t pw[BMW];
    __shared__ int wc[(BNT / WAVE) * RBINS];
    __shared__ int base[RBINS], tot[RBINS];
    __shared__ int32_t sm[BNT / WAVE + 1];
    constexpr int CAP = BIG_LDS / 8;
    const int nb = *nbig;
    for (int q = blockIdx.x; q < nb; q += gridDim.x) {
        const int64_t b = big[q];
        const int c = fill_src[b];
        const int m = c + (int)bucket_rows(b, g.SB, g.N);
        const int32_t off = bstart[b];
        const SegLds L{rc, ro, bm, pw, rank_g + off, wc, &flag};
        if (m <= CAP)
            csr_bucket<BNT>(g, b, dyn, dyn + CAP, false, c, off, node_ptr, keys, rowptr, ucnt, L, base, tot, sm);
        else   // in global memory: the bucket's own region (room for its self-loops) and the scratch twin
            csr_bucket<BNT>(g, b, keys + off, scratch + off, true, c, off, node_ptr, keys, rowptr, ucnt, L, base, tot,
                            sm);
    }
}

// one CSC bucket: its (key, CSR position) pairs in K / V, sorted in place (K2 / V2 staging), emit (or the fallback)
template <int NTH>
__device__ void csc_bucket(const Geo& g, int64_t b, uint32_t* K, uint32_t* K2, int32_t* V, int32_t* V2, int m,
                           int32_t o, const int64_t* __restrict__ node_ptr, int32_t* __restrict__ csc_ptr,
                           int32_t* __restrict__ csc_row, int32_t* __restrict__ csc_eid, int32_t* __restrict__ cpos,
                           SegLds L, int* colbase, int* sh_base, int* sh_tot, int32_t* sh_sm) {
    const int tid = threadIdx.x;
    const int64_t c0 = b << g.SB;
    const int nv = (int)bucket_rows(b, g.SB, g.N);
    const BucketBase nbase(node_ptr, g.G, c0);
    for (int j = tid; j < nv; j += NTH) colbase[j] = (int32_t)nbase(c0 + j);
    __syncthreads();
    if (seg_sort<NTH, true, false>(g, nv, K, K2, V, V2, m, L, sh_sm))
        csc_emit<NTH>(g, b, nv, K, V, m, L, colbase, o, csc_ptr, csc_row, csc_eid, cpos);
    else
        csc_lsd<NTH>(g, b, nv, K, K2, V, V2, m, o, colbase, csc_ptr, csc_row, csc_eid, cpos, sh_base, sh_tot, L.wc,
                     L.rc, sh_sm);
}

__global__ void __launch_bounds__(FNT) k_csc_finish(Geo g, const int32_t* __restrict__ cstart,
                                                    const int32_t* __restrict__ fill_dst,
                                                    const int32_t* __restrict__ coff,
                                                    const int64_t* __restrict__ node_ptr,
                                                    const uint32_t* __restrict__ ckey,
                                                    const int32_t* __restrict__ cval, int32_t* __restrict__ csc_ptr,
                                                    int32_t* __restrict__ csc_row, int32_t* __restrict__ csc_eid,
                                                    int32_t* __restrict__ cpos, int32_t* __restrict__ big,
                                                    int32_t* __restrict__ nbig) {
    constexpr int RK = CAP_C > (FNT / WAVE) * BMW * 3 / 2 ? CAP_C : (FNT / WAVE) * BMW * 3 / 2;
    static_assert(RK >= (FNT / WAVE) * RBINS, "the LSD count table aliases the rank array");
    __shared__ uint32_t K[CAP_C], K2[CAP_C];
    __shared__ int32_t V[CAP_C], V2[CAP_C];
    __shared__ int rc[1 << SB_MAX], ro[1 << SB_MAX], cb[1 << SB_MAX], flag;
    __shared__ int rk[RK];   // row slots, then the per-wave bitmaps / the LSD count table
    __shared__ int base[RBINS], tot[RBINS];
    __shared__ int32_t sm[FNT / WAVE + 1];
    const int64_t b = blockIdx.x;
    const int m = fill_dst[b];
    if (m > CAP_C) return;   // listed by k_big_list, finished by k_csc_finish_big
    const int32_t ro0 = cstart[b];
    gload_lds2<FNT, 8>(K, ckey + ro0, V, cval + ro0, m);
    const SegLds L{rc, ro, (uint32_t*)rk, (uint16_t*)(rk + (FNT / WAVE) * BMW), rk, rk, &flag};
    csc_bucket<FNT>(g, b, K, K2, V, V2, m, coff[b], node_ptr, csc_ptr, csc_row, csc_eid, cpos, L, cb, base,
                    tot, sm);
    if (b == g.NB - 1 && threadIdx.x == 0) csc_ptr[g.N] = coff[g.NB];
}

__global__ void __launch_bounds__(BNT) k_csc_finish_big(Geo g, const int32_t* __restrict__ cstart,
                                                        const int32_t* __restrict__ fill_dst,
                                                        const int32_t* __restrict__ coff,
                                                        const int64_t* __restrict__ node_ptr,
                                                        uint32_t* __restrict__ ckey, int32_t* __restrict__ cval,
                                                        uint32_t* __restrict__ sk, int32_t* __restrict__ sv,
                                                        int32_t* __restrict__ rank_g,
                                                        int32_t* __restrict__ csc_ptr, int32_t* __restrict__ csc_row,
                                                        int32_t* __restrict__ csc_eid, int32_t* __restrict__ cpos,
                                                        const int32_t* __restrict__ big,
                                                        const int32_t* __restrict__ nbig) {
    extern __shared__ __attribute__((aligned(16))) uint32_t dyn[];
    __shared__ int rc[1 << SB_MAX], ro[1 << SB_MAX], cb[1 << SB_MAX], flag;
    __shared__ uint32_t bm[BMW];   // one bitmap: the block ranks hub rows together
    __shared__ uint16_t pw[BMW];
    __shared__ int wc[(BNT / WAVE) * RBINS];
    __shared__ int base[RBINS], tot[RBINS];
    __shared__ int32_t sm[BNT / WAVE + 1];
    constexpr int CAP = BIG_LDS / 16;
    const int nb = nbig[1];
    for (int q = blockIdx.x; q < nb; q += gridDim.x) {
        const int64_t b = big[q];
        const int m = fill_dst[b];
        const int32_t ro0 = cstart[b];
        const SegLds L{rc, ro, bm, pw, rank_g + ro0, wc, &flag};
        if (m <= CAP) {
            uint32_t* K = dyn;
            uint32_t* K2 = dyn + CAP;
            int32_t* V = (int32_t*)(dyn + 2 * CAP);
            int32_t* V2 = (int32_t*)(dyn + 3 * CAP);
            gload_lds2<BNT, 4>(K, ckey + ro0, V, cval + ro0, m);
            csc_bucket<BNT>(g, b, K, K2, V, V2, m, coff[b], node_ptr, csc_ptr, csc_row, csc_eid, cpos, L,
                            cb, base, tot, sm);
        } else {
            csc_bucket<BNT>(g, b, ckey + ro0, sk + ro0, cval + ro0, sv + ro0, m, coff[b], node_ptr, csc_ptr, csc_row,
                            csc_eid, cpos, L, cb, base, tot, sm);
        }
        if (b == g.NB - 1 && threadIdx.x == 0) csc_ptr[g.N] = coff[g.NB];
        __syncthreads();
    }
}

// 6. place: CSR col, rowptr (+ the bucket's offset), each entry's local src (for the CSC pass), nnz
__global__ void __launch_bounds__(FNT) k_csr_place(Geo g, const int32_t* __restrict__ bstart,
                                                   const int32_t* __restrict__ uoff,
                                                   const int64_t* __restrict__ node_ptr,
                                                   const uint32_t* __restrict__ keys, int32_t* __restrict__ rowptr,
                                                   int32_t* __restrict__ col, int32_t* __restrict__ sloc,
                                                   int64_t* __restrict__ nnz_out) {
    __shared__ int32_t rb[1 << SB_MAX];
    const int64_t b = blockIdx.x;
    const int64_t r0 = b << g.SB;
    const int nv = (int)bucket_rows(b, g.SB, g.N);
    const int32_t off = bstart[b], u = uoff[b], cnt = uoff[b + 1] - u;
    const BucketBase nbase(node_ptr, g.G, r0);
    for (int j = threadIdx.x; j < nv; j += FNT) {
        rb[j] = (int32_t)nbase(r0 + j);
        rowptr[r0 + j] += u;
    }
    __syncthreads();
    const uint32_t lmask = (uint32_t)(((uint64_t)1 << g.LB) - 1);
    constexpr int PER = 8;   // loads in flight per thread (see gload_lds)
    for (int base = 0; base < cnt; base += FNT * PER) {
        uint32_t kr[PER];
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int i = base + q * FNT + (int)threadIdx.x;
            if (i < cnt) kr[q] = keys[off + i];
        }
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int i = base + q * FNT + (int)threadIdx.x;
            if (i >= cnt) continue;
            const uint32_t k = kr[q];
            const int j = (int)(k >> g.LB);
            if (TAGAN_DBAD(j < nv && u + i < g.E + g.N, j, u + i)) continue;   // row of the bucket, CSR capacity
            if (TAGAN_DBAD(rb[j] + (int64_t)(k & lmask) < g.N, rb[j], k & lmask)) continue;   // column id
            col[u + i] = rb[j] + (int32_t)(k & lmask);
            sloc[u + i] = (int32_t)(r0 + j) - rb[j];
        }
    }
    if (b == g.NB - 1 && threadIdx.x == 0) {
        rowptr[g.N] = uoff[g.NB];
        *nnz_out = uoff[g.NB];
    }
}

// 7a. CSR entries -> (bucket-in-bin << SB+LB | column-in-bucket << LB | local src, CSR position), coarse dst bins
// (SC = 0: straight into the dst buckets); snapshot by snapshot inside the block
__global__ void __launch_bounds__(PNT) k_part_csr(Geo g, const int32_t* __restrict__ rowptr,
                                                  const int32_t* __restrict__ col, const int32_t* __restrict__ sloc,
                                                  const int64_t* __restrict__ node_ptr,
                                                  const int64_t* __restrict__ nnz_p,
                                                  const int32_t* __restrict__ cstart, int32_t* __restrict__ fill,
                                                  uint32_t* __restrict__ okey, int32_t* __restrict__ oval) {
    __shared__ int h[PART_BINS];
    __shared__ int tcnt[PNB], tstart[PNB], gpos[PNB];
    __shared__ uint32_t stk[PTILE];
    __shared__ int32_t stv[PTILE];
    __shared__ int stp[PTILE];
    __shared__ int32_t sm[PNT / WAVE + 1];
    __shared__ int gr[2];
    for (int i = threadIdx.x; i < PNB; i += PNT) tcnt[i] = 0;
    const int64_t nnz = *nnz_p;
    const int64_t e0 = blockIdx.x * g.CHc, e1 = min(nnz, e0 + g.CHc);
    if (e0 >= e1) return;
    if (threadIdx.x < 2) {   // snapshots of the first / last entry's row (binary search of rowptr)
        const int64_t e = threadIdx.x == 0 ? e0 : e1 - 1;
        int64_t lo = 0, hi = g.N - 1;
        while (lo < hi) {
            const int64_t mid = (lo + hi + 1) >> 1;
            if (rowptr[mid] <= e) lo = mid; else hi = mid - 1;
        }
        gr[threadIdx.x] = find_graph(node_ptr, g.G, lo);
    }
    __syncthreads();
    const int shc = g.SB + g.SC;
    const uint32_t cmask = (1u << g.SB) - 1u, fmask = (1u << g.SC) - 1u;
    const int g0 = gr[0], g1 = gr[1];
    for (int gg = g0; gg <= g1; ++gg) {
        const int64_t v0 = node_ptr[gg], v1 = node_ptr[gg + 1];
        const int64_t a = max(e0, (int64_t)rowptr[v0]), z = min(e1, (int64_t)rowptr[v1]);
        const Span sp = span_of(v0, v1, shc, PART_BINS);
        const bool staged = sp.lds && sp.nb <= PNB;
        if (sp.lds && !(TAGAN_CSR_TILE_RES && staged)) {
            for (int i = threadIdx.x; i < sp.nb; i += PNT) h[i] = 0;
            __syncthreads();
            for (int64_t e4 = a + threadIdx.x; e4 < z; e4 += UNR * PNT) {
                int32_t d[UNR];
#pragma unroll
                for (int u = 0; u < UNR; ++u) d[u] = e4 + u * PNT < z ? col[e4 + u * PNT] : 0;
#pragma unroll
                for (int u = 0; u < UNR; ++u)
                    if (e4 + u * PNT < z) atomicAdd(&h[(d[u] >> shc) - sp.b0], 1);
            }
            __syncthreads();
            for (int i = threadIdx.x; i < sp.nb; i += PNT) {
                const int c = h[i];
                const int64_t bin = sp.b0 + i;
                if (c) h[i] = cstart[bin << g.SC] + atomicAdd(&fill[bin], c);
            }
            __syncthreads();
        }
        if (staged) {   // LDS-staged scatter
            const CsrEntryLoader ld{col, sloc, sp.b0, shc, g.SB, g.LB, cmask, fmask};
            tile_partition<PNT, PIPT, PNB, true, TAGAN_CSR_TILE_RES>(a, z, ld, h, tcnt, tstart, gpos, stk, stv, stp, sm,
                                                                     okey, oval, TileRes{cstart, fill, sp.b0, g.SC});
        } else {
            for (int64_t e4 = a + threadIdx.x; e4 < z; e4 += UNR * PNT) {
                int32_t dd[UNR], sl[UNR];
#pragma unroll
                for (int u = 0; u < UNR; ++u) {
                    const bool ok = e4 + u * PNT < z;
                    dd[u] = ok ? col[e4 + u * PNT] : 0;
                    sl[u] = ok ? sloc[e4 + u * PNT] : 0;
                }
#pragma unroll
                for (int u = 0; u < UNR; ++u) {
                    const int64_t e = e4 + u * PNT;
                    if (e >= z) break;
                    const int32_t d = dd[u];
                    const int64_t bin = d >> shc;
                    const int pos = sp.lds ? atomicAdd(&h[bin - sp.b0], 1)
                                           : cstart[bin << g.SC] + atomicAdd(&fill[bin], 1);
                    okey[pos] = ((((uint32_t)(d >> g.SB) & fmask) << g.SB | ((uint32_t)d & cmask)) << g.LB) |
                                (uint32_t)sl[u];
                    oval[pos] = (int32_t)e;
                }
            }
        }
        __syncthreads();
    }
}

// inverse of csc_eid: the CSC position of each CSR entry (graphs not built by tagan_csr_build)
__global__ void __launch_bounds__(BLK) k_csc_pos(const int32_t* __restrict__ csc_eid, const int64_t* __restrict__ nnz_p,
                                                 int32_t* __restrict__ cpos) {
    const int64_t nnz = *nnz_p;
    for (int64_t p = blockIdx.x * (int64_t)BLK + threadIdx.x; p < nnz; p += (int64_t)gridDim.x * BLK)
        cpos[csc_eid[p]] = (int32_t)p;
}

int grid_for(int64_t n) {
    int64_t gsz = (n + BLK - 1) / BLK;
    if (gsz > 256 * 16) gsz = 256 * 16;
    return (int)(gsz < 1 ? 1 : gsz);
}

struct CsrWs {
    size_t cap_src, fill_src, fillc_src, ucnt, cap_dst, fill_dst, fillc_dst, coff, big_src, big_dst, nbig, part,
        keys, stage, sloc, cval, sval, total;
};

CsrWs plan(const Geo& g) {
    const int64_t M = g.E + g.N;
    CsrWs w{};
    size_t off = 0;
    auto take = [&](size_t bytes) { size_t o = off; off = align_up(off + bytes, 256); return o; };
    w.cap_src = take((g.NB + 1) * 4);
    w.fill_src = take(g.NB * 4);
    w.fillc_src = take(g.NCB * 4);
    w.ucnt = take((g.NB + 1) * 4);
    w.cap_dst = take((g.NB + 1) * 4);
    w.fill_dst = take(g.NB * 4);
    w.fillc_dst = take(g.NCB * 4);
    w.coff = take((g.NB + 1) * 4);
    w.big_src = take(g.NB * 4);
    w.big_dst = take(g.NB * 4);
    w.nbig = take(2 * 4);
    w.part = take(scan::parts_len(g.NB) * 4);
    w.keys = take(M * 4);      // bucket layout: CSR keys, then the CSC keys
    w.stage = take(M * 4);     // coarse staging keys; the big buckets' global-memory sort twin
    w.sloc = take(M * 4);
    w.cval = take(M * 4);      // bucket layout CSC values
    w.sval = take(M * 4);      // staging values / value twin
    w.total = off;
    return w;
}


}  // namespace
}  // namespace tagan

extern "C" {

size_t tagan_csr_build_workspace(int64_t n_edges, int64_t n_nodes) {
    if (n_edges < 0 || n_nodes <= 0) return 0;
    // sized for both extremes of max_graph_nodes (the local-id width caps the bucket bits: more buckets)
    using namespace tagan;
    const Geo a = geometry(n_edges, n_nodes, 1, n_nodes), b = geometry(n_edges, n_nodes, 1, 1);
    return std::max(plan(a).total, plan(b).total);
}

int tagan_csr_build(const int64_t* edge_index, int64_t ld_ei, int64_t n_edges, const int64_t* edge_ptr,
                    const int64_t* node_ptr, int32_t n_graphs, int64_t n_nodes, int64_t max_graph_nodes,
                    int32_t* rowptr, int32_t* col,
                    int32_t* csc_ptr, int32_t* csc_row, int32_t* csc_eid, int64_t* nnz_out, int32_t* err_out,
                    int32_t* csr_cpos, void* workspace, size_t workspace_bytes, void* stream) {
    using namespace tagan;
    TAGAN_REQUIRE(n_nodes > 0 && n_nodes < (int64_t)INT32_MAX - 1, TAGAN_ERR_ARG,
                  "tagan_csr_build: n_nodes=%lld out of range", (long long)n_nodes);
    TAGAN_REQUIRE(n_edges >= 0 && (n_edges == 0 || (edge_index && ld_ei >= n_edges)), TAGAN_ERR_ARG,
                  "tagan_csr_build: bad edge_index (E=%lld ld=%lld)", (long long)n_edges, (long long)ld_ei);
    TAGAN_REQUIRE(n_edges + n_nodes < (int64_t)INT32_MAX, TAGAN_ERR_ARG, "tagan_csr_build: too many edges");
    TAGAN_REQUIRE(n_graphs >= 1 && edge_ptr && node_ptr, TAGAN_ERR_ARG, "tagan_csr_build: bad graph pointers");
    TAGAN_REQUIRE(rowptr && col && csc_ptr && csc_row && csc_eid && nnz_out && err_out, TAGAN_ERR_ARG,
                  "tagan_csr_build: null output");
    TAGAN_REQUIRE(max_graph_nodes <= n_nodes, TAGAN_ERR_ARG, "tagan_csr_build: max_graph_nodes > n_nodes");
    const int64_t NL = max_graph_nodes > 0 ? max_graph_nodes : n_nodes;
    const Geo g = geometry(n_edges, n_nodes, n_graphs, NL);
    const CsrWs w = plan(g);
    TAGAN_REQUIRE(workspace && workspace_bytes >= w.total, TAGAN_ERR_WORKSPACE,
                  "tagan_csr_build: workspace %zu < %zu", workspace_bytes, w.total);
    static const bool lds_ok = [] {
        hipError_t e1 = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_csr_finish_big),
                                            hipFuncAttributeMaxDynamicSharedMemorySize, BIG_LDS);
        hipError_t e2 = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_csc_finish_big),
                                            hipFuncAttributeMaxDynamicSharedMemorySize, BIG_LDS);
        return e1 == hipSuccess && e2 == hipSuccess;
    }();
    TAGAN_REQUIRE(lds_ok, TAGAN_ERR_LAUNCH, "tagan_csr_build: cannot enable %d B of dynamic LDS", BIG_LDS);
    hipStream_t s = as_stream(stream);
    char* ws = (char*)workspace;
    int32_t* cap_src = (int32_t*)(ws + w.cap_src);
    int32_t* fill_src = (int32_t*)(ws + w.fill_src);
    int32_t* fillc_src = (int32_t*)(ws + w.fillc_src);
    int32_t* ucnt = (int32_t*)(ws + w.ucnt);
    int32_t* cap_dst = (int32_t*)(ws + w.cap_dst);
    int32_t* fill_dst = (int32_t*)(ws + w.fill_dst);
    int32_t* fillc_dst = (int32_t*)(ws + w.fillc_dst);
    int32_t* coff = (int32_t*)(ws + w.coff);
    int32_t* big_src = (int32_t*)(ws + w.big_src);
    int32_t* big_dst = (int32_t*)(ws + w.big_dst);
    int32_t* nbig = (int32_t*)(ws + w.nbig);
    int32_t* part = (int32_t*)(ws + w.part);
    uint32_t* keys = (uint32_t*)(ws + w.keys);
    uint32_t* stage = (uint32_t*)(ws + w.stage);
    int32_t* sloc = (int32_t*)(ws + w.sloc);
    int32_t* cval = (int32_t*)(ws + w.cval);
    int32_t* sval = (int32_t*)(ws + w.sval);
    const scan::Plus plus;
    const bool two_level = g.SC > 0;

    k_init<<<grid_for(g.NB), BLK, 0, s>>>(g, cap_src, fill_src, cap_dst, fill_dst, fillc_src, fillc_dst, nbig, err_out);
    TAGAN_CHECK_LAUNCH("csr_build.init");
    const int64_t nblk = (n_edges + g.CH - 1) / g.CH, nblk_n = (n_edges + g.CHn - 1) / g.CHn;
    if (nblk > 0) {
        k_count<<<(unsigned)nblk_n, PNT, 0, s>>>(g, edge_index, ld_ei, edge_ptr, node_ptr, cap_src, cap_dst, err_out);
        TAGAN_CHECK_LAUNCH("csr_build.count");
    }
    scan::exclusive(cap_src, cap_src, g.NB, (int32_t)0, plus, part, true, s);     // -> src bucket regions
    scan::exclusive(cap_dst, cap_dst, g.NB, (int32_t)0, plus, part, true, s);     // -> dst bucket regions
    TAGAN_CHECK_LAUNCH("csr_build.scan_capacity");
    if (nblk > 0) {
        k_part_edges<<<(unsigned)nblk, PNT, 0, s>>>(g, edge_index, ld_ei, edge_ptr, node_ptr, cap_src,
                                                    two_level ? fillc_src : fill_src, two_level ? stage : keys);
        TAGAN_CHECK_LAUNCH("csr_build.part_edges");
        if (two_level) {
            k_refine<false><<<(unsigned)g.NCB, RNT, 0, s>>>(g, cap_src, fillc_src, stage, nullptr, fill_src, keys,
                                                            nullptr);
            TAGAN_CHECK_LAUNCH("csr_build.refine");
        }
    }
    k_big_list<false><<<grid_for(g.NB), BLK, 0, s>>>(g, fill_src, big_src, nbig);
    TAGAN_CHECK_LAUNCH("csr_build.big_list");
    k_csr_finish_big<<<BIG_WG, BNT, BIG_LDS, s>>>(g, cap_src, fill_src, node_ptr, keys, stage, sloc, rowptr, ucnt,
                                                        big_src, nbig);
    TAGAN_CHECK_LAUNCH("csr_build.csr_finish_big");
    k_csr_finish<<<(unsigned)g.NB, FNT, 0, s>>>(g, cap_src, fill_src, node_ptr, keys, rowptr, ucnt, big_src, nbig);
    TAGAN_CHECK_LAUNCH("csr_build.csr_finish");
    scan::exclusive(ucnt, ucnt, g.NB, (int32_t)0, plus, part, true, s);           // -> CSR bucket offsets
    TAGAN_CHECK_LAUNCH("csr_build.scan_unique");
    k_csr_place<<<(unsigned)g.NB, FNT, 0, s>>>(g, cap_src, ucnt, node_ptr, keys, rowptr, col, sloc, nnz_out);
    TAGAN_CHECK_LAUNCH("csr_build.csr_place");
    const int64_t nblk_c = (n_edges + n_nodes + g.CHc - 1) / g.CHc;   // capacity bound; blocks past nnz exit
    k_part_csr<<<(unsigned)nblk_c, PNT, 0, s>>>(g, rowptr, col, sloc, node_ptr, nnz_out, cap_dst,
                                                two_level ? fillc_dst : fill_dst, two_level ? stage : keys,
                                                two_level ? sval : cval);
    TAGAN_CHECK_LAUNCH("csr_build.part_csr");
    if (two_level) {
        k_refine<true><<<(unsigned)g.NCB, RNT, 0, s>>>(g, cap_dst, fillc_dst, stage, sval, fill_dst, keys, cval);
        TAGAN_CHECK_LAUNCH("csr_build.refine_csc");
    }
    scan::exclusive(fill_dst, coff, g.NB, (int32_t)0, plus, part, true, s);       // -> CSC bucket offsets
    TAGAN_CHECK_LAUNCH("csr_build.scan_csc");
    k_big_list<true><<<grid_for(g.NB), BLK, 0, s>>>(g, fill_dst, big_dst, nbig);
    TAGAN_CHECK_LAUNCH("csr_build.big_list_csc");
    k_csc_finish_big<<<BIG_WG, BNT, BIG_LDS, s>>>(g, cap_dst, fill_dst, coff, node_ptr, keys, cval, stage,
                                                        sval, sloc, csc_ptr, csc_row, csc_eid, csr_cpos, big_dst, nbig);
    TAGAN_CHECK_LAUNCH("csr_build.csc_finish_big");
    k_csc_finish<<<(unsigned)g.NB, FNT, 0, s>>>(g, cap_dst, fill_dst, coff, node_ptr, keys, cval, csc_ptr,
                                                csc_row, csc_eid, csr_cpos, big_dst, nbig);
    TAGAN_CHECK_LAUNCH("csr_build.csc_finish");
    return TAGAN_OK;
}

int tagan_csr_csc_pos(const int32_t* csc_eid, const int64_t* nnz, int64_t nnz_cap, int32_t* csr_cpos, void* stream) {
    using namespace tagan;
    TAGAN_REQUIRE(csc_eid && nnz && csr_cpos && nnz_cap > 0, TAGAN_ERR_ARG, "csr_csc_pos: bad argument");
    k_csc_pos<<<grid_for(nnz_cap), BLK, 0, as_stream(stream)>>>(csc_eid, nnz, csr_cpos);
    TAGAN_CHECK_LAUNCH("csr_csc_pos");
    return TAGAN_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------- chunked work lists
namespace tagan {
namespace {

// Per segment: {chunks, is_multi, partial slots}; ONE exclusive scan over the triple gives each
// segment's first chunk, its index among multi segments and its first partial slot.
struct Tri {
    int32_t a, b, c;
};
struct TriPlus {
    __host__ __device__ Tri operator()(const Tri& x, const Tri& y) const { return Tri{x.a + y.a, x.b + y.b, x.c + y.c}; }
};

__device__ __forceinline__ Tri shfl_up(const Tri& x, int o) {
    return Tri{__shfl_up(x.a, o, WAVE), __shfl_up(x.b, o, WAVE), __shfl_up(x.c, o, WAVE)};
}

__global__ void __launch_bounds__(BLK) k_chunk_count(const int32_t* __restrict__ ptr, int64_t n, int chunk,
                                                     Tri* __restrict__ cnt) {
    for (int64_t s = blockIdx.x * (int64_t)BLK + threadIdx.x; s < n; s += (int64_t)gridDim.x * BLK) {
        const int deg = ptr[s + 1] - ptr[s];
        const int c = deg <= chunk ? 1 : (deg + chunk - 1) / chunk;
        cnt[s] = Tri{c, c > 1 ? 1 : 0, c > 1 ? c : 0};
    }
}

__global__ void __launch_bounds__(BLK) k_chunk_fill(const int32_t* __restrict__ ptr, int64_t n, int chunk,
                                                    const Tri* __restrict__ cnt, const Tri* __restrict__ off,
                                                    int32_t* __restrict__ chunk_ptr, int32_t* __restrict__ seg,
                                                    int32_t* __restrict__ beg, int32_t* __restrict__ part,
                                                    int32_t* __restrict__ multi, int32_t* __restrict__ counts) {
    for (int64_t s = blockIdx.x * (int64_t)BLK + threadIdx.x; s < n; s += (int64_t)gridDim.x * BLK) {
        const int c = cnt[s].a, e0 = ptr[s];
        const Tri o = off[s];
        chunk_ptr[s] = o.a;
        for (int k = 0; k < c; ++k) {
            seg[o.a + k] = (int32_t)s;
            beg[o.a + k] = e0 + k * chunk;
            part[o.a + k] = c > 1 ? o.c + k : -1;
        }
        if (c > 1) multi[o.b] = (int32_t)s;
        if (s == n - 1) {
            chunk_ptr[n] = o.a + c;
            counts[0] = o.a + c;
            counts[1] = o.b + (c > 1);
            counts[2] = o.c + (c > 1 ? c : 0);
        }
    }
}

// One workgroup per window of 2^wbits consecutive segments (a contiguous chunk range): counting
// sort of the window's chunks by entry count, longest first, in LDS.  Positions inside a count
// bucket come from LDS atomics, so ties may run in any order; no result depends on the order.
constexpr int ORDER_BINS = 256;

__global__ void __launch_bounds__(BLK) k_chunk_order_window(const int32_t* __restrict__ ptr, int64_t n,
                                                            const int32_t* __restrict__ chunk_ptr,
                                                            const int32_t* __restrict__ seg,
                                                            const int32_t* __restrict__ beg, int chunk, int wbits,
                                                            int32_t* __restrict__ order) {
    __shared__ int hist[ORDER_BINS];
    __shared__ int base[ORDER_BINS];
    const int64_t s0 = (int64_t)blockIdx.x << wbits;
    const int64_t s1 = min(n, s0 + ((int64_t)1 << wbits));
    const int c0 = chunk_ptr[s0], c1 = chunk_ptr[s1];
    for (int i = threadIdx.x; i < ORDER_BINS; i += BLK) hist[i] = 0;
    __syncthreads();
    for (int c = c0 + threadIdx.x; c < c1; c += BLK) {
        const int cnt = min(chunk, ptr[seg[c] + 1] - beg[c]);
        atomicAdd(&hist[ORDER_BINS - 1 - cnt], 1);
    }
    __syncthreads();
    if (threadIdx.x < WAVE) {      // exclusive scan of the bins by one wave, 4 bins per lane
        const int l = threadIdx.x;
        int v[4], t = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) { v[k] = hist[4 * l + k]; t += v[k]; }
        int incl = t;
#pragma unroll
        for (int o = 1; o < WAVE; o <<= 1) {
            const int y = __shfl_up(incl, o, WAVE);
            if (l >= o) incl += y;
        }
        int run = incl - t;
#pragma unroll
        for (int k = 0; k < 4; ++k) { base[4 * l + k] = run; run += v[k]; }
    }
    __syncthreads();
    for (int c = c0 + threadIdx.x; c < c1; c += BLK) {
        const int cnt = min(chunk, ptr[seg[c] + 1] - beg[c]);
        order[c0 + atomicAdd(&base[ORDER_BINS - 1 - cnt], 1)] = c;
    }
}

}  // namespace
}  // namespace tagan

extern "C" {

int tagan_chunk_order(const int32_t* seg_ptr, int64_t n_segments, const int32_t* chunk_ptr,
                      const int32_t* chunk_seg, const int32_t* chunk_beg, int32_t chunk, int32_t window_bits,
                      int32_t* order, void* stream) {
    using namespace tagan;
    TAGAN_REQUIRE(n_segments > 0 && chunk > 0 && chunk < ORDER_BINS && window_bits >= 0 && window_bits < 31,
                  TAGAN_ERR_ARG, "tagan_chunk_order: n=%lld chunk=%d window_bits=%d", (long long)n_segments,
                  chunk, window_bits);
    TAGAN_REQUIRE(seg_ptr && chunk_ptr && chunk_seg && chunk_beg && order, TAGAN_ERR_ARG,
                  "tagan_chunk_order: null pointer");
    const int64_t windows = ((n_segments - 1) >> window_bits) + 1;
    TAGAN_REQUIRE(windows <= 0x7fffffff, TAGAN_ERR_ARG, "tagan_chunk_order: too many windows");
    hipStream_t s = as_stream(stream);
    k_chunk_order_window<<<(unsigned)windows, BLK, 0, s>>>(seg_ptr, n_segments, chunk_ptr, chunk_seg, chunk_beg,
                                                           chunk, window_bits, order);
    TAGAN_CHECK_LAUNCH("chunk_order");
    return TAGAN_OK;
}

int64_t tagan_chunk_capacity(int64_t n_segments, int64_t nnz_cap, int32_t chunk) {
    return chunk > 0 ? n_segments + nnz_cap / chunk + 1 : 0;
}

int64_t tagan_part_capacity(int64_t nnz_cap, int32_t chunk) {
    return chunk > 0 ? 2 * (nnz_cap / chunk) + 2 : 0;   // a multi segment with deg > chunk has <= 2*deg/chunk chunks
}

size_t tagan_graph_chunks_workspace(int64_t n) {
    using namespace tagan;
    if (n <= 0) return 0;
    return 2 * align_up((size_t)n * sizeof(Tri), 256) + align_up((size_t)scan::parts_len(n) * sizeof(Tri), 256);
}

int tagan_graph_chunks(const int32_t* seg_ptr, int64_t n, int32_t chunk, int32_t* chunk_ptr, int32_t* chunk_seg,
                       int32_t* chunk_beg, int32_t* chunk_part, int32_t* multi_seg, int32_t* counts,
                       void* workspace, size_t workspace_bytes, void* stream) {
    using namespace tagan;
    TAGAN_REQUIRE(n > 0 && chunk > 0, TAGAN_ERR_ARG, "tagan_graph_chunks: n=%lld chunk=%d", (long long)n, chunk);
    TAGAN_REQUIRE(seg_ptr && chunk_ptr && chunk_seg && chunk_beg && chunk_part && multi_seg && counts,
                  TAGAN_ERR_ARG, "tagan_graph_chunks: null pointer");
    const size_t need = tagan_graph_chunks_workspace(n);
    TAGAN_REQUIRE(workspace && workspace_bytes >= need, TAGAN_ERR_WORKSPACE, "tagan_graph_chunks: workspace");
    hipStream_t s = as_stream(stream);
    char* ws = (char*)workspace;
    const size_t a = align_up((size_t)n * sizeof(Tri), 256);
    Tri* cnt = (Tri*)ws;
    Tri* off = (Tri*)(ws + a);
    Tri* part = (Tri*)(ws + 2 * a);
    k_chunk_count<<<grid_for(n), BLK, 0, s>>>(seg_ptr, n, chunk, cnt);
    TAGAN_CHECK_LAUNCH("graph_chunks.count");
    scan::exclusive(cnt, off, n, Tri{0, 0, 0}, TriPlus(), part, false, s);
    TAGAN_CHECK_LAUNCH("graph_chunks.scan");
    k_chunk_fill<<<grid_for(n), BLK, 0, s>>>(seg_ptr, n, chunk, cnt, off, chunk_ptr, chunk_seg, chunk_beg,
                                             chunk_part, multi_seg, counts);
    TAGAN_CHECK_LAUNCH("graph_chunks.fill");
    return TAGAN_OK;
}

}  // extern "C"
