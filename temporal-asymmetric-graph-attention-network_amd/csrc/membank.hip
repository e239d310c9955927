// Device-resident NodeMemoryBank (replaces src/tagan/utils/memory_bank.py:14-360,
// a Python dict of per-node CPU tensors updated one node at a time).
//
// Layout in HBM: a dense slot table states[cap, H] + per-slot int arrays, an
// open-addressing hash (node id -> slot, splitmix64 probe start, linear probing,
// tombstones on prune) and a second never-pruned hash for the frequency counts.
// One update(ids, states, t) is a fixed sequence of kernels, each O(n) or O(cap):
//   age      inactivity += 1 for every stored slot                 (:88-90)
//   insert   claim hash keys by CAS (phase 1), allocate slots for the
//            new keys from the free list / bump pointer (phase 2), resolve (3)
//   fold     per unique slot, the reference's sequential per-occurrence update
//            (reappearance blend max(0.4, decay^min(dt,3)), NaN repair,
//            duplicates in one call) collapsed to its closed form     (:93-141)
//   decay    state *= decay^inactivity for stored slots not in this call (:148-153)
//   prune    inactivity > max_inactivity -> slot freed, key tombstoned (:155-166)
// Float rounding follows torch's CPU semantics for `python_float * tensor`
// (scalar rounded to fp32, one rounding per op, no FMA contraction), so states
// are bit-identical to the reference on NaN-free inputs.
#include "common.cuh"

namespace tagan {
namespace {

constexpr int BLK = 256;
constexpr int64_t KEY_EMPTY = INT64_MIN;
constexpr int64_t KEY_TOMB = INT64_MIN + 1;
constexpr int64_t UNSET = INT64_MIN;

__device__ __forceinline__ uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int grid_for(int64_t n) {
    int64_t g = (n + BLK - 1) / BLK;
    return (int)std::max<int64_t>(1, std::min<int64_t>(g, 4096));
}

#define GRID_LOOP(i, n) for (int64_t i = blockIdx.x * (int64_t)BLK + threadIdx.x; i < (n); i += (int64_t)gridDim.x * BLK)

// ---------------------------------------------------------------- hash primitives
// Find `id`; if `claim`, CAS an EMPTY bucket to `id`.  Returns bucket or -1 (absent / table full).
// *claimed = true iff this thread installed the key.
__device__ int64_t probe(unsigned long long* keys, int64_t tcap, int64_t id, bool claim, bool* claimed) {
    *claimed = false;
    int64_t h = (int64_t)(mix((uint64_t)id) & (uint64_t)(tcap - 1));
    for (int64_t step = 0; step < tcap; ++step) {
        const int64_t k = (int64_t)__hip_atomic_load(keys + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k == id) return h;
        if (k == KEY_EMPTY) {
            if (!claim) return -1;
            const unsigned long long prev = atomicCAS(keys + h, (unsigned long long)KEY_EMPTY, (unsigned long long)id);
            if ((int64_t)prev == KEY_EMPTY) {
                *claimed = true;
                return h;
            }
            if ((int64_t)prev == id) return h;
            // lost the race to another key: keep probing
        }
        h = (h + 1) & (tcap - 1);
    }
    return -1;
}

__global__ void __launch_bounds__(BLK) k_claim(tagan_membank B, const int64_t* __restrict__ ids, int64_t n, int claim,
                                               int32_t* __restrict__ tpos, int32_t* __restrict__ claimed) {
    GRID_LOOP(i, n) {
        bool c;
        const int64_t h = probe((unsigned long long*)B.tkeys, B.tcap, ids[i], claim != 0, &c);
        tpos[i] = (int32_t)h;
        claimed[i] = c ? 1 : 0;
        if (h < 0 && claim) atomicOr((int*)&B.ctl[5], 1);       // table full: host grows and retries
    }
}

// Allocate a slot for every newly claimed key and initialise it (zero state, counter 0).
__global__ void __launch_bounds__(BLK) k_alloc(tagan_membank B, const int64_t* __restrict__ ids, int64_t n,
                                               const int32_t* __restrict__ tpos, const int32_t* __restrict__ claimed,
                                               int32_t epoch) {
    GRID_LOOP(i, n) {
        if (!claimed[i]) continue;
        int32_t slot;
        const int64_t ft = atomicAdd((unsigned long long*)&B.ctl[1], (unsigned long long)-1ll);  // free_top--
        if (ft > 0) {
            slot = B.free_list[ft - 1];
        } else {
            atomicAdd((unsigned long long*)&B.ctl[1], 1ull);
            slot = (int32_t)atomicAdd((unsigned long long*)&B.ctl[0], 1ull);                      // bump
        }
        B.tvals[tpos[i]] = slot;
        B.slot_id[slot] = ids[i];
        B.slot_tpos[slot] = tpos[i];
        B.inact[slot] = 0;
        B.last_seen[slot] = UNSET;
        B.born[slot] = epoch;
        B.touch[slot] = -1;
        float* st = B.states + (int64_t)slot * B.H;
        for (int c = 0; c < B.H; ++c) st[c] = 0.f;
        atomicAdd((unsigned long long*)&B.ctl[2], 1ull);                                          // stored++
    }
}

__global__ void __launch_bounds__(BLK) k_resolve(tagan_membank B, int64_t n, const int32_t* __restrict__ tpos,
                                                 int32_t* __restrict__ slots) {
    GRID_LOOP(i, n) { slots[i] = tpos[i] >= 0 ? B.tvals[tpos[i]] : -1; }
}

// ---------------------------------------------------------------- update
__global__ void __launch_bounds__(BLK) k_age(tagan_membank B) {
    const int64_t used = B.ctl[0];
    GRID_LOOP(s, used) {
        if (B.slot_id[s] != KEY_EMPTY) B.inact[s] += 1;
    }
}

// Per occurrence: NaN flag of its row (one wave per row), first / last-non-NaN occurrence per slot.
__global__ void __launch_bounds__(BLK) k_occ(tagan_membank B, int64_t n, const int32_t* __restrict__ slots,
                                             const float* __restrict__ st, int64_t ld) {
    const int lane = threadIdx.x & (WAVE - 1);
    const int64_t i = blockIdx.x * (int64_t)(BLK / WAVE) + (threadIdx.x >> 6);
    if (i >= n) return;
    bool nan = false;
    for (int c = lane; c < B.H; c += WAVE) nan |= isnan(st[i * ld + c]);
    nan = __any(nan);
    if (lane == 0) {
        const int s = slots[i];
        atomicMin(&B.first_occ[s], (int32_t)i);
        if (!nan) atomicMax(&B.last_ok[s], (int32_t)i);
        atomicAdd(&B.occ_count[s], 1);
    }
}

__device__ __forceinline__ float mul_rn(float a, float b) { return __fmul_rn(a, b); }
__device__ __forceinline__ float add_rn(float a, float b) { return __fadd_rn(a, b); }

// One wave per first occurrence: closed form of the reference's sequential per-occurrence loop.
__global__ void __launch_bounds__(BLK) k_fold(tagan_membank B, const int64_t* __restrict__ ids, int64_t n,
                                              const int32_t* __restrict__ slots, const float* __restrict__ st,
                                              int64_t ld, int64_t t, double decay, int32_t epoch, uint64_t seed) {
    const int lane = threadIdx.x & (WAVE - 1);
    const int64_t i = blockIdx.x * (int64_t)(BLK / WAVE) + (threadIdx.x >> 6);
    if (i >= n) return;
    const int s = slots[i];
    if (B.first_occ[s] != (int32_t)i) return;
    const int32_t L = B.last_ok[s];
    const bool present = B.born[s] != epoch;
    const int64_t ls = B.last_seen[s];
    const bool reapp = present && ls != UNSET && ls < t - 1;
    float w = 0.f, w1 = 0.f;
    if (reapp) {
        const int64_t dt = t - ls;
        const double wd = fmax(0.4, pow(decay, (double)(dt < 3 ? dt : 3)));
        w = (float)wd;
        w1 = (float)(1.0 - wd);
    }
    float* row = B.states + (int64_t)s * B.H;
    for (int c = lane; c < B.H; c += WAVE) {
        float v;
        if (L > (int32_t)i) {
            v = st[(int64_t)L * ld + c];                                   // a later clean duplicate overwrites
        } else if (L == (int32_t)i) {
            const float cur = st[i * ld + c];
            v = reapp ? add_rn(mul_rn(w, row[c]), mul_rn(w1, cur)) : cur;
        } else if (present) {
            const float p = row[c];                                        // NaN row: recover from memory
            v = reapp ? add_rn(mul_rn(w, p), mul_rn(w1, p)) : p;
        } else {
            v = drop_u(drop_key(seed, (uint64_t)s), (uint32_t)c) * 0.01f;           // NaN on a new node: rand * 0.01
        }
        row[c] = v;
    }
    if (lane == 0) {
        B.inact[s] = 0;
        B.last_seen[s] = t;
        B.touch[s] = epoch;
        bool c;
        const int64_t h = probe((unsigned long long*)B.fkeys, B.fcap, ids[i], true, &c);
        if (h >= 0) atomicAdd((unsigned long long*)&B.fcount[h], (unsigned long long)B.occ_count[s]);
        else atomicOr((int*)&B.ctl[5], 2);
        if (c) atomicAdd((unsigned long long*)&B.ctl[4], 1ull);           // distinct ids ever seen
    }
}

// Decay untouched slots, prune, and reset the per-call scratch of every slot.
__global__ void __launch_bounds__(BLK) k_decay_prune(tagan_membank B, double decay, int32_t max_inact, int32_t epoch) {
    const int64_t used = B.ctl[0];
    GRID_LOOP(s, used) {
        B.first_occ[s] = INT32_MAX;
        B.last_ok[s] = -1;
        B.occ_count[s] = 0;
        if (B.slot_id[s] == KEY_EMPTY) continue;
        if (B.touch[s] != epoch) {
            const float f = (float)pow(decay, (double)B.inact[s]);
            float* row = B.states + s * B.H;
            for (int c = 0; c < B.H; ++c) row[c] = mul_rn(row[c], f);
        }
        if (B.inact[s] > max_inact) {
            B.tkeys[B.slot_tpos[s]] = KEY_TOMB;
            B.slot_id[s] = KEY_EMPTY;
            const int64_t ft = atomicAdd((unsigned long long*)&B.ctl[1], 1ull);
            B.free_list[ft] = (int32_t)s;
            atomicAdd((unsigned long long*)&B.ctl[2], (unsigned long long)-1ll);
            atomicAdd((unsigned long long*)&B.ctl[3], 1ull);               // tombstones
        }
    }
}

__global__ void __launch_bounds__(BLK) k_gather(tagan_membank B, const int32_t* __restrict__ slots, int64_t n,
                                                float* __restrict__ out) {
    GRID_LOOP(x, n * B.H) {
        const int64_t i = x / B.H;
        const int c = (int)(x - i * B.H);
        const int s = slots[i];
        if (TAGAN_DBAD(s < B.cap, s, B.cap)) continue;   // slot table index
        out[x] = s >= 0 ? B.states[(int64_t)s * B.H + c] : 0.f;
    }
}

__global__ void __launch_bounds__(BLK) k_scale_all(tagan_membank B, float f) {
    const int64_t used = B.ctl[0];
    GRID_LOOP(x, used * B.H) {
        if (B.slot_id[x / B.H] != KEY_EMPTY) B.states[x] = mul_rn(B.states[x], f);
    }
}

// Rebuild: copy every stored slot of `src` into `dst` (fresh tables, larger capacity), compacting slots.
__global__ void __launch_bounds__(BLK) k_rehash(tagan_membank S, tagan_membank D) {
    const int64_t used = S.ctl[0];
    GRID_LOOP(s, used) {
        const int64_t id = S.slot_id[s];
        if (id == KEY_EMPTY) continue;
        const int32_t d = (int32_t)atomicAdd((unsigned long long*)&D.ctl[0], 1ull);
        bool c;
        const int64_t h = probe((unsigned long long*)D.tkeys, D.tcap, id, true, &c);
        D.tvals[h] = d;
        D.slot_id[d] = id;
        D.slot_tpos[d] = (int32_t)h;
        D.inact[d] = S.inact[s];
        D.last_seen[d] = S.last_seen[s];
        D.born[d] = S.born[s];
        D.touch[d] = S.touch[s];
        D.first_occ[d] = INT32_MAX;
        D.last_ok[d] = -1;
        D.occ_count[d] = 0;
        for (int c2 = 0; c2 < S.H; ++c2) D.states[(int64_t)d * S.H + c2] = S.states[s * S.H + c2];
        atomicAdd((unsigned long long*)&D.ctl[2], 1ull);
    }
}

__global__ void __launch_bounds__(BLK) k_copy_freq(tagan_membank S, tagan_membank D) {
    GRID_LOOP(h, S.fcap) {
        const int64_t id = S.fkeys[h];
        if (id == KEY_EMPTY) continue;
        bool c;
        const int64_t d = probe((unsigned long long*)D.fkeys, D.fcap, id, true, &c);
        D.fcount[d] = S.fcount[h];
        atomicAdd((unsigned long long*)&D.ctl[4], 1ull);
    }
}

__global__ void __launch_bounds__(BLK) k_init(tagan_membank B) {
    GRID_LOOP(x, std::max(B.tcap, std::max(B.cap, B.fcap))) {
        if (x < B.tcap) { B.tkeys[x] = KEY_EMPTY; B.tvals[x] = -1; }
        if (x < B.fcap) { B.fkeys[x] = KEY_EMPTY; B.fcount[x] = 0; }
        if (x < B.cap) {
            B.slot_id[x] = KEY_EMPTY;
            B.first_occ[x] = INT32_MAX;
            B.last_ok[x] = -1;
            B.occ_count[x] = 0;
        }
        if (x < 8) B.ctl[x] = 0;
    }
}

int check_bank(const tagan_membank* B) {
    TAGAN_REQUIRE(B && B->cap > 0 && B->H > 0 && B->tcap >= 2 && (B->tcap & (B->tcap - 1)) == 0 && B->fcap >= 2 &&
                      (B->fcap & (B->fcap - 1)) == 0,
                  TAGAN_ERR_ARG, "membank: bad capacities");
    TAGAN_REQUIRE(B->tkeys && B->tvals && B->slot_id && B->slot_tpos && B->states && B->inact && B->last_seen &&
                      B->born && B->touch && B->first_occ && B->last_ok && B->occ_count && B->free_list && B->fkeys &&
                      B->fcount && B->ctl,
                  TAGAN_ERR_ARG, "membank: null array");
    return TAGAN_OK;
}

}  // namespace
}  // namespace tagan

extern "C" {

int tagan_membank_init(const tagan_membank* B, void* stream) {
    using namespace tagan;
    int rc = check_bank(B);
    if (rc) return rc;
    k_init<<<grid_for(std::max(B->tcap, std::max(B->cap, B->fcap))), BLK, 0, as_stream(stream)>>>(*B);
    TAGAN_CHECK_LAUNCH("membank_init");
    return TAGAN_OK;
}

int tagan_membank_lookup(const tagan_membank* B, const int64_t* ids, int64_t n, int insert, int32_t epoch,
                         int32_t* slots, int32_t* scratch, void* stream) {
    using namespace tagan;
    int rc = check_bank(B);
    if (rc) return rc;
    if (n == 0) return TAGAN_OK;
    TAGAN_REQUIRE(ids && slots && scratch, TAGAN_ERR_ARG, "membank_lookup: null pointer");
    hipStream_t s = as_stream(stream);
    int32_t* tpos = scratch;
    int32_t* claimed = scratch + n;
    k_claim<<<grid_for(n), BLK, 0, s>>>(*B, ids, n, insert, tpos, claimed);
    TAGAN_CHECK_LAUNCH("membank_claim");
    if (insert) {
        k_alloc<<<grid_for(n), BLK, 0, s>>>(*B, ids, n, tpos, claimed, epoch);
        TAGAN_CHECK_LAUNCH("membank_alloc");
    }
    k_resolve<<<grid_for(n), BLK, 0, s>>>(*B, n, tpos, slots);
    TAGAN_CHECK_LAUNCH("membank_resolve");
    return TAGAN_OK;
}

int tagan_membank_update(const tagan_membank* B, const int64_t* ids, int64_t n, const float* states, int64_t ld,
                         int64_t timestep, double decay, int32_t max_inactivity, int32_t epoch, uint64_t seed,
                         int32_t* slots, int32_t* scratch, void* stream) {
    using namespace tagan;
    int rc = check_bank(B);
    if (rc) return rc;
    TAGAN_REQUIRE(n == 0 || (ids && states && slots && scratch && ld >= B->H), TAGAN_ERR_ARG,
                  "membank_update: bad arguments");
    hipStream_t s = as_stream(stream);
    k_age<<<grid_for(B->cap), BLK, 0, s>>>(*B);
    TAGAN_CHECK_LAUNCH("membank_age");
    if (n > 0) {
        rc = tagan_membank_lookup(B, ids, n, 1, epoch, slots, scratch, stream);
        if (rc) return rc;
        const unsigned gw = (unsigned)((n + (BLK / WAVE) - 1) / (BLK / WAVE));
        k_occ<<<gw, BLK, 0, s>>>(*B, n, slots, states, ld);
        TAGAN_CHECK_LAUNCH("membank_occ");
        k_fold<<<gw, BLK, 0, s>>>(*B, ids, n, slots, states, ld, timestep, decay, epoch, seed);
        TAGAN_CHECK_LAUNCH("membank_fold");
    }
    k_decay_prune<<<grid_for(B->cap), BLK, 0, s>>>(*B, decay, max_inactivity, epoch);
    TAGAN_CHECK_LAUNCH("membank_decay_prune");
    return TAGAN_OK;
}

int tagan_membank_gather(const tagan_membank* B, const int32_t* slots, int64_t n, float* out, void* stream) {
    using namespace tagan;
    int rc = check_bank(B);
    if (rc) return rc;
    if (n == 0) return TAGAN_OK;
    TAGAN_REQUIRE(slots && out, TAGAN_ERR_ARG, "membank_gather: null pointer");
    k_gather<<<grid_for(n * B->H), BLK, 0, as_stream(stream)>>>(*B, slots, n, out);
    TAGAN_CHECK_LAUNCH("membank_gather");
    return TAGAN_OK;
}

int tagan_membank_scale(const tagan_membank* B, float factor, void* stream) {
    using namespace tagan;
    int rc = check_bank(B);
    if (rc) return rc;
    k_scale_all<<<grid_for(B->cap * B->H), BLK, 0, as_stream(stream)>>>(*B, factor);
    TAGAN_CHECK_LAUNCH("membank_scale");
    return TAGAN_OK;
}

int tagan_membank_rehash(const tagan_membank* src, const tagan_membank* dst, void* stream) {
    using namespace tagan;
    int rc = check_bank(src);
    if (rc) return rc;
    rc = check_bank(dst);
    if (rc) return rc;
    TAGAN_REQUIRE(src->H == dst->H && dst->cap >= src->cap, TAGAN_ERR_ARG, "membank_rehash: shapes");
    hipStream_t s = as_stream(stream);
    k_init<<<grid_for(std::max(dst->tcap, std::max(dst->cap, dst->fcap))), BLK, 0, s>>>(*dst);
    TAGAN_CHECK_LAUNCH("membank_rehash_init");
    k_rehash<<<grid_for(src->cap), BLK, 0, s>>>(*src, *dst);
    TAGAN_CHECK_LAUNCH("membank_rehash");
    k_copy_freq<<<grid_for(src->fcap), BLK, 0, s>>>(*src, *dst);
    TAGAN_CHECK_LAUNCH("membank_copy_freq");
    return TAGAN_OK;
}

}  // extern "C"
