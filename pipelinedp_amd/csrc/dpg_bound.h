// dpg_bound.h -- contribution bounding of privacy-id buckets (gfx950):
// parameters, LDS/global hash-table helpers, and the global-memory path for
// single buckets larger than the LDS chunk capacity (k_bound_big).
//
// Algorithm (same in k_bound_chunks, dpg_chunk.h, and here):
//   A  insert every record's pid (hash residual) and (pid slot, pk) pair into
//      hash tables; count records per pair, pairs (or records) per pid
//   B  every pid over its limit gets k cascade slots
//   C  mpc selection: per pid keep the mpc pairs with the smallest
//      philox(seed, pid, pk) key            (contribution_bounders.py:90-92)
//   D  pair state (dropped / kept / sampled) + mcpp cascade slots
//   E  mcpp selection: per kept pair keep the mcpp records with the smallest
//      philox(seed, pid, pk, global record id) key (:74-76); or, in
//      PER_PRIVACY_ID mode, the L records per pid (:123-124)
//   F  clipped per-pair accumulators of kept records, values gathered by
//      record index                         (combiners.py:255-500)
//   G  emit one Item per kept pair (pk, count, sum[, nsum, nsq])
// "k smallest" uses an atomicMin cascade over k slots per group; keys are
// distinct, so exactly k survive.
#pragma once

#include "dpg_common.h"

namespace dpg {

constexpr uint32_t kEmpty32 = 0xFFFFFFFFu;
constexpr uint64_t kEmpty64 = ~0ull;
constexpr uint32_t kNil = 0xFFFFFFFFu;
constexpr uint32_t kDropped = 0xFFFFFFFFu;
constexpr uint32_t kKeptAll = 0xFFFFFFFEu;

struct BoundParams {
    int mode;
    int sum_mode;
    uint32_t mask;
    uint32_t need_values;  // any value-dependent accumulator
    uint32_t mpc, mcpp, L;
    double lo, hi, lo_pp, hi_pp, mid;
    uint64_t seed;
    Fmt fmt;
    HashK hash;
    int64_t pid_min;
    int64_t rec_base;      // global id of input record 0
    const double *value;   // caller's value column (gathered by index)
    uint32_t *err;         // bit 1: internal table error
    uint32_t *progress;    // debug watchdog: last phase per workgroup (or null)
    unsigned long long *phase_cyc;  // debug: shader cycles per phase (or null)
    uint32_t *heavy_fb;    // heavy buckets handed back to k_bound_big (indices)
    uint32_t *heavy_nfb;   // their number
    float cand_mul;        // sort kernel: candidate records aimed at per filtered pid
    float defer_est;       // sort kernel, narrow / streamed passes: a chunk whose
                           // expected candidates exceed this is deferred before
                           // its pair priorities are drawn (0: off)
};

// privacy id of a bucket's pid-hash residual
__device__ __forceinline__ uint64_t pid_of(const BoundParams &bp, uint32_t d1, uint32_t hres) {
    const uint32_t hshift = bp.fmt.kbits - bp.fmt.b1;  // <= 31 (b1 >= 1)
    const uint32_t h = (d1 << hshift) | hres;
    return (uint64_t)(bp.pid_min + (int64_t)hk_inv(h, bp.hash));
}

// Debug hooks at phase boundaries: watchdog progress, and, in the timing
// build only (-DDPG_PHASE_TIMING: pipelinedp_amd/lib/libdpg_timing.so, loaded
// when the env var DPG_PHASE_TIMING is set), the shader cycles thread 0 spent
// since the previous mark, accumulated in registers and flushed once per
// workgroup.  The product build carries no timer state at all.
#ifdef DPG_PHASE_TIMING
struct PhaseTimer {
    uint64_t last;
    uint64_t pt[12];
};
#else
struct PhaseTimer {};
#endif
// The watchdog store is compiled into the debug builds only (-DDPG_WATCHDOG
// or the timing build): in the product kernels its pointer and branch cost
// scalar registers the bounding kernel spills.
__device__ __forceinline__ void mark(const BoundParams &bp, uint32_t phase, PhaseTimer &tm) {
#if defined(DPG_WATCHDOG) || defined(DPG_PHASE_TIMING)
    if (bp.progress && threadIdx.x == 0)
        __hip_atomic_store(&bp.progress[blockIdx.x], phase, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
#endif
#ifdef DPG_PHASE_TIMING
    if (bp.phase_cyc) {
        const uint64_t now = __builtin_amdgcn_s_memtime();
        tm.pt[phase] += now - tm.last;
        tm.last = now;
    }
#else
    (void)phase;
    (void)tm;
#endif
}
__device__ __forceinline__ void timer_start(const BoundParams &bp, PhaseTimer &tm) {
#ifdef DPG_PHASE_TIMING
    tm.last = bp.phase_cyc ? __builtin_amdgcn_s_memtime() : 0;
    for (int k = 0; k < 12; ++k) tm.pt[k] = 0;
#else
    (void)bp;
    (void)tm;
#endif
}
__device__ __forceinline__ void timer_flush(const BoundParams &bp, const PhaseTimer &tm) {
#ifdef DPG_PHASE_TIMING
    if (bp.phase_cyc && threadIdx.x == 0)
        for (int k = 0; k < 12; ++k) atomicAdd(&bp.phase_cyc[k], (unsigned long long)tm.pt[k]);
#else
    (void)bp;
    (void)tm;
#endif
}

__host__ __device__ __forceinline__ uint32_t next_pow2(uint32_t x) {
    uint32_t p = 64;
    while (p < x) p <<= 1;
    return p;
}

__host__ __device__ __forceinline__ size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

template <class Item>
struct ItemTraits;
// sum: the item carries the clipped sum (MEAN / VARIANCE without SUM need
// only the normalised moments: 24-byte items and one accumulator less)
template <>
struct ItemTraits<Item16> {
    static constexpr bool var = false;
    static constexpr bool preagg = false;
    static constexpr bool sum = true;
};
template <>
struct ItemTraits<Item32> {
    static constexpr bool var = true;
    static constexpr bool preagg = false;
    static constexpr bool sum = true;
};
template <>
struct ItemTraits<ItemV> {
    static constexpr bool var = true;
    static constexpr bool preagg = false;
    static constexpr bool sum = false;
};
// utility-analysis pre-aggregate: every pair kept (the host passes no-op
// bounds), each pair also carries its privacy id's partition and record
// counts (analysis/contribution_bounders.py:37-77)
template <>
struct ItemTraits<ItemPA> {
    static constexpr bool var = false;
    static constexpr bool preagg = true;
    static constexpr bool sum = true;
};

__device__ __forceinline__ uint32_t hslot(uint32_t key, uint32_t mask) {
    return fmix32(key * 0x9E3779B1u + 0x632BE5ABu) & mask;
}
__device__ __forceinline__ uint32_t hslot(uint64_t key, uint32_t mask) {
    return fmix32((uint32_t)key ^ fmix32((uint32_t)(key >> 32) + 0x7F4A7C15u)) & mask;
}

template <class K>
__device__ __forceinline__ K empty_key() {
    return (K)~(K)0;
}

// Insert `key` (linear probing); `won` = this lane created the entry.  Probe
// loops are bounded by the table size: a miss after a full sweep can only be
// a bug, which is reported through *err instead of spinning.
template <class K>
__device__ __forceinline__ uint32_t insert_key(K *keys, uint32_t mask, K key, bool &won,
                                               uint32_t *err) {
    uint32_t h = hslot(key, mask);
    for (uint32_t probe = 0; probe <= mask; ++probe) {
        // a slot goes empty -> key once: a key seen by a plain load is final,
        // so the records of a heavy privacy id (thousands on one slot) hit
        // without serialising on its L2 line; an empty or stale view CASes
        const K seen = __hip_atomic_load(&keys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (seen == key) {
            won = false;
            return h;
        }
        if (seen != empty_key<K>()) {
            h = (h + 1) & mask;
            continue;
        }
        K old;
        if constexpr (sizeof(K) == 8)
            old = (K)atomicCAS((unsigned long long *)&keys[h], (unsigned long long)empty_key<K>(),
                               (unsigned long long)key);
        else
            old = atomicCAS(&keys[h], empty_key<K>(), key);
        if (old == empty_key<K>()) {
            won = true;
            return h;
        }
        if (old == key) {
            won = false;
            return h;
        }
        h = (h + 1) & mask;
    }
    atomicOr(err, 2u);
    won = false;
    return 0;
}

// keep-the-k-smallest-distinct cascade (slot values only decrease)
__device__ __forceinline__ void cascade_insert(uint64_t *slots, uint32_t k, uint64_t x) {
    // slot values only decrease: a key above the current k-th smallest can
    // never enter (most records of a heavy pair stop at this load)
    if (x > __hip_atomic_load(&slots[k - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
        return;
    for (uint32_t j = 0; j < k; ++j) {
        uint64_t old = atomicMin((unsigned long long *)&slots[j], (unsigned long long)x);
        if (old == x) return;
        if (old > x) {
            if (old == kEmpty64) return;
            x = old;
        }
    }
}

// Per-pid candidate threshold of the mpc selection: a pid with m > k pairs
// cascades only the pairs whose 32-bit priority is below ~e / m of the range,
// e = k + 3 sqrt(k) + 3 (about 3 sigma above the k-th order statistic); the
// k smallest keys are among them whenever at least k fall below (any key
// above the threshold exceeds every candidate's), and the completion pass
// handles the rest (candidate count < k).  The threshold only steers work:
// the kept set does not depend on it.
// Candidate bound for an expected e candidates among m pairs.
__device__ __forceinline__ uint32_t cand_threshold_e(uint32_t m, float e) {
    if (e >= (float)m) return 0xFFFFFFFFu;
    return (uint32_t)(e / (float)m * 4294967040.0f);
}
// the same, for m pairs whose priorities are known to lie in [0, B]
__device__ __forceinline__ uint32_t cand_threshold_be(uint32_t m, float e, uint32_t B) {
    if (e >= (float)m) return 0xFFFFFFFFu;
    return (uint32_t)((float)B * (e / (float)m));
}
__device__ __forceinline__ uint32_t cand_threshold(uint32_t m, uint32_t k) {
    const float e = (float)k + 3.0f * sqrtf((float)k) + 3.0f;
    if (e >= (float)m) return 0xFFFFFFFFu;
    return (uint32_t)(e / (float)m * 4294967040.0f);
}

// Wave-aggregated counter allocation; call with the whole wave converged.
// Returns this lane's slot (meaningful where `want`).
template <class T>
__device__ __forceinline__ uint32_t wave_alloc(T *ctr, bool want, uint32_t per = 1) {
    const uint64_t b = __ballot(want);
    const int lane = __lane_id();
    uint32_t base = 0;
    if (b) {
        const int leader = __ffsll((long long)b) - 1;
        if (lane == leader) base = atomicAdd(ctr, (uint32_t)__popcll(b) * per);
        base = __builtin_amdgcn_readlane(base, leader);
    }
    return base + (uint32_t)__popcll(b & ((1ull << lane) - 1ull)) * per;
}

// ------------------------------------------------------------ global path
// Buckets beyond the LDS chunk capacity (a privacy id with thousands of
// records): one 1024-thread workgroup per bucket, working set in global
// memory.  The tables are written by L2 atomics and plain stores and re-read
// by plain loads of the same workgroup, i.e. of one CU, whose XCD L2 is the
// coherence point: every wave drains its memory operations before the
// barrier and drops this CU's possibly stale L1 lines after it (buffer_inv
// sc0, ~100 cycles).  An agent-scope release here would write back the whole
// XCD L2 at every phase of every bucket (buffer_wbl2 sc1): config 4's 1e5
// heavy privacy ids spent 458 ms in this kernel that way.
constexpr int kBigThreads = 1024;

__device__ __forceinline__ void big_sync() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    asm volatile("buffer_inv sc0" ::: "memory");
}

struct BigLayout {
    uint32_t Cq, Cp;
    size_t pidtab, pidm, pidc, pidslot, pairtab, paircnt, pairst, acc, pool, qs, ps, rkey, total;
    __host__ __device__ static BigLayout make(uint32_t n, bool var) {
        BigLayout L;
        L.Cq = next_pow2(n < 32 ? 32 : n);
        L.Cp = next_pow2(2 * (n < 32 ? 32 : n));
        size_t o = 0;
        L.pidtab = o;  o += align16((size_t)L.Cq * 4);
        L.pidm = o;    o += align16((size_t)L.Cq * 4);
        L.pidc = o;    o += align16((size_t)L.Cq * 4);
        L.pidslot = o; o += align16((size_t)L.Cq * 4);
        L.pairtab = o; o += align16((size_t)L.Cp * 8);
        L.paircnt = o; o += align16((size_t)L.Cp * 4);
        L.pairst = o;  o += align16((size_t)L.Cp * 4);
        L.acc = o;     o += align16((size_t)L.Cp * 8 * (var ? 3 : 1));
        L.pool = o;    o += align16((size_t)(2 * n + 2) * 8);
        L.qs = o;      o += align16((size_t)n * 4);
        L.ps = o;      o += align16((size_t)n * 4);
        L.rkey = o;    o += align16((size_t)n * 8);
        L.total = o;
        return L;
    }
};

template <class Item, class R>
__global__ __launch_bounds__(kBigThreads) void k_bound_big(
    const R *recs, const int64_t *bstart, const uint32_t *bcnt, const uint32_t *bd1,
    const size_t *scratch_off, char *scratch, BoundParams bp, Item *items, const int64_t *item_off,
    uint32_t *item_cursor) {
    constexpr bool kVar = ItemTraits<Item>::var;
    constexpr bool kPA = ItemTraits<Item>::preagg;
    __shared__ uint32_t sh_bump, sh_bump2;
    const uint32_t b = blockIdx.x;
    const int tid = threadIdx.x;
    const uint32_t n = __builtin_amdgcn_readfirstlane(bcnt[b]);
    const uint32_t d1 = __builtin_amdgcn_readfirstlane(bd1[b]);
    const R *rb = recs + bstart[b];
    char *base = scratch + scratch_off[b];
    const BigLayout Lb = BigLayout::make(n, kVar);
    const uint32_t Cq = __builtin_amdgcn_readfirstlane(Lb.Cq);
    const uint32_t Cp = __builtin_amdgcn_readfirstlane(Lb.Cp);
    uint32_t *pidtab = reinterpret_cast<uint32_t *>(base + Lb.pidtab);
    uint32_t *pidm = reinterpret_cast<uint32_t *>(base + Lb.pidm);
    uint32_t *pidc = reinterpret_cast<uint32_t *>(base + Lb.pidc);
    uint32_t *pidslot = reinterpret_cast<uint32_t *>(base + Lb.pidslot);
    uint64_t *pairtab = reinterpret_cast<uint64_t *>(base + Lb.pairtab);
    uint32_t *paircnt = reinterpret_cast<uint32_t *>(base + Lb.paircnt);
    uint32_t *pairst = reinterpret_cast<uint32_t *>(base + Lb.pairst);
    double *acc_sum = reinterpret_cast<double *>(base + Lb.acc);
    double *acc_nsum = acc_sum + Cp;
    double *acc_nsq = acc_nsum + Cp;
    uint64_t *pool = reinterpret_cast<uint64_t *>(base + Lb.pool);
    uint32_t *rqs = reinterpret_cast<uint32_t *>(base + Lb.qs);
    uint32_t *rps = reinterpret_cast<uint32_t *>(base + Lb.ps);
    uint64_t *rkey = reinterpret_cast<uint64_t *>(base + Lb.rkey);
    const Fmt f = bp.fmt;
    const uint32_t pkb = f.pkbits;
    const uint64_t pkmask = (pkb >= 64) ? ~0ull : ((1ull << pkb) - 1ull);
    const bool per_pid = bp.mode == DPG_MODE_PER_PRIVACY_ID;
    const bool need_v = bp.need_values != 0;
    const bool sample = bp.mode == DPG_MODE_CROSS_AND_PER_PARTITION && need_v;
    const bool part_clip = bp.sum_mode == DPG_SUM_CLIP_PARTITION;
    const uint32_t lim = per_pid ? bp.L : bp.mpc;
    PhaseTimer clk;
    timer_start(bp, clk);
    // ---- clear
    for (uint32_t i = tid; i < Cq; i += kBigThreads) {
        pidtab[i] = kEmpty32;
        pidm[i] = 0;
        pidc[i] = 0;
    }
    for (uint32_t i = tid; i < Cp; i += kBigThreads) {
        pairtab[i] = kEmpty64;
        paircnt[i] = 0;
        pairst[i] = 0;
        acc_sum[i] = 0.0;
        if (kVar) {
            acc_nsum[i] = 0.0;
            acc_nsq[i] = 0.0;
        }
    }
    if (tid == 0) {
        sh_bump = 0;
        sh_bump2 = n;
    }
    big_sync();
    mark(bp, 0, clk);
    // ---- A: inserts and counts
    for (uint32_t i = tid; i < n; i += kBigThreads) {
        const uint64_t key = RecOps<R>::key(rb[i], f);
        const uint32_t hres = (uint32_t)(key >> pkb);
        const uint32_t pk = (uint32_t)(key & pkmask);
        bool wq, wp;
        const uint32_t qs = insert_key<uint32_t>(pidtab, Cq - 1, hres, wq, bp.err);
        if (per_pid) atomicAdd(&pidm[qs], 1u);
        const uint32_t ps =
            insert_key<uint64_t>(pairtab, Cp - 1, ((uint64_t)qs << pkb) | pk, wp, bp.err);
        atomicAdd(&paircnt[ps], 1u);
        if (!per_pid && wp) atomicAdd(&pidm[qs], 1u);
        if (kPA) atomicAdd(&pidc[qs], 1u);  // records per pid (no pid is over a limit)
        rqs[i] = qs;
        rps[i] = ps;
    }
    big_sync();
    mark(bp, 1, clk);
    // ---- B: cascade slots for pids over their limit
    for (uint32_t q = tid; q < Cq; q += kBigThreads) {
        const bool occ = pidtab[q] != kEmpty32;
        const bool want = occ && pidm[q] > lim;
        if (want) {
            const uint32_t s = atomicAdd(&sh_bump, lim);
            for (uint32_t j = 0; j < lim; ++j) pool[s + j] = kEmpty64;
            pidslot[q] = s;
        } else if (occ) {
            pidslot[q] = kNil;
        }
    }
    big_sync();
    mark(bp, 2, clk);
    if (!per_pid) {
        // ---- C: mpc selection over pairs (candidates, then completion)
        for (uint32_t pass = 0; pass < 2; ++pass) {
            for (uint32_t p = tid; p < Cp; p += kBigThreads) {
                const uint64_t pkey = pairtab[p];
                if (pkey == kEmpty64) continue;
                const uint32_t q = (uint32_t)(pkey >> pkb);
                const uint32_t s = pidslot[q];
                if (s == kNil) continue;
                const uint32_t pk = (uint32_t)(pkey & pkmask);
                const uint32_t pr = pair_prio(bp.seed, pid_of(bp, d1, pidtab[q]), pk);
                const bool cand = pr < cand_threshold(pidm[q], bp.mpc);
                const uint64_t k64 = ((uint64_t)pr << 32) | pk;
                if (pass == 0 && cand) {
                    cascade_insert(pool + s, bp.mpc, k64);
                    atomicAdd(&pidc[q], 1u);
                } else if (pass == 1 && !cand && pidc[q] < bp.mpc) {
                    cascade_insert(pool + s, bp.mpc, k64);
                }
            }
            big_sync();
        }
        mark(bp, 3, clk);
        // ---- D: pair state + mcpp slots
        for (uint32_t p = tid; p < Cp; p += kBigThreads) {
            const uint64_t pkey = pairtab[p];
            if (pkey == kEmpty64) continue;
            const uint32_t q = (uint32_t)(pkey >> pkb);
            const uint32_t s = pidslot[q];
            bool kept = true;
            if (s != kNil) {
                const uint32_t pk = (uint32_t)(pkey & pkmask);
                const uint32_t pr = pair_prio(bp.seed, pid_of(bp, d1, pidtab[q]), pk);
                kept = (((uint64_t)pr << 32) | pk) <= pool[s + bp.mpc - 1];
            }
            uint32_t st = kept ? kKeptAll : kDropped;
            if (kept && sample && paircnt[p] > bp.mcpp) {
                st = atomicAdd(&sh_bump2, bp.mcpp);
                for (uint32_t j = 0; j < bp.mcpp; ++j) pool[st + j] = kEmpty64;
            }
            pairst[p] = st;
        }
        big_sync();
        mark(bp, 4, clk);
        // ---- E: mcpp cascade over record keys of over-full kept pairs
        if (sample) {
            for (uint32_t i = tid; i < n; i += kBigThreads) {
                const uint32_t st = pairst[rps[i]];
                if (st >= kKeptAll) continue;
                const uint64_t key = RecOps<R>::key(rb[i], f);
                const uint64_t rk = rec_prio(bp.seed, pid_of(bp, d1, pidtab[rqs[i]]),
                                             (uint32_t)(key & pkmask),
                                             (uint64_t)(bp.rec_base + RecOps<R>::idx(rb[i], f)));
                rkey[i] = rk;
                cascade_insert(pool + st, bp.mcpp, rk);
            }
            big_sync();
        }
        mark(bp, 5, clk);
        // ---- F: accumulators of kept records
        if (need_v) {
            for (uint32_t i = tid; i < n; i += kBigThreads) {
                const uint32_t p = rps[i];
                const uint32_t st = pairst[p];
                if (st == kDropped) continue;
                if (st != kKeptAll && rkey[i] > pool[st + bp.mcpp - 1]) continue;
                const double v = rec_value<R>(rb[i], bp.value, f);
                if (part_clip) {
                    atomicAdd(&acc_sum[p], v);
                } else {
                    const double x = clampd(v, bp.lo, bp.hi);
                    atomicAdd(&acc_sum[p], x);
                    if (kVar) {
                        const double y = x - bp.mid;
                        atomicAdd(&acc_nsum[p], y);
                        atomicAdd(&acc_nsq[p], y * y);
                    }
                }
            }
            big_sync();
        }
    } else {
        // ---- PER_PRIVACY_ID: keep the L records of each pid with the
        // smallest record key; pairst counts kept records per pair
        for (uint32_t i = tid; i < n; i += kBigThreads) {
            const uint32_t s = pidslot[rqs[i]];
            if (s == kNil) continue;
            const uint64_t key = RecOps<R>::key(rb[i], f);
            const uint64_t rk = rec_prio(bp.seed, pid_of(bp, d1, pidtab[rqs[i]]),
                                         (uint32_t)(key & pkmask),
                                         (uint64_t)(bp.rec_base + RecOps<R>::idx(rb[i], f)));
            rkey[i] = rk;
            cascade_insert(pool + s, bp.L, rk);
        }
        big_sync();
        for (uint32_t i = tid; i < n; i += kBigThreads) {
            const uint32_t s = pidslot[rqs[i]];
            if (s != kNil && rkey[i] > pool[s + bp.L - 1]) continue;
            const uint32_t p = rps[i];
            atomicAdd(&pairst[p], 1u);
            if (need_v) {
                const double v = rec_value<R>(rb[i], bp.value, f);
                if (part_clip) {
                    atomicAdd(&acc_sum[p], v);
                } else {
                    const double x = clampd(v, bp.lo, bp.hi);
                    atomicAdd(&acc_sum[p], x);
                    if (kVar) {
                        const double y = x - bp.mid;
                        atomicAdd(&acc_nsum[p], y);
                        atomicAdd(&acc_nsq[p], y * y);
                    }
                }
            }
        }
        big_sync();
    }
    mark(bp, 6, clk);
    // ---- G: emit kept pairs
    if constexpr (kPA) {
        // pid leader (leader bit set): the pair with the smallest slot of its
        // privacy id (pidslot is dead here: no pid is over a limit)
        for (uint32_t q = tid; q < Cq; q += kBigThreads) pidslot[q] = kNil;
        big_sync();
        for (uint32_t p = tid; p < Cp; p += kBigThreads) {
            const uint64_t pkey = pairtab[p];
            if (pkey != kEmpty64 && paircnt[p] > 0) atomicMin(&pidslot[(uint32_t)(pkey >> pkb)], p);
        }
        big_sync();
    }
    Item *out = items + *item_off;
    for (uint32_t p = tid; p < Cp; p += kBigThreads) {
        const uint64_t pkey = pairtab[p];
        if (pkey == kEmpty64) continue;
        const uint32_t st = pairst[p];
        uint32_t c;
        if (per_pid) c = st;
        else if (st == kDropped) c = 0;
        else if (bp.mode == DPG_MODE_CROSS_AND_PER_PARTITION) c = min(paircnt[p], bp.mcpp);
        else c = paircnt[p];
        if (c == 0) continue;
        Item it;
        it.pk = (uint32_t)(pkey & pkmask);
        it.cnt = c;
        double s = 0.0;
        if (need_v) {
            s = acc_sum[p];
            if (part_clip) s = clampd(s, bp.lo_pp, bp.hi_pp);
        }
        if constexpr (ItemTraits<Item>::sum) it.sum = s;
        if constexpr (kVar) {
            it.nsum = need_v ? acc_nsum[p] : 0.0;
            it.nsq = need_v ? acc_nsq[p] : 0.0;
        }
        if constexpr (kPA) {
            const uint32_t q = (uint32_t)(pkey >> pkb);
            it.npart = pidm[q];
            it.nl = ItemPA::pack_nl(pidc[q], pidslot[q] == p);
        }
        out[atomicAdd(item_cursor, 1u)] = it;
    }
    mark(bp, 7, clk);
    timer_flush(bp, clk);
}

}  // namespace dpg
