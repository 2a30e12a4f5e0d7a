// dpg_bound.h -- contribution bounding of one privacy-id bucket (gfx950).
//
// A bucket holds every record of a set of privacy ids (the top hash bits of
// fmix32(pid) are the bucket id).  One 1024-thread workgroup processes a
// bucket in a working set given by `base` (global scratch here):
//   A1  insert every record's pid and (pid, pk) into LDS hash tables
//   A2  dense ids for the occupied slots (block compaction)
//   A3  per-pair record counts + record lists, per-pid pair counts
//   C   mpc selection: per pid keep the mpc pairs with the smallest
//       philox(seed, pid, pk) key            (contribution_bounders.py:90-92)
//   D   mcpp selection: per kept pair keep the mcpp records with the
//       smallest philox(seed, pid, pk, value, occ) key (:74-76); or, in
//       PER_PRIVACY_ID mode, the L records per pid (:123-124)
//   E   clipped per-pair accumulators            (combiners.py:255-500)
//   F   emit one Item per kept pair (pk, count, sum[, nsum, nsq])
// This is the global-memory path for single buckets larger than the LDS chunk
// capacity (k_bound_global); the LDS path is process_chunk (dpg_chunk.h),
// which gives identical results.  "k smallest" uses an atomicMin cascade over k
// slots per group; keys are distinct, so exactly k survive.
#pragma once

#include "dpg_common.h"

namespace dpg {

constexpr int kBoundThreads = 1024;
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
    uint32_t *err;       // bit 1: internal table error
    uint32_t *progress;  // debug watchdog: last phase per workgroup (or null)
    unsigned long long *phase_cyc;  // debug: shader cycles per phase (or null)
};

// Debug hooks at phase boundaries: watchdog progress, and (DPG_PHASE_TIMING)
// the shader cycles thread 0 spent since the previous mark, added to the
// register accumulator pt[phase] (slot k = the phase that ends at mark k);
// the kernel flushes pt once at exit, so timing adds no memory traffic to
// the phases it measures.
struct PhaseTimer {
    uint64_t last;
    uint64_t pt[10];
};
__device__ __forceinline__ void mark(const BoundParams &bp, uint32_t phase, PhaseTimer &tm) {
    if (bp.progress && threadIdx.x == 0)
        __hip_atomic_store(&bp.progress[blockIdx.x], phase, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    if (bp.phase_cyc) {
        const uint64_t now = __builtin_amdgcn_s_memtime();
        tm.pt[phase] += now - tm.last;
        tm.last = now;
    }
}
__device__ __forceinline__ void timer_start(const BoundParams &bp, PhaseTimer &tm) {
    tm.last = bp.phase_cyc ? __builtin_amdgcn_s_memtime() : 0;
    for (int k = 0; k < 10; ++k) tm.pt[k] = 0;
}
__device__ __forceinline__ void timer_flush(const BoundParams &bp, const PhaseTimer &tm) {
    if (bp.phase_cyc && threadIdx.x == 0)
        for (int k = 0; k < 10; ++k) atomicAdd(&bp.phase_cyc[k], (unsigned long long)tm.pt[k]);
}

__host__ __device__ __forceinline__ uint32_t next_pow2(uint32_t x) {
    uint32_t p = 64;
    while (p < x) p <<= 1;
    return p;
}

__host__ __device__ __forceinline__ size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

// Byte layout of one bucket's working set for n records.
struct BucketLayout {
    uint32_t C;  // hash-table capacity (power of two)
    size_t t_off, p_off, q_off, r_off, total;
    __host__ __device__ static BucketLayout make(uint32_t n, bool var, int isz) {
        BucketLayout L;
        L.C = next_pow2(2 * (n < 32 ? 32 : n));
        size_t tables = (size_t)L.C * (4 + 8 + 2 * isz);
        size_t phase_d = (size_t)n * 8 * 3;                 // vstage, slots, rkey
        size_t phase_e = (size_t)n * 8 * (var ? 4 : 2);     // vstage + acc
        size_t T = tables;
        if (phase_d > T) T = phase_d;
        if (phase_e > T) T = phase_e;
        L.t_off = 0;
        L.p_off = align16(T);
        L.q_off = L.p_off + align16((size_t)n * 20);
        L.r_off = L.q_off + align16((size_t)n * 16);
        L.total = L.r_off + align16((size_t)n * 2 * isz);
        return L;
    }
};

template <class Item>
struct ItemTraits;
template <>
struct ItemTraits<Item16> {
    static constexpr bool var = false;
};
template <>
struct ItemTraits<Item32> {
    static constexpr bool var = true;
};

__device__ __forceinline__ uint32_t hslot32(uint32_t key, uint32_t mask) {
    return fmix32(key * 0x9E3779B1u + 0x632BE5ABu) & mask;
}
__device__ __forceinline__ uint32_t hslot64(uint64_t key, uint32_t mask) {
    return fmix32((uint32_t)key ^ fmix32((uint32_t)(key >> 32) + 0x7F4A7C15u)) & mask;
}

// Probe loops are bounded by the table size: a miss after a full sweep can
// only be a bug, which is reported through *err instead of spinning.
__device__ __forceinline__ uint32_t insert32(uint32_t *keys, uint32_t mask, uint32_t key,
                                             uint32_t *err) {
    uint32_t h = hslot32(key, mask);
    for (uint32_t probe = 0; probe <= mask; ++probe) {
        uint32_t old = atomicCAS(&keys[h], kEmpty32, key);
        if (old == kEmpty32 || old == key) return h;
        h = (h + 1) & mask;
    }
    atomicOr(err, 2u);
    return 0;
}
__device__ __forceinline__ uint32_t lookup32(const uint32_t *keys, uint32_t mask, uint32_t key,
                                             uint32_t *err) {
    uint32_t h = hslot32(key, mask);
    for (uint32_t probe = 0; probe <= mask; ++probe) {
        if (keys[h] == key) return h;
        h = (h + 1) & mask;
    }
    atomicOr(err, 2u);
    return 0;
}
__device__ __forceinline__ uint32_t insert64(uint64_t *keys, uint32_t mask, uint64_t key,
                                             uint32_t *err) {
    uint32_t h = hslot64(key, mask);
    for (uint32_t probe = 0; probe <= mask; ++probe) {
        uint64_t old = atomicCAS((unsigned long long *)&keys[h], (unsigned long long)kEmpty64,
                                 (unsigned long long)key);
        if (old == kEmpty64 || old == key) return h;
        h = (h + 1) & mask;
    }
    atomicOr(err, 2u);
    return 0;
}

// Workgroup barrier of a bucket pass.  With the working set in global memory
// (oversize buckets) the tables are written by L2 atomics and plain stores
// and re-read by plain loads, so each wave drops this CU's possibly stale L1
// lines after the barrier (agent-scope acquire, MI355X_MICROARCH.md
// "inter-workgroup visibility"); in LDS the plain barrier suffices.
template <bool kGlobal>
__device__ __forceinline__ void bucket_sync() {
    if (kGlobal) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __syncthreads();
    if (kGlobal) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

// keep-the-k-smallest-distinct cascade (slot values only decrease)
__device__ __forceinline__ void cascade_insert(uint64_t *slots, uint32_t k, uint64_t x) {
    for (uint32_t j = 0; j < k; ++j) {
        uint64_t old = atomicMin((unsigned long long *)&slots[j], (unsigned long long)x);
        if (old == x) return;
        if (old > x) {
            if (old == kEmpty64) return;
            x = old;
        }
    }
}

// Block compaction: dense id for every flagged slot in [0, C).  Returns count.
template <bool kGlobal, class Idx>
__device__ __forceinline__ uint32_t block_enumerate(uint32_t C, const uint32_t *keys32,
                                                   const uint64_t *keys64, Idx *s2i,
                                                   uint32_t *sh16, uint32_t *sh_total) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint32_t running = 0;
    for (uint32_t b = 0; b < C; b += kBoundThreads) {
        uint32_t s = b + tid;
        bool occ = false;
        if (s < C) occ = keys32 ? keys32[s] != kEmpty32 : keys64[s] != kEmpty64;
        uint64_t bal = __ballot(occ);
        if (lane == 0) sh16[w] = __popcll(bal);
        bucket_sync<kGlobal>();
        uint32_t pre = 0, tot = 0;
        for (int k = 0; k < 16; ++k) {
            uint32_t y = sh16[k];
            if (k < w) pre += y;
            tot += y;
        }
        if (occ) s2i[s] = (Idx)(running + pre + __popcll(bal & ((1ull << lane) - 1ull)));
        running += tot;
        bucket_sync<kGlobal>();
    }
    if (tid == 0) *sh_total = running;
    return running;
}

struct BucketShared {
    uint32_t npid, npair, bump, nkept, item_base, bucket, sh16[16];
};

// Processes records recs[0, n) of one bucket with working memory `base`
// (LDS or global scratch), appending Items to items[] via item_cursor.
template <class Item, class Idx>
__device__ __forceinline__ void process_bucket(const Rec16 *__restrict__ recs, uint32_t n,
                                               char *base, BucketShared *sh,
                                               const BoundParams &bp, Item *items,
                                               uint32_t *item_cursor, PhaseTimer &clk) {
    constexpr bool kVar = ItemTraits<Item>::var;
    constexpr bool kGlobal = sizeof(Idx) == 4;
    uint32_t *err = bp.err;
    const int tid = threadIdx.x;
    const BucketLayout L = BucketLayout::make(n, kVar, (int)sizeof(Idx));
    const uint32_t nilI = (uint32_t)(Idx)(~0u);
    const uint32_t C = __builtin_amdgcn_readfirstlane(L.C), cmask = C - 1;
    // T region (tables; reused in D/E)
    uint32_t *pidkey = reinterpret_cast<uint32_t *>(base + L.t_off);
    uint64_t *pairkey = reinterpret_cast<uint64_t *>(base + L.t_off + (size_t)C * 4);
    Idx *pid_s2i = reinterpret_cast<Idx *>(base + L.t_off + (size_t)C * 12);
    Idx *pair_s2i = pid_s2i + C;
    double *vstage = reinterpret_cast<double *>(base + L.t_off);
    uint64_t *slots = reinterpret_cast<uint64_t *>(base + L.t_off + (size_t)n * 8);
    uint64_t *rkey = reinterpret_cast<uint64_t *>(base + L.t_off + (size_t)n * 16);
    double *acc_sum = reinterpret_cast<double *>(base + L.t_off + (size_t)n * 8);
    double *acc_nsum = acc_sum + n;
    double *acc_nsq = acc_nsum + n;
    // P region: per pair
    uint32_t *pair_pk = reinterpret_cast<uint32_t *>(base + L.p_off);
    uint32_t *pair_pid = pair_pk + n;
    uint32_t *pair_cnt = pair_pid + n;
    uint32_t *pair_head = pair_cnt + n;  // list head; reused as kept count (PER_PID)
    uint32_t *pair_state = pair_head + n;
    // Q region: per pid
    uint32_t *pid_val = reinterpret_cast<uint32_t *>(base + L.q_off);
    uint32_t *pid_n = pid_val + n;  // #pairs (or #records in PER_PID mode)
    uint32_t *pid_slot = pid_n + n;
    // R region: per record
    Idx *rec_pair = reinterpret_cast<Idx *>(base + L.r_off);
    Idx *rec_next = rec_pair + n;  // pair list; reused as kept flag

    // ---- clear
    for (uint32_t i = tid; i < C; i += kBoundThreads) {
        pidkey[i] = kEmpty32;
        pairkey[i] = kEmpty64;
    }
    for (uint32_t i = tid; i < n; i += kBoundThreads) {
        pair_cnt[i] = 0;
        pair_head[i] = kNil;
        pid_n[i] = 0;
    }
    if (tid == 0) sh->bump = 0;
    bucket_sync<kGlobal>();
    mark(bp, 1, clk);
    // ---- A1: hash inserts
    for (uint32_t i = tid; i < n; i += kBoundThreads) {
        Rec16 r = recs[i];
        insert32(pidkey, cmask, r.pid, err);
        rec_pair[i] = (Idx)insert64(pairkey, cmask, ((uint64_t)r.pid << 32) | r.pk, err);
    }
    bucket_sync<kGlobal>();
    mark(bp, 2, clk);
    // ---- A2: dense ids
    const uint32_t npid = block_enumerate<kGlobal>(C, pidkey, nullptr, pid_s2i, sh->sh16, &sh->npid);
    const uint32_t npair = block_enumerate<kGlobal>(C, nullptr, pairkey, pair_s2i, sh->sh16, &sh->npair);
    for (uint32_t s = tid; s < C; s += kBoundThreads) {
        uint32_t k = pidkey[s];
        if (k != kEmpty32) pid_val[pid_s2i[s]] = k;
        uint64_t pk2 = pairkey[s];
        if (pk2 != kEmpty64) {
            uint32_t id = pair_s2i[s];
            pair_pk[id] = (uint32_t)pk2;
            pair_pid[id] = pid_s2i[lookup32(pidkey, cmask, (uint32_t)(pk2 >> 32), err)];
        }
    }
    bucket_sync<kGlobal>();
    mark(bp, 3, clk);
    // ---- A3: counts and lists
    const bool per_pid = bp.mode == DPG_MODE_PER_PRIVACY_ID;
    for (uint32_t i = tid; i < n; i += kBoundThreads) {
        uint32_t p = pair_s2i[rec_pair[i]];
        rec_pair[i] = (Idx)p;
        atomicAdd(&pair_cnt[p], 1u);
        rec_next[i] = (Idx)atomicExch(&pair_head[p], i);
        if (per_pid) atomicAdd(&pid_n[pair_pid[p]], 1u);
    }
    if (!per_pid)
        for (uint32_t p = tid; p < npair; p += kBoundThreads) atomicAdd(&pid_n[pair_pid[p]], 1u);
    bucket_sync<kGlobal>();  // tables dead from here on

    // ---- stage values (needed by D and E)
    if (bp.need_values)
        for (uint32_t i = tid; i < n; i += kBoundThreads) vstage[i] = recs[i].v;

    if (!per_pid) {
        mark(bp, 4, clk);
        // ---- C: cross-partition (mpc) selection over pairs
        for (uint32_t q = tid; q < npid; q += kBoundThreads) {
            uint32_t s = kNil;
            if (pid_n[q] > bp.mpc) {
                s = atomicAdd(&sh->bump, bp.mpc);
                for (uint32_t j = 0; j < bp.mpc; ++j) slots[s + j] = kEmpty64;
            }
            pid_slot[q] = s;
        }
        bucket_sync<kGlobal>();
        for (uint32_t p = tid; p < npair; p += kBoundThreads) {
            uint32_t q = pair_pid[p];
            if (pid_slot[q] != kNil) {
                uint64_t key = ((uint64_t)pair_prio(bp.seed, pid_val[q], pair_pk[p]) << 32) |
                               pair_pk[p];
                cascade_insert(slots + pid_slot[q], bp.mpc, key);
            }
        }
        bucket_sync<kGlobal>();
        for (uint32_t p = tid; p < npair; p += kBoundThreads) {
            uint32_t q = pair_pid[p];
            bool kept = true;
            if (pid_slot[q] != kNil) {
                uint64_t key = ((uint64_t)pair_prio(bp.seed, pid_val[q], pair_pk[p]) << 32) |
                               pair_pk[p];
                kept = key <= slots[pid_slot[q] + bp.mpc - 1];
            }
            pair_state[p] = kept ? kKeptAll : kDropped;
        }
        bucket_sync<kGlobal>();
        if (tid == 0) sh->bump = 0;
        bucket_sync<kGlobal>();
        mark(bp, 5, clk);
        // ---- D: per-partition (mcpp) sampling inside kept pairs
        const bool sample = bp.mode == DPG_MODE_CROSS_AND_PER_PARTITION && bp.need_values;
        if (sample) {
            for (uint32_t p = tid; p < npair; p += kBoundThreads) {
                if (pair_state[p] == kKeptAll && pair_cnt[p] > bp.mcpp) {
                    uint32_t s = atomicAdd(&sh->bump, bp.mcpp);
                    for (uint32_t j = 0; j < bp.mcpp; ++j) slots[s + j] = kEmpty64;
                    pair_state[p] = s;
                }
            }
            bucket_sync<kGlobal>();
            for (uint32_t i = tid; i < n; i += kBoundThreads) {
                uint32_t p = rec_pair[i];
                uint32_t st = pair_state[p];
                if (st < kKeptAll) {
                    uint64_t vb = __double_as_longlong(vstage[i]);
                    uint32_t occ = 0;
                    for (uint32_t j = pair_head[p]; j != kNil;) {
                        if (j < i && (uint64_t)__double_as_longlong(vstage[j]) == vb) ++occ;
                        uint32_t nx = rec_next[j];
                        j = nx == nilI ? kNil : nx;
                    }
                    uint64_t key = rec_prio(bp.seed, pid_val[pair_pid[p]], pair_pk[p], vb, occ);
                    rkey[i] = key;
                    cascade_insert(slots + st, bp.mcpp, key);
                }
            }
            bucket_sync<kGlobal>();
        }
        // kept flag per record -> rec_next
        for (uint32_t i = tid; i < n; i += kBoundThreads) {
            uint32_t st = pair_state[rec_pair[i]];
            bool k = st != kDropped;
            if (sample && st < kKeptAll) k = rkey[i] <= slots[st + bp.mcpp - 1];
            rec_next[i] = k ? 1 : 0;
        }
        bucket_sync<kGlobal>();
    } else {
        // ---- PER_PRIVACY_ID: keep the L records of each pid with the
        // smallest record key (pid_n holds the pid's record count)
        for (uint32_t q = tid; q < npid; q += kBoundThreads) {
            uint32_t s = kNil;
            if (pid_n[q] > bp.L) {
                s = atomicAdd(&sh->bump, bp.L);
                for (uint32_t j = 0; j < bp.L; ++j) slots[s + j] = kEmpty64;
            }
            pid_slot[q] = s;
        }
        bucket_sync<kGlobal>();
        for (uint32_t i = tid; i < n; i += kBoundThreads) {
            uint32_t p = rec_pair[i];
            uint32_t q = pair_pid[p];
            if (pid_slot[q] != kNil) {
                uint64_t vb = bp.need_values ? __double_as_longlong(vstage[i]) : 0ull;
                uint32_t occ = 0;
                for (uint32_t j = pair_head[p]; j != kNil;) {
                    if (j < i && (!bp.need_values ||
                                  (uint64_t)__double_as_longlong(vstage[j]) == vb))
                        ++occ;
                    uint32_t nx = rec_next[j];
                    j = nx == nilI ? kNil : nx;
                }
                uint64_t key = rec_prio(bp.seed, pid_val[q], pair_pk[p], vb, occ);
                rkey[i] = key;
                cascade_insert(slots + pid_slot[q], bp.L, key);
            }
        }
        bucket_sync<kGlobal>();
        for (uint32_t p = tid; p < npair; p += kBoundThreads) pair_head[p] = 0;  // kept count
        bucket_sync<kGlobal>();
        for (uint32_t i = tid; i < n; i += kBoundThreads) {
            uint32_t p = rec_pair[i];
            uint32_t q = pair_pid[p];
            bool k = pid_slot[q] == kNil || rkey[i] <= slots[pid_slot[q] + bp.L - 1];
            rec_next[i] = k ? 1 : 0;
            if (k) atomicAdd(&pair_head[p], 1u);
        }
        bucket_sync<kGlobal>();
    }

    mark(bp, 6, clk);
    // ---- E: accumulators of kept records (slots/rkey dead; acc overlays)
    const bool part_clip = bp.sum_mode == DPG_SUM_CLIP_PARTITION;
    if (bp.need_values) {
        for (uint32_t p = tid; p < npair; p += kBoundThreads) {
            acc_sum[p] = 0.0;
            if (kVar) {
                acc_nsum[p] = 0.0;
                acc_nsq[p] = 0.0;
            }
        }
        bucket_sync<kGlobal>();
        for (uint32_t i = tid; i < n; i += kBoundThreads) {
            if (!rec_next[i]) continue;
            uint32_t p = rec_pair[i];
            double v = vstage[i];
            if (part_clip) {
                atomicAdd(&acc_sum[p], v);
            } else {
                double x = clampd(v, bp.lo, bp.hi);
                atomicAdd(&acc_sum[p], x);
                if (kVar) {
                    double y = x - bp.mid;
                    atomicAdd(&acc_nsum[p], y);
                    atomicAdd(&acc_nsq[p], y * y);
                }
            }
        }
        bucket_sync<kGlobal>();
    }
    mark(bp, 7, clk);
    // ---- F: emit kept pairs
    uint32_t kept_here = 0;
    for (uint32_t p = tid; p < npair; p += kBoundThreads) {
        uint32_t c;
        if (per_pid) c = pair_head[p];
        else if (pair_state[p] == kDropped) c = 0;
        else if (bp.mode == DPG_MODE_CROSS_AND_PER_PARTITION) c = min(pair_cnt[p], bp.mcpp);
        else c = pair_cnt[p];
        kept_here += c > 0;
    }
    // block total of kept pairs
    {
        const int lane = tid & 63, w = tid >> 6;
        uint32_t x = kept_here;
        for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
        if (lane == 0) sh->sh16[w] = x;
        bucket_sync<kGlobal>();
        if (tid == 0) {
            uint32_t tot = 0;
            for (int k = 0; k < 16; ++k) tot += sh->sh16[k];
            sh->item_base = tot ? atomicAdd(item_cursor, tot) : 0;
            sh->nkept = 0;
        }
        bucket_sync<kGlobal>();
    }
    for (uint32_t p = tid; p < npair; p += kBoundThreads) {
        uint32_t c;
        if (per_pid) c = pair_head[p];
        else if (pair_state[p] == kDropped) c = 0;
        else if (bp.mode == DPG_MODE_CROSS_AND_PER_PARTITION) c = min(pair_cnt[p], bp.mcpp);
        else c = pair_cnt[p];
        if (c == 0) continue;
        uint32_t slot = sh->item_base + atomicAdd(&sh->nkept, 1u);
        Item it;
        it.pk = pair_pk[p];
        it.cnt = c;
        double s = 0.0;
        if (bp.need_values) {
            s = acc_sum[p];
            if (part_clip) s = clampd(s, bp.lo_pp, bp.hi_pp);
        }
        it.sum = s;
        if constexpr (kVar) {
            it.nsum = bp.need_values ? acc_nsum[p] : 0.0;
            it.nsq = bp.need_values ? acc_nsq[p] : 0.0;
        }
        items[slot] = it;
    }
    bucket_sync<kGlobal>();
    mark(bp, 8, clk);
}

// Buckets beyond the LDS chunk capacity (a privacy id with thousands of
// records): one workgroup per bucket, working set in global memory.
template <class Item>
__global__ __launch_bounds__(kBoundThreads) void k_bound_global(
    const Rec16 *recs, const int64_t *bstart, const uint32_t *bcnt, const size_t *scratch_off,
    char *scratch, BoundParams bp, Item *items, const int64_t *item_off, uint32_t *item_cursor) {
    __shared__ BucketShared sh;
    const uint32_t b = blockIdx.x;
    PhaseTimer clk;
    BoundParams bq = bp;
    bq.phase_cyc = nullptr;
    timer_start(bq, clk);
    process_bucket<Item, uint32_t>(recs + bstart[b], __builtin_amdgcn_readfirstlane(bcnt[b]),
                                   scratch + scratch_off[blockIdx.x], &sh, bq, items + *item_off,
                                   item_cursor, clk);
    mark(bq, 9, clk);
}

}  // namespace dpg
