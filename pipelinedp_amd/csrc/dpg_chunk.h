// dpg_chunk.h -- contribution bounding over packed chunks of privacy-id
// buckets, records resident in registers (gfx950).
//
// After the partition levels, consecutive fine buckets (disjoint privacy-id
// sets) are packed greedily into chunks of at most kCap records
// (k_make_chunks).  One 1024-thread workgroup per CU walks the chunk list;
// thread t owns records t and t + 1024 of a chunk in registers, and the next
// chunk's records are prefetched into registers while the current one is
// processed.  Phases (one barrier each):
//   A1  hash-insert (pid, pk), and pid for the first record of each pair; the
//       inserting lane of a new key takes a dense id (wave-aggregated LDS
//       counter) and initialises its rows
//   A2  per-pair record counts + record lists, per-pid pair (or record) counts
//   C1  value staging; each pid over its limit gets k cascade slots
//   C2  mpc selection, one lane per dense pair id: the pairs of a pid over
//       mpc cascade philox(seed, pid, pk) keys -- candidates below a
//       threshold first, the rest only if a pid got fewer than mpc
//                                               (contribution_bounders.py:90-92)
//   C3  pair state (dropped / kept / sampled) + item slot reservation in
//       the workgroup's item region
//   D   mcpp sampling: records of over-full kept pairs are compacted into a
//       work list, then cascade philox(seed, pid, pk, value, occ) keys
//       (:74-76); dense lanes keep the Philox cost proportional to the work
//   E   clipped accumulators of kept records         (combiners.py:255-500)
//   F   emit one Item per kept pair; clear the tables for the next chunk
// PER_PRIVACY_ID mode (:123-124) replaces C2..E with a per-pid cascade over
// record keys.  Results are identical to process_bucket (dpg_bound.h), which
// stays as the path for single buckets larger than kCap.
#pragma once

#include "dpg_bound.h"

namespace dpg {

constexpr int kChunkThreads = 1024;
constexpr uint16_t kNil16 = 0xFFFFu;

__host__ __device__ constexpr uint32_t pow2_at_least(uint32_t x) {
    uint32_t p = 64;
    while (p < x) p <<= 1;
    return p;
}
__host__ __device__ constexpr size_t cmax(size_t a, size_t b) { return a > b ? a : b; }
__host__ __device__ constexpr size_t a16(size_t x) { return (x + 15) & ~(size_t)15; }

struct ChunkShared {
    uint32_t npid, npair, bump, nwork;
    uint32_t nitems;  // this workgroup's items so far
    uint32_t pad[3];
};

// LDS layout of one chunk of at most kCap records.
template <class Item, int kCap>
struct ChunkLayout {
    static constexpr bool var = ItemTraits<Item>::var;
    static constexpr int RPT = (kCap + kChunkThreads - 1) / kChunkThreads;
    static constexpr uint32_t C = pow2_at_least(2 * kCap);  // load factor <= 1/2
    // T: tables (A1-A2), then vstage f64[kCap] + slots u64[2 kCap] +
    // rkey u64[kCap] (C1-E)
    static constexpr size_t tables = (size_t)C * (4 + 8 + 2 + 2);
    static constexpr size_t late = (size_t)kCap * 8 * 4;
    static constexpr size_t T = a16(cmax(tables, late));
    static constexpr size_t P_OFF = T;                                  // 5 x u32 per pair
    static constexpr size_t A_OFF = P_OFF + a16((size_t)kCap * 20);    // f64 acc per pair
    static constexpr size_t Q_OFF = A_OFF + a16((size_t)kCap * 8 * (var ? 3 : 1));
    static constexpr size_t R_OFF = Q_OFF + a16((size_t)kCap * 12);   // 3 x u32 per pid
    static constexpr size_t W_OFF = R_OFF + a16((size_t)kCap * 2);    // u16 next per record
    static constexpr size_t SH_OFF = W_OFF + a16((size_t)kCap * 4);   // u32 work list
    static constexpr size_t TOTAL = SH_OFF + a16(sizeof(ChunkShared));
    static_assert(TOTAL <= 160 * 1024, "chunk working set exceeds LDS");
};

// Insert `key`; `won` = this lane created the entry.
__device__ __forceinline__ uint32_t insert32w(uint32_t *keys, uint32_t mask, uint32_t key,
                                              bool &won, uint32_t *err) {
    uint32_t h = hslot32(key, mask);
    for (uint32_t probe = 0; probe <= mask; ++probe) {
        uint32_t old = atomicCAS(&keys[h], kEmpty32, key);
        if (old == kEmpty32) {
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
__device__ __forceinline__ uint32_t insert64w(uint64_t *keys, uint32_t mask, uint64_t key,
                                              bool &won, uint32_t *err) {
    uint32_t h = hslot64(key, mask);
    for (uint32_t probe = 0; probe <= mask; ++probe) {
        uint64_t old = atomicCAS((unsigned long long *)&keys[h], (unsigned long long)kEmpty64,
                                 (unsigned long long)key);
        if (old == kEmpty64) {
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
        base = __shfl(base, leader, 64);
    }
    return base + (uint32_t)__popcll(b & ((1ull << lane) - 1ull)) * per;
}

template <class Item, int kCap>
__device__ __forceinline__ void clear_tables(char *smem) {
    using L = ChunkLayout<Item, kCap>;
    uint4 *t = reinterpret_cast<uint4 *>(smem);  // pidkey + pairkey: C * 12 bytes
    const uint4 ones = make_uint4(~0u, ~0u, ~0u, ~0u);
    for (uint32_t i = threadIdx.x; i < L::C * 12 / 16; i += kChunkThreads) t[i] = ones;
}

// occurrence index of record i among identical (pid, pk, value) records of
// its pair (the canonical label, DESIGN.md "Randomness")
__device__ __forceinline__ uint32_t occurrence(uint32_t i, uint32_t head, const uint16_t *next,
                                               const double *vstage, bool use_v, uint64_t vb) {
    uint32_t occ = 0;
    for (uint32_t j = head; j != kNil16;) {
        if (j < i && (!use_v || (uint64_t)__double_as_longlong(vstage[j]) == vb)) ++occ;
        j = next[j];
    }
    return occ;
}

// Per-pid candidate threshold of the mpc selection: a pid with m > k pairs
// cascades only the pairs whose 32-bit priority is below ~(2k + 16) / m of
// the range; the k smallest are among them unless fewer than k fall below,
// which the second pass detects (slot k - 1 still empty) and completes.
__device__ __forceinline__ uint32_t cand_threshold(uint32_t m, uint32_t k) {
    const uint32_t e = 2 * k + 16;
    if (e >= m) return 0xFFFFFFFFu;
    return (uint32_t)(((uint64_t)e << 32) / m);
}

template <class Item, int kCap>
__device__ __forceinline__ void process_chunk(const Rec16 (&r)[ChunkLayout<Item, kCap>::RPT],
                                              uint32_t n, const Rec16 *next_base, uint32_t next_n,
                                              Rec16 (&rn)[ChunkLayout<Item, kCap>::RPT],
                                              char *smem, const BoundParams &bp, Item *items,
                                              PhaseTimer &clk) {
    using L = ChunkLayout<Item, kCap>;
    constexpr int RPT = L::RPT;
    constexpr bool kVar = L::var;
    constexpr uint32_t C = L::C, cmask = C - 1;
    uint32_t *err = bp.err;
    const int tid = threadIdx.x;
    // T region
    uint32_t *pidkey = reinterpret_cast<uint32_t *>(smem);
    uint64_t *pairkey = reinterpret_cast<uint64_t *>(smem + (size_t)C * 4);
    uint16_t *pid_s2i = reinterpret_cast<uint16_t *>(smem + (size_t)C * 12);
    uint16_t *pair_s2i = pid_s2i + C;
    double *vstage = reinterpret_cast<double *>(smem);
    uint64_t *slots = reinterpret_cast<uint64_t *>(smem + (size_t)kCap * 8);
    uint64_t *rkey = reinterpret_cast<uint64_t *>(smem + (size_t)kCap * 24);
    // per pair
    uint32_t *pair_pk = reinterpret_cast<uint32_t *>(smem + L::P_OFF);
    uint32_t *pair_pid = pair_pk + kCap;
    uint32_t *pair_cnt = pair_pid + kCap;
    uint32_t *pair_head = pair_cnt + kCap;
    uint32_t *pair_state = pair_head + kCap;  // slot base / kKeptAll / kDropped; kept count (per pid)
    double *acc_sum = reinterpret_cast<double *>(smem + L::A_OFF);
    double *acc_nsum = acc_sum + kCap;
    double *acc_nsq = acc_nsum + kCap;
    // per pid
    uint32_t *pid_val = reinterpret_cast<uint32_t *>(smem + L::Q_OFF);
    uint32_t *pid_n = pid_val + kCap;
    uint32_t *pid_slot = pid_n + kCap;
    uint16_t *rec_next = reinterpret_cast<uint16_t *>(smem + L::R_OFF);
    uint32_t *work = reinterpret_cast<uint32_t *>(smem + L::W_OFF);  // record | pair << 16
    ChunkShared *sh = reinterpret_cast<ChunkShared *>(smem + L::SH_OFF);

    const bool per_pid = bp.mode == DPG_MODE_PER_PRIVACY_ID;
    const bool need_v = bp.need_values != 0;
    const bool sample = bp.mode == DPG_MODE_CROSS_AND_PER_PARTITION && need_v;
    const bool part_clip = bp.sum_mode == DPG_SUM_CLIP_PARTITION;

    // record-major state (record i = tid + k * 1024)
    bool valid[RPT], pw[RPT], qw[RPT];
    uint32_t ps[RPT], rs[RPT], pp[RPT], qq[RPT];
    // pair-major state (dense pair id p = tid + k * 1024)
    uint64_t pkey[RPT];
    uint32_t islot[RPT];
    bool emit[RPT];

    // ---- A1: inserts, dense ids for new keys.  The pid table is probed by
    // the first record of each pair only (by every record in PER_PRIVACY_ID
    // mode, which counts records per pid).
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        const uint32_t i = tid + k * kChunkThreads;
        valid[k] = i < n;
        pw[k] = qw[k] = false;
        ps[k] = rs[k] = 0;
        if (valid[k])
            rs[k] = insert64w(pairkey, cmask, ((uint64_t)r[k].pid << 32) | r[k].pk, pw[k], err);
        const uint32_t p = wave_alloc(&sh->npair, pw[k]);
        if (pw[k]) {
            pair_s2i[rs[k]] = (uint16_t)p;
            pair_pk[p] = r[k].pk;
            pair_cnt[p] = 0;
            pair_head[p] = kNil16;
        }
        if (pw[k] || (per_pid && valid[k])) ps[k] = insert32w(pidkey, cmask, r[k].pid, qw[k], err);
        const uint32_t q = wave_alloc(&sh->npid, qw[k]);
        if (qw[k]) {
            pid_s2i[ps[k]] = (uint16_t)q;
            pid_val[q] = r[k].pid;
            pid_n[q] = 0;
        }
    }
    __syncthreads();
    mark(bp, 2, clk);
    // prefetch the next chunk's records (in flight during the phases below)
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        const uint32_t i = tid + k * kChunkThreads;
        if (i < next_n) rn[k] = next_base[i];
    }
    const uint32_t npair = __builtin_amdgcn_readfirstlane(sh->npair);
    // ---- A2: counts and record lists
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        if (!valid[k]) continue;
        const uint32_t i = tid + k * kChunkThreads;
        const uint32_t p = pair_s2i[rs[k]];
        pp[k] = p;
        if (per_pid || pw[k]) {
            const uint32_t q = pid_s2i[ps[k]];
            qq[k] = q;
            if (pw[k]) pair_pid[p] = q;
            atomicAdd(&pid_n[q], 1u);
        }
        atomicAdd(&pair_cnt[p], 1u);
        rec_next[i] = (uint16_t)atomicExch(&pair_head[p], i);
    }
    __syncthreads();  // tables dead from here on
    mark(bp, 3, clk);
    // ---- C1: value staging; cascade slots for pids over their limit
    const uint32_t lim = per_pid ? bp.L : bp.mpc;
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        if (!valid[k]) continue;
        const uint32_t i = tid + k * kChunkThreads;
        if (need_v) vstage[i] = r[k].v;
        if (qw[k]) {
            uint32_t s = kNil;
            if (pid_n[qq[k]] > lim) {
                s = atomicAdd(&sh->bump, lim);
                for (uint32_t j = 0; j < lim; ++j) slots[s + j] = kEmpty64;
            }
            pid_slot[qq[k]] = s;
            work[qq[k]] = 0;  // C2 candidate count of this pid
        }
    }
    if (tid == 0) sh->nwork = 0;
    __syncthreads();
    mark(bp, 4, clk);

    if (!per_pid) {
        // ---- C2: mpc cascade over pair keys, pair-major (dense lanes);
        // candidates first, then the rare completion pass
        bool cand[RPT], over[RPT];
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            const uint32_t p = tid + k * kChunkThreads;
            pkey[k] = 0;
            cand[k] = over[k] = false;
            if (p >= npair) continue;
            const uint32_t q = pair_pid[p];
            const uint32_t s = pid_slot[q];
            if (s == kNil) continue;
            over[k] = true;
            const uint32_t pk = pair_pk[p];
            const uint32_t pr = pair_prio(bp.seed, pid_val[q], pk);
            pkey[k] = ((uint64_t)pr << 32) | pk;
            cand[k] = pr < cand_threshold(pid_n[q], bp.mpc);
            if (cand[k]) {
                cascade_insert(slots + s, bp.mpc, pkey[k]);
                atomicAdd(&work[q], 1u);
            }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            if (!over[k] || cand[k]) continue;
            const uint32_t q = pair_pid[tid + k * kChunkThreads];
            if (work[q] < bp.mpc) cascade_insert(slots + pid_slot[q], bp.mpc, pkey[k]);
        }
        __syncthreads();
        // ---- C3: pair state, accumulator init, item slots (pair-major)
        bool kept[RPT];
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            const uint32_t p = tid + k * kChunkThreads;
            kept[k] = false;
            if (p < npair) {
                const uint32_t s = pid_slot[pair_pid[p]];
                kept[k] = s == kNil || pkey[k] <= slots[s + bp.mpc - 1];
                pair_state[p] = kept[k] ? kKeptAll : kDropped;
                if (need_v) {
                    acc_sum[p] = 0.0;
                    if (kVar) {
                        acc_nsum[p] = 0.0;
                        acc_nsq[p] = 0.0;
                    }
                }
            }
            emit[k] = kept[k];
        }
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            const uint32_t p = tid + k * kChunkThreads;
            const bool want = sample && kept[k] && pair_cnt[p] > bp.mcpp;
            const uint32_t s2 = wave_alloc(&sh->bump, want, bp.mcpp);
            if (want) {
                for (uint32_t j = 0; j < bp.mcpp; ++j) slots[s2 + j] = kEmpty64;
                pair_state[p] = s2;
            }
            islot[k] = wave_alloc(&sh->nitems, emit[k]);
        }
        __syncthreads();
        mark(bp, 5, clk);
        // ---- D: mcpp cascade over record keys inside over-full kept pairs:
        // the records needing a key are compacted into a work list first
        if (sample) {
#pragma unroll
            for (int k = 0; k < RPT; ++k) {
                const bool want = valid[k] && pair_state[pp[k]] < kKeptAll;
                const uint32_t w = wave_alloc(&sh->nwork, want);
                if (want) work[w] = (tid + k * kChunkThreads) | (pp[k] << 16);
            }
            __syncthreads();
            const uint32_t nwork = __builtin_amdgcn_readfirstlane(sh->nwork);
            for (uint32_t w = tid; w < nwork; w += kChunkThreads) {
                const uint32_t e = work[w], i = e & 0xFFFFu, p = e >> 16;
                const uint64_t vb = __double_as_longlong(vstage[i]);
                const uint32_t occ = occurrence(i, pair_head[p], rec_next, vstage, true, vb);
                const uint64_t key = rec_prio(bp.seed, pid_val[pair_pid[p]], pair_pk[p], vb, occ);
                rkey[i] = key;
                cascade_insert(slots + pair_state[p], bp.mcpp, key);
            }
            __syncthreads();
        }
        mark(bp, 6, clk);
        // ---- E: accumulators of kept records
        if (need_v) {
#pragma unroll
            for (int k = 0; k < RPT; ++k) {
                if (!valid[k]) continue;
                const uint32_t i = tid + k * kChunkThreads;
                const uint32_t p = pp[k];
                const uint32_t st = pair_state[p];
                bool keep = st != kDropped;
                if (sample && st < kKeptAll) keep = rkey[i] <= slots[st + bp.mcpp - 1];
                if (!keep) continue;
                const double v = r[k].v;
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
            __syncthreads();
        }
        mark(bp, 7, clk);
    } else {
        // ---- PER_PRIVACY_ID: keep the L records of each pid with the
        // smallest record key; pair_state counts kept records per pair
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            const uint32_t p = tid + k * kChunkThreads;
            if (p < npair) {
                pair_state[p] = 0;
                if (need_v) {
                    acc_sum[p] = 0.0;
                    if (kVar) {
                        acc_nsum[p] = 0.0;
                        acc_nsq[p] = 0.0;
                    }
                }
            }
            const bool want = valid[k] && pid_slot[qq[k]] != kNil;
            const uint32_t w = wave_alloc(&sh->nwork, want);
            if (want) work[w] = (tid + k * kChunkThreads) | (pp[k] << 16);
        }
        __syncthreads();
        const uint32_t nwork = __builtin_amdgcn_readfirstlane(sh->nwork);
        for (uint32_t w = tid; w < nwork; w += kChunkThreads) {
            const uint32_t e = work[w], i = e & 0xFFFFu, p = e >> 16;
            const uint32_t q = pair_pid[p];
            const uint64_t vb = need_v ? (uint64_t)__double_as_longlong(vstage[i]) : 0ull;
            const uint32_t occ = occurrence(i, pair_head[p], rec_next, vstage, need_v, vb);
            const uint64_t key = rec_prio(bp.seed, pid_val[q], pair_pk[p], vb, occ);
            rkey[i] = key;
            cascade_insert(slots + pid_slot[q], bp.L, key);
        }
        __syncthreads();
        mark(bp, 5, clk);
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            if (!valid[k]) continue;
            const uint32_t i = tid + k * kChunkThreads;
            const uint32_t p = pp[k];
            const uint32_t s = pid_slot[qq[k]];
            const bool keep = s == kNil || rkey[i] <= slots[s + bp.L - 1];
            if (!keep) continue;
            atomicAdd(&pair_state[p], 1u);
            if (need_v) {
                const double v = r[k].v;
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
        __syncthreads();
        mark(bp, 7, clk);
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            const uint32_t p = tid + k * kChunkThreads;
            emit[k] = p < npair && pair_state[p] > 0;
            islot[k] = wave_alloc(&sh->nitems, emit[k]);
        }
    }
    // ---- F: emit kept pairs (pair-major); clear the tables for the next chunk
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        if (!emit[k]) continue;
        const uint32_t p = tid + k * kChunkThreads;
        uint32_t c;
        if (per_pid) c = pair_state[p];
        else if (bp.mode == DPG_MODE_CROSS_AND_PER_PARTITION) c = min(pair_cnt[p], bp.mcpp);
        else c = pair_cnt[p];
        Item it;
        it.pk = pair_pk[p];
        it.cnt = c;
        double s = 0.0;
        if (need_v) {
            s = acc_sum[p];
            if (part_clip) s = clampd(s, bp.lo_pp, bp.hi_pp);
        }
        it.sum = s;
        if constexpr (kVar) {
            it.nsum = need_v ? acc_nsum[p] : 0.0;
            it.nsq = need_v ? acc_nsq[p] : 0.0;
        }
        items[islot[k]] = it;
    }
    clear_tables<Item, kCap>(smem);
    if (tid == 0) {
        sh->npid = 0;
        sh->npair = 0;
        sh->bump = 0;
    }
    __syncthreads();
    mark(bp, 8, clk);
}

// Chunk descriptor: records [x, x + (y & 0x7FFFFFFF)) of buffer (y >> 31).
__device__ __forceinline__ const Rec16 *chunk_base(uint2 d, const Rec16 *b0, const Rec16 *b1) {
    return ((d.y >> 31) ? b1 : b0) + d.x;
}

// Persistent workgroups walk the chunk list statically (w, w + G, ...): the
// loop bound, the chunk size and every branch around a barrier are uniform.
// Workgroup g appends its items to its own region items[wg_off[g], ...) (the
// records of its chunks bound the count) and leaves the count in wg_cnt[g]:
// no global atomics in the loop.
template <class Item, int kCap>
__global__ __launch_bounds__(kChunkThreads) void k_bound_chunks(
    const Rec16 *recs, const Rec16 *refined, const uint2 *chunks, const uint32_t *n_chunks,
    BoundParams bp, Item *items, const int64_t *wg_off, uint32_t *wg_cnt) {
    using L = ChunkLayout<Item, kCap>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    PhaseTimer clk;
    timer_start(bp, clk);
    const uint32_t nch = __builtin_amdgcn_readfirstlane(*n_chunks);
    ChunkShared *sh = reinterpret_cast<ChunkShared *>(smem + L::SH_OFF);
    Item *my_items = items + wg_off[blockIdx.x];
    clear_tables<Item, kCap>(smem);
    if (threadIdx.x == 0) {
        sh->npid = 0;
        sh->npair = 0;
        sh->bump = 0;
        sh->nwork = 0;
        sh->nitems = 0;
    }
    // software pipeline: records of chunk w in r, descriptor of w + G in dn;
    // the descriptor of w + 2G and the records of w + G load during w
    Rec16 r[L::RPT], rn[L::RPT];
    const uint32_t G = gridDim.x;
    uint32_t w = blockIdx.x;
    uint32_t n = 0;
    uint2 dn = make_uint2(0, 0);
    if (w < nch) {
        const uint2 d = chunks[w];
        n = __builtin_amdgcn_readfirstlane(d.y & 0x7FFFFFFFu);
        const Rec16 *b = chunk_base(d, recs, refined);
#pragma unroll
        for (int k = 0; k < L::RPT; ++k) {
            const uint32_t i = threadIdx.x + k * kChunkThreads;
            if (i < n) r[k] = b[i];
        }
        if (w + G < nch) dn = chunks[w + G];
    }
    __syncthreads();
    for (; w < nch; w += G) {
        uint2 dnn = make_uint2(0, 0);
        if (w + 2 * G < nch) dnn = chunks[w + 2 * G];
        const uint32_t nn = __builtin_amdgcn_readfirstlane(dn.y & 0x7FFFFFFFu);
        const Rec16 *nb = chunk_base(make_uint2(__builtin_amdgcn_readfirstlane(dn.x),
                                                __builtin_amdgcn_readfirstlane(dn.y)),
                                     recs, refined);
        process_chunk<Item, kCap>(r, n, nb, nn, rn, smem, bp, my_items, clk);
#pragma unroll
        for (int k = 0; k < L::RPT; ++k) r[k] = rn[k];
        n = nn;
        dn = dnn;
    }
    if (threadIdx.x == 0) wg_cnt[blockIdx.x] = sh->nitems;
    timer_flush(bp, clk);
}

// wg_rec[g] = records of the chunks workgroup g of G will process (w = g mod G)
__global__ __launch_bounds__(256) void k_wg_records(const uint2 *chunks, const uint32_t *n_chunks,
                                                    uint32_t G, uint32_t *wg_rec) {
    __shared__ uint32_t part[4];
    const uint32_t nch = *n_chunks, g = blockIdx.x;
    uint32_t acc = 0;
    for (uint32_t w = g + threadIdx.x * G; w < nch; w += 256 * G) acc += chunks[w].y & 0x7FFFFFFFu;
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) wg_rec[g] = part[0] + part[1] + part[2] + part[3];
}

// out[i] = sum(in[0, i)) for i <= m (m < 1024); optionally *total32 = out[m]
__global__ __launch_bounds__(1024) void k_scan_small(const uint32_t *in, uint32_t m, int64_t *out,
                                                     uint32_t *total32) {
    __shared__ int64_t sh[1024];
    const uint32_t t = threadIdx.x;
    sh[t] = t < m ? (int64_t)in[t] : 0;
    __syncthreads();
    for (uint32_t o = 1; o < 1024; o <<= 1) {
        int64_t x = t >= o ? sh[t - o] : 0;
        __syncthreads();
        sh[t] += x;
        __syncthreads();
    }
    if (t <= m) out[t] = t ? sh[t - 1] : 0;
    if (t == 0 && total32) *total32 = m ? (uint32_t)sh[m - 1] : 0u;
}

// Greedy packing of consecutive fine buckets into chunks of <= cap records,
// one thread per group of `group` buckets.  Buckets larger than cap go to
// the oversize list (start, count).  sel = buffer the buckets live in.
__global__ void k_make_chunks(const int64_t *bstart, const uint32_t *bcnt, uint32_t B,
                              uint32_t group, uint32_t cap, uint32_t sel, uint2 *chunks,
                              uint32_t *n_chunks, int64_t *over_start, uint32_t *over_cnt,
                              uint32_t *n_over, unsigned long long *over_records) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t b0 = g * group;
    if (b0 >= B) return;
    const uint32_t b1 = min(B, b0 + group);
    // pass 1: count chunks
    uint32_t nc = 0, cur = 0;
    int64_t cend = -1;
    for (uint32_t b = b0; b < b1; ++b) {
        const uint32_t c = bcnt[b];
        if (c == 0) continue;
        if (c > cap) continue;
        const int64_t st = bstart[b];
        if (cur == 0 || cur + c > cap || st != cend) {
            ++nc;
            cur = 0;
        }
        cur += c;
        cend = st + c;
    }
    uint32_t base = nc ? atomicAdd(n_chunks, nc) : 0;
    // pass 2: write
    cur = 0;
    cend = -1;
    int64_t cst = 0;
    for (uint32_t b = b0; b < b1; ++b) {
        const uint32_t c = bcnt[b];
        if (c == 0) continue;
        const int64_t st = bstart[b];
        if (c > cap) {
            const uint32_t o = atomicAdd(n_over, 1u);
            over_start[o] = st;
            over_cnt[o] = c;
            atomicAdd(over_records, (unsigned long long)c);
            continue;
        }
        if (cur == 0 || cur + c > cap || st != cend) {
            if (cur) chunks[base++] = make_uint2((uint32_t)cst, cur | (sel << 31));
            cur = 0;
            cst = st;
        }
        cur += c;
        cend = st + c;
    }
    if (cur) chunks[base++] = make_uint2((uint32_t)cst, cur | (sel << 31));
}

}  // namespace dpg
