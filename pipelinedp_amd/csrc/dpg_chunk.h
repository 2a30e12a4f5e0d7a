// dpg_chunk.h -- contribution bounding over packed chunks of privacy-id
// buckets in LDS (gfx950).
//
// After the partition levels, consecutive fine buckets of one level-1 bucket
// (disjoint privacy-id sets) are packed greedily into chunks of at most
// kBCap = 1024 records (k_make_chunks).  Persistent 256-thread workgroups --
// three per CU at ~48 KB of LDS each, so one workgroup's barriers and LDS
// round trips overlap the others' work -- walk the chunk list statically;
// thread t keeps records t + 256 k (k < 4) of a chunk in registers and
// prefetches the next chunk's records while the current one is processed.
//
// Tables are indexed by hash slot (no compaction): pid slot q <- the pid's
// hash residual, pair slot p <- (q, pk).  Phases (one barrier each) follow
// dpg_bound.h: A inserts/counts, B pid cascade slots, C mpc selection over
// pair keys (candidates below a per-pid threshold first, then a rare
// completion pass), D pair state + mcpp slots, E mcpp cascade over record
// keys (values of kept pairs are gathered meanwhile), F clipped
// accumulators, G emit + clear.  PER_PRIVACY_ID mode replaces C..F with a
// per-pid cascade over record keys.
#pragma once

#include "dpg_bound.h"

namespace dpg {

constexpr int kBT = 256;             // threads per bound workgroup
constexpr int kBCap = 1024;          // records per chunk
constexpr int kRPT = kBCap / kBT;    // records per thread
constexpr uint32_t kCq = 1024;       // pid table slots (pids <= records)
constexpr uint32_t kCp = 1024;       // pair table slots (pairs <= records)
constexpr uint32_t kPool = 2048;     // selection keys: per-pid regions in [0, 1024), per-pair above
constexpr uint32_t kMcppBase = 1024;
constexpr int kQPT = kCq / kBT;      // pid slots per thread
constexpr int kPPT = kCp / kBT;      // pair slots per thread

// small chunks: one wave each (dpg_wave.h)
#ifndef DPG_WCAP
#define DPG_WCAP 512
#endif
constexpr int kWCap = DPG_WCAP;        // records per small chunk
constexpr int kWRPT = kWCap / 64;      // records per lane
constexpr uint32_t kWCq = 128;         // direct pid slots per small chunk
constexpr uint32_t kWCp = kWCap;       // pairs (dense ids) per small chunk
constexpr uint32_t kWCk = 2 * kWCap;   // pair key table slots (load <= 1/2)
constexpr uint32_t kWPool = kWCap;     // selection keys (mpc regions, then mcpp regions)
constexpr int kWQPL = kWCq / 64;       // pid slots per lane
constexpr int kWPPL = kWCp / 64;       // pair slots per lane

struct ChunkShared {
    uint32_t bump, bump2, nitems, npair, npid, pad[3];
};

// LDS layout of one workgroup (KeyT: pair key width).  Pid slots are direct:
// q = hash residual - chunk base (< kCq, the chunk packer guarantees it).
template <class KeyT, class Item>
struct ChunkLayout {
    static constexpr bool var = ItemTraits<Item>::var;
    static constexpr size_t PIDV = 0;                 // privacy id - pid_min
    static constexpr size_t PIDM = PIDV + 4 * kCq;    // low 16: pairs/records, high: appends
    static constexpr size_t PIDSLOT = PIDM + 4 * kCq; // pool base (+ appends << 16) or kNil
    static constexpr size_t QLIST = PIDSLOT + 4 * kCq;  // dense list of occupied pid slots
    static constexpr size_t PAIRTAB = QLIST + 2 * kCq;
    static constexpr size_t PAIRCNT = PAIRTAB + sizeof(KeyT) * kCp;
    static constexpr size_t PAIRST = PAIRCNT + 4 * kCp;
    static constexpr size_t PLIST = PAIRST + 4 * kCp;  // dense list of occupied pair slots
    static constexpr size_t POOL = PLIST + 2 * kCp;
    static constexpr size_t ACC = POOL + 8 * kPool;
    static constexpr size_t SH = ACC + 8 * kCp * (var ? 3 : 1);
    static constexpr size_t TOTAL = SH + sizeof(ChunkShared);
    static constexpr int PER_CU = TOTAL <= 53 * 1024 ? 3 : 2;
    static_assert(TOTAL <= 80 * 1024, "chunk working set too large");
};

// Full clear (kernel start); chunks clear only their occupied slots.
template <class KeyT, class Item>
__device__ __forceinline__ void clear_tables(char *smem) {
    using L = ChunkLayout<KeyT, Item>;
    uint32_t *pidm = reinterpret_cast<uint32_t *>(smem + L::PIDM);
    KeyT *pairtab = reinterpret_cast<KeyT *>(smem + L::PAIRTAB);
    uint32_t *paircnt = reinterpret_cast<uint32_t *>(smem + L::PAIRCNT);
#pragma unroll
    for (int j = 0; j < kQPT; ++j) pidm[threadIdx.x + j * kBT] = 0;
#pragma unroll
    for (int j = 0; j < kPPT; ++j) {
        pairtab[threadIdx.x + j * kBT] = empty_key<KeyT>();
        paircnt[threadIdx.x + j * kBT] = 0;
    }
}

// Linear probing continued from slot h (the home slot's CAS already failed on
// a different key); `won` = this lane created the entry.
template <class K>
__device__ __forceinline__ uint32_t probe_from(K *keys, uint32_t mask, K key, uint32_t h,
                                               bool &won, uint32_t *err) {
    for (uint32_t probe = 1; probe <= mask; ++probe) {
        h = (h + 1) & mask;
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
    }
    atomicOr(err, 2u);
    won = false;
    return 0;
}

template <class K>
__device__ __forceinline__ K cas_home(K *keys, uint32_t h, K key) {
    if constexpr (sizeof(K) == 8)
        return (K)atomicCAS((unsigned long long *)&keys[h], (unsigned long long)empty_key<K>(),
                            (unsigned long long)key);
    else
        return atomicCAS(&keys[h], empty_key<K>(), key);
}

// Variable-size wave-aggregated allocation (amount 0: nothing); call with
// the whole wave converged.
template <class T>
__device__ __forceinline__ uint32_t wave_alloc_var(T *ctr, uint32_t amount) {
    uint32_t total;
    const uint32_t ex = wave_excl_scan(amount, total);
    uint32_t base = 0;
    if (total) {
        if (__lane_id() == 0) base = atomicAdd(ctr, total);
        base = __shfl(base, 0, 64);
    }
    return base + ex;
}

// Batched wave-aggregated allocation: lane slot k gets one entry where
// want[k]; one LDS atomic per wave for all K (call with the wave converged).
__device__ __forceinline__ uint32_t lanes_below(uint64_t b) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
}
template <int K>
__device__ __forceinline__ void wave_alloc_batch(uint32_t *ctr, const bool (&want)[K],
                                                 uint32_t (&slot)[K]) {
    uint64_t b[K];
    uint32_t tot = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        b[k] = __ballot(want[k]);
        tot += (uint32_t)__popcll(b[k]);
    }
    uint32_t base = 0;
    if (tot) {
        if (__lane_id() == 0) base = atomicAdd(ctr, tot);
        base = __builtin_amdgcn_readfirstlane(base);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        slot[k] = base + lanes_below(b[k]);
        base += (uint32_t)__popcll(b[k]);
    }
}

// Number of keys in a[0, cnt) below x (cnt >= 1): loads are unconditional
// (index clamped) in batches of 8 so that a batch is in flight together.
__device__ __forceinline__ uint32_t rank_below(const uint64_t *a, uint32_t cnt, uint64_t x) {
    uint32_t r = 0;
    for (uint32_t j = 0; j < cnt; j += 8) {
        uint64_t y[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) y[u] = a[min(j + u, cnt - 1)];
#pragma unroll
        for (int u = 0; u < 8; ++u) r += (j + u < cnt && y[u] < x) ? 1u : 0u;
    }
    return r;
}

// Records past the chunk end hold a copy of its last record (loads are
// unconditional): they take part in the table inserts, whose keys exist
// anyway, and in nothing that counts.
template <class KeyT, class Item, class R>
__device__ __forceinline__ void bound_chunk(const R (&r)[kRPT], uint32_t n, uint32_t d1,
                                            uint32_t hbase, const R *next_base, uint32_t next_n,
                                            R (&rn)[kRPT], char *smem, const BoundParams &bp,
                                            Item *items, PhaseTimer &clk) {
    using L = ChunkLayout<KeyT, Item>;
    constexpr bool kVar = L::var;
    uint32_t *pidv = reinterpret_cast<uint32_t *>(smem + L::PIDV);
    uint32_t *pidm = reinterpret_cast<uint32_t *>(smem + L::PIDM);
    uint32_t *pidslot = reinterpret_cast<uint32_t *>(smem + L::PIDSLOT);
    uint16_t *qlist = reinterpret_cast<uint16_t *>(smem + L::QLIST);
    KeyT *pairtab = reinterpret_cast<KeyT *>(smem + L::PAIRTAB);
    uint32_t *paircnt = reinterpret_cast<uint32_t *>(smem + L::PAIRCNT);
    uint32_t *pairst = reinterpret_cast<uint32_t *>(smem + L::PAIRST);
    uint16_t *plist = reinterpret_cast<uint16_t *>(smem + L::PLIST);
    uint64_t *pool = reinterpret_cast<uint64_t *>(smem + L::POOL);
    double *acc_sum = reinterpret_cast<double *>(smem + L::ACC);
    double *acc_nsum = acc_sum + kCp;
    double *acc_nsq = acc_nsum + kCp;
    ChunkShared *sh = reinterpret_cast<ChunkShared *>(smem + L::SH);

    const int tid = threadIdx.x;
    const Fmt f = bp.fmt;
    const uint32_t pkb = f.pkbits;
    const uint64_t pkmask = (1ull << pkb) - 1ull;
    const bool per_pid = bp.mode == DPG_MODE_PER_PRIVACY_ID;
    const bool need_v = bp.need_values != 0;
    const bool sample = bp.mode == DPG_MODE_CROSS_AND_PER_PARTITION && need_v;
    const bool part_clip = bp.sum_mode == DPG_SUM_CLIP_PARTITION;
    const uint32_t lim = per_pid ? bp.L : bp.mpc;

    // ---- A: pair inserts and counts (record-major); the pid slot is the
    // hash residual minus the chunk base.  The home-slot CAS of all kRPT
    // records is issued back to back; only collisions probe on.  Lanes past
    // the chunk end aim their CAS at a lane-private dummy word in the (still
    // idle) pool, so they neither touch the table nor serialise on one
    // address.  The first pair (record, PER_PRIVACY_ID) of a pid appends the
    // pid slot to the dense pid list.
    uint32_t qs[kRPT], ps[kRPT];
    bool valid[kRPT];
    {
        KeyT pkey[kRPT], op[kRPT];
#pragma unroll
        for (int k = 0; k < kRPT; ++k) {
            valid[k] = tid + k * kBT < n;
            const uint64_t key = RecOps<R>::key(r[k], f);
            qs[k] = ((uint32_t)(key >> pkb) - hbase) & (kCq - 1);
            pkey[k] = ((KeyT)qs[k] << pkb) | (KeyT)(key & pkmask);
            ps[k] = hslot(pkey[k], kCp - 1);
            KeyT *tgt = valid[k] ? pairtab + ps[k]
                                 : reinterpret_cast<KeyT *>(pool) + (tid + k * kBT);
            op[k] = cas_home<KeyT>(tgt, 0, pkey[k]);
        }
        mark(bp, 0, clk);
        bool won[kRPT], first[kRPT];
        uint32_t oldm[kRPT];
#pragma unroll
        for (int k = 0; k < kRPT; ++k) {
            won[k] = valid[k] && op[k] == empty_key<KeyT>();
            if (valid[k] && !won[k] && op[k] != pkey[k])
                ps[k] = probe_from<KeyT>(pairtab, kCp - 1, pkey[k], ps[k], won[k], bp.err);
        }
        // counts; the returned pid count (all kRPT in flight together; lanes
        // not counting add 0 to a valid slot) tells the pid's first toucher
#pragma unroll
        for (int k = 0; k < kRPT; ++k) {
            if (valid[k]) atomicAdd(&paircnt[ps[k]], 1u);
            const bool touch = per_pid ? valid[k] : won[k];
            // pre-aggregate: records per pid in the high half (no pid is
            // over a limit, so no candidate appends use it)
            const uint32_t rec = (ItemTraits<Item>::preagg && valid[k]) ? 1u << 16 : 0u;
            oldm[k] = atomicAdd(&pidm[qs[k]], (touch ? 1u : 0u) + rec);
        }
#pragma unroll
        for (int k = 0; k < kRPT; ++k)
            first[k] = (per_pid ? valid[k] : won[k]) && (oldm[k] & 0xFFFFu) == 0u;
        uint32_t qi[kRPT], li[kRPT];
        wave_alloc_batch<kRPT>(&sh->npid, first, qi);
        wave_alloc_batch<kRPT>(&sh->npair, won, li);
#pragma unroll
        for (int k = 0; k < kRPT; ++k) {
            if (first[k]) qlist[qi[k]] = (uint16_t)qs[k];
            if (won[k]) plist[li[k]] = (uint16_t)ps[k];
        }
        mark(bp, 1, clk);
    }
    __syncthreads();
    mark(bp, 2, clk);
    // prefetch the next chunk's records (in flight during the phases below)
    if (next_n > 0) {
#pragma unroll
        for (int k = 0; k < kRPT; ++k) rn[k] = next_base[min((uint32_t)(tid + k * kBT), next_n - 1)];
    }
    const uint32_t npair = __builtin_amdgcn_readfirstlane(sh->npair);
    const uint32_t npid = __builtin_amdgcn_readfirstlane(sh->npid);
    // ---- B: privacy id of every pid (pid-major, dense) and, for pids over
    // their limit, one pool slot per pair (per record in PER_PRIVACY_ID
    // mode) for the selection keys; pair accumulators (pair-major, dense)
    const uint32_t hshift = f.kbits - f.b1;
#pragma unroll
    for (int j = 0; j < kQPT; ++j) {
        const uint32_t li = tid + j * kBT;
        const bool occ = li < npid;
        const uint32_t q = occ ? qlist[li] : 0u;
        const uint32_t m = occ ? (pidm[q] & 0xFFFFu) : 0u;
        const bool want = m > lim;
        const uint32_t s = want ? atomicAdd(&sh->bump, m) : 0u;
        if (occ) {
            pidslot[q] = want ? s : kNil;
            pidv[q] = hk_inv((d1 << hshift) | (hbase + q), bp.hash);
        }
    }
#pragma unroll
    for (int j = 0; j < kPPT; ++j) {
        const uint32_t li = tid + j * kBT;
        if (li >= npair) continue;
        const uint32_t p = plist[li];
        if (need_v) {
            acc_sum[p] = 0.0;
            if (kVar) {
                acc_nsum[p] = 0.0;
                acc_nsq[p] = 0.0;
            }
        }
        if (per_pid) pairst[p] = 0;
    }
    __syncthreads();
    mark(bp, 3, clk);

    bool emit[kPPT];
    uint32_t ecnt[kPPT], pslot_of[kPPT];
    if (!per_pid) {
        // ---- C1: mpc selection over pair keys (pair-major, dense): pairs of
        // over-limit pids whose priority is below the candidate threshold
        // append their key to the pid's pool region
        uint64_t k64[kPPT];
        uint32_t pbase[kPPT];
        bool over[kPPT], cand[kPPT], kept[kPPT];
#pragma unroll
        for (int j = 0; j < kPPT; ++j) {
            const uint32_t li = tid + j * kBT;
            over[j] = cand[j] = false;
            kept[j] = li < npair;
            k64[j] = 0;
            pbase[j] = 0;
            pslot_of[j] = 0;
            if (li >= npair) continue;
            const uint32_t p = plist[li];
            pslot_of[j] = p;
            const KeyT pkey = pairtab[p];
            const uint32_t q = (uint32_t)(pkey >> pkb);
            const uint32_t s = pidslot[q];
            if (s == kNil) continue;
            over[j] = true;
            pbase[j] = s;
            const uint32_t pk = (uint32_t)(pkey & (KeyT)pkmask);
            const uint32_t pr =
                pair_prio(bp.seed, (uint64_t)(bp.pid_min + (int64_t)pidv[q]), pk);
            k64[j] = ((uint64_t)pr << 32) | pk;
            cand[j] = pr < cand_threshold(pidm[q] & 0xFFFFu, bp.mpc);
            if (cand[j]) pool[s + (atomicAdd(&pidm[q], 1u << 16) >> 16)] = k64[j];
        }
        __syncthreads();
        // ---- C2: with >= mpc candidates a candidate is kept iff fewer than
        // mpc candidates have a smaller key (every non-candidate key exceeds
        // every candidate key); with fewer (rare), all candidates are kept and
        // the non-candidates append after them for C3
        uint32_t ncd[kPPT];
#pragma unroll
        for (int j = 0; j < kPPT; ++j) {
            ncd[j] = 0;
            if (!over[j]) continue;
            const uint32_t q = (uint32_t)(pairtab[pslot_of[j]] >> pkb);
            const uint32_t nc = pidm[q] >> 16;
            ncd[j] = nc;
            if (nc >= bp.mpc) {
                kept[j] = cand[j] && rank_below(pool + pbase[j], nc, k64[j]) < bp.mpc;
            } else if (!cand[j]) {
                pool[pbase[j] + nc + (atomicAdd(&pidslot[q], 1u << 16) >> 16)] = k64[j];
            }
        }
        __syncthreads();
        mark(bp, 4, clk);
        // ---- D: (C3) non-candidates of pids short of candidates rank among
        // the appended non-candidates; pair state; every over-full kept pair
        // reserves one pool slot per record for its record keys
#pragma unroll
        for (int j = 0; j < kPPT; ++j) {
            const uint32_t li = tid + j * kBT;
            const bool occ = li < npair;
            const uint32_t p = pslot_of[j];
            if (over[j] && !cand[j] && ncd[j] < bp.mpc) {
                const uint32_t q = (uint32_t)(pairtab[p] >> pkb);
                const uint32_t nn = pidslot[q] >> 16;
                kept[j] = rank_below(pool + pbase[j] + ncd[j], nn, k64[j]) < bp.mpc - ncd[j];
            }
            const uint32_t c = occ ? paircnt[p] : 0u;
            const bool need = sample && kept[j] && c > bp.mcpp;
            const uint32_t b2 = need ? atomicAdd(&sh->bump2, c) : 0u;
            if (occ) pairst[p] = !kept[j] ? kDropped : (need ? b2 : kKeptAll);
            emit[j] = kept[j];
            ecnt[j] = bp.mode == DPG_MODE_CROSS_AND_PER_PARTITION ? min(c, bp.mcpp) : c;
        }
        __syncthreads();
        mark(bp, 5, clk);
        // ---- E: records of over-full kept pairs append their record key to
        // the pair's pool region (the low 16 bits of pairst hold its base, the
        // high 16 count appends); the values of records of kept pairs are
        // gathered meanwhile
        uint64_t rkey[kRPT];
        double v[kRPT];
        uint32_t st[kRPT];
#pragma unroll
        for (int k = 0; k < kRPT; ++k) {
            rkey[k] = 0;
            v[k] = 0.0;
            // other records of the pair may already have appended (high 16
            // bits), so a sampled pair's base is the low 16 bits
            st[k] = valid[k] ? pairst[ps[k]] : kDropped;
            if (st[k] < kKeptAll) st[k] &= 0xFFFFu;
            if (need_v && st[k] != kDropped) v[k] = rec_value<R>(r[k], bp.value, f);
        }
        if (sample) {
#pragma unroll
            for (int k = 0; k < kRPT; ++k) {
                if (st[k] >= kKeptAll) continue;
                const uint64_t key = RecOps<R>::key(r[k], f);
                rkey[k] = rec_prio(bp.seed, (uint64_t)(bp.pid_min + (int64_t)pidv[qs[k]]),
                                   (uint32_t)(key & pkmask),
                                   (uint64_t)(bp.rec_base + RecOps<R>::idx(r[k], f)));
                pool[st[k] + (atomicAdd(&pairst[ps[k]], 1u << 16) >> 16)] = rkey[k];
            }
            __syncthreads();
        }
        mark(bp, 6, clk);
        // ---- F: a sampled record is kept iff fewer than mcpp records of its
        // pair have a smaller key; accumulators of kept records
        if (need_v) {
#pragma unroll
            for (int k = 0; k < kRPT; ++k) {
                if (st[k] == kDropped) continue;
                if (st[k] != kKeptAll &&
                    rank_below(pool + st[k], paircnt[ps[k]], rkey[k]) >= bp.mcpp)
                    continue;
                const uint32_t p = ps[k];
                if (part_clip) {
                    atomicAdd(&acc_sum[p], v[k]);
                } else {
                    const double x = clampd(v[k], bp.lo, bp.hi);
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
        // ---- PER_PRIVACY_ID: records of pids over L append their record key
        // to the pid's pool region; a record is kept iff fewer than L records
        // of its pid have a smaller key; pairst counts kept records per pair
        uint64_t rkey[kRPT];
        uint32_t s[kRPT];
#pragma unroll
        for (int k = 0; k < kRPT; ++k) {
            rkey[k] = 0;
            s[k] = kNil;
            if (!valid[k]) continue;
            s[k] = pidslot[qs[k]];
            if (s[k] == kNil) continue;
            const uint64_t key = RecOps<R>::key(r[k], f);
            rkey[k] = rec_prio(bp.seed, (uint64_t)(bp.pid_min + (int64_t)pidv[qs[k]]),
                               (uint32_t)(key & pkmask),
                               (uint64_t)(bp.rec_base + RecOps<R>::idx(r[k], f)));
            pool[s[k] + (atomicAdd(&pidm[qs[k]], 1u << 16) >> 16)] = rkey[k];
        }
        __syncthreads();
        mark(bp, 5, clk);
#pragma unroll
        for (int k = 0; k < kRPT; ++k) {
            if (!valid[k]) continue;
            if (s[k] != kNil && rank_below(pool + s[k], pidm[qs[k]] & 0xFFFFu, rkey[k]) >= bp.L)
                continue;
            const uint32_t p = ps[k];
            atomicAdd(&pairst[p], 1u);
            if (need_v) {
                const double v = rec_value<R>(r[k], bp.value, f);
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
        for (int j = 0; j < kPPT; ++j) {
            const uint32_t li = tid + j * kBT;
            pslot_of[j] = li < npair ? plist[li] : 0u;
            ecnt[j] = li < npair ? pairst[pslot_of[j]] : 0u;
            emit[j] = ecnt[j] > 0;
        }
    }
    // ---- G: emit kept pairs (pair-major, dense); clear the tables for the
    // next chunk
    if constexpr (ItemTraits<Item>::preagg) {
        // pid leader (leader bit set): the pair with the smallest slot of its
        // privacy id (pidv is dead here; phase B rewrites it per chunk)
#pragma unroll
        for (int j = 0; j < kQPT; ++j) {
            const uint32_t li = tid + j * kBT;
            if (li < npid) pidv[qlist[li]] = 0xFFFFFFFFu;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kPPT; ++j)
            if (emit[j])
                atomicMin(&pidv[(uint32_t)(pairtab[pslot_of[j]] >> pkb) & (kCq - 1)], pslot_of[j]);
        __syncthreads();
    }
    uint32_t islot[kPPT];
    wave_alloc_batch<kPPT>(&sh->nitems, emit, islot);
#pragma unroll
    for (int j = 0; j < kPPT; ++j) {
        const uint32_t p = pslot_of[j];
        const uint32_t slot = islot[j];
        if (!emit[j]) continue;
        Item it;
        it.pk = (uint32_t)(pairtab[p] & (KeyT)pkmask);
        it.cnt = ecnt[j];
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
        if constexpr (ItemTraits<Item>::preagg) {
            const uint32_t q = (uint32_t)(pairtab[p] >> pkb) & (kCq - 1);
            const uint32_t pm = pidm[q];
            it.npart = pm & 0xFFFFu;
            it.nl = ItemPA::pack_nl(pm >> 16, pidv[q] == p);
        }
        items[slot] = it;
    }
    __syncthreads();
    // clear the occupied slots for the next chunk
#pragma unroll
    for (int j = 0; j < kPPT; ++j) {
        const uint32_t li = tid + j * kBT;
        if (li < npair) {
            const uint32_t p = plist[li];
            pairtab[p] = empty_key<KeyT>();
            paircnt[p] = 0;
        }
        if (li < npid) pidm[qlist[li]] = 0;
    }
    if (tid == 0) {
        sh->bump = 0;
        sh->bump2 = kMcppBase;
        sh->npair = 0;
        sh->npid = 0;
    }
    __syncthreads();
    mark(bp, 8, clk);
}

// Chunk descriptor: records [x, x + (y & kChunkCount)) of buffer (y >> 31),
// level-1 bucket z, pid hash-residual base w.  Heavy chunks (bit 30 of y,
// small-chunk list only, dpg_wave.h) hold the candidate records of one heavy
// privacy id in their own buffer, with the candidate cut in z >> 16.
constexpr uint32_t kChunkCount = 0x3FFFFFFFu;
constexpr uint32_t kChunkHeavy = 0x40000000u;
template <class R>
__device__ __forceinline__ const R *chunk_base(uint4 d, const R *b0, const R *b1) {
    return ((d.y >> 31) ? b1 : b0) + d.x;
}

// Persistent workgroups walk the chunk list statically (w, w + G, ...): the
// loop bound, the chunk size and every branch around a barrier are uniform.
// Workgroup g appends its items to its own region items[wg_off[g], ...) (the
// records of its chunks bound the count) and leaves the count in wg_cnt[g]:
// no global atomics in the loop.
template <class KeyT, class Item, class R>
__global__ __launch_bounds__(kBT) void k_bound_chunks(const R *recs, const R *refined,
                                                      const uint4 *chunks,
                                                      const uint32_t *n_chunks, BoundParams bp,
                                                      Item *items, const int64_t *wg_off,
                                                      uint32_t *wg_cnt) {
    using L = ChunkLayout<KeyT, Item>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    PhaseTimer clk;
    timer_start(bp, clk);
    const uint32_t nch = __builtin_amdgcn_readfirstlane(*n_chunks);
    ChunkShared *sh = reinterpret_cast<ChunkShared *>(smem + L::SH);
    Item *my_items = items + wg_off[blockIdx.x];
    clear_tables<KeyT, Item>(smem);
    if (threadIdx.x == 0) {
        sh->bump = 0;
        sh->bump2 = kMcppBase;
        sh->nitems = 0;
        sh->npair = 0;
        sh->npid = 0;
    }
    // software pipeline: records of chunk w in r, descriptor of w + G in dn;
    // the descriptor of w + 2G and the records of w + G load during w
    R r[kRPT], rn[kRPT];
    const uint32_t G = gridDim.x;
    uint32_t w = blockIdx.x;
    uint32_t n = 0, d1 = 0, hb = 0;
    uint4 dn = make_uint4(0, 0, 0, 0);
    if (w < nch) {
        const uint4 d = chunks[w];
        n = __builtin_amdgcn_readfirstlane(d.y & 0x7FFFFFFFu);
        d1 = __builtin_amdgcn_readfirstlane(d.z);
        hb = __builtin_amdgcn_readfirstlane(d.w);
        const R *b = chunk_base(d, recs, refined);
#pragma unroll
        for (int k = 0; k < kRPT; ++k) r[k] = b[min((uint32_t)(threadIdx.x + k * kBT), n - 1)];
        if (w + G < nch) dn = chunks[w + G];
    }
    __syncthreads();
    for (; w < nch; w += G) {
        uint4 dnn = make_uint4(0, 0, 0, 0);
        if (w + 2 * G < nch) dnn = chunks[w + 2 * G];
        const uint4 du = make_uint4(__builtin_amdgcn_readfirstlane(dn.x),
                                    __builtin_amdgcn_readfirstlane(dn.y),
                                    __builtin_amdgcn_readfirstlane(dn.z),
                                    __builtin_amdgcn_readfirstlane(dn.w));
        const uint32_t nn = du.y & 0x7FFFFFFFu;
        bound_chunk<KeyT, Item, R>(r, n, d1, hb, chunk_base(du, recs, refined), nn, rn, smem,
                                   bp, my_items, clk);
#pragma unroll
        for (int k = 0; k < kRPT; ++k) r[k] = rn[k];
        n = nn;
        d1 = du.z;
        hb = du.w;
        dn = dnn;
    }
    if (threadIdx.x == 0) wg_cnt[blockIdx.x] = sh->nitems;
    timer_flush(bp, clk);
}

// The medium chunks the streamed sort pass (dpg_sortb.h, tier 3) deferred
// (defer[w] set: more candidates than its working set holds): workgroup g2
// takes the streamed pass's workgroups g = g2, g2 + gridDim.x, ... (of G1)
// and bounds their flagged chunks, appending behind wg_cnt[g].
template <class KeyT, class Item, class R>
__global__ __launch_bounds__(kBT) void k_bound_chunks_deferred(
    const R *recs, const R *refined, const uint4 *chunks, const uint32_t *n_chunks, BoundParams bp,
    Item *items, const int64_t *wg_off, uint32_t *wg_cnt, const uint8_t *defer, uint32_t G1) {
    using L = ChunkLayout<KeyT, Item>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    PhaseTimer clk;
    timer_start(bp, clk);
    const uint32_t nch = __builtin_amdgcn_readfirstlane(*n_chunks);
    ChunkShared *sh = reinterpret_cast<ChunkShared *>(smem + L::SH);
    clear_tables<KeyT, Item>(smem);
    if (threadIdx.x == 0) {
        sh->bump = 0;
        sh->bump2 = kMcppBase;
        sh->npair = 0;
        sh->npid = 0;
    }
    R r[kRPT], rn[kRPT];
    for (uint32_t g = blockIdx.x; g < G1; g += gridDim.x) {
        __syncthreads();
        if (threadIdx.x == 0) sh->nitems = wg_cnt[g];
        bool any = false;
        for (uint32_t w = g; w < nch; w += G1) {
            if (!__builtin_amdgcn_readfirstlane((int)defer[w])) continue;  // one flag per chunk
            any = true;
            const uint4 d = make_uint4(__builtin_amdgcn_readfirstlane(chunks[w].x),
                                       __builtin_amdgcn_readfirstlane(chunks[w].y),
                                       __builtin_amdgcn_readfirstlane(chunks[w].z),
                                       __builtin_amdgcn_readfirstlane(chunks[w].w));
            const uint32_t n = d.y & kChunkCount;
            const R *b = chunk_base(d, recs, refined);
#pragma unroll
            for (int k = 0; k < kRPT; ++k) r[k] = b[min((uint32_t)(threadIdx.x + k * kBT), n - 1)];
            __syncthreads();
            bound_chunk<KeyT, Item, R>(r, n, d.z, d.w, b, 0u, rn, smem, bp, items + wg_off[g], clk);
        }
        __syncthreads();
        if (any && threadIdx.x == 0) wg_cnt[g] = sh->nitems;
    }
    timer_flush(bp, clk);
}

// Oversize buckets (start, count, level-1 bucket, residual base) appended to
// the medium-chunk list behind its n_m0 entries (sel: the buffer they live
// in), for the streamed sort pass (dpg_sortb.h tier 3).
__global__ void k_over_to_medium(const int64_t *st, const uint32_t *cnt, const uint32_t *d1,
                                 const uint32_t *hb, uint32_t n, uint32_t sel, uint4 *mchunks,
                                 uint32_t *n_mchunks, uint32_t n_m0) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) mchunks[n_m0 + i] = make_uint4((uint32_t)st[i], cnt[i] | (sel << 31), d1[i], hb[i]);
    if (i == 0) *n_mchunks = n_m0 + n;
}

// wg_rec[g] = records of the chunks workgroup g of G will process (w = g mod G)
__global__ __launch_bounds__(256) void k_wg_records(const uint4 *chunks, const uint32_t *n_chunks,
                                                    uint32_t G, uint32_t *wg_rec) {
    __shared__ uint32_t part[4];
    const uint32_t nch = *n_chunks, g = blockIdx.x;
    uint32_t acc = 0;
    for (uint32_t w = g + threadIdx.x * G; w < nch; w += 256 * G) acc += chunks[w].y & kChunkCount;
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) wg_rec[g] = part[0] + part[1] + part[2] + part[3];
}

// out[i] = sum(in[0, i)) for i <= m (one workgroup, 1024 entries per round);
// optionally *total32 = out[m]
__global__ __launch_bounds__(1024) void k_scan_small(const uint32_t *in, uint32_t m, int64_t *out,
                                                     uint32_t *total32) {
    __shared__ int64_t sh[1024];
    __shared__ int64_t carry;
    const uint32_t t = threadIdx.x;
    if (t == 0) carry = 0;
    __syncthreads();
    for (uint32_t b = 0; b <= m; b += 1024) {
        const uint32_t i = b + t;
        sh[t] = i < m ? (int64_t)in[i] : 0;
        __syncthreads();
        for (uint32_t o = 1; o < 1024; o <<= 1) {
            int64_t x = t >= o ? sh[t - o] : 0;
            __syncthreads();
            sh[t] += x;
            __syncthreads();
        }
        if (i <= m) out[i] = carry + (t ? sh[t - 1] : 0);
        __syncthreads();
        if (t == 0) carry += sh[1023];
        __syncthreads();
    }
    if (t == 0 && total32) *total32 = (uint32_t)carry;
}

// Greedy packing of consecutive fine buckets into small chunks of <= capS
// records (single-wave kernel, dpg_wave.h), one thread per group of `group`
// buckets; a group never spans two level-1 buckets: bucket b belongs to
// level-1 bucket b >> d1_shift (group divides 1 << d1_shift), or to
// d1_map[b >> d1_shift] for refined buckets.  A bucket's pid hash-residual
// base is (b mod 2^d1_shift) << plb (plus hb_map[b >> d1_shift] for refined
// buckets); a small chunk spans at most kWCq >> plb bucket indices, so its
// pid slots (residual - chunk base) stay below kWCq.  Buckets of (capS, capM]
// records become single-bucket medium chunks (workgroup kernel above), larger
// ones go to the oversize list (start, count, level-1 bucket, residual base).
// sel = buffer the buckets live in.
__global__ __launch_bounds__(256) void k_make_chunks(
    const int64_t *bstart, const uint32_t *bcnt, uint32_t B, uint32_t group, uint32_t capS,
    uint32_t capM, uint32_t sel, uint32_t d1_shift, const uint32_t *d1_map, const uint32_t *hb_map,
    uint32_t plb, uint4 *chunks, uint32_t *n_chunks, uint4 *mchunks, uint32_t *n_mchunks,
    int64_t *over_start, uint32_t *over_cnt, uint32_t *over_d1, uint32_t *over_hb,
    uint32_t *n_over, unsigned long long *over_records) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t b0 = g * group;
    const bool active = b0 < B;  // every lane takes part in the reservations below
    const uint32_t b1 = active ? min(B, b0 + group) : b0;
    const uint32_t maxspan = max(1u, kWCq >> plb);
    const uint32_t lmask = (1u << d1_shift) - 1u;
    const uint32_t d1 = !active ? 0u : d1_map ? d1_map[b0 >> d1_shift] : (b0 >> d1_shift);
    const uint32_t hb0 = active && hb_map ? hb_map[b0 >> d1_shift] : 0u;
    // the group's first kMkPre counts and starts, all loads in flight at
    // once (the two passes below used to load them bucket by bucket: 0.25
    // ms of dependent loads at config 2 for 48 MB); a group of more buckets
    // (the refine level's) reads the rest directly
    constexpr uint32_t kMkPre = 32;
    uint32_t cpre[kMkPre];
    int64_t spre[kMkPre];
#pragma unroll
    for (uint32_t j = 0; j < kMkPre; ++j) {
        const uint32_t b = active ? min(b0 + j, b1 - 1) : 0u;
        cpre[j] = active ? bcnt[b] : 0u;
        spre[j] = active ? bstart[b] : 0;
    }
    // pass 1: count small chunks, medium chunks, oversize buckets (records)
    uint32_t nc = 0, nm = 0, no = 0, cur = 0, bfirst = 0;
    double orec = 0.0;  // exact: < 2^53
    int64_t cend = -1;
    auto count_step = [&](uint32_t b, uint32_t c, int64_t st) {
        if (c == 0) return;
        if (c > capM) {
            ++no;
            orec += (double)c;
            return;
        }
        if (c > capS) {
            ++nm;
            return;
        }
        if (cur == 0 || cur + c > capS || st != cend || b - bfirst >= maxspan) {
            ++nc;
            cur = 0;
            bfirst = b;
        }
        cur += c;
        cend = st + c;
    };
#pragma unroll
    for (uint32_t j = 0; j < kMkPre; ++j)
        if (b0 + j < b1) count_step(b0 + j, cpre[j], spre[j]);
    for (uint32_t b = b0 + kMkPre; b < b1; ++b) count_step(b, bcnt[b], bstart[b]);
    // one reservation per wave and list (per-entry atomics on one counter
    // serialise in L2: 0.9 ms for config 2's buckets at a 384-record cap)
    uint32_t tc, tm, to;
    uint32_t base = wave_excl_scan(nc, tc), mbase = wave_excl_scan(nm, tm),
             obase = wave_excl_scan(no, to);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) orec += __shfl_xor(orec, o, 64);
    uint32_t rc = 0, rm = 0, ro = 0;
    if (__lane_id() == 0) {
        if (tc) rc = atomicAdd(n_chunks, tc);
        if (tm) rm = atomicAdd(n_mchunks, tm);
        if (to) {
            ro = atomicAdd(n_over, to);
            atomicAdd(over_records, (unsigned long long)orec);
        }
    }
    base += __builtin_amdgcn_readfirstlane(rc);
    mbase += __builtin_amdgcn_readfirstlane(rm);
    obase += __builtin_amdgcn_readfirstlane(ro);
    if (!active) return;
    // pass 2: write
    cur = 0;
    cend = -1;
    bfirst = 0;
    int64_t cst = 0;
    auto write_step = [&](uint32_t b, uint32_t c, int64_t st) {
        if (c == 0) return;
        const uint32_t hb = hb0 + ((b & lmask) << plb);
        if (c > capM) {
            const uint32_t o = obase++;
            over_start[o] = st;
            over_cnt[o] = c;
            over_d1[o] = d1;
            over_hb[o] = hb;
            return;
        }
        if (c > capS) {
            mchunks[mbase++] = make_uint4((uint32_t)st, c | (sel << 31), d1, hb);
            return;
        }
        if (cur == 0 || cur + c > capS || st != cend || b - bfirst >= maxspan) {
            if (cur)
                chunks[base++] = make_uint4((uint32_t)cst, cur | (sel << 31), d1,
                                            hb0 + ((bfirst & lmask) << plb));
            cur = 0;
            cst = st;
            bfirst = b;
        }
        cur += c;
        cend = st + c;
    };
#pragma unroll
    for (uint32_t j = 0; j < kMkPre; ++j)
        if (b0 + j < b1) write_step(b0 + j, cpre[j], spre[j]);
    for (uint32_t b = b0 + kMkPre; b < b1; ++b) write_step(b, bcnt[b], bstart[b]);
    if (cur)
        chunks[base++] =
            make_uint4((uint32_t)cst, cur | (sel << 31), d1, hb0 + ((bfirst & lmask) << plb));
}

}  // namespace dpg
