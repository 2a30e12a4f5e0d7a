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
constexpr uint32_t kPool = 2048;     // cascade slots: mpc in [0, 1024), mcpp above
constexpr uint32_t kMcppBase = 1024;
constexpr int kQPT = kCq / kBT;      // pid slots per thread
constexpr int kPPT = kCp / kBT;      // pair slots per thread

struct ChunkShared {
    uint32_t bump, bump2, nitems, pad;
};

// LDS layout of one workgroup (KeyT: pair key width).
template <class KeyT, class Item>
struct ChunkLayout {
    static constexpr bool var = ItemTraits<Item>::var;
    static constexpr size_t PIDTAB = 0;
    static constexpr size_t PIDM = PIDTAB + 4 * kCq;  // low 16: pairs/records, high: candidates
    static constexpr size_t PIDSLOT = PIDM + 4 * kCq;
    static constexpr size_t PAIRTAB = PIDSLOT + 4 * kCq;
    static constexpr size_t PAIRCNT = PAIRTAB + sizeof(KeyT) * kCp;
    static constexpr size_t PAIRST = PAIRCNT + 4 * kCp;
    static constexpr size_t POOL = PAIRST + 4 * kCp;
    static constexpr size_t ACC = POOL + 8 * kPool;
    static constexpr size_t SH = ACC + 8 * kCp * (var ? 3 : 1);
    static constexpr size_t TOTAL = SH + sizeof(ChunkShared);
    static constexpr int PER_CU = TOTAL <= 53 * 1024 ? 3 : 2;
    static_assert(TOTAL <= 80 * 1024, "chunk working set too large");
};

template <class KeyT, class Item>
__device__ __forceinline__ void clear_tables(char *smem) {
    using L = ChunkLayout<KeyT, Item>;
    uint32_t *pidtab = reinterpret_cast<uint32_t *>(smem + L::PIDTAB);
    uint32_t *pidm = reinterpret_cast<uint32_t *>(smem + L::PIDM);
    KeyT *pairtab = reinterpret_cast<KeyT *>(smem + L::PAIRTAB);
    uint32_t *paircnt = reinterpret_cast<uint32_t *>(smem + L::PAIRCNT);
#pragma unroll
    for (int j = 0; j < kQPT; ++j) {
        pidtab[threadIdx.x + j * kBT] = kEmpty32;
        pidm[threadIdx.x + j * kBT] = 0;
    }
#pragma unroll
    for (int j = 0; j < kPPT; ++j) {
        pairtab[threadIdx.x + j * kBT] = empty_key<KeyT>();
        paircnt[threadIdx.x + j * kBT] = 0;
    }
}

template <class KeyT, class Item, class R>
__device__ __forceinline__ void bound_chunk(const R (&r)[kRPT], uint32_t n, uint32_t d1,
                                            const R *next_base, uint32_t next_n,
                                            R (&rn)[kRPT], char *smem, const BoundParams &bp,
                                            Item *items, PhaseTimer &clk) {
    using L = ChunkLayout<KeyT, Item>;
    constexpr bool kVar = L::var;
    uint32_t *pidtab = reinterpret_cast<uint32_t *>(smem + L::PIDTAB);
    uint32_t *pidm = reinterpret_cast<uint32_t *>(smem + L::PIDM);
    uint32_t *pidslot = reinterpret_cast<uint32_t *>(smem + L::PIDSLOT);
    KeyT *pairtab = reinterpret_cast<KeyT *>(smem + L::PAIRTAB);
    uint32_t *paircnt = reinterpret_cast<uint32_t *>(smem + L::PAIRCNT);
    uint32_t *pairst = reinterpret_cast<uint32_t *>(smem + L::PAIRST);
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

    // ---- A: pid and pair inserts, counts (record-major)
    uint32_t qs[kRPT], ps[kRPT];
#pragma unroll
    for (int k = 0; k < kRPT; ++k) {
        const uint32_t i = tid + k * kBT;
        qs[k] = ps[k] = 0;
        if (i < n) {
            const uint64_t key = RecOps<R>::key(r[k], f);
            bool wq, wp;
            qs[k] = insert_key<uint32_t>(pidtab, kCq - 1, (uint32_t)(key >> pkb), wq, bp.err);
            if (per_pid) atomicAdd(&pidm[qs[k]], 1u);
            const KeyT pkey = ((KeyT)qs[k] << pkb) | (KeyT)(key & pkmask);
            ps[k] = insert_key<KeyT>(pairtab, kCp - 1, pkey, wp, bp.err);
            atomicAdd(&paircnt[ps[k]], 1u);
            if (!per_pid && wp) atomicAdd(&pidm[qs[k]], 1u);
        }
    }
    __syncthreads();
    mark(bp, 2, clk);
    // prefetch the next chunk's records (in flight during the phases below)
#pragma unroll
    for (int k = 0; k < kRPT; ++k) {
        const uint32_t i = tid + k * kBT;
        if (i < next_n) rn[k] = next_base[i];
    }
    // ---- B: cascade slots for pids over their limit (pid-major); pair
    // accumulators / counters (pair-major)
#pragma unroll
    for (int j = 0; j < kQPT; ++j) {
        const uint32_t q = tid + j * kBT;
        const bool occ = pidtab[q] != kEmpty32;
        const bool want = occ && (pidm[q] & 0xFFFFu) > lim;
        const uint32_t s = wave_alloc(&sh->bump, want, lim);
        if (want)
            for (uint32_t t = 0; t < lim; ++t) pool[s + t] = kEmpty64;
        if (occ) pidslot[q] = want ? s : kNil;
    }
#pragma unroll
    for (int j = 0; j < kPPT; ++j) {
        const uint32_t p = tid + j * kBT;
        if (pairtab[p] == empty_key<KeyT>()) continue;
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
    uint32_t ecnt[kPPT];
    if (!per_pid) {
        // ---- C: mpc cascade over pair keys (pair-major): candidates first,
        // then the rare completion pass for pids with < mpc candidates
        uint64_t k64[kPPT];
        uint32_t pslot[kPPT];
        bool over[kPPT], cand[kPPT];
#pragma unroll
        for (int j = 0; j < kPPT; ++j) {
            const uint32_t p = tid + j * kBT;
            const KeyT pkey = pairtab[p];
            over[j] = cand[j] = false;
            k64[j] = 0;
            pslot[j] = kNil;
            if (pkey == empty_key<KeyT>()) continue;
            const uint32_t q = (uint32_t)(pkey >> pkb);
            const uint32_t s = pidslot[q];
            pslot[j] = s;
            if (s == kNil) continue;
            over[j] = true;
            const uint32_t pk = (uint32_t)(pkey & (KeyT)pkmask);
            const uint32_t pr = pair_prio(bp.seed, pid_of(bp, d1, pidtab[q]), pk);
            k64[j] = ((uint64_t)pr << 32) | pk;
            cand[j] = pr < cand_threshold(pidm[q] & 0xFFFFu, bp.mpc);
            if (cand[j]) {
                cascade_insert(pool + s, bp.mpc, k64[j]);
                atomicAdd(&pidm[q], 1u << 16);
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kPPT; ++j) {
            if (!over[j] || cand[j]) continue;
            const uint32_t q = (uint32_t)(pairtab[tid + j * kBT] >> pkb);
            if ((pidm[q] >> 16) < bp.mpc) cascade_insert(pool + pslot[j], bp.mpc, k64[j]);
        }
        __syncthreads();
        mark(bp, 4, clk);
        // ---- D: pair state; mcpp cascade slots for over-full kept pairs
#pragma unroll
        for (int j = 0; j < kPPT; ++j) {
            const uint32_t p = tid + j * kBT;
            const bool occ = pairtab[p] != empty_key<KeyT>();
            const bool kept = occ && (!over[j] || k64[j] <= pool[pslot[j] + bp.mpc - 1]);
            const uint32_t c = occ ? paircnt[p] : 0u;
            const bool need = sample && kept && c > bp.mcpp;
            const uint32_t b2 = wave_alloc(&sh->bump2, need, bp.mcpp);
            if (need)
                for (uint32_t t = 0; t < bp.mcpp; ++t) pool[b2 + t] = kEmpty64;
            if (occ) pairst[p] = !kept ? kDropped : (need ? b2 : kKeptAll);
            emit[j] = kept;
            ecnt[j] = bp.mode == DPG_MODE_CROSS_AND_PER_PARTITION ? min(c, bp.mcpp) : c;
        }
        __syncthreads();
        mark(bp, 5, clk);
        // ---- E: mcpp cascade over record keys inside over-full kept pairs;
        // the values of records of kept pairs are gathered meanwhile
        uint64_t rkey[kRPT];
        double v[kRPT];
        uint32_t st[kRPT];
#pragma unroll
        for (int k = 0; k < kRPT; ++k) {
            const uint32_t i = tid + k * kBT;
            rkey[k] = 0;
            v[k] = 0.0;
            st[k] = kDropped;
            if (i >= n) continue;
            st[k] = pairst[ps[k]];
            if (need_v && st[k] != kDropped) v[k] = bp.value[RecOps<R>::idx(r[k], f)];
        }
        if (sample) {
#pragma unroll
            for (int k = 0; k < kRPT; ++k) {
                if (st[k] >= kKeptAll) continue;
                const uint64_t key = RecOps<R>::key(r[k], f);
                rkey[k] = rec_prio(bp.seed, pid_of(bp, d1, pidtab[qs[k]]),
                                   (uint32_t)(key & pkmask),
                                   (uint64_t)(bp.rec_base + RecOps<R>::idx(r[k], f)));
                cascade_insert(pool + st[k], bp.mcpp, rkey[k]);
            }
            __syncthreads();
        }
        mark(bp, 6, clk);
        // ---- F: accumulators of kept records
        if (need_v) {
#pragma unroll
            for (int k = 0; k < kRPT; ++k) {
                if (st[k] == kDropped) continue;
                if (st[k] != kKeptAll && rkey[k] > pool[st[k] + bp.mcpp - 1]) continue;
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
        // ---- PER_PRIVACY_ID: keep the L records of each pid with the
        // smallest record key; pairst counts kept records per pair
        uint64_t rkey[kRPT];
        uint32_t s[kRPT];
#pragma unroll
        for (int k = 0; k < kRPT; ++k) {
            const uint32_t i = tid + k * kBT;
            rkey[k] = 0;
            s[k] = kNil;
            if (i >= n) continue;
            s[k] = pidslot[qs[k]];
            if (s[k] == kNil) continue;
            const uint64_t key = RecOps<R>::key(r[k], f);
            rkey[k] = rec_prio(bp.seed, pid_of(bp, d1, pidtab[qs[k]]), (uint32_t)(key & pkmask),
                               (uint64_t)(bp.rec_base + RecOps<R>::idx(r[k], f)));
            cascade_insert(pool + s[k], bp.L, rkey[k]);
        }
        __syncthreads();
        mark(bp, 5, clk);
#pragma unroll
        for (int k = 0; k < kRPT; ++k) {
            const uint32_t i = tid + k * kBT;
            if (i >= n) continue;
            if (s[k] != kNil && rkey[k] > pool[s[k] + bp.L - 1]) continue;
            const uint32_t p = ps[k];
            atomicAdd(&pairst[p], 1u);
            if (need_v) {
                const double v = bp.value[RecOps<R>::idx(r[k], f)];
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
            const uint32_t p = tid + j * kBT;
            const bool occ = pairtab[p] != empty_key<KeyT>();
            ecnt[j] = occ ? pairst[p] : 0u;
            emit[j] = ecnt[j] > 0;
        }
    }
    // ---- G: emit kept pairs (pair-major); clear the tables for the next chunk
#pragma unroll
    for (int j = 0; j < kPPT; ++j) {
        const uint32_t p = tid + j * kBT;
        const uint32_t slot = wave_alloc(&sh->nitems, emit[j]);
        if (!emit[j]) continue;
        Item it;
        it.pk = (uint32_t)(pairtab[p] & (KeyT)pkmask);
        it.cnt = ecnt[j];
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
        items[slot] = it;
    }
    __syncthreads();
    clear_tables<KeyT, Item>(smem);
    if (tid == 0) {
        sh->bump = 0;
        sh->bump2 = kMcppBase;
    }
    __syncthreads();
    mark(bp, 8, clk);
}

// Chunk descriptor: records [x, x + (y & 0x7FFFFFFF)) of buffer (y >> 31),
// level-1 bucket z.
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
    }
    // software pipeline: records of chunk w in r, descriptor of w + G in dn;
    // the descriptor of w + 2G and the records of w + G load during w
    R r[kRPT], rn[kRPT];
    const uint32_t G = gridDim.x;
    uint32_t w = blockIdx.x;
    uint32_t n = 0, d1 = 0;
    uint4 dn = make_uint4(0, 0, 0, 0);
    if (w < nch) {
        const uint4 d = chunks[w];
        n = __builtin_amdgcn_readfirstlane(d.y & 0x7FFFFFFFu);
        d1 = __builtin_amdgcn_readfirstlane(d.z);
        const R *b = chunk_base(d, recs, refined);
#pragma unroll
        for (int k = 0; k < kRPT; ++k) {
            const uint32_t i = threadIdx.x + k * kBT;
            if (i < n) r[k] = b[i];
        }
        if (w + G < nch) dn = chunks[w + G];
    }
    __syncthreads();
    for (; w < nch; w += G) {
        uint4 dnn = make_uint4(0, 0, 0, 0);
        if (w + 2 * G < nch) dnn = chunks[w + 2 * G];
        const uint4 du = make_uint4(__builtin_amdgcn_readfirstlane(dn.x),
                                    __builtin_amdgcn_readfirstlane(dn.y),
                                    __builtin_amdgcn_readfirstlane(dn.z), 0u);
        const uint32_t nn = du.y & 0x7FFFFFFFu;
        bound_chunk<KeyT, Item, R>(r, n, d1, chunk_base(du, recs, refined), nn, rn, smem, bp,
                                   my_items, clk);
#pragma unroll
        for (int k = 0; k < kRPT; ++k) r[k] = rn[k];
        n = nn;
        d1 = du.z;
        dn = dnn;
    }
    if (threadIdx.x == 0) wg_cnt[blockIdx.x] = sh->nitems;
    timer_flush(bp, clk);
}

// wg_rec[g] = records of the chunks workgroup g of G will process (w = g mod G)
__global__ __launch_bounds__(256) void k_wg_records(const uint4 *chunks, const uint32_t *n_chunks,
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
// one thread per group of `group` buckets; a group never spans two level-1
// buckets: bucket b belongs to level-1 bucket b >> d1_shift, or to
// d1_map[b >> d1_shift] when a map is given (refined buckets), and group
// divides 1 << d1_shift.  Buckets larger than cap go to the oversize list
// (start, count, level-1 bucket).  sel = buffer the buckets live in.
__global__ void k_make_chunks(const int64_t *bstart, const uint32_t *bcnt, uint32_t B,
                              uint32_t group, uint32_t cap, uint32_t sel, uint32_t d1_shift,
                              const uint32_t *d1_map, uint4 *chunks, uint32_t *n_chunks,
                              int64_t *over_start, uint32_t *over_cnt, uint32_t *over_d1,
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
    const uint32_t d1 = d1_map ? d1_map[b0 >> d1_shift] : (b0 >> d1_shift);
    for (uint32_t b = b0; b < b1; ++b) {
        const uint32_t c = bcnt[b];
        if (c == 0) continue;
        const int64_t st = bstart[b];
        if (c > cap) {
            const uint32_t o = atomicAdd(n_over, 1u);
            over_start[o] = st;
            over_cnt[o] = c;
            over_d1[o] = d1;
            atomicAdd(over_records, (unsigned long long)c);
            continue;
        }
        if (cur == 0 || cur + c > cap || st != cend) {
            if (cur) chunks[base++] = make_uint4((uint32_t)cst, cur | (sel << 31), d1, 0u);
            cur = 0;
            cst = st;
        }
        cur += c;
        cend = st + c;
    }
    if (cur) chunks[base++] = make_uint4((uint32_t)cst, cur | (sel << 31), d1, 0u);
}

}  // namespace dpg
