// dpg_wave.h -- contribution bounding of small chunks by single waves (gfx950).
//
// The hot path of the bound stage.  Every 64-lane workgroup is one wave that
// owns a private ~17 KB LDS working set and walks its share of the chunk list
// (chunks of <= kWCap = 512 records: the fine buckets of the partition
// levels, packed).  Nothing is shared between waves, so there is no
// workgroup barrier at all: phases are ordered by the wave's own program
// order (LDS instructions of one wave execute in order; a wavefront fence
// keeps the compiler from reordering them), counters live in scalar
// registers and allocations are ballot + mbcnt instead of LDS atomics.
// Nine such waves share a CU, so one wave's LDS round trips overlap the
// others' work.
//
// Per chunk (same algorithm as dpg_bound.h / dpg_chunk.h, identical results):
//   A  pair inserts (pid slot = pid hash residual - chunk base: direct, no
//      table), counts, dense pair / pid lists, pid values
//   B  every pid over its limit reserves one pool slot per pair (record in
//      PER_PRIVACY_ID mode)
//   C  mpc selection: candidates (priority below a per-pid threshold) append
//      their pair key to the pid's pool region and are kept iff fewer than
//      mpc candidates have a smaller key; pids short of candidates rank their
//      non-candidates too (rare)          (contribution_bounders.py:90-92)
//   D  pair state; over-full kept pairs reserve one pool slot per record
//   E  their records append philox(seed, pid, pk, record id) keys; values of
//      records of kept pairs are gathered by record index
//   F  a sampled record is kept iff fewer than mcpp keys of its pair are
//      smaller (:74-76); clipped accumulators (combiners.py:255-500)
//   G  emit one Item per kept pair; clear the occupied slots
#pragma once

#include "dpg_chunk.h"

namespace dpg {


// Hide a uniform value from the compiler's uniformity analysis so that it
// lives in a VGPR: the wave kernel runs short of scalar registers (spills
// cost v_writelane / v_readlane issue slots), while vector registers have
// headroom.  For parameters used in few places only.
template <class T>
__device__ __forceinline__ T vreg(T x) {
    static_assert(sizeof(T) == 4 || sizeof(T) == 8, "vreg");
    asm volatile("" : "=v"(x) : "0"(x));
    return x;
}

template <class KeyT, class Item>
struct WaveLayout {
    static constexpr bool var = ItemTraits<Item>::var;
    static constexpr size_t PIDV = 0;                   // pid_hash of the privacy id
    static constexpr size_t PIDM = PIDV + 4 * kWCq;     // low 16: pairs/records, high: appends
    static constexpr size_t PIDSLOT = PIDM + 4 * kWCq;  // pool base (+ appends << 16) or kNil
    // pair key table (kWCk slots); once every insert has settled, a slot
    // holds its pair's dense id instead of the key
    static constexpr size_t CBND = PIDSLOT + 4 * kWCq;  // candidate bound per pid slot
    static constexpr size_t KEYS = CBND + 4 * kWCq;
    static constexpr size_t PKEY = KEYS + sizeof(KeyT) * kWCk;  // dense: pair key
    static constexpr size_t PCNT = PKEY + sizeof(KeyT) * kWCp;  // dense: records
    static constexpr size_t PST = PCNT + 4 * kWCp;              // dense: state
    static constexpr size_t POOL = PST + 4 * kWCp;
    static constexpr size_t ACC = POOL + 8 * kWPool;
    static constexpr size_t END = ACC + 8 * kWCp * (var ? (ItemTraits<Item>::sum ? 3 : 2) : 1);
    // padded to a multiple of 4 KB so that the allocation granularity of LDS
    // cannot cost a resident wave (20 KB: 8 per CU)
    static constexpr size_t TOTAL = (END + 4095) & ~(size_t)4095;
    static constexpr int PER_CU = (int)((160 * 1024) / TOTAL) < 16 ? (int)((160 * 1024) / TOTAL) : 16;
    static_assert(TOTAL <= 40 * 1024, "wave working set too large");
    static_assert(8 * kWPool >= sizeof(KeyT) * kWCap, "pool hosts the dummy CAS words");
    static_assert(KEYS % 16 == 0, "key table cleared by 16-byte stores");
};

#ifndef DPG_RT_W
#define DPG_RT_W 8
#endif
// same-box A/B, config 2: late gathers cut the value traffic of the
// bounding kernel but cost 13.0 -> 13.75 ms (their latency is exposed)
#ifndef DPG_LATE_GATHER
#define DPG_LATE_GATHER 0
#endif
// candidate bounds: round-0 mpc candidates ~ k + E0 sqrt(k) + E0 per pid,
// pre-filter ~ CAND x (k + 2 sqrt(k) + 2) records per pid (same-box A/B,
// config 2 / config 4 bound ms: (2.0, 2.0) 14.2 / 31.7; (1.5, 1.25) 13.1 /
// 29.6; (1.5, 1.0) 13.0 / 29.4-29.6; (1.0, 2.0) 19.9 -- restarts)
#ifndef DPG_E0_C
#define DPG_E0_C 1.25f
#endif
#ifndef DPG_CAND_C
#define DPG_CAND_C 1.5f
#endif

// Heavy chunks (k_heavy_filter): the candidate records of one privacy id
// whose bucket exceeds every LDS chunk, in their own buffer, kWCap slots per
// heavy bucket; the candidate bound is (cut << 20) - 1 with cut = z >> 16.
constexpr uint32_t kHvBins = 4096;  // cut granularity: 2^20 of the 2^32 priority range
__device__ __forceinline__ uint32_t heavy_bound(uint4 d) {
    if (!(d.y & kChunkHeavy)) return 0u;
    const uint32_t cut = d.z >> 16;
    return cut >= kHvBins ? 0xFFFFFFFFu : (cut << 20) - 1u;
}
template <class R>
__device__ __forceinline__ const R *wave_chunk_base(uint4 d, const R *recs, const R *refined,
                                                    const R *heavy) {
    return ((d.y & kChunkHeavy) ? heavy : (d.y >> 31) ? refined : recs) + d.x;
}

// Compiler-level ordering of one wave's LDS accesses between phases (the
// hardware already executes them in order).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Threshold search over key regions of the pool.  `mask` (uniform) selects
// lanes whose (vb, vc) describe a region [vb, vb + vc) with vc >= K keys; for
// every such region the K-th smallest key T is found and written over the
// region's first entry, so that a key of the region is among the K smallest
// iff it is <= T (keys are distinct).
//
// Regions of <= 64 keys are packed side by side into the wave's lanes (lane
// = one entry of one region); each lane counts the smaller keys of its own
// region, 4 per load batch, and the entry of rank K - 1 writes the
// threshold itself.  Larger regions (rare) take region_thresholds_wide.
__device__ __forceinline__ void region_thresholds_wide(uint64_t *pool, uint64_t mask, uint32_t vb,
                                                       uint32_t vc, uint32_t K) {
    const uint32_t lane = __lane_id();
    while (mask) {
        const int l = __builtin_ctzll(mask);
        mask &= mask - 1;
        const uint32_t sb = __builtin_amdgcn_readlane(vb, l);
        const uint32_t nc = __builtin_amdgcn_readlane(vc, l);
        if (nc <= 128) {
            // two entries per lane, one pass over the region's keys (mpc ~ 50:
            // k + 2 sqrt(k) + 2 candidates just above one wave)
            const uint64_t x0 = pool[sb + min(lane, nc - 1)];
            const uint64_t x1 = pool[sb + min(lane + 64u, nc - 1)];
            uint32_t r0 = 0, r1 = 0;
            for (uint32_t t = 0; t < nc; t += 8) {
                uint64_t y[8];
#pragma unroll
                for (int w = 0; w < 8; ++w) y[w] = pool[sb + min(t + w, nc - 1)];
#pragma unroll
                for (int w = 0; w < 8; ++w) {
                    const bool in = t + w < nc;
                    r0 += (in && y[w] < x0) ? 1u : 0u;
                    r1 += (in && y[w] < x1) ? 1u : 0u;
                }
            }
            // keys are distinct: exactly one entry has rank K - 1
            const uint64_t b0 = __ballot(r0 == K - 1 && lane < nc);
            const uint64_t b1 = __ballot(r1 == K - 1 && lane + 64u < nc);
            if (b0 | b1) {
                const int m = __builtin_ctzll(b0 ? b0 : b1);
                const uint64_t x = b0 ? x0 : x1;
                const uint64_t T = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(x >> 32), m) << 32) |
                                   __builtin_amdgcn_readlane((uint32_t)x, m);
                if (lane == 0) pool[sb] = T;
            } else if (lane == 0) {
                pool[sb] = ~0ull;
            }
            continue;
        }
        uint64_t T = ~0ull;
        for (uint32_t l0 = 0; l0 < nc; l0 += 64) {
            const uint32_t e = l0 + lane;
            const uint64_t x = pool[sb + min(e, nc - 1)];
            uint32_t rk = 0;
            for (uint32_t t = 0; t < nc; t += 4) {
                uint64_t y[4];
#pragma unroll
                for (int w = 0; w < 4; ++w) y[w] = pool[sb + min(t + w, nc - 1)];
#pragma unroll
                for (int w = 0; w < 4; ++w) rk += (t + w < nc && y[w] < x) ? 1u : 0u;
            }
            const uint64_t b = __ballot(e < nc && rk == K - 1);
            if (b) {
                const int m = __builtin_ctzll(b);
                T = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(x >> 32), m) << 32) |
                    __builtin_amdgcn_readlane((uint32_t)x, m);
            }
        }
        if (lane == 0) pool[sb] = T;
    }
}

// sel[j] (per lane) selects the region (vb[j], vc[j]) of slot j; regions of
// all J slots share the packed passes.
template <int J>
__device__ __forceinline__ void region_thresholds(uint64_t *pool, const bool (&sel)[J],
                                                  const uint32_t (&vb)[J], const uint32_t (&vc)[J],
                                                  uint32_t K) {
    const uint32_t lane = __lane_id();
    uint64_t mask[J];
    uint64_t any = 0;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        mask[j] = __ballot(sel[j]);
        const uint64_t big = mask[j] & __ballot(vc[j] > 64);
        mask[j] &= ~big;
        if (big) region_thresholds_wide(pool, big, vb[j], vc[j], K);
        any |= mask[j];
    }
    while (any) {
        // pack regions into lanes [off, off + c) until the wave is full
        uint32_t my_b = 0, my_c = 0, my_off = 0, used = 0, maxc = 0;
        bool full = false;
        any = 0;
#pragma unroll
        for (int j = 0; j < J; ++j) {
            for (uint64_t m = mask[j]; m && !full; m &= m - 1) {
                const int l = __builtin_ctzll(m);
                const uint32_t c = __builtin_amdgcn_readlane(vc[j], l);
                if (used + c > 64) {
                    full = true;
                    break;
                }
                const uint32_t b = __builtin_amdgcn_readlane(vb[j], l);
                const bool inr = lane >= used && lane < used + c;
                my_b = inr ? b : my_b;
                my_c = inr ? c : my_c;
                my_off = inr ? used : my_off;
                used += c;
                maxc = max(maxc, c);
                mask[j] &= ~(1ull << l);
            }
            any |= mask[j];
        }
        const bool act = lane < used;
        const uint32_t last = my_c ? my_c - 1 : 0u;
        const uint64_t x = pool[my_b + min(lane - my_off, last)];
        uint32_t rk = 0;
        constexpr int W = DPG_RT_W;
        for (uint32_t t = 0; t < maxc; t += W) {
            uint64_t y[W];
#pragma unroll
            for (int w = 0; w < W; ++w) y[w] = pool[my_b + min(t + w, last)];
#pragma unroll
            for (int w = 0; w < W; ++w) rk += (t + w < my_c && y[w] < x) ? 1u : 0u;
        }
        // every lane of the pass has read its region: the threshold may land
        if (act && rk == K - 1) pool[my_b] = x;
    }
}

// Records past the chunk end hold a copy of its last record (loads are
// unconditional); they aim their table CAS at lane-private dummy words and
// take part in nothing that counts.  Every phase is written stage-wise over
// the lane's kWRPT records / kWPPL pairs (all loads of a stage issued before
// any use), so one wave keeps many LDS round trips in flight.  Pairs get
// dense ids 0..npair-1 when they are created; every per-pair array is dense.
template <class KeyT, class Item, class R, bool kPerPid>
__device__ __forceinline__ uint32_t wave_chunk(const R (&r)[kWRPT], uint32_t n, uint32_t d1,
                                               uint32_t hbase, char *smem, const BoundParams &bp,
                                               Item *items, uint32_t nitems, PhaseTimer &clk,
                                               uint32_t hbound = 0, uint32_t hidx = 0) {
    using L = WaveLayout<KeyT, Item>;
    constexpr bool kVar = L::var;
    constexpr bool kSum = ItemTraits<Item>::sum;  // false: MEAN / VARIANCE moments only
    uint32_t *pidv = reinterpret_cast<uint32_t *>(smem + L::PIDV);
    uint32_t *pidm = reinterpret_cast<uint32_t *>(smem + L::PIDM);
    uint32_t *pidslot = reinterpret_cast<uint32_t *>(smem + L::PIDSLOT);
    KeyT *keys = reinterpret_cast<KeyT *>(smem + L::KEYS);
    KeyT *pkey_d = reinterpret_cast<KeyT *>(smem + L::PKEY);
    uint32_t *pcnt = reinterpret_cast<uint32_t *>(smem + L::PCNT);
    uint32_t *pst = reinterpret_cast<uint32_t *>(smem + L::PST);
    uint64_t *pool = reinterpret_cast<uint64_t *>(smem + L::POOL);
    double *acc_sum = reinterpret_cast<double *>(smem + L::ACC);
    double *acc_nsum = acc_sum + (kSum ? kWCp : 0);
    double *acc_nsq = acc_nsum + kWCp;

    const uint32_t lane = __lane_id();
    const Fmt f = bp.fmt;
    const uint32_t pkb = f.pkbits;
    const uint64_t pkmask = (1ull << pkb) - 1ull;
    constexpr bool per_pid = kPerPid;  // bp.mode == DPG_MODE_PER_PRIVACY_ID
    const bool need_v = bp.need_values != 0;
    const bool sample = bp.mode == DPG_MODE_CROSS_AND_PER_PARTITION && need_v;
    const bool part_clip = bp.sum_mode == DPG_SUM_CLIP_PARTITION;
    const uint32_t lim = per_pid ? bp.L : bp.mpc;
    const uint32_t hshift = f.kbits - f.b1;
    uint32_t kn = (n + 63) >> 6;  // occupied record slots per lane (uniform)

    // ---- A-: candidate pre-filter (cross-partition modes).  A pair's
    // priority is a function of (pid, pk), so every record of a pair shares
    // it: records whose priority is above a per-pid bound belong to pairs
    // the mpc sample can only keep if fewer than mpc pairs lie below it.
    // The bound aims at ~DPG_CAND_C x (mpc + 2 sqrt(mpc) + 2) records per
    // pid, so only those records are inserted into the pair table; a pid
    // left short of mpc candidate pairs restarts the chunk with every record
    // (rare).  Pids with <= mpc records keep all of them.
    uint32_t qs[kWRPT], dn[kWRPT];
    uint32_t validm = 0;  // per-lane bit k: record slot occupied
    uint32_t insm = 0;    // records inserted into the pair table
    uint32_t npair = 0;
    uint32_t *cbnd = reinterpret_cast<uint32_t *>(smem + L::CBND);
#pragma unroll
    for (int k = 0; k < kWRPT && k < (int)kn; ++k) {
        validm |= lane + 64u * k < n ? 1u << k : 0u;
        qs[k] = ((uint32_t)(RecOps<R>::key(r[k], f) >> pkb) - hbase) & (kWCq - 1);
    }
    if constexpr (!kPerPid) {
#pragma unroll
        for (int k = 0; k < kWRPT && k < (int)kn; ++k)
            if ((validm >> k) & 1u) atomicAdd(&pidslot[qs[k]], 1u);  // records per pid
        wave_sync();
    }
    // pid_hash of every pid slot of the chunk's residual range: 2 per lane,
    // no first-toucher detection (slots without a pid get a value nobody
    // reads); the candidate bound from the pid's record count
    if constexpr (!kPerPid) {
        // occupied slots only (typically a handful): compacted into lanes
        const float cmul = DPG_CAND_C * ((float)bp.mpc + 2.0f * sqrtf((float)bp.mpc) + 2.0f);
        uint32_t *olist = reinterpret_cast<uint32_t *>(pool);
        uint32_t nocc = 0;
#pragma unroll
        for (int j = 0; j < kWQPL; ++j) {
            const uint32_t q = lane + 64u * j;
            const bool occ = pidslot[q] > 0;
            const uint64_t bo = __ballot(occ);
            if (occ) olist[nocc + lanes_below(bo)] = q;
            else cbnd[q] = 0xFFFFFFFFu;
            nocc += (uint32_t)__popcll(bo);
        }
        wave_sync();
        for (uint32_t o = 0; o < nocc; o += 64) {
            if (o + lane < nocc) {
                const uint32_t q = olist[o + lane];
                pidv[q] = pid_hash(bp.seed, (uint64_t)(bp.pid_min + (int64_t)hk_inv(
                                                           (d1 << hshift) | (hbase + q), bp.hash)));
                const uint32_t rc = pidslot[q];
                const float fr = cmul / (float)rc;
                // a heavy chunk holds the candidates of one pid, filtered by
                // k_heavy_filter with the bound hbound
                cbnd[q] = hbound ? hbound
                                 : (rc <= bp.mpc || fr >= 1.0f ? 0xFFFFFFFFu
                                                               : (uint32_t)(fr * 4294967296.0f));
            }
        }
    } else {
        // pid_hash of every pid slot of the chunk's residual range: 2 per
        // lane (slots without a pid get a value nobody reads)
#pragma unroll
        for (int j = 0; j < kWQPL; ++j) {
            const uint32_t q = lane + 64u * j;
            pidv[q] = pid_hash(bp.seed, (uint64_t)(bp.pid_min + (int64_t)hk_inv(
                                                                     (d1 << hshift) | (hbase + q), bp.hash)));
        }
    }
    wave_sync();
    mark(bp, 10, clk);
    if constexpr (!kPerPid) {
        uint32_t pv[kWRPT], cb[kWRPT];
#pragma unroll
        for (int k = 0; k < kWRPT && k < (int)kn; ++k) {
            pv[k] = pidv[qs[k]];
            cb[k] = cbnd[qs[k]];
        }
#pragma unroll
        for (int k = 0; k < kWRPT && k < (int)kn; ++k) {
            const uint32_t pk = (uint32_t)(RecOps<R>::key(r[k], f) & pkmask);
            if (((validm >> k) & 1u) && pair_prio_h(pv[k], pk) <= cb[k]) insm |= 1u << k;
        }
    } else {
        insm = validm;
    }
    mark(bp, 11, clk);
    // the candidates, compacted into the first slots (pool + accumulator
    // area: idle until phase A), are the records the phases below work on;
    // a restart switches back to all of them
    R cur[kWRPT];
    uint32_t ncand = n;
    if constexpr (!kPerPid) {
        R *lst = reinterpret_cast<R *>(pool);
        static_assert(8 * kWPool + 8 * kWCp >= sizeof(R) * kWCap, "candidate list");
        ncand = 0;
#pragma unroll
        for (int k = 0; k < kWRPT && k < (int)kn; ++k) {
            const bool c = (insm >> k) & 1u;
            const uint64_t bc = __ballot(c);
            if (c) lst[ncand + lanes_below(bc)] = r[k];
            ncand += (uint32_t)__popcll(bc);
        }
        wave_sync();
#pragma unroll
        for (int k = 0; k < kWRPT; ++k)
            if (64u * k < ncand) cur[k] = lst[min(lane + 64u * k, ncand - 1)];
        wave_sync();
    }
    // ---- A: pair inserts: home-slot CAS of all records in flight; a record
    // whose home holds another key tries a second slot (other bits of the same
    // hash), then probes linearly from there -- one probe step of all of them
    // per round (table load <= 1/2; both choices taken ~ load^2)
    for (uint32_t round = (kPerPid || ncand == 0) ? 1u : 0u;; ++round) {
        // round 0: the compacted candidates; round 1: every record
        const uint32_t nn = round ? n : ncand;
        kn = (nn + 63) >> 6;
        validm = 0;
#pragma unroll
        for (int k = 0; k < kWRPT && k < (int)kn; ++k) {
            if (round) cur[k] = r[k];
            validm |= lane + 64u * k < nn ? 1u << k : 0u;
            qs[k] = ((uint32_t)(RecOps<R>::key(cur[k], f) >> pkb) - hbase) & (kWCq - 1);
        }
        insm = validm;
        uint32_t ps[kWRPT], alt[kWRPT], wonm = 0;
        KeyT pkey[kWRPT], op[kWRPT];
#pragma unroll
        for (int k = 0; k < kWRPT && k < (int)kn; ++k) {
            const bool valid = (insm >> k) & 1u;
            const uint64_t key = RecOps<R>::key(cur[k], f);
            pkey[k] = ((KeyT)qs[k] << pkb) | (KeyT)(key & pkmask);
            const uint32_t hh = hslot(pkey[k], 0xFFFFFFFFu);
            ps[k] = hh & (kWCk - 1);
            alt[k] = (hh >> 16) & (kWCk - 1);  // second choice (other hash bits)
            KeyT *tgt = valid ? keys + ps[k] : reinterpret_cast<KeyT *>(pool) + (lane + 64u * k);
            op[k] = cas_home<KeyT>(tgt, 0, pkey[k]);
        }
        mark(bp, 0, clk);
        uint32_t pend = 0;
#pragma unroll
        for (int k = 0; k < kWRPT && k < (int)kn; ++k) {
            if (!((insm >> k) & 1u)) continue;
            if (op[k] == empty_key<KeyT>()) wonm |= 1u << k;
            else if (op[k] != pkey[k]) pend |= 1u << k;
        }
        // records whose home slot holds another key are compacted into a
        // dense list (one per lane; the pool -- its dummy words are spent --
        // holds the keys, the idle accumulator area the second-choice slot
        // and the record's position) and probe there: second-choice slot,
        // then linearly; the final slot (and whether the record created the
        // entry) returns through the idle pair-state array by position
        {
            KeyT *ckey = reinterpret_cast<KeyT *>(pool);
            uint32_t *cmeta = reinterpret_cast<uint32_t *>(acc_sum);
            uint32_t *cres = pst;
            uint32_t npend = 0;
#pragma unroll
            for (int k = 0; k < kWRPT && k < (int)kn; ++k) {
                const bool pk_ = (pend >> k) & 1u;
                const uint64_t b = __ballot(pk_);
                if (pk_) {
                    const uint32_t e = npend + lanes_below(b);
                    ckey[e] = pkey[k];
                    cmeta[e] = alt[k] | ((lane + 64u * k) << 16);
                }
                npend += (uint32_t)__popcll(b);
            }
            if (npend) {
                wave_sync();
                for (uint32_t e0 = 0; e0 < npend; e0 += 64) {
                    const uint32_t e = min(e0 + lane, npend - 1);
                    const bool act = e0 + lane < npend;
                    const KeyT key = ckey[e];
                    const uint32_t meta = cmeta[e];
                    uint32_t slot = meta & 0xFFFFu;
                    bool done = !act, won = false;
                    for (uint32_t it = 0; __ballot(!done); ++it) {
                        if (it >= kWCk) {
                            if (!done) atomicOr(bp.err, 2u);
                            break;
                        }
                        if (!done) {
                            const KeyT o = cas_home<KeyT>(keys, slot, key);
                            if (o == empty_key<KeyT>()) {
                                won = true;
                                done = true;
                            } else if (o == key) {
                                done = true;
                            } else {
                                slot = (slot + 1) & (kWCk - 1);
                            }
                        }
                    }
                    if (act) cres[meta >> 16] = slot | (won ? 0x8000u : 0u);
                }
                wave_sync();
                uint32_t res[kWRPT];
#pragma unroll
                for (int k = 0; k < kWRPT && k < (int)kn; ++k) res[k] = cres[lane + 64u * k];
#pragma unroll
                for (int k = 0; k < kWRPT && k < (int)kn; ++k) {
                    if ((pend >> k) & 1u) {
                        ps[k] = res[k] & (kWCk - 1);
                        if (res[k] & 0x8000u) wonm |= 1u << k;
                    }
                }
            }
        }
        mark(bp, 9, clk);
        // winners: dense pair ids (the probing is over: slots now hold ids)
#pragma unroll
        for (int k = 0; k < kWRPT && k < (int)kn; ++k) {
            const bool won = (wonm >> k) & 1u;
            const uint64_t bw = __ballot(won);
            if (won) {
                const uint32_t d = npair + lanes_below(bw);
                keys[ps[k]] = (KeyT)d;
                pkey_d[d] = pkey[k];
                pcnt[d] = 0;
                if (need_v) {
                    if (kSum) acc_sum[d] = 0.0;
                    if (kVar) {
                        acc_nsum[d] = 0.0;
                        acc_nsq[d] = 0.0;
                    }
                }
                if (per_pid) pst[d] = 0;
            }
            npair += (uint32_t)__popcll(bw);
        }
        wave_sync();
#pragma unroll
        for (int k = 0; k < kWRPT && k < (int)kn; ++k) dn[k] = min((uint32_t)keys[ps[k]], kWCp - 1);
        // counts: records per pair; pairs (records in PER_PRIVACY_ID mode)
        // per pid
        const uint32_t touchm = per_pid ? insm : wonm;
#pragma unroll
        for (int k = 0; k < kWRPT && k < (int)kn; ++k) {
            if ((insm >> k) & 1u) atomicAdd(&pcnt[dn[k]], 1u);
            if constexpr (ItemTraits<Item>::preagg) {
                // pre-aggregate: records per pid in the high half (no pid is
                // over a limit, so no candidate appends use it)
                if ((insm >> k) & 1u)
                    atomicAdd(&pidm[qs[k]], (1u << 16) + ((touchm >> k) & 1u));
            } else {
                if ((touchm >> k) & 1u) atomicAdd(&pidm[qs[k]], 1u);
            }
        }
        if (kPerPid || round > 0) break;
        // a pid with more than mpc records but fewer than mpc candidate pairs
        // may own kept pairs above its bound: restart with every record
        wave_sync();
        bool shrt = false;
#pragma unroll
        for (int j = 0; j < kWQPL; ++j) {
            const uint32_t q = lane + 64u * j;
            shrt |= cbnd[q] != 0xFFFFFFFFu && (pidm[q] & 0xFFFFu) < bp.mpc;
        }
        if (!__ballot(shrt)) break;
        // restart: clear the pair table and the pair counts per pid
        constexpr int kClr0 = (int)(sizeof(KeyT) * kWCk / (16 * 64));
#pragma unroll
        for (int i = 0; i < kClr0; ++i)
            reinterpret_cast<uint4 *>(keys)[lane + 64u * i] = make_uint4(~0u, ~0u, ~0u, ~0u);
#pragma unroll
        for (int j = 0; j < kWQPL; ++j) pidm[lane + 64u * j] = 0;
        npair = 0;
        if (hbound) {
            // a heavy chunk holds only its pid's candidates: the bucket goes
            // back to the global-memory kernel (rare)
#pragma unroll
            for (int j = 0; j < kWQPL; ++j) pidslot[lane + 64u * j] = 0;
            if (lane == 0) bp.heavy_fb[atomicAdd(bp.heavy_nfb, 1u)] = hidx;
            wave_sync();
            return nitems;
        }
        wave_sync();
    }
    const uint32_t jn = (npair + 63) >> 6;  // occupied pair slots per lane (uniform)
    wave_sync();
    mark(bp, 1, clk);
    // ---- B: pool regions for pids over their limit (every pid slot;
    // empty ones count 0)
    uint32_t qv[kWQPL];
#pragma unroll
    for (int j = 0; j < kWQPL; ++j) qv[j] = lane + 64u * j;
    {
        uint32_t m[kWQPL];
#pragma unroll
        for (int j = 0; j < kWQPL; ++j) m[j] = pidm[qv[j]] & 0xFFFFu;
        // region offsets by a wave prefix sum (registers only)
        uint32_t run = 0;
#pragma unroll
        for (int j = 0; j < kWQPL; ++j) {
            const bool want = m[j] > lim;
            uint32_t tot;
            const uint32_t ex = wave_excl_scan(want ? m[j] : 0u, tot);
            pidslot[qv[j]] = want ? run + ex : kNil;
            run += tot;
        }
    }
    wave_sync();
    mark(bp, 2, clk);

    // pair-major state: pair j of this lane is dense id lane + 64 j (< npair)
    KeyT pkv[kWPPL];
    uint32_t keptm = 0, ecnt[kWPPL];
#pragma unroll
    for (int j = 0; j < kWPPL && j < (int)jn; ++j) pkv[j] = pkey_d[lane + 64u * j];
    if constexpr (ItemTraits<Item>::preagg) {
        // ---- pre-aggregate (no bounds): every pair is kept with all of its
        // records, so phases C-F reduce to the pair counts and one value
        // sum per record (no thresholds, states or samples to compute)
#pragma unroll
        for (int j = 0; j < kWPPL && j < (int)jn; ++j) {
            if (lane + 64u * j < npair) keptm |= 1u << j;
            ecnt[j] = pcnt[lane + 64u * j];
        }
        if (need_v) {
            double v[kWRPT];
#pragma unroll
            for (int k = 0; k < kWRPT && k < (int)kn; ++k)
                v[k] = ((insm >> k) & 1u) ? rec_value<R>(cur[k], bp.value, f) : 0.0;
#pragma unroll
            for (int k = 0; k < kWRPT && k < (int)kn; ++k)
                if ((insm >> k) & 1u) atomicAdd(&acc_sum[dn[k]], v[k]);
            wave_sync();
        }
        mark(bp, 7, clk);
    } else if constexpr (!per_pid) {
        // ---- C1: candidates (priority below the pid's threshold) append
        // their pair key to the pid's region
        uint32_t sb[kWPPL], m[kWPPL];
        uint64_t k64[kWPPL];
        uint32_t overm = 0, candm = 0;
        // round-0 candidate bound: about k + 2 sqrt(k) + 2 expected
        // candidates per pid (~1.5 % of pids need a second round)
        const float e0 = (float)bp.mpc + DPG_E0_C * sqrtf((float)bp.mpc) + DPG_E0_C;
        uint32_t bq[kWPPL];  // the pid's pre-filter bound: its pairs' priorities are <= it
        {
            uint32_t pv[kWPPL];
#pragma unroll
            for (int j = 0; j < kWPPL && j < (int)jn; ++j) {
                const uint32_t q = (uint32_t)(pkv[j] >> pkb) & (kWCq - 1);
                sb[j] = pidslot[q];
                pv[j] = pidv[q];
                m[j] = pidm[q] & 0xFFFFu;
                bq[j] = cbnd[q];
            }
#pragma unroll
            for (int j = 0; j < kWPPL && j < (int)jn; ++j) {
                const bool occ = lane + 64u * j < npair;
                k64[j] = 0;
                if (occ) keptm |= 1u << j;
                if (!occ || sb[j] == kNil) continue;
                overm |= 1u << j;
                const uint32_t pk = (uint32_t)(pkv[j] & (KeyT)pkmask);
                const uint32_t pr = pair_prio_h(pv[j], pk);
                k64[j] = ((uint64_t)pr << 32) | pk;
                if (pr < cand_threshold_be(m[j], e0, bq[j])) candm |= 1u << j;
            }
            uint32_t pos[kWPPL];
#pragma unroll
            for (int j = 0; j < kWPPL && j < (int)jn; ++j) {
                const uint32_t q = (uint32_t)(pkv[j] >> pkb) & (kWCq - 1);
                pos[j] = ((candm >> j) & 1u) ? atomicAdd(&pidm[q], 1u << 16) >> 16 : 0u;
            }
#pragma unroll
            for (int j = 0; j < kWPPL && j < (int)jn; ++j)
                if ((candm >> j) & 1u) pool[sb[j] + pos[j]] = k64[j];
        }
        wave_sync();
        mark(bp, 3, clk);
        // ---- C2: every pid with >= mpc candidates gets its threshold, the
        // mpc-th smallest candidate key (every non-candidate key exceeds every
        // candidate key); pids short of candidates widen their priority bound
        // and append the next pairs (round 1: 4 x e0; round 2: every pair),
        // whose keys all exceed the earlier candidates', and try again
        {
            uint32_t donem = 0;  // pid slots whose threshold is set (bit j)
            for (uint32_t rnd = 0;; ++rnd) {
                uint32_t psb[kWQPL], pnc[kWQPL];
#pragma unroll
                for (int j = 0; j < kWQPL; ++j) {
                    psb[j] = pidslot[qv[j]];
                    pnc[j] = pidm[qv[j]] >> 16;
                }
                bool shortq = false, ready[kWQPL];
#pragma unroll
                for (int j = 0; j < kWQPL; ++j) {
                    const bool over = psb[j] != kNil;
                    ready[j] = over && pnc[j] >= bp.mpc && !((donem >> j) & 1u);
                    if (ready[j]) donem |= 1u << j;
                    shortq |= over && pnc[j] < bp.mpc;
                }
                region_thresholds<kWQPL>(pool, ready, psb, pnc, bp.mpc);
                if (!__ballot(shortq)) break;
                wave_sync();
                uint32_t ncp[kWPPL], pos[kWPPL], newm = 0;
#pragma unroll
                for (int j = 0; j < kWPPL && j < (int)jn; ++j) {
                    const uint32_t q = (uint32_t)(pkv[j] >> pkb) & (kWCq - 1);
                    ncp[j] = pidm[q] >> 16;
                }
#pragma unroll
                for (int j = 0; j < kWPPL && j < (int)jn; ++j) {
                    const bool over = (overm >> j) & 1u, cand = (candm >> j) & 1u;
                    if (over && !cand && ncp[j] < bp.mpc &&
                        (rnd > 0 ||
                         (uint32_t)(k64[j] >> 32) < cand_threshold_be(m[j], 4.0f * e0, bq[j])))
                        newm |= 1u << j;
                }
#pragma unroll
                for (int j = 0; j < kWPPL && j < (int)jn; ++j) {
                    const uint32_t q = (uint32_t)(pkv[j] >> pkb) & (kWCq - 1);
                    pos[j] = ((newm >> j) & 1u) ? atomicAdd(&pidm[q], 1u << 16) >> 16 : 0u;
                }
#pragma unroll
                for (int j = 0; j < kWPPL && j < (int)jn; ++j)
                    if ((newm >> j) & 1u) pool[sb[j] + pos[j]] = k64[j];
                candm |= newm;
                wave_sync();
            }
        }
        wave_sync();
        {
            uint64_t thr[kWPPL];
#pragma unroll
            for (int j = 0; j < kWPPL && j < (int)jn; ++j) thr[j] = pool[((overm >> j) & 1u) ? sb[j] : 0u];
#pragma unroll
            for (int j = 0; j < kWPPL && j < (int)jn; ++j) {
                const bool over = (overm >> j) & 1u, cand = (candm >> j) & 1u;
                if (over && !(cand && k64[j] <= thr[j])) keptm &= ~(1u << j);
            }
        }
        wave_sync();
        mark(bp, 4, clk);
        // ---- D: pair state; over-full kept pairs reserve one pool slot per
        // record (the pool's mpc regions are dead now)
        uint32_t c[kWPPL], b2[kWPPL];
        {
#pragma unroll
            for (int j = 0; j < kWPPL && j < (int)jn; ++j) c[j] = pcnt[lane + 64u * j];
            uint32_t run = 0;
#pragma unroll
            for (int j = 0; j < kWPPL && j < (int)jn; ++j) {
                const bool need = sample && ((keptm >> j) & 1u) && c[j] > bp.mcpp;
                uint32_t tot;
                const uint32_t ex = wave_excl_scan(need ? c[j] : 0u, tot);
                b2[j] = need ? run + ex : kKeptAll;
                run += tot;
            }
#pragma unroll
            for (int j = 0; j < kWPPL && j < (int)jn; ++j) {
                if (lane + 64u * j < npair)
                    pst[lane + 64u * j] = ((keptm >> j) & 1u) ? b2[j] : kDropped;
                ecnt[j] = bp.mode == DPG_MODE_CROSS_AND_PER_PARTITION ? min(c[j], bp.mcpp) : c[j];
            }
        }
        wave_sync();
        mark(bp, 5, clk);
        // ---- E: values of records of kept pairs are gathered; records of
        // over-full kept pairs append their record key
        uint64_t rkey[kWRPT];
        double v[kWRPT];
        uint32_t st[kWRPT];
#pragma unroll
        for (int k = 0; k < kWRPT && k < (int)kn; ++k) st[k] = pst[dn[k]];
#pragma unroll
        for (int k = 0; k < kWRPT && k < (int)kn; ++k) {
            if (!((insm >> k) & 1u)) st[k] = kDropped;
            if (st[k] < kKeptAll) st[k] &= 0xFFFFu;  // base (appends in the high bits)
            v[k] = 0.0;
            rkey[k] = 0;
            // values of records whose pair keeps every record load now; the
            // records of over-full pairs load once their sample is known
            // (DPG_LATE_GATHER: most of them are not kept, and every gather
            // pulls a whole sector)
            if (need_v && (DPG_LATE_GATHER ? st[k] == kKeptAll : st[k] != kDropped))
                v[k] = rec_value<R>(cur[k], bp.value, f);
        }
        if (sample) {
            uint32_t pv[kWRPT], pos[kWRPT];
#pragma unroll
            for (int k = 0; k < kWRPT && k < (int)kn; ++k) pv[k] = pidv[qs[k]];
#pragma unroll
            for (int k = 0; k < kWRPT && k < (int)kn; ++k) {
                if (st[k] >= kKeptAll) continue;
                const uint64_t key = RecOps<R>::key(cur[k], f);
                rkey[k] = rec_prio_h(pv[k], (uint32_t)(key & pkmask),
                                     (uint64_t)(bp.rec_base + RecOps<R>::idx(cur[k], f)));
            }
#pragma unroll
            for (int k = 0; k < kWRPT && k < (int)kn; ++k)
                pos[k] = st[k] < kKeptAll ? atomicAdd(&pst[dn[k]], 1u << 16) >> 16 : 0u;
#pragma unroll
            for (int k = 0; k < kWRPT && k < (int)kn; ++k)
                if (st[k] < kKeptAll) pool[st[k] + pos[k]] = rkey[k];
            wave_sync();
        }
        mark(bp, 6, clk);
        // ---- F: a sampled record is kept iff fewer than mcpp keys of its
        // pair are smaller; clipped accumulators of kept records
        if (need_v) {
            uint32_t keepm = 0;
#pragma unroll
            for (int k = 0; k < kWRPT && k < (int)kn; ++k) keepm |= st[k] == kKeptAll ? 1u << k : 0u;
            if (sample) {
                // threshold of every over-full kept pair; a sampled record is
                // kept iff its key is <= the threshold
                bool needp[kWPPL];
#pragma unroll
                for (int j = 0; j < kWPPL; ++j) needp[j] = j < (int)jn && b2[j] < kKeptAll;
                region_thresholds<kWPPL>(pool, needp, b2, c, bp.mcpp);
                wave_sync();
                uint64_t thr[kWRPT];
#pragma unroll
                for (int k = 0; k < kWRPT && k < (int)kn; ++k) thr[k] = pool[st[k] < kKeptAll ? st[k] : 0u];
#pragma unroll
                for (int k = 0; k < kWRPT && k < (int)kn; ++k)
                    if (st[k] < kKeptAll && rkey[k] <= thr[k]) keepm |= 1u << k;
#if DPG_LATE_GATHER
#pragma unroll
                for (int k = 0; k < kWRPT && k < (int)kn; ++k)
                    if (st[k] < kKeptAll && rkey[k] <= thr[k]) v[k] = rec_value<R>(cur[k], bp.value, f);
#endif
            }
#pragma unroll
            for (int k = 0; k < kWRPT && k < (int)kn; ++k) {
                if (!((keepm >> k) & 1u)) continue;
                const uint32_t p = dn[k];
                if (part_clip) {
                    atomicAdd(&acc_sum[p], v[k]);
                } else {
                    const double x = clampd(v[k], bp.lo, bp.hi);
                    if (kSum) atomicAdd(&acc_sum[p], x);
                    if (kVar) {
                        const double y = x - bp.mid;
                        atomicAdd(&acc_nsum[p], y);
                        atomicAdd(&acc_nsq[p], y * y);
                    }
                }
            }
            wave_sync();
        }
        mark(bp, 7, clk);
    } else {
        // ---- PER_PRIVACY_ID: records of pids over L append their record key
        // to the pid's region; a record is kept iff fewer than L records of
        // its pid have a smaller key; pst counts kept records per pair
        uint64_t rkey[kWRPT];
        uint32_t sb[kWRPT], pv[kWRPT], pos[kWRPT], overm = 0;
#pragma unroll
        for (int k = 0; k < kWRPT && k < (int)kn; ++k) {
            sb[k] = pidslot[qs[k]];
            pv[k] = pidv[qs[k]];
        }
#pragma unroll
        for (int k = 0; k < kWRPT && k < (int)kn; ++k) {
            rkey[k] = 0;
            if (!((validm >> k) & 1u) || sb[k] == kNil) continue;
            overm |= 1u << k;
            const uint64_t key = RecOps<R>::key(cur[k], f);
            rkey[k] = rec_prio_h(pv[k], (uint32_t)(key & pkmask),
                                 (uint64_t)(bp.rec_base + RecOps<R>::idx(cur[k], f)));
        }
#pragma unroll
        for (int k = 0; k < kWRPT && k < (int)kn; ++k)
            pos[k] = ((overm >> k) & 1u) ? atomicAdd(&pidm[qs[k]], 1u << 16) >> 16 : 0u;
#pragma unroll
        for (int k = 0; k < kWRPT && k < (int)kn; ++k)
            if ((overm >> k) & 1u) pool[sb[k] + pos[k]] = rkey[k];
        wave_sync();
        mark(bp, 5, clk);
        {
            uint32_t psb[kWQPL], pnc[kWQPL];
#pragma unroll
            for (int j = 0; j < kWQPL; ++j) {
                psb[j] = pidslot[qv[j]];
                pnc[j] = pidm[qv[j]] & 0xFFFFu;
            }
bool overp[kWQPL];
#pragma unroll
            for (int j = 0; j < kWQPL; ++j) overp[j] = psb[j] != kNil;
            region_thresholds<kWQPL>(pool, overp, psb, pnc, bp.L);
        }
        wave_sync();
        uint64_t thr[kWRPT];
#pragma unroll
        for (int k = 0; k < kWRPT && k < (int)kn; ++k) thr[k] = pool[((overm >> k) & 1u) ? sb[k] : 0u];
        double v[kWRPT];
#pragma unroll
        for (int k = 0; k < kWRPT && k < (int)kn; ++k) {
            v[k] = 0.0;
            if (((overm >> k) & 1u) && rkey[k] > thr[k]) validm &= ~(1u << k);
            if (need_v && ((validm >> k) & 1u)) v[k] = rec_value<R>(cur[k], bp.value, f);
        }
#pragma unroll
        for (int k = 0; k < kWRPT && k < (int)kn; ++k) {
            if (!((validm >> k) & 1u)) continue;
            const uint32_t p = dn[k];
            atomicAdd(&pst[p], 1u);
            if (need_v) {
                if (part_clip) {
                    atomicAdd(&acc_sum[p], v[k]);
                } else {
                    const double x = clampd(v[k], bp.lo, bp.hi);
                    if (kSum) atomicAdd(&acc_sum[p], x);
                    if (kVar) {
                        const double y = x - bp.mid;
                        atomicAdd(&acc_nsum[p], y);
                        atomicAdd(&acc_nsq[p], y * y);
                    }
                }
            }
        }
        wave_sync();
        mark(bp, 7, clk);
#pragma unroll
        for (int j = 0; j < kWPPL && j < (int)jn; ++j) ecnt[j] = pst[lane + 64u * j];
#pragma unroll
        for (int j = 0; j < kWPPL && j < (int)jn; ++j)
            if (lane + 64u * j < npair && ecnt[j] > 0) keptm |= 1u << j;
    }
    // ---- G: emit kept pairs; clear the key table
    {
        if constexpr (ItemTraits<Item>::preagg) {
            // pid leader: the pair with the smallest dense id of its privacy
            // id carries the leader bit, so dataset histograms count every privacy
            // id once (pidv, the pid hashes, is dead here and is rewritten
            // for the next chunk's occupied slots)
#pragma unroll
            for (int j = 0; j < kWQPL; ++j) pidv[qv[j]] = 0xFFFFFFFFu;
            wave_sync();
#pragma unroll
            for (int j = 0; j < kWPPL && j < (int)jn; ++j)
                if ((keptm >> j) & 1u)
                    atomicMin(&pidv[(uint32_t)(pkv[j] >> pkb) & (kWCq - 1)], lane + 64u * j);
            wave_sync();
        }
        double a0[kWPPL], a1[kWPPL], a2[kWPPL];
#pragma unroll
        for (int j = 0; j < kWPPL && j < (int)jn; ++j) {
            const uint32_t d = lane + 64u * j;
            a0[j] = (kSum && need_v) ? acc_sum[d] : 0.0;
            if constexpr (kVar) {
                a1[j] = need_v ? acc_nsum[d] : 0.0;
                a2[j] = need_v ? acc_nsq[d] : 0.0;
            }
        }
#pragma unroll
        for (int j = 0; j < kWPPL && j < (int)jn; ++j) {
            const bool e = (keptm >> j) & 1u;
            const uint64_t be = __ballot(e);
            if (e) {
                Item it;
                it.pk = (uint32_t)(pkv[j] & (KeyT)pkmask);
                it.cnt = ecnt[j];
                if constexpr (kSum)
                    it.sum = (need_v && part_clip) ? clampd(a0[j], bp.lo_pp, bp.hi_pp) : a0[j];
                if constexpr (kVar) {
                    it.nsum = a1[j];
                    it.nsq = a2[j];
                }
                if constexpr (ItemTraits<Item>::preagg) {
                    const uint32_t q = (uint32_t)(pkv[j] >> pkb) & (kWCq - 1);
                    const uint32_t pm = pidm[q];
                    it.npart = pm & 0xFFFFu;
                    it.nl = ItemPA::pack_nl(pm >> 16, pidv[q] == lane + 64u * j);
                }
                items[nitems + lanes_below(be)] = it;
            }
            nitems += (uint32_t)__popcll(be);
        }
        constexpr int kClr = (int)(sizeof(KeyT) * kWCk / (16 * 64));
#pragma unroll
        for (int i = 0; i < kClr; ++i)
            reinterpret_cast<uint4 *>(keys)[lane + 64u * i] = make_uint4(~0u, ~0u, ~0u, ~0u);
    }
#pragma unroll
    for (int j = 0; j < kWQPL; ++j) {
        pidm[qv[j]] = 0;
        pidslot[qv[j]] = 0;
    }
    wave_sync();
    mark(bp, 8, clk);
    return nitems;
}

// Persistent single-wave workgroups walk the small-chunk list statically
// (w, w + G, ...); workgroup g appends its items to items[wg_off[g], ...)
// and leaves the count in wg_cnt[g].
template <class KeyT, class Item, class R, bool kPerPid>
__global__ __launch_bounds__(64, kWCap <= 384 ? 3 : 2) void k_bound_waves(const R *recs, const R *refined,
                                                    const R *heavy, const uint4 *chunks,
                                                    const uint32_t *n_chunks,
                                                    BoundParams bp, Item *items,
                                                    const int64_t *wg_off, uint32_t *wg_cnt) {
    using L = WaveLayout<KeyT, Item>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    PhaseTimer clk;
    timer_start(bp, clk);
    // parameters used in one phase each: vector registers (see vreg)
    bp.lo = vreg(bp.lo);
    bp.hi = vreg(bp.hi);
    bp.lo_pp = vreg(bp.lo_pp);
    bp.hi_pp = vreg(bp.hi_pp);
    bp.mid = vreg(bp.mid);
    bp.seed = vreg(bp.seed);
    bp.pid_min = vreg(bp.pid_min);
    bp.rec_base = vreg(bp.rec_base);
    bp.hash.mask = vreg(bp.hash.mask);
    // bounds and record-format fields only meet vector operands
    bp.mpc = vreg(bp.mpc);
    bp.mcpp = vreg(bp.mcpp);
    bp.L = vreg(bp.L);
    bp.fmt.ib = vreg(bp.fmt.ib);
    bp.fmt.pkbits = vreg(bp.fmt.pkbits);
    bp.fmt.kbits = vreg(bp.fmt.kbits);
    bp.fmt.b1 = vreg(bp.fmt.b1);
    // pointers used by one phase each (or only on errors)
    bp.value = vreg(bp.value);
    bp.err = vreg(bp.err);
    bp.heavy_fb = vreg(bp.heavy_fb);
    bp.heavy_nfb = vreg(bp.heavy_nfb);
    bp.hash.i1 = vreg(bp.hash.i1);
    bp.hash.i2 = vreg(bp.hash.i2);
    const uint32_t nch = __builtin_amdgcn_readfirstlane(*n_chunks);
    Item *my_items = items + wg_off[blockIdx.x];
    const uint32_t lane = __lane_id();
    {
        uint32_t *pidm = reinterpret_cast<uint32_t *>(smem + L::PIDM);
        uint32_t *pidslot = reinterpret_cast<uint32_t *>(smem + L::PIDSLOT);
        KeyT *keys = reinterpret_cast<KeyT *>(smem + L::KEYS);
        for (uint32_t i = lane; i < kWCq; i += 64) pidm[i] = pidslot[i] = 0;
        for (uint32_t i = lane; i < kWCk; i += 64) keys[i] = empty_key<KeyT>();
    }
    wave_sync();
    R r[kWRPT], rn[kWRPT];
    const uint32_t G = gridDim.x;
    uint32_t w = blockIdx.x;
    uint32_t n = 0, d1 = 0, hb = 0, hbound = 0, hidx = 0, nitems = 0;
    uint4 dn = make_uint4(0, 0, 0, 0);
    if (w < nch) {
        const uint4 d = make_uint4(__builtin_amdgcn_readfirstlane(chunks[w].x),
                                   __builtin_amdgcn_readfirstlane(chunks[w].y),
                                   __builtin_amdgcn_readfirstlane(chunks[w].z),
                                   __builtin_amdgcn_readfirstlane(chunks[w].w));
        n = d.y & kChunkCount;
        d1 = d.z & 0xFFFFu;
        hb = d.w;
        hbound = heavy_bound(d);
        hidx = d.x / (uint32_t)kWCap;
        const R *b = wave_chunk_base(d, recs, refined, heavy);
#pragma unroll
        for (int k = 0; k < kWRPT; ++k) r[k] = b[min(lane + 64u * k, n - 1)];
        if (w + G < nch) dn = chunks[w + G];
    }
    for (; w < nch; w += G) {
        uint4 dnn = make_uint4(0, 0, 0, 0);
        if (w + 2 * G < nch) dnn = chunks[w + 2 * G];
        const uint4 du = make_uint4(__builtin_amdgcn_readfirstlane(dn.x),
                                    __builtin_amdgcn_readfirstlane(dn.y),
                                    __builtin_amdgcn_readfirstlane(dn.z),
                                    __builtin_amdgcn_readfirstlane(dn.w));
        const uint32_t nn = du.y & kChunkCount;
        // the next chunk's records load while this one is processed
        if (nn > 0) {
            const R *nb = wave_chunk_base(du, recs, refined, heavy);
#pragma unroll
            for (int k = 0; k < kWRPT; ++k) rn[k] = nb[min(lane + 64u * k, nn - 1)];
        }
        nitems = wave_chunk<KeyT, Item, R, kPerPid>(r, n, d1, hb, smem, bp, my_items, nitems, clk,
                                                    hbound, hidx);
#pragma unroll
        for (int k = 0; k < kWRPT; ++k) r[k] = rn[k];
        n = nn;
        d1 = du.z & 0xFFFFu;
        hb = du.w;
        hbound = heavy_bound(du);
        hidx = du.x / (uint32_t)kWCap;
        dn = dnn;
    }
    if (lane == 0) wg_cnt[blockIdx.x] = nitems;
    timer_flush(bp, clk);
}

// Heavy buckets (cross-partition modes): a single privacy id with more
// records than any LDS chunk holds (config 4's Pareto tail: 1e5 ids with up
// to ~2e4 records each).  Only pairs of low priority can be among its mpc
// kept pairs, and a pair's records share its priority, so one workgroup per
// bucket histograms the records' pair priorities (4096 bins), picks the
// largest bin cut with <= kWCap records below it and writes those records --
// every record of every pair below the cut -- to a heavy chunk that the wave
// kernel bounds like any other, with the cut as the pid's candidate bound.
// When fewer than mpc pairs lie below the cut (many records per pair) the
// wave kernel hands the bucket back to k_bound_big (heavy_fb), as does this
// kernel for a bucket of several privacy ids.  Two reads of the bucket's
// records (the second mostly from L2), no global atomics but one per bucket.
constexpr int kHvThreads = 256;
template <class R>
__global__ __launch_bounds__(kHvThreads) void k_heavy_filter(
    const R *base, const int64_t *bstart, const uint32_t *bcnt, const uint32_t *bd1,
    BoundParams bp, R *hrec, uint4 *chunks, uint32_t *n_chunks) {
    __shared__ uint32_t hist[kHvBins];
    __shared__ uint32_t wtot[kHvThreads / 64];
    __shared__ uint32_t sh_le, sh_n;
    const uint32_t b = blockIdx.x;
    const uint32_t tid = threadIdx.x, lane = __lane_id(), wid = tid >> 6;
    const uint32_t n = bcnt[b];
    const uint32_t d1 = bd1[b];
    const R *rb = base + bstart[b];
    const Fmt f = bp.fmt;
    const uint32_t pkb = f.pkbits;
    const uint64_t pkmask = (1ull << pkb) - 1ull;
    const uint32_t hres = (uint32_t)(RecOps<R>::key(rb[0], f) >> pkb);
    const uint32_t pv = pid_hash(bp.seed, pid_of(bp, d1, hres));
    for (uint32_t i = tid; i < kHvBins; i += kHvThreads) hist[i] = 0;
    if (tid == 0) sh_le = sh_n = 0;
    __syncthreads();
    bool multi = false;
    for (uint32_t i = tid; i < n; i += kHvThreads) {
        const uint64_t key = RecOps<R>::key(rb[i], f);
        multi |= (uint32_t)(key >> pkb) != hres;
        atomicAdd(&hist[pair_prio_h(pv, (uint32_t)(key & pkmask)) >> 20], 1u);
    }
    if (__syncthreads_or(multi)) {
        if (tid == 0) bp.heavy_fb[atomicAdd(bp.heavy_nfb, 1u)] = b;
        return;
    }
    // cut = max{c : records in bins [0, c) <= kWCap}: cum(c) is
    // non-decreasing, so the cut is the number of c in [1, 4096] that qualify
    constexpr uint32_t kPer = kHvBins / kHvThreads;
    uint32_t s = 0;
#pragma unroll
    for (uint32_t j = 0; j < kPer; ++j) s += hist[tid * kPer + j];
    uint32_t tot;
    uint32_t run = wave_excl_scan(s, tot);
    if (lane == 0) wtot[wid] = tot;
    __syncthreads();
    for (uint32_t w = 0; w < wid; ++w) run += wtot[w];
    uint32_t le = 0;
#pragma unroll
    for (uint32_t j = 0; j < kPer; ++j) {
        run += hist[tid * kPer + j];
        le += run <= (uint32_t)kWCap ? 1u : 0u;
    }
    atomicAdd(&sh_le, le);
    __syncthreads();
    const uint32_t cut = sh_le;
    const uint32_t B = cut >= kHvBins ? 0xFFFFFFFFu : cut ? (cut << 20) - 1u : 0u;
    R *out = hrec + (size_t)b * kWCap;
    if (cut) {
        for (uint32_t i0 = 0; i0 < n; i0 += kHvThreads) {
            const uint32_t i = i0 + tid;
            bool c = false;
            R rec{};
            if (i < n) {
                rec = rb[i];
                c = pair_prio_h(pv, (uint32_t)(RecOps<R>::key(rec, f) & pkmask)) <= B;
            }
            const uint64_t bal = __ballot(c);
            uint32_t o = 0;
            if (bal) {
                if (lane == 0) o = atomicAdd(&sh_n, (uint32_t)__popcll(bal));
                o = __shfl(o, 0, 64);
            }
            if (c) out[o + lanes_below(bal)] = rec;
        }
    }
    __syncthreads();
    if (tid == 0) {
        const uint32_t cnt = sh_n;
        if (cnt == 0)
            bp.heavy_fb[atomicAdd(bp.heavy_nfb, 1u)] = b;
        else
            chunks[atomicAdd(n_chunks, 1u)] =
                make_uint4(b * (uint32_t)kWCap, cnt | kChunkHeavy, d1 | (cut << 16), hres);
    }
}

// The buckets handed back (heavy_fb) as an oversize list for k_bound_big.
__global__ void k_gather_heavy(const uint32_t *fb, const uint32_t *nfb, const int64_t *st,
                               const uint32_t *cnt, const uint32_t *d1, int64_t *ost,
                               uint32_t *ocnt, uint32_t *od1) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= *nfb) return;
    const uint32_t b = fb[i];
    ost[i] = st[b];
    ocnt[i] = cnt[b];
    od1[i] = d1[b];
}

}  // namespace dpg
