// dpg_sortb.h -- sort-based contribution bounding of small chunks by single
// waves (gfx950): the default bounding kernel of the cross-partition modes.
//
// A small chunk (<= kWCap = 512 records of <= kWCq = 128 privacy-id hash
// slots, dpg_chunk.h) is bounded by one 64-lane wave that owns a private LDS
// working set.  Instead of a hash table of pairs (dpg_wave.h) the wave SORTS
// the chunk's candidate records in registers by the key the reference's
// sampler orders pairs by (contribution_bounders.py:90-92; oracle
// dp_oracle.c: key = pair_priority << 32 | pk per privacy id):
//
//   skey = pid slot q (7 bits) | pair priority pp (32 bits) | pk (24 bits)
//
// so that the records of one pair are adjacent, the pairs of one privacy id
// follow each other in ascending (pp, pk) order, and a pair is kept iff
// fewer than mpc pairs of its privacy id precede it -- a segmented count
// over the sorted sequence instead of hash inserts, probing and a per-pid
// threshold search.  Per chunk:
//
//   A  records per pid slot (LDS atomics), pid hash and candidate bound of
//      every occupied slot: a pid with more than mpc records only sends the
//      records whose pair priority is below a bound aimed at ~CAND x (mpc +
//      2 sqrt(mpc) + 2) records (a pair's records share its priority, so
//      whole pairs pass or fail); candidates are compacted into LDS
//   S  bitonic sort of the candidates' (skey, record index) in registers: E =
//      1, 2, 4 or 8 elements per lane (64 E >= candidates), cross-lane steps
//      by DPP / ds_swizzle / bpermute
//   P  pair starts, pair ordinals (wave scan), pair rank inside the pid; a
//      filtered pid that shows fewer than mpc candidate pairs restarts the
//      chunk with all of its records, re-read from HBM (rare); a pair is
//      kept iff rank < mpc
//   M  records of kept pairs gather their values; pairs over mcpp rank their
//      records by record priority (contribution_bounders.py:74-76) inside
//      the pair's segment
//   F  clipped accumulators (combiners.py:255-500) per pair in LDS; one Item
//      per kept pair.
//
// Kept sets are bit-identical to the oracle's: the order is the oracle's
// key order whenever pk < 2^24 (the host uses the hash kernel otherwise).
// PER_PRIVACY_ID bounding and the utility pre-aggregate keep dpg_wave.h.
#pragma once

#include "dpg_wave.h"

namespace dpg {

// candidate bound of the sort kernel (records per pid aimed at, times
// mpc + 2 sqrt(mpc) + 2: BoundParams::cand_mul); restarts (a pid short of
// mpc candidate pairs) cost a second round, candidates past 64 / 128 / 256
// per chunk a sort twice as wide
// same-box A/Bs of the config-2 bounding stage: 2.0 9.03 ms, 1.5 7.49, 1.25
// 7.47 (round 3); with the float64 network 1.75 7.38, 1.5 6.83, 1.35 6.70,
// 1.25 6.81 (round 4, profiles/r4/r4p_cand_mult_ab.txt)
constexpr float kSortCandC = 1.35f;

constexpr uint32_t kSkPkBits = 24;  // partition-key bits of the sort key
#ifndef DPG_SORT_PACKED
#define DPG_SORT_PACKED 1  // narrow kernel: keys with the position packed in, no payload
#endif
constexpr uint64_t kSkPad = ~0ull;  // padding elements (real keys have bit 63 clear)
#ifndef DPG_SORT_LATE
#define DPG_SORT_LATE 1  // value gathers of over-full pairs after their mcpp sample
#endif
constexpr bool kSortLate = DPG_SORT_LATE != 0;
#ifndef DPG_SORT_PF
#define DPG_SORT_PF 0  // 8-byte records: the narrow pass prefetches the next chunk (see kSortPF)
#endif

// The wave's LDS working set is kept under 10 KB (COUNT / SUM items) so that
// 16 waves share a CU: the kernel is latency-bound per wave (same-box A/B,
// config 2: 4 waves per CU 24.2 ms, 8 waves per CU 12.5 ms), so resident
// waves are what hides the LDS round trips and the value gathers.  The sort
// payload is the record index itself (no per-position copy of the records),
// pair starts are 16-bit, and the candidate area is reused: candidate keys
// and indices -> record keys of over-full pairs (phase M) -> accumulators
// per pair (phase F).
// kC: candidates the working set holds -- kTierCand of the pass (kNarrowCand
// for the narrow one (round 5: a smaller working set is what lets more waves
// share a CU, see k_bound_sorted)
template <class Item, class R, bool kWPk = false, int kC = kWCap>
struct SortLayout {
    static constexpr int NACC = ItemTraits<Item>::var ? (ItemTraits<Item>::sum ? 3 : 2) : 1;
    static constexpr uint32_t CAP = kC;
    static constexpr size_t PIDC = 0;                  // records per pid slot
    static constexpr size_t PIDV = PIDC + 4 * kWCq;    // pid hash
    static constexpr size_t CBND = PIDV + 4 * kWCq;    // candidate bound
    static constexpr size_t PBASE = CBND + 4 * kWCq;   // ordinal of the pid's first pair
    static constexpr size_t FULL = PBASE + 4 * kWCq;   // pid shows >= mpc candidate pairs
    // first position per pair (u16); before the sort: occupied pid slots (u32)
    static constexpr size_t PSTART = FULL + 4 * kWCq;
    static constexpr size_t CK = PSTART + a16(2 * (kC + 1) > 4 * kWCq ? 2 * (kC + 1) : 4 * kWCq);
    // candidate keys u64[kC] + record indices u32[kC]; then record keys by
    // position (u64); then NACC accumulators per pair (f64)
    static constexpr size_t CIDX = CK + 8 * kC;
    static constexpr size_t CKSZ = 12 * kC > 8 * NACC * kC ? 12 * kC : 8 * NACC * kC;
    // wide partition keys (kWPk): the low pk bits the sort key has no room
    // for, per candidate (u8)
    static constexpr size_t CPKL = CK + CKSZ;
    static constexpr size_t END = CPKL + (kWPk ? kC : 0);
    static constexpr size_t TOTAL = (END + 255) & ~(size_t)255;
    static_assert(TOTAL <= 40 * 1024, "sort working set too large");
};

// Passes of the kernel over the small-chunk list (kTier):
//  * 0, narrow: chunks of <= kNarrowCand<R> candidates, a working set sized
//    for them and registers for kNarrowWPS<R> waves per SIMD; a chunk with
//    more candidates is only flagged (defer[w] = 1) and left to
//  * 1, mid (only with a narrow capacity below 256, DPG_NARROW_CAND):
//    <= 256 candidates (E <= 4 elements per lane), 4 waves per SIMD, over
//    the flagged chunks of the narrow workgroups; it clears the flags of the
//    chunks it bounds and leaves the rest to
//  * 2, wide: E <= 8, 2 waves per SIMD (the 8-element sort network needs
//    ~230 VGPRs), or the 2-wave kernel of dpg_sortmw.h.
// The deferred passes walk the flagged chunks of the narrow workgroups and
// append to their item regions.  With 8-byte records the narrow pass runs
// at 5 waves per SIMD (96 VGPRs: no next-chunk prefetch, 7 spilled VGPRs)
// over a working set sized for its 256 candidates (6 KB): same-box A/B at
// config 2, bounding 6.61-6.64 -> 6.27-6.31 ms per step
// (profiles/r5/r5w_sort_5wps_ab.txt).  A 128-candidate narrow pass (4.5 KB,
// 96 VGPRs without spills) bounds the chunks it keeps faster still, but
// about half of config 2's chunks hold more than 128 candidates, and a mid
// pass for them costs more than it saves (r5h, r5j).  Chunks of many small
// privacy ids (every record a candidate) reach the wide pass.
#ifndef DPG_NARROW_CAND
#define DPG_NARROW_CAND 256  // 8-byte records; 12-byte ones: 256
#endif
#ifndef DPG_NARROW_WPS
#define DPG_NARROW_WPS 5
#endif
template <class R>
constexpr uint32_t kNarrowCand = sizeof(R) == 8 ? DPG_NARROW_CAND : 256;
template <class R>
constexpr int kNarrowWPS = sizeof(R) == 8 ? DPG_NARROW_WPS : 4;  // waves per SIMD by registers
// the narrow pass loads the next chunk's records during the current one
// (8-byte records: not at 5 waves per SIMD, where the prefetch registers spill)
template <class R>
constexpr bool kSortPF = sizeof(R) == 8 ? DPG_SORT_PF != 0 : true;
constexpr uint32_t kMidCand = 256;
constexpr int kMidWPS = 4;
template <class R>
constexpr bool kHasMid = kNarrowCand<R> < kMidCand;
constexpr int kWideWPS = 2;
// tier 3: medium chunks (one fine bucket of kWCap + 1 .. capM records),
// streamed (stream_bound_chunk below) with the narrow pass's working set
template <class R, int kTier>
constexpr int kTierCand = kTier == 0 || kTier == 3 ? (int)kNarrowCand<R> : kTier == 1 ? (int)kMidCand : kWCap;
template <class R, int kTier>
constexpr int kTierWPS = kTier == 0 || kTier == 3 ? kNarrowWPS<R> : kTier == 1 ? kMidWPS : kWideWPS;
// candidate records aimed at per privacy id of more than kStreamBig records in
// a streamed chunk: up to kStreamMul x cand_mul, at most half the working set
// (a pid's records crowd into its few Zipf-heavy pairs, so cand_mul records
// -- ~mpc pairs at one record per pair -- would restart most such pids)
constexpr uint32_t kStreamBig = 256;
constexpr float kStreamMul = 4.0f;
#ifndef DPG_SORT_VREG
#define DPG_SORT_VREG 0  // bound parameters the narrow kernel keeps in VGPRs (0, 1 or 2 groups; 5 waves per SIMD: 0, r5z)
#endif

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, o, 64));
    return x;
}

// x of lane (lane ^ m), m < 64 either a power of two or 2^t - 1: quad DPP
// for 1, 2, 3, half-row / row mirrors for 7 and 15, the ds_swizzle bit-mask
// mode inside 32 lanes for 4, 8, 16 and 31, bpermute for 32 and 63.  The
// callers' loops are fully unrolled, so m is a constant and one case stays.
__device__ __forceinline__ uint32_t xlane(uint32_t x, int m) {
    switch (m) {
        case 1:
            return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);  // [1,0,3,2]
        case 2:
            return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);  // [2,3,0,1]
        case 3:
            return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x1B, 0xF, 0xF, false);  // [3,2,1,0]
        case 7:
            return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, false);  // half mirror
        case 15:
            return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xF, 0xF, false);  // row mirror
        case 4:
            return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x101F);
        case 8:
            return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x201F);
        case 16:
            return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x401F);
        case 31:
            return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x7C1F);
        default:
            return (uint32_t)__shfl_xor((int)x, m, 64);
    }
}
__device__ __forceinline__ uint64_t xlane64(uint64_t x, int m) {
    return ((uint64_t)xlane((uint32_t)(x >> 32), m) << 32) | xlane((uint32_t)x, m);
}

// Ascending sort of 64 E (key, payload) elements, element i = lane E + j in
// k[j], o[j]: a bitonic network in the form whose comparators all put the
// minimum at the lower index -- each merge of block size kk first compares
// i with its mirror i ^ (kk - 1), then half-cleans with i ^ s.  Steps inside
// a lane's E elements need no exchange; the others read the partner lane's
// element through xlane.  The only lane-dependent decision is "is this the
// lower index", one lane bit.  Equal keys never move, so partners agree.
template <int E, bool kLex = false>
__device__ __forceinline__ void bitonic_sort(uint64_t (&k)[E], uint32_t (&o)[E]) {
    constexpr int LOG_S = E == 1 ? 6 : E == 2 ? 7 : E == 4 ? 8 : 9;
    constexpr int LOG_E = LOG_S - 6;
    // a fresh copy per call: keeps the lane-bit masks from being hoisted out
    // of the chunk loop (they would live in scalar registers all along)
    uint32_t lid = __lane_id();
    asm volatile("" : "+v"(lid));
    // kLex: (key, payload) lexicographically (every element distinct)
    auto less = [](uint64_t a, uint32_t oa, uint64_t b, uint32_t ob) {
        return kLex ? (a < b || (a == b && oa < ob)) : a < b;
    };
    auto cex = [&](int j, int j2) {  // in-lane compare-exchange, min to j
        const bool sw = less(k[j2], o[j2], k[j], o[j]);
        const uint64_t a = k[j], b = k[j2];
        const uint32_t oa = o[j], ob = o[j2];
        k[j] = sw ? b : a;
        k[j2] = sw ? a : b;
        o[j] = sw ? ob : oa;
        o[j2] = sw ? oa : ob;
    };
#pragma unroll
    for (int lk = 1; lk <= LOG_S; ++lk) {
        const int kk = 1 << lk;
        // mirror step
        if (lk <= LOG_E) {
#pragma unroll
            for (int j = 0; j < E; ++j) {
                const int j2 = j ^ (kk - 1);
                if (j < j2) cex(j, j2);
            }
        } else {
            const int m = (kk >> LOG_E) - 1;            // partner lane = lane ^ m, slot E-1-j
            const bool lower = (lid & (uint32_t)((m + 1) >> 1)) == 0;
            uint64_t y[E];
            uint32_t yo[E];
#pragma unroll
            for (int j = 0; j < E; ++j) {
                y[j] = xlane64(k[E - 1 - j], m);
                yo[j] = xlane(o[E - 1 - j], m);
            }
#pragma unroll
            for (int j = 0; j < E; ++j) {
                const bool take = lower ? less(y[j], yo[j], k[j], o[j]) : less(k[j], o[j], y[j], yo[j]);
                k[j] = take ? y[j] : k[j];
                o[j] = take ? yo[j] : o[j];
            }
        }
        // half-cleaners
#pragma unroll
        for (int ls = lk - 2; ls >= 0; --ls) {
            const int sd = 1 << ls;
            if (ls < LOG_E) {
#pragma unroll
                for (int j = 0; j < E; ++j)
                    if (!(j & sd)) cex(j, j | sd);
            } else {
                const int m = sd >> LOG_E;
                const bool lower = (lid & (uint32_t)m) == 0;
#pragma unroll
                for (int j = 0; j < E; ++j) {
                    const uint64_t y = xlane64(k[j], m);
                    const uint32_t yo = xlane(o[j], m);
                    const bool take = lower ? less(y, yo, k[j], o[j]) : less(k[j], o[j], y, yo);
                    k[j] = take ? y : k[j];
                    o[j] = take ? yo : o[j];
                }
            }
        }
    }
}

// The same network over keys alone (unique keys: the candidate position
// rides in the low bits, see sort_chunk), on keys that are finite positive
// normal doubles when read as float64 (bit 63 clear, bits 62..61 = 01, see sort_chunk's packed
// keys; padding +inf): for those, float64 order is the unsigned order of the
// bits, so a compare-exchange is one v_min_f64 and one v_max_f64 (bare, in
// inline asm: fmin / fmax would first canonicalise both operands) instead of
// a 64-bit compare and four selects.
__device__ __forceinline__ uint64_t fmin_bits(uint64_t a, uint64_t b) {
    double x = __builtin_bit_cast(double, a), y = __builtin_bit_cast(double, b), r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
    return __builtin_bit_cast(uint64_t, r);
}
__device__ __forceinline__ uint64_t fmax_bits(uint64_t a, uint64_t b) {
    double x = __builtin_bit_cast(double, a), y = __builtin_bit_cast(double, b), r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
    return __builtin_bit_cast(uint64_t, r);
}
constexpr uint64_t kSkPadF = 0x7FF0000000000000ull;  // +inf: above every packed key
constexpr uint64_t kSkTagF = 1ull << 61;              // exponent bits 01...: normal, finite

template <int E>
__device__ __forceinline__ void bitonic_sort_keys_f64(uint64_t (&k)[E]) {
    constexpr int LOG_S = E == 1 ? 6 : E == 2 ? 7 : E == 4 ? 8 : 9;
    constexpr int LOG_E = LOG_S - 6;
    uint32_t lid = __lane_id();
    asm volatile("" : "+v"(lid));
    auto cex = [&](int j, int j2) {
        const uint64_t a = k[j], b = k[j2];
        k[j] = fmin_bits(a, b);
        k[j2] = fmax_bits(a, b);
    };
#pragma unroll
    for (int lk = 1; lk <= LOG_S; ++lk) {
        const int kk = 1 << lk;
        if (lk <= LOG_E) {
#pragma unroll
            for (int j = 0; j < E; ++j) {
                const int j2 = j ^ (kk - 1);
                if (j < j2) cex(j, j2);
            }
        } else {
            const int m = (kk >> LOG_E) - 1;
            const bool lower = (lid & (uint32_t)((m + 1) >> 1)) == 0;
            uint64_t y[E];
#pragma unroll
            for (int j = 0; j < E; ++j) y[j] = xlane64(k[E - 1 - j], m);
#pragma unroll
            for (int j = 0; j < E; ++j)
                k[j] = lower ? fmin_bits(k[j], y[j]) : fmax_bits(k[j], y[j]);
        }
#pragma unroll
        for (int ls = lk - 2; ls >= 0; --ls) {
            const int sd = 1 << ls;
            if (ls < LOG_E) {
#pragma unroll
                for (int j = 0; j < E; ++j)
                    if (!(j & sd)) cex(j, j | sd);
            } else {
                const int m = sd >> LOG_E;
                const bool lower = (lid & (uint32_t)m) == 0;
#pragma unroll
                for (int j = 0; j < E; ++j) {
                    const uint64_t y = xlane64(k[j], m);
                    k[j] = lower ? fmin_bits(k[j], y) : fmax_bits(k[j], y);
                }
            }
        }
    }
}

// Sorts the nc candidates and bounds them (phases S, P, M, F of the header).
// Returns kRoundRestart when the chunk must restart: the filtered pids short
// of mpc candidate pairs have had their bound lifted (their CBND set to
// all-pass).  Per-element flags live in per-lane bit masks (bit j = element
// j).
//
// kWPk (partition keys of 25..32 bits): the sort key carries the top 24 pk
// bits, the payload the candidate's position e (9 bits) and the low pk bits
// (idx is read back from CIDX by e).  Pairs then differ in (key, low bits);
// two pairs of one pid with equal key (same priority, same top bits; ~2^-56
// per pair of pairs) may interleave under a key-only comparator, so the
// narrow kernel defers such a chunk (kRoundDefer) to the wide kernel, whose
// comparator (kLex) orders by (key, payload).
constexpr int kRoundRestart = 0, kRoundDone = 1, kRoundDefer = 2;
template <class Item, class R, int E, bool kWPk, bool kLex, int kC>
__device__ __forceinline__ int sort_chunk(uint32_t nc, char *smem, const BoundParams &bp,
                                           bool last_round, uint32_t hbound, uint32_t hidx,
                                           Item *items, uint32_t &nitems, PhaseTimer &clk) {
    using L = SortLayout<Item, R, kWPk, kC>;
    static_assert(64 * E <= kC || E == 1, "sort width beyond the working set");
    constexpr bool kVar = ItemTraits<Item>::var;
    constexpr bool kSum = ItemTraits<Item>::sum;
    const uint8_t *cpkl = reinterpret_cast<const uint8_t *>(smem + L::CPKL);
    uint32_t *pidv = reinterpret_cast<uint32_t *>(smem + L::PIDV);
    uint32_t *pidc = reinterpret_cast<uint32_t *>(smem + L::PIDC);
    uint32_t *cbnd = reinterpret_cast<uint32_t *>(smem + L::CBND);
    uint32_t *pbase = reinterpret_cast<uint32_t *>(smem + L::PBASE);
    uint32_t *full = reinterpret_cast<uint32_t *>(smem + L::FULL);
    uint64_t *ckey = reinterpret_cast<uint64_t *>(smem + L::CK);
    const uint32_t *cidx = reinterpret_cast<const uint32_t *>(smem + L::CIDX);
    uint64_t *rks = ckey;  // after the sort (phase M)
    uint16_t *pstart = reinterpret_cast<uint16_t *>(smem + L::PSTART);
    double *acc = reinterpret_cast<double *>(smem + L::CK);  // phase F
    double *acc_nsum = acc + (kSum ? L::CAP : 0);
    double *acc_nsq = acc_nsum + L::CAP;
    const uint32_t lane = __lane_id();
    const Fmt f = bp.fmt;
    const bool need_v = bp.need_values != 0;
    const bool cap_pp = bp.mode == DPG_MODE_CROSS_AND_PER_PARTITION;
    const bool sample = cap_pp && need_v;
    const bool part_clip = bp.sum_mode == DPG_SUM_CLIP_PARTITION;
    constexpr uint32_t kPkMask = (1u << kSkPkBits) - 1u;
    const uint32_t pksh = kWPk ? f.pkbits - kSkPkBits : 0u;  // low pk bits in the payload

    // ---- S: sort (key, record index | kWPk: position e | low pk bits << 9)
    uint64_t k[E];
    uint32_t o[E];
#pragma unroll
    for (int j = 0; j < E; ++j) {
        const uint32_t i = lane * E + j;
        const uint32_t ic = min(i, L::CAP - 1);
        const uint64_t x = ckey[ic];
        const uint32_t y = kWPk ? (ic | ((uint32_t)cpkl[ic] << 9)) : cidx[ic];
        k[j] = i < nc ? x : kSkPad;
        o[j] = i < nc ? y : 0u;
    }
    full[lane] = 0;
    full[lane + 64u] = 0;
    bool sorted_packed = false;
    if constexpr (!kWPk && !kLex && E <= 4 && DPG_SORT_PACKED) {
        // keys alone (2 VALU per in-lane compare-exchange, see
        // bitonic_sort_keys_f64): tag bits 01 | pid slot (7 bits) | top
        // min(32, 45 - pkbits) bits of the pair priority | pk | candidate
        // position (9 bits); the full keys and record indices are read back by position.
        // Two pairs of one pid whose priorities agree in the kept bits (~24^2
        // / 2^26 per pid at pkbits 20) may come out in pk order instead of
        // priority order: the full keys are then not ascending and the chunk
        // is sorted again with key and payload.
        const uint32_t pkb = f.pkbits;
        const uint32_t ppb = min(32u, 45u - pkb);  // all 32 bits when pk is narrow
        const uint64_t pkm = (1ull << pkb) - 1ull;
        uint64_t pk64[E];
#pragma unroll
        for (int j = 0; j < E; ++j) {
            const uint32_t i = lane * E + j;
            const uint64_t x = k[j];
            const uint64_t pp = (x >> kSkPkBits) & 0xFFFFFFFFull;
            pk64[j] = i < nc ? (kSkTagF | ((x >> 56) << 54) | ((pp >> (32u - ppb)) << (9u + pkb)) |
                                ((x & pkm) << 9) | (uint64_t)i)
                             : kSkPadF;
        }
        bitonic_sort_keys_f64<E>(pk64);
#pragma unroll
        for (int j = 0; j < E; ++j) {
            const uint32_t i = lane * E + j;
            const uint32_t pos = (uint32_t)pk64[j] & 511u;
            k[j] = i < nc ? ckey[min(pos, L::CAP - 1)] : kSkPad;
            o[j] = i < nc ? cidx[min(pos, L::CAP - 1)] : 0u;
        }
        const uint64_t pl = (uint64_t)__shfl_up((long long)k[E - 1], 1, 64);
        bool bad = false;
#pragma unroll
        for (int j = 0; j < E; ++j) {
            const uint32_t i = lane * E + j;
            bad |= i > 0 && i < nc && k[j] < (j ? k[j - 1] : pl);
        }
        sorted_packed = __ballot(bad) == 0;
        if (!sorted_packed) {
#pragma unroll
            for (int j = 0; j < E; ++j) {
                const uint32_t i = lane * E + j;
                const uint32_t ic = min(i, L::CAP - 1);
                k[j] = i < nc ? ckey[ic] : kSkPad;
                o[j] = i < nc ? cidx[ic] : 0u;
            }
        }
    }
    if (!sorted_packed) bitonic_sort<E, kLex>(k, o);
    mark(bp, 1, clk);

    // ---- P: pair starts, ordinals, rank inside the pid
    const uint64_t prev_last = (uint64_t)__shfl_up((long long)k[E - 1], 1, 64);
    const uint32_t prev_o = kWPk ? (uint32_t)__shfl_up((int)o[E - 1], 1, 64) : 0u;
    uint32_t validm = 0, psm = 0, pidm = 0;
    uint32_t a[E];
    uint32_t cnt = 0;
    bool coll = false;  // kWPk: two pairs with one key (see above)
#pragma unroll
    for (int j = 0; j < E; ++j) {
        const uint32_t i = lane * E + j;
        const uint64_t pv = j ? k[j - 1] : prev_last;
        const bool val = i < nc;
        const bool lodiff = kWPk && ((o[j] >> 9) != ((j ? o[j - 1] : prev_o) >> 9));
        const bool p = val && (i == 0 || k[j] != pv || lodiff);
        coll |= val && i > 0 && k[j] == pv && lodiff;
        const bool d = val && (i == 0 || (k[j] >> 56) != (pv >> 56));
        validm |= val ? 1u << j : 0u;
        psm |= p ? 1u << j : 0u;
        pidm |= d ? 1u << j : 0u;
        cnt += p ? 1u : 0u;
        a[j] = cnt;  // inclusive within the lane
    }
    if constexpr (kWPk && !kLex) {
        if (__ballot(coll)) return kRoundDefer;
    }
    uint32_t npairs;
    const uint32_t before = wave_excl_scan(cnt, npairs) - 1u;
#pragma unroll
    for (int j = 0; j < E; ++j) {
        a[j] += before;  // pair ordinal
        if ((psm >> j) & 1u) pstart[a[j]] = (uint16_t)(lane * E + j);
        if ((pidm >> j) & 1u) pbase[(uint32_t)(k[j] >> 56) & (kWCq - 1)] = a[j];
    }
    if (lane == 0) pstart[npairs] = (uint16_t)nc;
    wave_sync();
    uint32_t kpm = 0;
    {
        uint32_t pb[E];
#pragma unroll
        for (int j = 0; j < E; ++j) pb[j] = pbase[(uint32_t)(k[j] >> 56) & (kWCq - 1)];
#pragma unroll
        for (int j = 0; j < E; ++j) {
            const uint32_t rank = a[j] - pb[j];
            if (((psm >> j) & 1u) && rank == bp.mpc - 1)
                full[(uint32_t)(k[j] >> 56) & (kWCq - 1)] = 1u;
            kpm |= (((validm >> j) & 1u) && rank < bp.mpc) ? 1u << j : 0u;
        }
    }
    wave_sync();
    // pids filtered by their bound that show fewer than mpc candidate pairs
    // may own kept pairs above the bound
    {
        bool shrt = false;
#pragma unroll
        for (int jj = 0; jj < (int)(kWCq / 64); ++jj) {
            const uint32_t qq = lane + 64u * jj;
            const bool sh = pidc[qq] > 0 && cbnd[qq] != 0xFFFFFFFFu && full[qq] == 0;
            if (sh && !hbound) cbnd[qq] = 0xFFFFFFFFu;
            shrt |= sh;
        }
        if (__ballot(shrt) && !last_round) {
            wave_sync();
            if (hbound) {
                // a heavy chunk holds only its pid's candidates: the bucket
                // goes back to the global-memory kernel (rare)
                if (lane == 0) bp.heavy_fb[atomicAdd(bp.heavy_nfb, 1u)] = hidx;
                return kRoundDone;
            }
            return kRoundRestart;
        }
    }
    mark(bp, 2, clk);

    // ---- M: kept pairs; values of their records; mcpp sample of over-full
    // pairs by record priority
    uint32_t st[E], len[E], idx[E], pkf[E];  // pkf: the full partition key
    double v[E];
#pragma unroll
    for (int j = 0; j < E; ++j) {
        st[j] = pstart[min(a[j], L::CAP - 1)];
        len[j] = pstart[min(a[j] + 1, L::CAP)];
        idx[j] = kWPk ? cidx[min(o[j] & 511u, L::CAP - 1)] : o[j];
        pkf[j] = kWPk ? ((((uint32_t)k[j] & kPkMask) << pksh) | (o[j] >> 9)) : ((uint32_t)k[j] & kPkMask);
    }
    uint32_t overm = 0, maxlen = 0;
#pragma unroll
    for (int j = 0; j < E; ++j) {
        len[j] -= st[j];
        const bool kp = (kpm >> j) & 1u;
        const bool ov = sample && kp && len[j] > bp.mcpp;
        overm |= ov ? 1u << j : 0u;
        maxlen = max(maxlen, ov ? len[j] : 0u);
        // records of kept pairs within mcpp gather now; those of over-full
        // pairs only once the sample below has kept them (DPG_SORT_LATE 0:
        // every record of a kept pair gathers here)
        v[j] = (need_v && kp && (!kSortLate || !ov)) ? gather_value(bp.value, idx[j]) : 0.0;
    }
    uint32_t keepm = kpm;
    maxlen = __builtin_amdgcn_readfirstlane(wave_max_u32(maxlen));
    if (maxlen) {
        // record keys of over-full kept pairs, by sorted position; a record
        // is kept iff fewer than mcpp keys of its pair are smaller
#pragma unroll
        for (int j = 0; j < E; ++j) {
            if (!((overm >> j) & 1u)) continue;
            const uint32_t q = (uint32_t)(k[j] >> 56) & (kWCq - 1);
            rks[lane * E + j] = rec_prio_h(pidv[q], pkf[j], (uint64_t)(bp.rec_base + idx[j]));
        }
        wave_sync();
#pragma unroll
        for (int j = 0; j < E; ++j) {
            if (!__ballot((overm >> j) & 1u)) continue;
            const bool ov = (overm >> j) & 1u;
            const uint64_t mine = rks[lane * E + j];
            const uint32_t lm = max(len[j], 1u) - 1u;
            uint32_t below = 0;
            for (uint32_t t = 0; t < maxlen; t += 2) {
                const uint64_t y0 = rks[min(st[j] + min(t, lm), L::CAP - 1)];
                const uint64_t y1 = rks[min(st[j] + min(t + 1, lm), L::CAP - 1)];
                below += (t < len[j] && y0 < mine) ? 1u : 0u;
                below += (t + 1 < len[j] && y1 < mine) ? 1u : 0u;
            }
            if (ov && below >= bp.mcpp) keepm &= ~(1u << j);
        }
        if constexpr (kSortLate) {
            if (need_v) {
#pragma unroll
                for (int j = 0; j < E; ++j)
                    if ((overm & keepm) >> j & 1u) v[j] = gather_value(bp.value, idx[j]);
            }
        }
    }
    mark(bp, 3, clk);

    // ---- F: accumulators of kept records, one item per kept pair
    const uint32_t em = psm & kpm;
    if (need_v) {
        wave_sync();  // the accumulators overwrite the record keys of phase M
#pragma unroll
        for (int j = 0; j < E; ++j) {
            if (!((em >> j) & 1u)) continue;
            if (kSum) acc[a[j]] = 0.0;
            if (kVar) {
                acc_nsum[a[j]] = 0.0;
                acc_nsq[a[j]] = 0.0;
            }
        }
        wave_sync();
#pragma unroll
        for (int j = 0; j < E; ++j) {
            if (!((keepm >> j) & 1u)) continue;
            if (part_clip) {
                atomicAdd(&acc[a[j]], v[j]);
            } else {
                const double x = clampd(v[j], bp.lo, bp.hi);
                if (kSum) atomicAdd(&acc[a[j]], x);
                if (kVar) {
                    const double y = x - bp.mid;
                    atomicAdd(&acc_nsum[a[j]], y);
                    atomicAdd(&acc_nsq[a[j]], y * y);
                }
            }
        }
        wave_sync();
    }
#pragma unroll
    for (int j = 0; j < E; ++j) {
        const bool e = (em >> j) & 1u;
        const uint64_t be = __ballot(e);
        if (e) {
            Item it;
            it.pk = pkf[j];
            it.cnt = cap_pp ? min(len[j], bp.mcpp) : len[j];
            if constexpr (kSum) {
                const double s = need_v ? acc[a[j]] : 0.0;
                it.sum = (need_v && part_clip) ? clampd(s, bp.lo_pp, bp.hi_pp) : s;
            }
            if constexpr (kVar) {
                it.nsum = need_v ? acc_nsum[a[j]] : 0.0;
                it.nsq = need_v ? acc_nsq[a[j]] : 0.0;
            }
            items[nitems + lanes_below(be)] = it;
        }
        nitems += (uint32_t)__popcll(be);
    }
    mark(bp, 4, clk);
    return kRoundDone;
}

// One round: (first round only) records per pid slot, pid hashes and
// candidate bounds; pair priorities; candidates compacted into LDS; sort and
// bound.  Returns kRoundDone, kRoundRestart (see sort_chunk) or, in the
// narrow and mid passes, kRoundDefer (more than kC candidates, or a key
// collision of wide partition keys).
template <class Item, class R, bool kFirst, bool kWide, bool kWPk, int kC>
__device__ __forceinline__ int sort_round(const R (&r)[kWRPT], uint32_t n, uint32_t d1,
                                           uint32_t hbase, char *smem, const BoundParams &bp,
                                           Item *items, uint32_t &nitems, PhaseTimer &clk,
                                           uint32_t hbound, uint32_t hidx) {
    using L = SortLayout<Item, R, kWPk, kC>;
    uint32_t *pidv = reinterpret_cast<uint32_t *>(smem + L::PIDV);
    uint32_t *pidc = reinterpret_cast<uint32_t *>(smem + L::PIDC);
    uint32_t *cbnd = reinterpret_cast<uint32_t *>(smem + L::CBND);
    uint64_t *ckey = reinterpret_cast<uint64_t *>(smem + L::CK);
    uint32_t *cidx = reinterpret_cast<uint32_t *>(smem + L::CIDX);
    uint8_t *cpkl = reinterpret_cast<uint8_t *>(smem + L::CPKL);
    uint32_t *olist = reinterpret_cast<uint32_t *>(smem + L::PSTART);
    const uint32_t lane = __lane_id();
    const Fmt f = bp.fmt;
    const uint32_t pkb = f.pkbits;
    const uint64_t pkmask = (1ull << pkb) - 1ull;
    const uint32_t hshift = f.kbits - f.b1;
    const uint32_t kn = (n + 63) >> 6;  // occupied record slots per lane (uniform)
    const uint32_t pksh = kWPk ? pkb - kSkPkBits : 0u;

    // ---- A: records per pid slot, pair priorities, candidates
    uint64_t sk[kWRPT];  // q << 56 | pk (pp << 24 | pk >> pksh below)
    uint32_t ix[kWRPT];
    uint32_t validm = 0;
#pragma unroll
    for (int k = 0; k < kWRPT && k < (int)kn; ++k) {
        validm |= lane + 64u * k < n ? 1u << k : 0u;
        const uint64_t key = RecOps<R>::key(r[k], f);
        const uint32_t q = ((uint32_t)(key >> pkb) - hbase) & (kWCq - 1);
        sk[k] = ((uint64_t)q << 56) | (key & pkmask);
        ix[k] = RecOps<R>::idx(r[k], f);
    }
    if constexpr (kFirst) {
#pragma unroll
        for (int k = 0; k < kWRPT && k < (int)kn; ++k)
            if ((validm >> k) & 1u) atomicAdd(&pidc[(uint32_t)(sk[k] >> 56)], 1u);
        wave_sync();
        // pid hash and candidate bound of the occupied slots (compacted)
        const float cmul = bp.cand_mul;
        uint32_t nocc = 0;
#pragma unroll
        for (int j = 0; j < (int)(kWCq / 64); ++j) {
            const uint32_t qq = lane + 64u * j;
            const bool occ = pidc[qq] > 0;
            const uint64_t bo = __ballot(occ);
            if (occ) olist[nocc + lanes_below(bo)] = qq;
            nocc += (uint32_t)__popcll(bo);
        }
        wave_sync();
        float est = 0.0f;  // expected candidates: all records of unfiltered pids, ~cmul of the others
        for (uint32_t o = 0; o < nocc; o += 64) {
            if (o + lane < nocc) {
                const uint32_t qq = olist[o + lane];
                pidv[qq] = pid_hash(bp.seed, (uint64_t)(bp.pid_min + (int64_t)hk_inv(
                                                            (d1 << hshift) | (hbase + qq), bp.hash)));
                const uint32_t rc = pidc[qq];
                const float fr = cmul / (float)rc;
                const bool all = hbound || rc <= bp.mpc || fr >= 1.0f;
                cbnd[qq] = hbound ? hbound : all ? 0xFFFFFFFFu : (uint32_t)(fr * 4294967296.0f);
                est += all ? (float)rc : cmul;
            }
        }
        wave_sync();
        if constexpr (!kWide) {
            // a chunk that will hold more candidates than the working set goes
            // to the wide pass before its priorities are drawn
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) est += __shfl_xor(est, o, 64);
            if (bp.defer_est > 0.0f && est > bp.defer_est) return kRoundDefer;
        }
    }
    uint32_t nc = 0;
    {
        uint32_t pv[kWRPT], cb[kWRPT];
#pragma unroll
        for (int k = 0; k < kWRPT && k < (int)kn; ++k) {
            pv[k] = pidv[(uint32_t)(sk[k] >> 56)];
            cb[k] = cbnd[(uint32_t)(sk[k] >> 56)];
        }
#pragma unroll
        for (int k = 0; k < kWRPT && k < (int)kn; ++k) {
            const uint32_t pk = (uint32_t)sk[k];
            const uint32_t pp = pair_prio_h(pv[k], pk);
            if constexpr (kWPk) sk[k] = (sk[k] & ~(uint64_t)0xFFFFFFFFu) | (pk >> pksh);
            sk[k] |= (uint64_t)pp << kSkPkBits;
            const bool c = ((validm >> k) & 1u) && pp <= cb[k];
            const uint64_t bc = __ballot(c);
            // the working set holds kC candidates: past them the chunk is
            // deferred below (narrow and mid passes), so the rest need no slot
            const uint32_t e = nc + lanes_below(bc);
            if (c && e < L::CAP) {
                ckey[e] = sk[k];
                cidx[e] = ix[k];
                if constexpr (kWPk) cpkl[e] = (uint8_t)(pk & ((1u << pksh) - 1u));
            }
            nc += (uint32_t)__popcll(bc);
        }
    }
    wave_sync();
    mark(bp, 0, clk);
    if constexpr (!kWide) {
        if (nc > (uint32_t)kC) return kRoundDefer;
    }
    constexpr bool last = !kFirst;
    constexpr bool kLex = kWide && kWPk;
    int st;
    if (nc <= 64) {
        st = sort_chunk<Item, R, 1, kWPk, kLex, L::CAP>(nc, smem, bp, last, hbound, hidx, items, nitems, clk);
    } else if (nc <= 128 || (!kWide && kC <= 128)) {
        st = sort_chunk<Item, R, 2, kWPk, kLex, L::CAP>(nc, smem, bp, last, hbound, hidx, items, nitems, clk);
    } else if constexpr (kWide || kC > 128) {
        if (!kWide || nc <= 256)
            st = sort_chunk<Item, R, 4, kWPk, kLex, L::CAP>(nc, smem, bp, last, hbound, hidx, items, nitems,
                                                    clk);
        else
            st = sort_chunk<Item, R, kWide ? 8 : 4, kWPk, kLex, L::CAP>(nc, smem, bp, last, hbound, hidx,
                                                                items, nitems, clk);
    }
    wave_sync();
    return st;
}

// One small chunk.  When the first round finds a filtered pid short of mpc
// candidate pairs, the chunk's records are loaded again (L2-hot) and a
// second round runs with that pid's bound lifted: keeping the records in
// registers across the sort would cost the occupancy the kernel lives on.
// Returns true when the chunk was deferred to the wide kernel (nothing
// emitted).
template <class Item, class R, bool kWide, bool kWPk, int kC>
__device__ __forceinline__ bool sort_bound_chunk(const R (&r0)[kWRPT], const R *base, uint32_t n,
                                                 uint32_t d1, uint32_t hbase, char *smem,
                                                 const BoundParams &bp, Item *items,
                                                 uint32_t &nitems, PhaseTimer &clk,
                                                 uint32_t hbound, uint32_t hidx) {
    using L = SortLayout<Item, R, kWPk, kC>;
    uint32_t *pidc = reinterpret_cast<uint32_t *>(smem + L::PIDC);
    const uint32_t lane = __lane_id();
    int st = sort_round<Item, R, true, kWide, kWPk, kC>(r0, n, d1, hbase, smem, bp, items, nitems, clk,
                                              hbound, hidx);
    if (st == kRoundRestart) {
        R r[kWRPT];
#pragma unroll
        for (int k = 0; k < kWRPT; ++k) r[k] = base[min(lane + 64u * k, n - 1)];
        st = sort_round<Item, R, false, kWide, kWPk, kC>(r, n, d1, hbase, smem, bp, items, nitems, clk,
                                               hbound, hidx);
    }
#pragma unroll
    for (int j = 0; j < (int)(kWCq / 64); ++j) pidc[lane + 64u * j] = 0;
    wave_sync();
    mark(bp, 5, clk);
    return st == kRoundDefer;
}

// One round over a medium chunk (n > kWCap records of one fine bucket, <= 128
// pid slots) in pieces of kWCap records, re-read from memory (L2-hot after
// the first pass): (first round only) records per pid slot over every piece,
// then pid hashes and candidate bounds; then the candidates of every piece
// compacted into LDS -- the working set holds the candidates, never the
// chunk.  Returns as sort_round; kRoundDefer when more than kC candidates
// pass (the chunk is left to the hash-table kernel).
template <class Item, class R, bool kFirst, bool kWPk, int kC>
__device__ __forceinline__ int stream_round(const R *base, uint32_t n, uint32_t d1, uint32_t hbase,
                                            char *smem, const BoundParams &bp, Item *items,
                                            uint32_t &nitems, PhaseTimer &clk) {
    using L = SortLayout<Item, R, kWPk, kC>;
    uint32_t *pidv = reinterpret_cast<uint32_t *>(smem + L::PIDV);
    uint32_t *pidc = reinterpret_cast<uint32_t *>(smem + L::PIDC);
    uint32_t *cbnd = reinterpret_cast<uint32_t *>(smem + L::CBND);
    uint64_t *ckey = reinterpret_cast<uint64_t *>(smem + L::CK);
    uint32_t *cidx = reinterpret_cast<uint32_t *>(smem + L::CIDX);
    uint8_t *cpkl = reinterpret_cast<uint8_t *>(smem + L::CPKL);
    uint32_t *olist = reinterpret_cast<uint32_t *>(smem + L::PSTART);
    const uint32_t lane = __lane_id();
    const Fmt f = bp.fmt;
    const uint32_t pkb = f.pkbits;
    const uint64_t pkmask = (1ull << pkb) - 1ull;
    const uint32_t hshift = f.kbits - f.b1;
    const uint32_t pksh = kWPk ? pkb - kSkPkBits : 0u;
    auto load = [&](uint32_t p0, uint32_t m, R (&r)[kWRPT]) {
#pragma unroll
        for (int k = 0; k < kWRPT; ++k) r[k] = base[p0 + min(lane + 64u * k, m - 1)];
    };
    if constexpr (kFirst) {
        for (uint32_t p0 = 0; p0 < n; p0 += kWCap) {
            const uint32_t m = min(n - p0, (uint32_t)kWCap);
            R r[kWRPT];
            load(p0, m, r);
#pragma unroll
            for (int k = 0; k < kWRPT; ++k) {
                const uint32_t q = ((uint32_t)(RecOps<R>::key(r[k], f) >> pkb) - hbase) & (kWCq - 1);
                if (lane + 64u * k < m) atomicAdd(&pidc[q], 1u);
            }
        }
        wave_sync();
        const float cmul = bp.cand_mul;
        const float big = fmaxf(cmul, fminf(kStreamMul * cmul, 0.5f * (float)kC));
        uint32_t nocc = 0;
#pragma unroll
        for (int j = 0; j < (int)(kWCq / 64); ++j) {
            const uint32_t qq = lane + 64u * j;
            const bool occ = pidc[qq] > 0;
            const uint64_t bo = __ballot(occ);
            if (occ) olist[nocc + lanes_below(bo)] = qq;
            nocc += (uint32_t)__popcll(bo);
        }
        wave_sync();
        float est = 0.0f;  // expected candidates (see sort_round)
        for (uint32_t o = 0; o < nocc; o += 64) {
            if (o + lane < nocc) {
                const uint32_t qq = olist[o + lane];
                pidv[qq] = pid_hash(bp.seed, (uint64_t)(bp.pid_min + (int64_t)hk_inv(
                                                            (d1 << hshift) | (hbase + qq), bp.hash)));
                const uint32_t rc = pidc[qq];
                const float aim = rc > kStreamBig ? big : cmul;
                const float fr = aim / (float)rc;
                const bool all = rc <= bp.mpc || fr >= 1.0f;
                cbnd[qq] = all ? 0xFFFFFFFFu : (uint32_t)(fr * 4294967296.0f);
                est += all ? (float)rc : aim;
            }
        }
        wave_sync();
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) est += __shfl_xor(est, o, 64);
        if (bp.defer_est > 0.0f && est > bp.defer_est) return kRoundDefer;
    }
    uint32_t nc = 0;
    for (uint32_t p0 = 0; p0 < n; p0 += kWCap) {
        const uint32_t m = min(n - p0, (uint32_t)kWCap);
        R r[kWRPT];
        load(p0, m, r);
#pragma unroll
        for (int k = 0; k < kWRPT; ++k) {
            const uint64_t key = RecOps<R>::key(r[k], f);
            const uint32_t q = ((uint32_t)(key >> pkb) - hbase) & (kWCq - 1);
            const uint32_t pk = (uint32_t)(key & pkmask);
            const uint32_t pp = pair_prio_h(pidv[q], pk);
            uint64_t sk = ((uint64_t)q << 56) | (uint64_t)(kWPk ? (pk >> pksh) : pk);
            sk |= (uint64_t)pp << kSkPkBits;
            const bool c = lane + 64u * k < m && pp <= cbnd[q];
            const uint64_t bc = __ballot(c);
            const uint32_t e = nc + lanes_below(bc);
            if (c && e < L::CAP) {
                ckey[e] = sk;
                cidx[e] = RecOps<R>::idx(r[k], f);
                if constexpr (kWPk) cpkl[e] = (uint8_t)(pk & ((1u << pksh) - 1u));
            }
            nc += (uint32_t)__popcll(bc);
        }
    }
    wave_sync();
    mark(bp, 0, clk);
    if (nc > (uint32_t)kC) return kRoundDefer;
    constexpr bool last = !kFirst;
    int st;
    if (nc <= 64)
        st = sort_chunk<Item, R, 1, kWPk, false, L::CAP>(nc, smem, bp, last, 0u, 0u, items, nitems, clk);
    else if (nc <= 128)
        st = sort_chunk<Item, R, 2, kWPk, false, L::CAP>(nc, smem, bp, last, 0u, 0u, items, nitems, clk);
    else
        st = sort_chunk<Item, R, 4, kWPk, false, L::CAP>(nc, smem, bp, last, 0u, 0u, items, nitems, clk);
    wave_sync();
    return st;
}

// One medium chunk by stream_round (a second round when a filtered pid is
// short of mpc candidate pairs).  Returns true when the chunk was deferred
// (nothing emitted: a restart or a deferral happens before any item).
template <class Item, class R, bool kWPk, int kC>
__device__ __forceinline__ bool stream_bound_chunk(const R *base, uint32_t n, uint32_t d1,
                                                   uint32_t hbase, char *smem, const BoundParams &bp,
                                                   Item *items, uint32_t &nitems, PhaseTimer &clk) {
    using L = SortLayout<Item, R, kWPk, kC>;
    uint32_t *pidc = reinterpret_cast<uint32_t *>(smem + L::PIDC);
    const uint32_t lane = __lane_id();
    int st = stream_round<Item, R, true, kWPk, kC>(base, n, d1, hbase, smem, bp, items, nitems, clk);
    if (st == kRoundRestart)
        st = stream_round<Item, R, false, kWPk, kC>(base, n, d1, hbase, smem, bp, items, nitems, clk);
#pragma unroll
    for (int j = 0; j < (int)(kWCq / 64); ++j) pidc[lane + 64u * j] = 0;
    wave_sync();
    mark(bp, 5, clk);
    return st == kRoundDefer;
}

// Persistent single-wave workgroups walk the small-chunk list statically
// (w, w + G1, ...), as k_bound_waves; narrow workgroup g appends its items
// to items[wg_off[g], ...) and leaves the count in wg_cnt[g], and flags the
// chunks it defers in defer[w].  A deferred pass's workgroup g2 then takes
// the narrow workgroups g = g2, g2 + gridDim.x, ... and bounds their flagged
// chunks, appending behind wg_cnt[g] (the mid pass clears the flag of a
// chunk it bounds).  The narrow pass may load the next chunk's records while
// the current one is bounded (kSortPF).
template <class Item, class R, int kTier, bool kWPk>
__global__ __launch_bounds__(64, (kTierWPS<R, kTier>)) void k_bound_sorted(
    const R *recs, const R *refined, const R *heavy, const uint4 *chunks, const uint32_t *n_chunks,
    BoundParams bp, Item *items, const int64_t *wg_off, uint32_t *wg_cnt, uint8_t *defer,
    uint32_t G1) {
    constexpr bool kWide = kTier == 2;
    constexpr int kC = kTierCand<R, kTier>;
    using L = SortLayout<Item, R, kWPk, kC>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    PhaseTimer clk;
    timer_start(bp, clk);
    // parameters used in one phase each: vector registers (see vreg).  The
    // wide kernel is short of scalar registers, not of vector ones: all of
    // them; the narrow one (<= 128 VGPRs) moves the 64-bit ones only, and
    // only with 8-byte records (the 12-byte ones need those registers)
    constexpr int kVreg = sizeof(R) == 8 ? DPG_SORT_VREG : 0;
    if constexpr (kWide || kVreg >= 1) {
        bp.lo = vreg(bp.lo);
        bp.hi = vreg(bp.hi);
        bp.lo_pp = vreg(bp.lo_pp);
        bp.hi_pp = vreg(bp.hi_pp);
        bp.mid = vreg(bp.mid);
        bp.seed = vreg(bp.seed);
        bp.pid_min = vreg(bp.pid_min);
        bp.rec_base = vreg(bp.rec_base);
        bp.value = vreg(bp.value);
    }
    if constexpr (kWide || kVreg >= 2) {
        bp.hash.mask = vreg(bp.hash.mask);
        bp.hash.i1 = vreg(bp.hash.i1);
        bp.hash.i2 = vreg(bp.hash.i2);
        bp.mpc = vreg(bp.mpc);
        bp.mcpp = vreg(bp.mcpp);
        bp.fmt.ib = vreg(bp.fmt.ib);
        bp.fmt.pkbits = vreg(bp.fmt.pkbits);
        bp.fmt.kbits = vreg(bp.fmt.kbits);
        bp.fmt.b1 = vreg(bp.fmt.b1);
        bp.heavy_fb = vreg(bp.heavy_fb);
        bp.heavy_nfb = vreg(bp.heavy_nfb);
    }
    const uint32_t nch = __builtin_amdgcn_readfirstlane(*n_chunks);
    const uint32_t lane = __lane_id();
    {
        uint32_t *pidc = reinterpret_cast<uint32_t *>(smem + L::PIDC);
        for (uint32_t i = lane; i < kWCq; i += 64) pidc[i] = 0;
    }
    wave_sync();
    auto desc = [&](uint32_t w) {
        return make_uint4(__builtin_amdgcn_readfirstlane(chunks[w].x),
                          __builtin_amdgcn_readfirstlane(chunks[w].y),
                          __builtin_amdgcn_readfirstlane(chunks[w].z),
                          __builtin_amdgcn_readfirstlane(chunks[w].w));
    };
    if constexpr (kTier == 0) {
        constexpr bool kPF = kSortPF<R>;
        uint32_t nitems = 0;
        Item *my_items = items + wg_off[blockIdx.x];
        R r[kWRPT], rn[kWRPT];
        uint4 d = make_uint4(0, 0, 0, 0);
        if (blockIdx.x < nch) {
            d = desc(blockIdx.x);
            const uint32_t n = d.y & kChunkCount;
            const R *b = wave_chunk_base(d, recs, refined, heavy);
#pragma unroll
            for (int k = 0; k < kWRPT; ++k) r[k] = b[min(lane + 64u * k, n - 1)];
        }
        for (uint32_t w = blockIdx.x; w < nch; w += G1) {
            uint4 du = make_uint4(0, 0, 0, 0);
            if (kPF && w + G1 < nch) {
                du = desc(w + G1);
                const uint32_t nn = du.y & kChunkCount;
                const R *nb = wave_chunk_base(du, recs, refined, heavy);
#pragma unroll
                for (int k = 0; k < kWRPT; ++k) rn[k] = nb[min(lane + 64u * k, nn - 1)];
            }
            const bool df = sort_bound_chunk<Item, R, false, kWPk, kC>(
                r, wave_chunk_base(d, recs, refined, heavy), d.y & kChunkCount, d.z & 0xFFFFu, d.w,
                smem, bp, my_items, nitems, clk, heavy_bound(d), d.x / (uint32_t)kWCap);
            if (lane == 0) defer[w] = df ? 1 : 0;
            if constexpr (kPF) {
#pragma unroll
                for (int k = 0; k < kWRPT; ++k) r[k] = rn[k];
                d = du;
            } else if (w + G1 < nch) {
                d = desc(w + G1);
                const uint32_t nn = d.y & kChunkCount;
                const R *nb = wave_chunk_base(d, recs, refined, heavy);
#pragma unroll
                for (int k = 0; k < kWRPT; ++k) r[k] = nb[min(lane + 64u * k, nn - 1)];
            }
        }
        if (lane == 0) wg_cnt[blockIdx.x] = nitems;
    } else if constexpr (kTier == 3) {
        // the medium-chunk list, statically (w, w + G, ...); workgroup g
        // appends to items[wg_off[g], ...) and flags the chunks it defers --
        // except entries w >= G1, oversize buckets (k_over_to_medium), which
        // go back to the global-memory kernel as oversize bucket w - G1
        uint32_t nitems = 0;
        Item *my_items = items + wg_off[blockIdx.x];
        for (uint32_t w = blockIdx.x; w < nch; w += gridDim.x) {
            const uint4 d = desc(w);
            const bool df = stream_bound_chunk<Item, R, kWPk, kC>(
                wave_chunk_base(d, recs, refined, heavy), d.y & kChunkCount, d.z & 0xFFFFu, d.w,
                smem, bp, my_items, nitems, clk);
            if (lane == 0) {
                const bool over = w >= G1;
                if (df && over) bp.heavy_fb[atomicAdd(bp.heavy_nfb, 1u)] = w - G1;
                defer[w] = df && !over ? 1 : 0;
            }
        }
        if (lane == 0) wg_cnt[blockIdx.x] = nitems;
    } else {
        for (uint32_t g = blockIdx.x; g < G1; g += gridDim.x) {
            uint32_t nitems = __builtin_amdgcn_readfirstlane(wg_cnt[g]);
            Item *my_items = items + wg_off[g];
            bool any = false;
            // the flags of 64 of g's chunks per load, then the set ones
            for (uint32_t i0 = 0; g + i0 * G1 < nch; i0 += 64) {
                const uint32_t wl = g + (i0 + lane) * G1;
                for (uint64_t fm = __ballot(wl < nch && defer[min(wl, nch - 1)] != 0); fm;
                     fm &= fm - 1) {
                    const uint32_t w = g + (i0 + (uint32_t)__builtin_ctzll(fm)) * G1;
                    any = true;
                    const uint4 d = desc(w);
                    const uint32_t n = d.y & kChunkCount;
                    const R *b = wave_chunk_base(d, recs, refined, heavy);
                    R r[kWRPT];
#pragma unroll
                    for (int k = 0; k < kWRPT; ++k) r[k] = b[min(lane + 64u * k, n - 1)];
                    const bool df = sort_bound_chunk<Item, R, kWide, kWPk, kC>(
                        r, b, n, d.z & 0xFFFFu, d.w, smem, bp, my_items, nitems, clk,
                        heavy_bound(d), d.x / (uint32_t)kWCap);
                    if (kTier == 1 && lane == 0) defer[w] = df ? 1 : 0;
                }
            }
            if (any && lane == 0) wg_cnt[g] = nitems;
        }
    }
    timer_flush(bp, clk);
}

}  // namespace dpg
