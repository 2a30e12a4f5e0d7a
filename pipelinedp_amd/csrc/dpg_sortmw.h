// dpg_sortmw.h -- sort-based contribution bounding of one chunk by a
// workgroup of NW waves (gfx950): the chunks the single-wave sort kernel
// (dpg_sortb.h) cannot hold at 4 waves per SIMD.
//
//  * NW = 2 (k_bound_sorted_w2): small chunks (<= 512 records) with more
//    than kNarrowCand = 256 candidate records.  The single-wave version
//    sorts 8 elements per lane and needs ~230 VGPRs (2 waves per SIMD); two
//    waves of 4 elements per lane stay under 128 VGPRs (4 waves per SIMD).
//  * NW = 4 (k_bound_sorted_m4): medium chunks (one fine bucket of 513..1024
//    records), instead of the 256-thread hash-table kernel (dpg_chunk.h).
//
// Same algorithm, same sort key and hence bit-identical kept sets as
// dpg_sortb.h (pid slot | pair priority | pk; contribution_bounders.py:
// 56-105 -- a pair is kept iff fewer than mpc pairs of its pid precede it in
// (priority, pk) order, a record iff fewer than mcpp records of its pair
// have a smaller record priority).  Element i of the chunk's sorted
// candidates lives in thread i / 4, slot i % 4: each wave sorts its 256
// elements with the single-wave network (bitonic_sort<4>); the merges of
// 512- and 1024-element blocks add three (NW = 4) or one (NW = 2)
// compare-exchange steps across waves, through LDS.  The scans, ballots and
// maxima of the single-wave kernel become workgroup-wide (two barriers
// each); per-element state and the LDS tables (pid slots, pair starts,
// accumulators by pair ordinal) keep their meaning.
#pragma once

#include "dpg_sortb.h"

namespace dpg {

template <class Item, class R, bool kWPk, int NW>
struct SortLayoutMW {
    static constexpr int T = 64 * NW;    // threads
    static constexpr int CAP = 4 * T;    // records / candidates per chunk
    static constexpr int PB = NW == 2 ? 9 : 10;  // bits of a candidate position
    static_assert((1 << PB) == CAP, "position bits");
    static constexpr int NACC = ItemTraits<Item>::var ? (ItemTraits<Item>::sum ? 3 : 2) : 1;
    static constexpr size_t PIDC = 0;                  // records per pid slot
    static constexpr size_t PIDV = PIDC + 4 * kWCq;    // pid hash
    static constexpr size_t CBND = PIDV + 4 * kWCq;    // candidate bound
    static constexpr size_t PBASE = CBND + 4 * kWCq;   // ordinal of the pid's first pair
    static constexpr size_t FULL = PBASE + 4 * kWCq;   // pid shows >= mpc candidate pairs
    static constexpr size_t PSTART = FULL + 4 * kWCq;  // first position per pair (u16)
    static constexpr size_t CK = PSTART + a16(2 * (CAP + 1));
    // candidate keys u64[CAP] + record indices u32[CAP]; then record keys by
    // position (u64); then NACC accumulators per pair (f64)
    static constexpr size_t CIDX = CK + 8 * CAP;
    static constexpr size_t CKSZ = 12 * CAP > 8 * NACC * CAP ? 12 * CAP : 8 * NACC * CAP;
    static constexpr size_t CPKL = CK + CKSZ;  // kWPk: low pk bits per candidate (u8)
    // cross-wave exchange of the sort (u64 keys, u32 payloads), then each
    // thread's last element (the next thread's predecessor)
    static constexpr size_t XCH = a16(CPKL + (kWPk ? CAP : 0));
    static constexpr size_t SCR = XCH + 12 * CAP;  // u32[32]: wave partials, flags
    static constexpr size_t END = SCR + 128;
    static constexpr size_t TOTAL = (END + 255) & ~(size_t)255;
};

// ---- workgroup primitives (all threads call them, control flow uniform)
template <int NW>
__device__ __forceinline__ uint32_t mw_excl_scan(uint32_t x, uint32_t &total, uint32_t *scr) {
    const uint32_t w = threadIdx.x >> 6;
    uint32_t wt;
    const uint32_t e = wave_excl_scan(x, wt);
    if (__lane_id() == 0) scr[w] = wt;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
        const uint32_t y = scr[k];
        pre += k < (int)w ? y : 0u;
        tot += y;
    }
    __syncthreads();
    total = tot;
    return e + pre;
}

template <int NW>
__device__ __forceinline__ uint32_t mw_max(uint32_t x, uint32_t *scr) {
    x = wave_max_u32(x);
    if (__lane_id() == 0) scr[threadIdx.x >> 6] = x;
    __syncthreads();
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < NW; ++k) m = max(m, scr[k]);
    __syncthreads();
    return m;
}

template <int NW>
__device__ __forceinline__ bool mw_any(bool b, uint32_t *scr) {
    return mw_max<NW>(__ballot(b) != 0 ? 1u : 0u, scr) != 0;
}

// Half-cleaners of a 256-element block inside one wave (E = 4 elements per
// lane): partner distances 128 .. 1, minimum to the lower index (the tail
// of bitonic_sort<4>'s last merge).
template <bool kLex>
__device__ __forceinline__ void half_clean_256(uint64_t (&k)[4], uint32_t (&o)[4]) {
    uint32_t lid = __lane_id();
    asm volatile("" : "+v"(lid));
    auto less = [](uint64_t a, uint32_t oa, uint64_t b, uint32_t ob) {
        return kLex ? (a < b || (a == b && oa < ob)) : a < b;
    };
#pragma unroll
    for (int ls = 7; ls >= 0; --ls) {
        const int sd = 1 << ls;
        if (ls < 2) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (j & sd) continue;
                const int j2 = j | sd;
                const bool sw = less(k[j2], o[j2], k[j], o[j]);
                const uint64_t a = k[j], b = k[j2];
                const uint32_t oa = o[j], ob = o[j2];
                k[j] = sw ? b : a;
                k[j2] = sw ? a : b;
                o[j] = sw ? ob : oa;
                o[j2] = sw ? oa : ob;
            }
        } else {
            const int m = sd >> 2;
            const bool lower = (lid & (uint32_t)m) == 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint64_t y = xlane64(k[j], m);
                const uint32_t yo = xlane(o[j], m);
                const bool take = lower ? less(y, yo, k[j], o[j]) : less(k[j], o[j], y, yo);
                k[j] = take ? y : k[j];
                o[j] = take ? yo : o[j];
            }
        }
    }
}

// One compare-exchange step across waves through LDS: element (wave w,
// lane l, slot j) meets (pw, mirror ? 63 - l : l, mirror ? 3 - j : j); the
// lower index keeps the minimum.
template <bool kLex>
__device__ __forceinline__ void cross_wave_step(uint64_t (&k)[4], uint32_t (&o)[4], uint64_t *xk,
                                                uint32_t *xo, uint32_t pw, bool mirror,
                                                bool lower) {
    auto less = [](uint64_t a, uint32_t oa, uint64_t b, uint32_t ob) {
        return kLex ? (a < b || (a == b && oa < ob)) : a < b;
    };
    const uint32_t t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        xk[4 * t + j] = k[j];
        xo[4 * t + j] = o[j];
    }
    __syncthreads();
    const uint32_t l = __lane_id();
    const uint32_t pt = pw * 64 + (mirror ? 63 - l : l);
    uint64_t y[4];
    uint32_t yo[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t pj = mirror ? 3 - j : j;
        y[j] = xk[4 * pt + pj];
        yo[j] = xo[4 * pt + pj];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const bool take = lower ? less(y[j], yo[j], k[j], o[j]) : less(k[j], o[j], y[j], yo[j]);
        k[j] = take ? y[j] : k[j];
        o[j] = take ? yo[j] : o[j];
    }
}

// The same two steps over float64-packed keys alone (bitonic_sort_keys_f64,
// dpg_sortb.h): one v_min_f64 / v_max_f64 per compare-exchange.
__device__ __forceinline__ void half_clean_256_f64(uint64_t (&k)[4]) {
    uint32_t lid = __lane_id();
    asm volatile("" : "+v"(lid));
#pragma unroll
    for (int ls = 7; ls >= 0; --ls) {
        const int sd = 1 << ls;
        if (ls < 2) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (j & sd) continue;
                const int j2 = j | sd;
                const uint64_t a = k[j], b = k[j2];
                k[j] = fmin_bits(a, b);
                k[j2] = fmax_bits(a, b);
            }
        } else {
            const int m = sd >> 2;
            const bool lower = (lid & (uint32_t)m) == 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint64_t y = xlane64(k[j], m);
                k[j] = lower ? fmin_bits(k[j], y) : fmax_bits(k[j], y);
            }
        }
    }
}

__device__ __forceinline__ void cross_wave_step_f64(uint64_t (&k)[4], uint64_t *xk, uint32_t pw,
                                                    bool mirror, bool lower) {
    const uint32_t t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) xk[4 * t + j] = k[j];
    __syncthreads();
    const uint32_t l = __lane_id();
    const uint32_t pt = pw * 64 + (mirror ? 63 - l : l);
    uint64_t y[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) y[j] = xk[4 * pt + (mirror ? 3 - j : j)];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j) k[j] = lower ? fmin_bits(k[j], y[j]) : fmax_bits(k[j], y[j]);
}

// Ascending sort of the workgroup's 256 NW elements (element i in thread
// i / 4, slot i % 4).
template <int NW, bool kLex>
__device__ __forceinline__ void mw_sort(uint64_t (&k)[4], uint32_t (&o)[4], uint64_t *xk,
                                        uint32_t *xo) {
    bitonic_sort<4, kLex>(k, o);  // every wave's 256 elements
    const uint32_t w = threadIdx.x >> 6;
    // 512-element blocks: mirror step between waves w and w ^ 1
    cross_wave_step<kLex>(k, o, xk, xo, w ^ 1u, true, (w & 1u) == 0);
    half_clean_256<kLex>(k, o);
    if constexpr (NW == 4) {
        // 1024: mirror step between waves w and 3 - w, half-cleaner at 256
        cross_wave_step<kLex>(k, o, xk, xo, 3u - w, true, w < 2u);
        cross_wave_step<kLex>(k, o, xk, xo, w ^ 1u, false, (w & 1u) == 0);
        half_clean_256<kLex>(k, o);
    }
}

// Phases S, P, M, F of sort_chunk (dpg_sortb.h) for a workgroup of NW
// waves; returns kRoundRestart / kRoundDone as there.
template <class Item, class R, bool kWPk, int NW>
__device__ __forceinline__ int mw_sort_chunk(uint32_t nc, char *smem, const BoundParams &bp,
                                              bool last_round, uint32_t hbound, uint32_t hidx,
                                              Item *items, uint32_t &nitems, PhaseTimer &clk) {
    using L = SortLayoutMW<Item, R, kWPk, NW>;
    constexpr int T = L::T, CAP = L::CAP, PB = L::PB;
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
    double *acc_nsum = acc + (kSum ? CAP : 0);
    double *acc_nsq = acc_nsum + CAP;
    uint64_t *xk = reinterpret_cast<uint64_t *>(smem + L::XCH);
    uint32_t *xo = reinterpret_cast<uint32_t *>(smem + L::XCH + 8 * CAP);
    uint32_t *scr = reinterpret_cast<uint32_t *>(smem + L::SCR);
    const uint32_t tid = threadIdx.x;
    const Fmt f = bp.fmt;
    const bool need_v = bp.need_values != 0;
    const bool cap_pp = bp.mode == DPG_MODE_CROSS_AND_PER_PARTITION;
    const bool sample = cap_pp && need_v;
    const bool part_clip = bp.sum_mode == DPG_SUM_CLIP_PARTITION;
    constexpr uint32_t kPkMask = (1u << kSkPkBits) - 1u;
    const uint32_t pksh = kWPk ? f.pkbits - kSkPkBits : 0u;

    // ---- S: sort (key, record index | kWPk: position | low pk bits << PB)
    uint64_t k[4];
    uint32_t o[4];
    auto load = [&]() {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t i = 4 * tid + j;
            const uint32_t ic = min(i, (uint32_t)CAP - 1);
            const uint64_t x = ckey[ic];
            const uint32_t y = kWPk ? (ic | ((uint32_t)cpkl[ic] << PB)) : cidx[ic];
            k[j] = i < nc ? x : kSkPad;
            o[j] = i < nc ? y : 0u;
        }
    };
    load();
    for (uint32_t q = tid; q < kWCq; q += T) full[q] = 0;
    bool sorted_packed = false;
    if constexpr (NW == 2 && DPG_SORT_PACKED) {
        // keys alone, packed as positive normal float64 (dpg_sortb.h
        // sort_chunk): tag 01 | pid slot | top 45 - pkbits bits of the pair
        // priority | the full partition key | position (9 bits); the keys
        // and payloads are read back by position.  Pairs of one pid whose
        // priorities agree in the kept bits may come out in pk order: the
        // order is checked on (key, low pk bits) and, if broken, the chunk
        // is sorted again the payload way below.  Partition keys over 29
        // bits keep too few priority bits for this to pay.
        const uint32_t pkb = f.pkbits;
        if (pkb <= 29) {
            const uint32_t ppb = min(32u, 45u - pkb);
            const uint64_t pkm = (1ull << pkb) - 1ull;
            uint64_t pk64[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t i = 4 * tid + j;
                const uint64_t x = k[j];
                const uint64_t pp = (x >> kSkPkBits) & 0xFFFFFFFFull;
                const uint64_t pkfull = kWPk ? ((((uint64_t)x & kPkMask) << pksh) | (uint64_t)(o[j] >> PB))
                                             : (x & pkm);
                pk64[j] = i < nc ? (kSkTagF | ((x >> 56) << 54) | ((pp >> (32u - ppb)) << (9u + pkb)) |
                                    (pkfull << 9) | (uint64_t)i)
                                 : kSkPadF;
            }
            bitonic_sort_keys_f64<4>(pk64);
            const uint32_t w = threadIdx.x >> 6;
            cross_wave_step_f64(pk64, xk, w ^ 1u, true, (w & 1u) == 0);
            half_clean_256_f64(pk64);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t pos = (uint32_t)pk64[j] & 511u;
                const bool v = pk64[j] != kSkPadF;
                k[j] = v ? ckey[pos] : kSkPad;
                o[j] = v ? (kWPk ? (pos | ((uint32_t)cpkl[pos] << PB)) : cidx[pos]) : 0u;
            }
            __syncthreads();  // xk: the sort's exchange area, now each thread's last element
            xk[tid] = k[3];
            xo[tid] = o[3];
            __syncthreads();
            const uint64_t pk0 = tid ? xk[tid - 1] : 0ull;
            const uint32_t po0 = tid ? xo[tid - 1] : 0u;
            bool bad = false;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t i = 4 * tid + j;
                const uint64_t pv = j ? k[j - 1] : pk0;
                const uint32_t pvl = (j ? o[j - 1] : po0) >> PB;
                const uint32_t lo = o[j] >> PB;
                bad |= i > 0 && i < nc && (k[j] < pv || (kWPk && k[j] == pv && lo < pvl));
            }
            sorted_packed = __builtin_amdgcn_readfirstlane(mw_any<NW>(bad, scr) ? 0 : 1) != 0;
            if (!sorted_packed) load();
        }
    }
    // by key only; wide partition keys (kWPk) whose low bits ride in the
    // payload re-sort by (key, payload) when two pairs of one pid share a
    // key (same priority and top 24 pk bits, ~2^-56 per pair of pairs):
    // the lexicographic comparator costs the common case a third more
    if (!sorted_packed) mw_sort<NW, false>(k, o, xk, xo);
    if (kWPk && !sorted_packed) {
        xk[tid] = k[3];
        xo[tid] = o[3];
        __syncthreads();
        const uint64_t pk0 = tid ? xk[tid - 1] : 0ull;
        const uint32_t po0 = tid ? xo[tid - 1] : 0u;
        bool coll = false;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t i = 4 * tid + j;
            const uint64_t pv = j ? k[j - 1] : pk0;
            const uint32_t pvo = j ? o[j - 1] : po0;
            coll |= i < nc && i > 0 && k[j] == pv && (o[j] >> PB) != (pvo >> PB);
        }
        if (mw_any<NW>(coll, scr)) {
            load();
            mw_sort<NW, true>(k, o, xk, xo);
        }
    }
    mark(bp, 1, clk);

    // ---- P: pair starts, ordinals, rank inside the pid
    xk[tid] = k[3];
    xo[tid] = o[3];
    __syncthreads();
    const uint64_t prev_last = tid ? xk[tid - 1] : 0ull;
    const uint32_t prev_o = tid ? xo[tid - 1] : 0u;
    uint32_t validm = 0, psm = 0, pidm = 0;
    uint32_t a[4];
    uint32_t cnt = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t i = 4 * tid + j;
        const uint64_t pv = j ? k[j - 1] : prev_last;
        const bool val = i < nc;
        const bool lodiff = kWPk && ((o[j] >> PB) != ((j ? o[j - 1] : prev_o) >> PB));
        const bool p = val && (i == 0 || k[j] != pv || lodiff);
        const bool d = val && (i == 0 || (k[j] >> 56) != (pv >> 56));
        validm |= val ? 1u << j : 0u;
        psm |= p ? 1u << j : 0u;
        pidm |= d ? 1u << j : 0u;
        cnt += p ? 1u : 0u;
        a[j] = cnt;  // inclusive within the thread
    }
    uint32_t npairs;
    const uint32_t before = mw_excl_scan<NW>(cnt, npairs, scr) - 1u;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        a[j] += before;  // pair ordinal
        if ((psm >> j) & 1u) pstart[a[j]] = (uint16_t)(4 * tid + j);
        if ((pidm >> j) & 1u) pbase[(uint32_t)(k[j] >> 56) & (kWCq - 1)] = a[j];
    }
    if (tid == 0) pstart[npairs] = (uint16_t)nc;
    __syncthreads();
    uint32_t kpm = 0;
    {
        uint32_t pb[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) pb[j] = pbase[(uint32_t)(k[j] >> 56) & (kWCq - 1)];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t rank = a[j] - pb[j];
            if (((psm >> j) & 1u) && rank == bp.mpc - 1)
                full[(uint32_t)(k[j] >> 56) & (kWCq - 1)] = 1u;
            kpm |= (((validm >> j) & 1u) && rank < bp.mpc) ? 1u << j : 0u;
        }
    }
    __syncthreads();
    // pids filtered by their bound that show fewer than mpc candidate pairs
    // may own kept pairs above the bound
    {
        bool shrt = false;
        for (uint32_t q = tid; q < kWCq; q += T) {
            const bool sh = pidc[q] > 0 && cbnd[q] != 0xFFFFFFFFu && full[q] == 0;
            if (sh && !hbound) cbnd[q] = 0xFFFFFFFFu;
            shrt |= sh;
        }
        if (mw_any<NW>(shrt, scr) && !last_round) {
            if (hbound) {
                // a heavy chunk holds only its pid's candidates: the bucket
                // goes back to the global-memory kernel (rare)
                if (tid == 0) bp.heavy_fb[atomicAdd(bp.heavy_nfb, 1u)] = hidx;
                return kRoundDone;
            }
            return kRoundRestart;
        }
    }
    mark(bp, 2, clk);

    // ---- M: kept pairs; values of their records; mcpp sample of over-full
    // pairs by record priority
    uint32_t st[4], len[4], idx[4], pkf[4];
    double v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        st[j] = pstart[min(a[j], (uint32_t)CAP - 1)];
        len[j] = pstart[min(a[j] + 1, (uint32_t)CAP)];
        idx[j] = kWPk ? cidx[o[j] & (CAP - 1)] : o[j];
        pkf[j] = kWPk ? ((((uint32_t)k[j] & kPkMask) << pksh) | (o[j] >> PB)) : ((uint32_t)k[j] & kPkMask);
    }
    uint32_t overm = 0, maxlen = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        len[j] -= st[j];
        const bool kp = (kpm >> j) & 1u;
        const bool ov = sample && kp && len[j] > bp.mcpp;
        overm |= ov ? 1u << j : 0u;
        maxlen = max(maxlen, ov ? len[j] : 0u);
        v[j] = (need_v && kp && (!kSortLate || !ov)) ? gather_value(bp.value, idx[j]) : 0.0;  // see dpg_sortb.h
    }
    uint32_t keepm = kpm;
    maxlen = __builtin_amdgcn_readfirstlane(mw_max<NW>(maxlen, scr));
    if (maxlen) {
        // record keys of over-full kept pairs, by sorted position; a record
        // is kept iff fewer than mcpp keys of its pair are smaller
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (!((overm >> j) & 1u)) continue;
            const uint32_t q = (uint32_t)(k[j] >> 56) & (kWCq - 1);
            rks[4 * tid + j] = rec_prio_h(pidv[q], pkf[j], (uint64_t)(bp.rec_base + idx[j]));
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool ov = (overm >> j) & 1u;
            // this wave's longest over-full pair in slot j (the sorted
            // order puts a long pair in few neighbouring threads)
            const uint32_t mj = __builtin_amdgcn_readfirstlane(wave_max_u32(ov ? len[j] : 0u));
            if (!mj) continue;
            const uint64_t mine = rks[4 * tid + j];
            const uint32_t lm = max(len[j], 1u) - 1u;
            uint32_t below = 0;
            for (uint32_t t = 0; t < mj; t += 2) {
                const uint64_t y0 = rks[min(st[j] + min(t, lm), (uint32_t)CAP - 1)];
                const uint64_t y1 = rks[min(st[j] + min(t + 1, lm), (uint32_t)CAP - 1)];
                below += (t < len[j] && y0 < mine) ? 1u : 0u;
                below += (t + 1 < len[j] && y1 < mine) ? 1u : 0u;
            }
            if (ov && below >= bp.mcpp) keepm &= ~(1u << j);
        }
        if constexpr (kSortLate) {
            if (need_v) {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if ((overm & keepm) >> j & 1u) v[j] = gather_value(bp.value, idx[j]);
            }
        }
    }

    mark(bp, 3, clk);

    // ---- F: accumulators of kept records, one item per kept pair
    const uint32_t em = psm & kpm;
    if (need_v) {
        __syncthreads();  // the accumulators overwrite the record keys of phase M
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (!((em >> j) & 1u)) continue;
            if (kSum) acc[a[j]] = 0.0;
            if (kVar) {
                acc_nsum[a[j]] = 0.0;
                acc_nsq[a[j]] = 0.0;
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 4; ++j) {
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
        __syncthreads();
    }
    uint32_t nem;
    uint32_t oe = nitems + mw_excl_scan<NW>((uint32_t)__popc(em), nem, scr);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (!((em >> j) & 1u)) continue;
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
        items[oe++] = it;
    }
    nitems += nem;
    mark(bp, 4, clk);
    return kRoundDone;
}

// One round of a chunk (phase A of sort_round, dpg_sortb.h): (first round
// only) records per pid slot, pid hashes, candidate bounds; pair priorities;
// candidates compacted into LDS; then sort and bound.
template <class Item, class R, bool kFirst, bool kWPk, int NW>
__device__ __forceinline__ int mw_round(const R (&r)[4], uint32_t n, uint32_t d1, uint32_t hbase,
                                         char *smem, const BoundParams &bp, Item *items,
                                         uint32_t &nitems, uint32_t hbound, uint32_t hidx,
                                         PhaseTimer &clk) {
    using L = SortLayoutMW<Item, R, kWPk, NW>;
    constexpr int T = L::T;
    uint32_t *pidv = reinterpret_cast<uint32_t *>(smem + L::PIDV);
    uint32_t *pidc = reinterpret_cast<uint32_t *>(smem + L::PIDC);
    uint32_t *cbnd = reinterpret_cast<uint32_t *>(smem + L::CBND);
    uint64_t *ckey = reinterpret_cast<uint64_t *>(smem + L::CK);
    uint32_t *cidx = reinterpret_cast<uint32_t *>(smem + L::CIDX);
    uint8_t *cpkl = reinterpret_cast<uint8_t *>(smem + L::CPKL);
    uint32_t *scr = reinterpret_cast<uint32_t *>(smem + L::SCR);
    const uint32_t tid = threadIdx.x;
    const Fmt f = bp.fmt;
    const uint32_t pkb = f.pkbits;
    const uint64_t pkmask = (1ull << pkb) - 1ull;
    const uint32_t hshift = f.kbits - f.b1;
    const uint32_t pksh = kWPk ? pkb - kSkPkBits : 0u;

    uint64_t sk[4];  // q << 56 | pk (pp << 24 | pk >> pksh below)
    uint32_t ix[4];
    uint32_t validm = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        validm |= tid + T * j < n ? 1u << j : 0u;
        const uint64_t key = RecOps<R>::key(r[j], f);
        const uint32_t q = ((uint32_t)(key >> pkb) - hbase) & (kWCq - 1);
        sk[j] = ((uint64_t)q << 56) | (key & pkmask);
        ix[j] = RecOps<R>::idx(r[j], f);
    }
    if constexpr (kFirst) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if ((validm >> j) & 1u) atomicAdd(&pidc[(uint32_t)(sk[j] >> 56)], 1u);
        __syncthreads();
        const float cmul = bp.cand_mul;
        for (uint32_t q = tid; q < kWCq; q += T) {
            const uint32_t rc = pidc[q];
            if (rc == 0) continue;
            pidv[q] = pid_hash(bp.seed, (uint64_t)(bp.pid_min + (int64_t)hk_inv(
                                                 (d1 << hshift) | (hbase + q), bp.hash)));
            const float fr = cmul / (float)rc;
            cbnd[q] = hbound ? hbound
                             : (rc <= bp.mpc || fr >= 1.0f ? 0xFFFFFFFFu
                                                           : (uint32_t)(fr * 4294967296.0f));
        }
        __syncthreads();
    }
    uint32_t cm = 0;
    uint32_t pkl[4];  // kWPk: the low pk bits the sort key has no room for
    {
        uint32_t pv[4], cb[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            pv[j] = pidv[(uint32_t)(sk[j] >> 56)];
            cb[j] = cbnd[(uint32_t)(sk[j] >> 56)];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t pk = (uint32_t)sk[j];
            const uint32_t pp = pair_prio_h(pv[j], pk);
            pkl[j] = kWPk ? (pk & ((1u << pksh) - 1u)) : 0u;
            if constexpr (kWPk) sk[j] = (sk[j] & ~(uint64_t)0xFFFFFFFFu) | (pk >> pksh);
            sk[j] |= (uint64_t)pp << kSkPkBits;
            cm |= (((validm >> j) & 1u) && pp <= cb[j]) ? 1u << j : 0u;
        }
    }
    uint32_t nc;
    uint32_t e = mw_excl_scan<NW>((uint32_t)__popc(cm), nc, scr);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (!((cm >> j) & 1u)) continue;
        ckey[e] = sk[j];
        cidx[e] = ix[j];
        if constexpr (kWPk) cpkl[e] = (uint8_t)pkl[j];
        ++e;
    }
    __syncthreads();
    mark(bp, 0, clk);
    const int st = mw_sort_chunk<Item, R, kWPk, NW>(nc, smem, bp, !kFirst, hbound, hidx, items,
                                                    nitems, clk);
    __syncthreads();
    return st;
}

// One chunk; a restart (a filtered pid short of mpc candidate pairs)
// re-reads the records (L2-hot) for a second round with that pid's bound
// lifted.
template <class Item, class R, bool kWPk, int NW>
__device__ __forceinline__ void mw_bound_chunk(const R (&r0)[4], const R *base, uint32_t n,
                                               uint32_t d1, uint32_t hbase, char *smem,
                                               const BoundParams &bp, Item *items, uint32_t &nitems,
                                               uint32_t hbound, uint32_t hidx, PhaseTimer &clk) {
    using L = SortLayoutMW<Item, R, kWPk, NW>;
    constexpr int T = L::T;
    uint32_t *pidc = reinterpret_cast<uint32_t *>(smem + L::PIDC);
    const uint32_t tid = threadIdx.x;
    int st = mw_round<Item, R, true, kWPk, NW>(r0, n, d1, hbase, smem, bp, items, nitems, hbound,
                                              hidx, clk);
    if (st == kRoundRestart) {
        R r[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = base[min(tid + (uint32_t)T * j, n - 1)];
        mw_round<Item, R, false, kWPk, NW>(r, n, d1, hbase, smem, bp, items, nitems, hbound, hidx,
                                           clk);
    }
    for (uint32_t q = tid; q < kWCq; q += T) pidc[q] = 0;
    __syncthreads();
    mark(bp, 5, clk);
}

template <class R>
__device__ __forceinline__ void mw_params(BoundParams &bp) {
    // parameters used in one phase each: vector registers (see vreg)
    bp.lo = vreg(bp.lo);
    bp.hi = vreg(bp.hi);
    bp.lo_pp = vreg(bp.lo_pp);
    bp.hi_pp = vreg(bp.hi_pp);
    bp.mid = vreg(bp.mid);
    bp.seed = vreg(bp.seed);
    bp.pid_min = vreg(bp.pid_min);
    bp.rec_base = vreg(bp.rec_base);
    bp.value = vreg(bp.value);
    bp.hash.mask = vreg(bp.hash.mask);
    bp.hash.i1 = vreg(bp.hash.i1);
    bp.hash.i2 = vreg(bp.hash.i2);
    bp.mcpp = vreg(bp.mcpp);
    bp.heavy_fb = vreg(bp.heavy_fb);
    bp.heavy_nfb = vreg(bp.heavy_nfb);
}

// NW = 2: the chunks the single-wave narrow kernel deferred (defer[w] set),
// walked like k_bound_sorted's wide instantiation: workgroup g2 takes the
// narrow workgroups g = g2, g2 + gridDim.x, ... and appends to their item
// regions behind wg_cnt[g].
template <class Item, class R, bool kWPk>
__global__ __launch_bounds__(128, 4) void k_bound_sorted_w2(
    const R *recs, const R *refined, const R *heavy, const uint4 *chunks, const uint32_t *n_chunks,
    BoundParams bp, Item *items, const int64_t *wg_off, uint32_t *wg_cnt, const uint8_t *defer,
    uint32_t G1) {
    using L = SortLayoutMW<Item, R, kWPk, 2>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    PhaseTimer clk;
    timer_start(bp, clk);
    mw_params<R>(bp);
    const uint32_t nch = __builtin_amdgcn_readfirstlane(*n_chunks);
    const uint32_t lane = __lane_id(), tid = threadIdx.x;
    uint32_t *pidc = reinterpret_cast<uint32_t *>(smem + L::PIDC);
    for (uint32_t q = tid; q < kWCq; q += L::T) pidc[q] = 0;
    __syncthreads();
    for (uint32_t g = blockIdx.x; g < G1; g += gridDim.x) {
        uint32_t nitems = __builtin_amdgcn_readfirstlane(wg_cnt[g]);
        Item *my_items = items + wg_off[g];
        bool any = false;
        for (uint32_t i0 = 0; g + i0 * G1 < nch; i0 += 64) {
            const uint32_t wl = g + (i0 + lane) * G1;
            // every wave computes the same mask (it depends on the lane only)
            for (uint64_t fm = __ballot(wl < nch && defer[min(wl, nch - 1)] != 0); fm;
                 fm &= fm - 1) {
                const uint32_t w = g + (i0 + (uint32_t)__builtin_ctzll(fm)) * G1;
                any = true;
                const uint4 d = make_uint4(__builtin_amdgcn_readfirstlane(chunks[w].x),
                                           __builtin_amdgcn_readfirstlane(chunks[w].y),
                                           __builtin_amdgcn_readfirstlane(chunks[w].z),
                                           __builtin_amdgcn_readfirstlane(chunks[w].w));
                const uint32_t n = d.y & kChunkCount;
                const R *b = wave_chunk_base(d, recs, refined, heavy);
                R r[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) r[j] = b[min(tid + (uint32_t)L::T * j, n - 1)];
                mw_bound_chunk<Item, R, kWPk, 2>(r, b, n, d.z & 0xFFFFu, d.w, smem, bp, my_items,
                                                 nitems, heavy_bound(d), d.x / (uint32_t)kWCap, clk);
            }
        }
        if (any && tid == 0) wg_cnt[g] = nitems;
    }
    timer_flush(bp, clk);
}

// NW = 4: medium chunks (one fine bucket of <= 1024 records, <= 128 pid
// hash values), workgroup g takes chunks g, g + gridDim.x, ... (the static
// schedule k_wg_records sized the item regions for) and loads the next
// chunk's records while bounding the current one.
template <class Item, class R, bool kWPk>
__global__ __launch_bounds__(256, 4) void k_bound_sorted_m4(
    const R *recs, const R *refined, const uint4 *chunks, const uint32_t *n_chunks, BoundParams bp,
    Item *items, const int64_t *wg_off, uint32_t *wg_cnt) {
    using L = SortLayoutMW<Item, R, kWPk, 4>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    PhaseTimer clk;
    timer_start(bp, clk);
    mw_params<R>(bp);
    const uint32_t nch = __builtin_amdgcn_readfirstlane(*n_chunks);
    const uint32_t tid = threadIdx.x;
    uint32_t *pidc = reinterpret_cast<uint32_t *>(smem + L::PIDC);
    for (uint32_t q = tid; q < kWCq; q += L::T) pidc[q] = 0;
    __syncthreads();
    uint32_t nitems = 0;
    Item *my_items = items + wg_off[blockIdx.x];
    auto desc = [&](uint32_t w) {
        return make_uint4(__builtin_amdgcn_readfirstlane(chunks[w].x),
                          __builtin_amdgcn_readfirstlane(chunks[w].y),
                          __builtin_amdgcn_readfirstlane(chunks[w].z),
                          __builtin_amdgcn_readfirstlane(chunks[w].w));
    };
    R r[4], rn[4];
    uint4 d = make_uint4(0, 0, 0, 0);
    const uint32_t G = gridDim.x;
    if (blockIdx.x < nch) {
        d = desc(blockIdx.x);
        const uint32_t n = d.y & kChunkCount;
        const R *b = wave_chunk_base(d, recs, refined, recs);
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = b[min(tid + (uint32_t)L::T * j, n - 1)];
    }
    for (uint32_t w = blockIdx.x; w < nch; w += G) {
        uint4 du = make_uint4(0, 0, 0, 0);
        if (w + G < nch) {
            du = desc(w + G);
            const uint32_t nn = du.y & kChunkCount;
            const R *nb = wave_chunk_base(du, recs, refined, recs);
#pragma unroll
            for (int j = 0; j < 4; ++j) rn[j] = nb[min(tid + (uint32_t)L::T * j, nn - 1)];
        }
        mw_bound_chunk<Item, R, kWPk, 4>(r, wave_chunk_base(d, recs, refined, recs),
                                         d.y & kChunkCount, d.z & 0xFFFFu, d.w, smem, bp,
                                         my_items, nitems, 0u, 0u, clk);
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = rn[j];
        d = du;
    }
    if (tid == 0) wg_cnt[blockIdx.x] = nitems;
    timer_flush(bp, clk);
}

}  // namespace dpg
