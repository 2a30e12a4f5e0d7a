// dpg_partition.h -- MSD radix partitioning of records by privacy-id hash
// (and of kept pairs by partition-key range) for gfx950.
//
// One level = hist -> scan -> digit-base -> scatter.  A level splits every
// segment of its input into F <= 2048 digit buckets.  The scatter stages a
// sub-tile of records through LDS, ranked per digit with wave-aggregated LDS
// atomics, so each digit leaves as one contiguous run per sub-tile: coalesced
// writes without per-record global atomics.  Order inside a digit is not
// preserved (nothing downstream depends on it: the samplers key on the
// global record id, see DESIGN.md "Randomness").
//
// Sources expose fetch(i) -> Raw (the global loads, issued one sub-tile ahead)
// and decode(Raw, i, rec, digit) -> keep; sources whose records still carry
// their digit recompute it at write-out, the level-1 source (whose records
// drop the level-1 digit) stages it in LDS beside the record.
#pragma once

#include "dpg_common.h"

#include <type_traits>

namespace dpg {

#ifndef DPG_HIST_U
#define DPG_HIST_U 8
#endif
#ifndef DPG_SCAT_WB
#define DPG_SCAT_WB 2  // same-box A/B: 8 -> 4 level-1 scatter 7.51 -> 7.45 ms, 4 -> 2 pieces 7.24 -> 7.07 ms (r5zd; fewer live registers)
#endif
constexpr int kPartThreads = 1024;  // 16 waves
// scatter workgroups (512 threads with twice the records per thread measured
// slower on the level-1 scatter)
constexpr int kScatThreads = 1024;

__host__ __device__ constexpr size_t a16(size_t x) { return (x + 15) & ~(size_t)15; }

typedef int64_t i64x2 __attribute__((ext_vector_type(2)));
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
typedef uint64_t u64x2a8 __attribute__((ext_vector_type(2), aligned(8)));

template <class Src, class = void>
struct HasFetchPairs {
    static constexpr bool value = false;
};
template <class Src>
struct HasFetchPairs<Src, decltype((void)Src::kFetchPairs)> {
    static constexpr bool value = Src::kFetchPairs;
};

// Sources whose fetch is a plain indexed load may prefetch across tiles (the
// XCD-local scatter's next tile; SrcSeg's fetch holds a per-lane search).
#ifndef DPG_XTILE_PF
#define DPG_XTILE_PF 1
#endif
template <class Src, class = void>
struct HasTilePrefetch {
    static constexpr bool value = false;
};
template <class Src>
struct HasTilePrefetch<Src, decltype((void)Src::kTilePrefetch)> {
    static constexpr bool value = Src::kTilePrefetch && DPG_XTILE_PF;
};

// Piece-mode sources (k_scatter without a histogram pass, see there).
template <class Src, class = void>
struct HasPieces {
    static constexpr bool value = false;
};
template <class Src>
struct HasPieces<Src, decltype((void)Src::kPieces)> {
    static constexpr bool value = Src::kPieces;
};

// Sources without a pair view (kPairs false) take the one-record loop.
template <class Src, class = void>
struct HasPairs {
    static constexpr bool value = false;
};
template <class Src>
struct HasPairs<Src, decltype((void)Src::kPairs)> {
    static constexpr bool value = Src::kPairs;
};

struct TileDesc {
    int64_t begin, end;
    uint32_t seg;
    uint32_t pad;
};

// A tile descriptor read by a uniform index, kept in scalar registers (the
// loops over its sub-tiles hold barriers: their trip counts must be
// visibly wave-uniform).
__device__ __forceinline__ TileDesc uniform_tile(const TileDesc *tiles, uint32_t t) {
    const TileDesc d = tiles[t];
    auto u64 = [](int64_t x) {
        return (int64_t)(((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)x >> 32)) << 32) |
                         (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)x));
    };
    TileDesc r;
    r.begin = u64(d.begin);
    r.end = u64(d.end);
    r.seg = __builtin_amdgcn_readfirstlane(d.seg);
    r.pad = __builtin_amdgcn_readfirstlane(d.pad);
    return r;
}

// ---------------------------------------------------------------- sources
// Level 1: the caller's int64 pid / pk columns -> R (key residual, index).
// Drops records of non-public partitions.  Keys outside the declared ranges
// raise err bit 1 (the call then fails before any bucket is bounded); such a
// record is still kept so that the scatter agrees with the histogram.
//
// kFull (the histogram-free level 1, k_scatter's piece mode): the scatter
// loads the whole privacy id and raises the range error itself.
template <class R, bool kFull = false>
struct SrcSoAKey {
    static constexpr bool kDigitFromRec = false;
    static constexpr bool kTilePrefetch = true;
    static constexpr bool kPieces = kFull;
    // the scatter loads only the low word of the privacy id: the digit and
    // the stored key depend on (pid - pid_min) mod 2^32 alone, and the
    // histogram pass, which reads the whole column, raises the range error
    // (12 fewer VGPRs per thread in flight: the level-1 scatter spilled)
    // R16 records carry the value column too (the utility pre-aggregate)
    static constexpr bool kV = sizeof(R) == 16;
    using PidW = std::conditional_t<kFull, uint64_t, uint32_t>;
    struct RawK {
        PidW pid;
        int64_t pk;
    };
    struct RawV {
        PidW pid;
        int64_t pk;
        double v;
    };
    using Raw = std::conditional_t<kV, RawV, RawK>;
    const int64_t *pid;
    const int64_t *pk;
    const uint8_t *pub;  // public-partition bitmap or null
    int64_t P;
    int64_t pid_min;
    uint64_t U;          // privacy ids in [pid_min, pid_min + U)
    HashK H;
    Fmt f;
    uint64_t kmask;      // stored key bits
    uint32_t dshift;     // kbits - b1
    uint32_t *err;
    const double *value = nullptr;  // R16 only
#ifndef DPG_L1_NT
#define DPG_L1_NT 1  // same-box A/B: level-1 scatter 8.15 -> 7.86 ms
#endif
#if DPG_L1_NT
    // the key columns are read once: non-temporal loads leave L2 to the
    // scattered runs being written
    __device__ __forceinline__ PidW fetch_pid(int64_t i) const {
        if constexpr (kFull)
            return (uint64_t)__builtin_nontemporal_load(pid + i);
        else
            return __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(pid) + 2 * i);
    }
    __device__ __forceinline__ Raw fetch(int64_t i) const {
        if constexpr (kV)
            return Raw{fetch_pid(i), __builtin_nontemporal_load(pk + i),
                       __builtin_nontemporal_load(value + i)};
        else
            return Raw{fetch_pid(i), __builtin_nontemporal_load(pk + i)};
    }
#else
    __device__ __forceinline__ PidW fetch_pid(int64_t i) const {
        if constexpr (kFull)
            return (uint64_t)pid[i];
        else
            return reinterpret_cast<const uint32_t *>(pid)[2 * i];
    }
    __device__ __forceinline__ Raw fetch(int64_t i) const {
        if constexpr (kV)
            return Raw{fetch_pid(i), pk[i], value[i]};
        else
            return Raw{fetch_pid(i), pk[i]};
    }
#endif
    // keep decision shared by the histogram and the scatter (they must agree
    // record for record): from the low word of pid - pid_min and pk
    __device__ __forceinline__ bool keep(uint32_t a, int64_t b) const {
        if (!pub) return true;
        const bool in_range = (uint64_t)a < U && (uint64_t)b < (uint64_t)P;
        return !(in_range && !((pub[b >> 3] >> (b & 7)) & 1));
    }
    __device__ __forceinline__ bool decode(const Raw &x, int64_t i, R &r, uint32_t &d) const {
        uint32_t a;
        if constexpr (kFull) {
            const uint64_t a64 = x.pid - (uint64_t)pid_min;
            if (a64 >= U || (uint64_t)x.pk >= (uint64_t)P) atomicOr(err, 1u);
            a = (uint32_t)a64;
        } else {
            a = x.pid - (uint32_t)pid_min;
            if ((uint64_t)x.pk >= (uint64_t)P) atomicOr(err, 1u);
        }
        const uint32_t h = hk(a, H);
        d = h >> dshift;
        const uint64_t key = (((uint64_t)h << f.pkbits) | (uint64_t)x.pk) & kmask;
        r = RecOps<R>::make(key, (uint32_t)i, f);
        if constexpr (kV) r.v = x.v;
        return keep(a, x.pk);
    }
    // histogram view: the same digit and keep decision from pid (and pk
    // only when a public-partition filter applies); the privacy-id range
    // check of the whole 64-bit id
    __device__ __forceinline__ bool hist(int64_t i, uint32_t &d) const {
        const uint64_t a = (uint64_t)(pid[i] - pid_min);
        if (a >= U) atomicOr(err, 1u);
        d = hk((uint32_t)a, H) >> dshift;
        if (!pub) return true;
        return keep((uint32_t)a, pk[i]);
    }
    // the scatter's pair view: two consecutive records by one 16-byte load
    // per column (8-byte aligned, any tile start), half the vector memory
    // instructions of the 8-byte loads (DPG_L1_PAIRS; the scatter takes it
    // with an even records-per-thread count: the piece mode and 12-byte
    // records)
#ifndef DPG_L1_PAIRS
#define DPG_L1_PAIRS 1
#endif
    static constexpr bool kFetchPairs = DPG_L1_PAIRS != 0;
    __device__ __forceinline__ void fetch2(int64_t i, Raw &x0, Raw &x1) const {
#if DPG_L1_NT
        const u64x2a8 p = __builtin_nontemporal_load(reinterpret_cast<const u64x2a8 *>(pid + i));
        const u64x2a8 q = __builtin_nontemporal_load(reinterpret_cast<const u64x2a8 *>(pk + i));
#else
        const u64x2a8 p = *reinterpret_cast<const u64x2a8 *>(pid + i);
        const u64x2a8 q = *reinterpret_cast<const u64x2a8 *>(pk + i);
#endif
        if constexpr (kV) {
#if DPG_L1_NT
            const u64x2a8 v = __builtin_nontemporal_load(reinterpret_cast<const u64x2a8 *>(value + i));
#else
            const u64x2a8 v = *reinterpret_cast<const u64x2a8 *>(value + i);
#endif
            x0 = Raw{(PidW)p.x, (int64_t)q.x, __builtin_bit_cast(double, v.x)};
            x1 = Raw{(PidW)p.y, (int64_t)q.y, __builtin_bit_cast(double, v.y)};
        } else {
            x0 = Raw{(PidW)p.x, (int64_t)q.x};
            x1 = Raw{(PidW)p.y, (int64_t)q.y};
        }
    }
    // two consecutive records (i even) by 16-byte loads: the histogram pass
    // streams at the 16-B/lane rate instead of the 8-B one
    static constexpr bool kPairs = true;
    __device__ __forceinline__ bool pairs_ok() const {
        return ((uintptr_t)pid & 15) == 0 && (!pub || ((uintptr_t)pk & 15) == 0);
    }
    __device__ __forceinline__ void hist2(int64_t i, uint32_t (&d)[2], bool (&ok)[2]) const {
        const i64x2 p = *reinterpret_cast<const i64x2 *>(pid + i);
        const uint64_t a0 = (uint64_t)(p.x - pid_min), a1 = (uint64_t)(p.y - pid_min);
        if (a0 >= U || a1 >= U) atomicOr(err, 1u);
        d[0] = hk((uint32_t)a0, H) >> dshift;
        d[1] = hk((uint32_t)a1, H) >> dshift;
        ok[0] = ok[1] = true;
        if (pub) {
            const i64x2 q = *reinterpret_cast<const i64x2 *>(pk + i);
            ok[0] = keep((uint32_t)a0, q.x);
            ok[1] = keep((uint32_t)a1, q.y);
        }
    }
};

// Bucketed records; digit = bits [shift, shift + log2 F) of the stored key.
template <class R>
struct SrcAoS {
    static constexpr bool kDigitFromRec = true;
    static constexpr bool kTilePrefetch = true;
    using Raw = R;
    const R *a;
    Fmt f;
    uint32_t shift, mask;
    __device__ __forceinline__ R fetch(int64_t i) const { return a[i]; }
    __device__ __forceinline__ uint32_t digit(const R &r) const {
        return (uint32_t)(RecOps<R>::key(r, f) >> shift) & mask;
    }
    __device__ __forceinline__ bool decode(const R &x, int64_t, R &r, uint32_t &d) const {
        r = x;
        d = digit(x);
        return true;
    }
    __device__ __forceinline__ bool hist(int64_t i, uint32_t &d) const {
        d = digit(a[i]);
        return true;
    }
    // 8-byte records: pairs by 16-byte loads (see SrcSoAKey::hist2); the
    // scatter's fetch2 needs only 8-byte alignment (any tile start)
    static constexpr bool kPairs = sizeof(R) == 8;
    static constexpr bool kFetchPairs = sizeof(R) == 8;
    __device__ __forceinline__ void fetch2(int64_t i, R &x0, R &x1) const {
        if constexpr (sizeof(R) == 8) {
            const u64x2a8 w = *reinterpret_cast<const u64x2a8 *>(a + i);
            x0 = R{w.x};
            x1 = R{w.y};
        }
    }
    __device__ __forceinline__ bool pairs_ok() const { return ((uintptr_t)a & 15) == 0; }
    __device__ __forceinline__ void hist2(int64_t i, uint32_t (&d)[2], bool (&ok)[2]) const {
        if constexpr (sizeof(R) == 8) {
            const u64x2 w = *reinterpret_cast<const u64x2 *>(a + i);
            d[0] = digit(R{w.x});
            d[1] = digit(R{w.y});
        }
        ok[0] = ok[1] = true;
    }
};

// Items of S per-workgroup regions read as one sequence: element i lives in
// region s with pre[s] <= i < pre[s + 1], at a[off[s] + i - pre[s]].  Each
// thread walks increasing i, so the region found last is cached in
// registers and the binary search runs only when i leaves it.  Digit =
// pk >> shift (partition-key ranges).
template <class T>
struct SrcSeg {
    static constexpr bool kDigitFromRec = true;
    using Raw = T;
    const T *a;
    const int64_t *pre;  // [S + 1]
    const int64_t *off;  // [S]
    uint32_t S;
    uint32_t shift;
    int64_t lo = 0, hi = 0, base = 0;  // cached region [lo, hi), a index = base + i
    __device__ __forceinline__ T fetch(int64_t i) {
        if (i < lo || i >= hi) {
            uint32_t l = 0, h = S;
            while (h - l > 1) {
                const uint32_t mid = (l + h) >> 1;
                if (pre[mid] <= i) l = mid;
                else h = mid;
            }
            lo = pre[l];
            hi = pre[l + 1];
            base = off[l] - lo;
        }
        return a[base + i];
    }
    __device__ __forceinline__ uint32_t digit(const T &r) const { return r.pk >> shift; }
    __device__ __forceinline__ bool decode(const T &x, int64_t, T &r, uint32_t &d) const {
        r = x;
        d = digit(x);
        return true;
    }
    __device__ __forceinline__ bool hist(int64_t i, uint32_t &d) {
        d = digit(fetch(i));
        return true;
    }
};

// Contiguous items (or any T with a .pk field); digit = (pk >> shift) & mask
// (the second partition-key level of the merge).
template <class T>
struct SrcItems {
    static constexpr bool kDigitFromRec = true;
    using Raw = T;
    const T *a;
    uint32_t shift, mask;
    __device__ __forceinline__ T fetch(int64_t i) const { return a[i]; }
    __device__ __forceinline__ uint32_t digit(const T &r) const { return (r.pk >> shift) & mask; }
    __device__ __forceinline__ bool decode(const T &x, int64_t, T &r, uint32_t &d) const {
        r = x;
        d = digit(x);
        return true;
    }
    __device__ __forceinline__ bool hist(int64_t i, uint32_t &d) const {
        d = digit(a[i]);
        return true;
    }
};

// ------------------------------------------------------------ tile table
// One thread per segment: allocate ceil(n / tile) tiles.  With XCD queues
// (xq != null) the segment's tile ids are also appended to the queue of XCD
// s % 8, so that one XCD's workgroups take all tiles of a segment together
// (k_scatter's XCD-local mode).
struct XcdQueues {
    uint32_t *q;      // [8][stride] global tile ids
    uint32_t *n;      // [8] queue lengths
    uint32_t *next;   // [8] work counters (zeroed)
    uint32_t stride;
};

// One segment cut into many one-sub-tile tiles (level 1 in XCD-local mode):
// one thread per tile.  Groups of G consecutive tiles go to the XCD queues
// round-robin, so the ~G workgroups of one XCD write adjacent runs of every
// digit at the same time (they meet in that XCD's L2).
__global__ void k_build_tiles_single(int64_t n, int64_t tile, uint32_t G, TileDesc *tiles,
                                     uint32_t *seg_tile_base, uint32_t *seg_ntiles,
                                     uint32_t *ntiles_total, XcdQueues xq) {
    const uint32_t nt = (uint32_t)((n + tile - 1) / tile);
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t == 0) {
        seg_tile_base[0] = 0;
        seg_ntiles[0] = nt;
        *ntiles_total = nt;
    }
    if (t >= nt) return;
    TileDesc d;
    d.begin = (int64_t)t * tile;
    d.end = min((int64_t)(t + 1) * tile, n);
    d.seg = 0;
    d.pad = 0;
    tiles[t] = d;
    if (!xq.q) return;
    const uint32_t g = t / G, x = g & 7u;
    xq.q[(size_t)x * xq.stride + (g >> 3) * G + t % G] = t;
    atomicAdd(&xq.n[x], 1u);
}

// Grouped mode: the work items of the scatter are the sub-tiles of the
// histogram tiles ("groups"): one thread per group appends its sub-tiles
// (pad = group id) and queues them, in order, to XCD group % 8.
__global__ void k_build_subtiles(const TileDesc *groups, const uint32_t *ngroups, int64_t sub,
                                 TileDesc *tiles, uint32_t *ntiles_total, XcdQueues xq) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= *ngroups) return;
    const TileDesc gd = groups[g];
    const uint32_t nt = (uint32_t)((gd.end - gd.begin + sub - 1) / sub);
    if (!nt) return;
    const uint32_t b = atomicAdd(ntiles_total, nt);
    for (uint32_t j = 0; j < nt; ++j) {
        TileDesc d;
        d.begin = gd.begin + (int64_t)j * sub;
        d.end = min(gd.begin + (int64_t)(j + 1) * sub, gd.end);
        d.seg = gd.seg;
        d.pad = g;
        tiles[b + j] = d;
    }
    const uint32_t x = g & 7u;
    const uint32_t qb = atomicAdd(&xq.n[x], nt);
    for (uint32_t j = 0; j < nt; ++j) xq.q[(size_t)x * xq.stride + qb + j] = b + j;
}

// One wave per segment (launch build_tiles_blocks(S) blocks of 256): lane 0
// reserves the segment's tile range, the lanes write its tiles.  (One thread
// per segment left a single segment of thousands of tiles -- the item level
// -- to one thread's serial loop: 92 us per release at config 2.)
__global__ __launch_bounds__(256) void k_build_tiles(const int64_t *seg_start,
                                                     const uint32_t *seg_cnt,
                                                     const int64_t *seg_cnt64, uint32_t S,
                                                     int64_t tile, TileDesc *tiles,
                                                     uint32_t *seg_tile_base,
                                                     uint32_t *seg_ntiles,
                                                     uint32_t *ntiles_total,
                                                     XcdQueues xq = XcdQueues{}) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t s = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (s >= S) return;  // wave-uniform
    const int64_t st = seg_start ? seg_start[s] : 0;
    const int64_t n = seg_cnt64 ? seg_cnt64[s] : (int64_t)seg_cnt[s];
    const uint32_t nt = (uint32_t)((n + tile - 1) / tile);
    const uint32_t x = s & 7u;
    uint32_t b = 0, qb = 0;
    if (lane == 0 && nt) {
        b = atomicAdd(ntiles_total, nt);
        if (xq.q) qb = atomicAdd(&xq.n[x], nt);
    }
    b = (uint32_t)__shfl((int)b, 0, 64);
    qb = (uint32_t)__shfl((int)qb, 0, 64);
    if (lane == 0) {
        seg_tile_base[s] = b;
        seg_ntiles[s] = nt;
    }
    for (uint32_t j = lane; j < nt; j += 64) {
        TileDesc d;
        d.begin = st + (int64_t)j * tile;
        d.end = st + min((int64_t)(j + 1) * tile, n);
        d.seg = s;
        d.pad = 0;
        tiles[b + j] = d;
        if (xq.q) xq.q[(size_t)x * xq.stride + qb + j] = b + j;
    }
}

inline uint32_t build_tiles_blocks(uint32_t S) { return (S + 3) / 4; }

// ---------------------------------------------------------------- hist
template <class Src>
__global__ __launch_bounds__(kPartThreads) void k_hist(Src src_in, const TileDesc *tiles,
                                                       const uint32_t *ntiles, uint32_t F,
                                                       uint32_t *hist) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lh[];  // [4][F]
    const uint32_t t = blockIdx.x;
    if (t >= *ntiles) return;
    const TileDesc td = tiles[t];
    const int tid = threadIdx.x;
    const uint32_t copy = (tid >> 6) & 3;
    for (uint32_t d = tid; d < 4 * F; d += kPartThreads) lh[d] = 0;
    __syncthreads();
    uint32_t *my = lh + copy * F;
    Src src = src_in;  // per-thread copy (sources may cache lookup state)
    constexpr int U = DPG_HIST_U;  // loads per thread in flight per round
    if constexpr (HasPairs<Src>::value) {
        if (src.pairs_ok()) {
            // pairs (i even, 16-byte aligned): an odd first record alone,
            // then U / 2 pair loads per thread in flight, a last odd record
            int64_t b = td.begin;
            const int64_t e = td.end;
            if (b & 1) {
                uint32_t d;
                if (tid == 0 && b < e && src.hist(b, d)) atomicAdd(&my[d], 1u);
                ++b;
            }
            constexpr int U2 = U / 2 > 0 ? U / 2 : 1;
            int64_t i = b + 2 * tid;
            for (; i + 2 * (U2 - 1) * kPartThreads + 1 < e; i += 2 * U2 * kPartThreads) {
                uint32_t d[U2][2];
                bool ok[U2][2];
#pragma unroll
                for (int u = 0; u < U2; ++u) src.hist2(i + 2 * u * kPartThreads, d[u], ok[u]);
#pragma unroll
                for (int u = 0; u < U2; ++u) {
                    if (ok[u][0]) atomicAdd(&my[d[u][0]], 1u);
                    if (ok[u][1]) atomicAdd(&my[d[u][1]], 1u);
                }
            }
            for (; i + 1 < e; i += 2 * kPartThreads) {
                uint32_t d[2];
                bool ok[2];
                src.hist2(i, d, ok);
                if (ok[0]) atomicAdd(&my[d[0]], 1u);
                if (ok[1]) atomicAdd(&my[d[1]], 1u);
            }
            if (i < e) {
                uint32_t d;
                if (src.hist(i, d)) atomicAdd(&my[d], 1u);
            }
            __syncthreads();
            for (uint32_t d = tid; d < F; d += kPartThreads)
                hist[(size_t)t * F + d] = lh[d] + lh[F + d] + lh[2 * F + d] + lh[3 * F + d];
            return;
        }
    }
    int64_t i = td.begin + tid;
    for (; i + (U - 1) * kPartThreads < td.end; i += U * kPartThreads) {
        uint32_t d[U];
        bool ok[U];
#pragma unroll
        for (int u = 0; u < U; ++u) ok[u] = src.hist(i + u * kPartThreads, d[u]);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (ok[u]) atomicAdd(&my[d[u]], 1u);
    }
    for (; i < td.end; i += kPartThreads) {
        uint32_t d;
        if (src.hist(i, d)) atomicAdd(&my[d], 1u);
    }
    __syncthreads();
    for (uint32_t d = tid; d < F; d += kPartThreads)
        hist[(size_t)t * F + d] = lh[d] + lh[F + d] + lh[2 * F + d] + lh[3 * F + d];
}

// ---------------------------------------------------------------- scan
// grid (S, ceil(F/64), C); 16 waves split chunk c of a segment's tiles (C
// chunks of ceil(nt / C) tiles), lane = digit.  hist[t][d] <- exclusive
// prefix over the chunk's tiles; ctot[s][c][d] = the chunk's total (C = 1:
// the segment total).
__global__ __launch_bounds__(1024) void k_scan_tiles(const uint32_t *seg_tile_base,
                                                     const uint32_t *seg_ntiles, uint32_t F,
                                                     uint32_t *hist, uint32_t *ctot) {
    __shared__ uint32_t part[16][64];
    const uint32_t s = blockIdx.x, c = blockIdx.z, C = gridDim.z;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t d = blockIdx.y * 64 + lane;
    const uint32_t nt_all = seg_ntiles[s];
    const uint32_t per = (nt_all + C - 1) / C;
    const uint32_t c0 = min(nt_all, c * per), c1 = min(nt_all, c0 + per);
    const uint32_t nt = c1 - c0, tb = seg_tile_base[s] + c0;
    const uint32_t ch = (nt + 15) / 16;
    const uint32_t t0 = min(nt, w * ch), t1 = min(nt, (w + 1) * ch);
    uint32_t acc = 0;
    if (d < F)
        for (uint32_t t = t0; t < t1; ++t) acc += hist[(size_t)(tb + t) * F + d];
    part[w][lane] = acc;
    __syncthreads();
    uint32_t pre = 0, total = 0;
    for (int k = 0; k < 16; ++k) {
        uint32_t x = part[k][lane];
        if (k < w) pre += x;
        total += x;
    }
    if (d < F) {
        uint32_t run = pre;
        for (uint32_t t = t0; t < t1; ++t) {
            size_t o = (size_t)(tb + t) * F + d;
            uint32_t x = hist[o];
            hist[o] = run;
            run += x;
        }
        if (w == 0) ctot[((size_t)s * C + c) * F + d] = total;
    }
}

// C > 1 chunks: ctot[s][c][d] <- exclusive prefix over c (the chunk base the
// scatter adds to its tile offsets), tot[s][d] = the segment total.
__global__ void k_scan_chunks(uint32_t S, uint32_t C, uint32_t F, uint32_t *ctot, uint32_t *tot) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= S * F) return;
    const uint32_t s = i / F, d = i % F;
    uint32_t run = 0;
    for (uint32_t c = 0; c < C; ++c) {
        uint32_t &x = ctot[((size_t)s * C + c) * F + d];
        const uint32_t v = x;
        x = run;
        run += v;
    }
    tot[(size_t)s * F + d] = run;
}

// Block-wide exclusive scan of one value per thread (1024 threads).
__device__ __forceinline__ uint32_t block_excl_scan_1024(uint32_t x, uint32_t *sh16,
                                                         uint32_t &total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t wt;
    uint32_t e = wave_excl_scan(x, wt);
    if (lane == 63) sh16[w] = wt;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
    for (int k = 0; k < 16; ++k) {
        uint32_t y = sh16[k];
        if (k < w) pre += y;
        tot += y;
    }
    __syncthreads();
    total = tot;
    return e + pre;
}

// Exclusive scan of cnt[0, F) (F <= 2048) into dstart by 1024 threads
// (two consecutive digits per thread); returns the total.  Ends with a
// barrier: every dstart entry is visible to every thread on return.
__device__ __forceinline__ uint32_t block_scan_digits(const uint32_t *cnt, uint32_t *dstart,
                                                      uint32_t F, uint32_t *sh16) {
    const uint32_t d0 = 2 * threadIdx.x;
    const uint32_t c0 = d0 < F ? cnt[d0] : 0u;
    const uint32_t c1 = d0 + 1 < F ? cnt[d0 + 1] : 0u;
    uint32_t total;
    const uint32_t e = block_excl_scan_1024(c0 + c1, sh16, total);
    if (d0 < F) dstart[d0] = e;
    if (d0 + 1 < F) dstart[d0 + 1] = e + c0;
    __syncthreads();
    return total;
}

// Block-wide exclusive scan of one value per thread (T threads, T / 64
// waves <= 16).
template <int T>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t *sh16, uint32_t &total) {
    constexpr int NW = T / 64;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t wt;
    uint32_t e = wave_excl_scan(x, wt);
    if (lane == 63) sh16[w] = wt;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
        uint32_t y = sh16[k];
        if (k < w) pre += y;
        tot += y;
    }
    __syncthreads();
    total = tot;
    return e + pre;
}

// Exclusive scan of cnt[0, F) (F <= DPT * T) into dstart by T threads (DPT
// consecutive digits per thread); returns the total.  Ends with a barrier.
template <int T, int DPT>
__device__ __forceinline__ uint32_t block_scan_digits_t(const uint32_t *cnt, uint32_t *dstart,
                                                        uint32_t F, uint32_t *sh16) {
    const uint32_t d0 = DPT * threadIdx.x;
    uint32_t c[DPT], s = 0;
#pragma unroll
    for (int u = 0; u < DPT; ++u) {
        c[u] = d0 + u < F ? cnt[d0 + u] : 0u;
        s += c[u];
    }
    uint32_t total;
    uint32_t e = block_excl_scan<T>(s, sh16, total);
#pragma unroll
    for (int u = 0; u < DPT; ++u) {
        if (d0 + u < F) dstart[d0 + u] = e;
        e += c[u];
    }
    __syncthreads();
    return total;
}

// Scatter's per-sub-tile digit scan: dstart[0, F] <- exclusive prefix of
// cnt (dstart[F] = total), and for every digit cur[d] += cnt[d], cnt[d] = 0
// (the write-out then addresses cur[d] - dstart[d + 1] + k).  Grouped mode
// (goff: the group's digit offsets): the sub-tile reserves its run of every
// digit it holds inside its group by one atomic add, cur[d] += reserved
// start + cnt[d].  Each reservation sits behind its own branch (its
// s_waitcnt vmcnt(0) waits for the returned offset before the next is
// issued): issuing a thread's two atomics together, unconditionally, costs
// the level-1 scatter 10 more spilled VGPRs (6 -> 16), and keeping the
// offsets in registers until after the staging measured 7.1 -> 7.55 ms
// (round 5, profiles/r5/r5c_ab.txt).  Two barriers: the wave totals' buffer is
// next written one sub-tile later, behind the caller's own barriers.  Piece
// mode (kCap): goff are the cursors of fixed-capacity regions; a run that
// does not fit raises err bit 16 and goes to the dump area at `dump` instead
// (the host redoes the level with the histogram path).
#ifndef DPG_SCAT_RSV_PAIR
#define DPG_SCAT_RSV_PAIR 1
#endif
#ifndef DPG_SCAT_RSV_PAIR_EARLY
#define DPG_SCAT_RSV_PAIR_EARLY 1
#endif
template <int T, int DPT, bool kCap = false>
__device__ __forceinline__ uint32_t scatter_scan_update(uint32_t *cnt, uint32_t *dstart,
                                                        uint32_t *cur, uint32_t F,
                                                        uint32_t *sh16, uint32_t *goff = nullptr,
                                                        uint32_t cap = 0, uint32_t dump = 0,
                                                        uint32_t *err = nullptr,
                                                        const uint32_t *lb = nullptr) {
    constexpr int NW = T / 64;
    const uint32_t d0 = DPT * threadIdx.x;
    uint32_t c[DPT], x = 0;
#pragma unroll
    for (int u = 0; u < DPT; ++u) {
        c[u] = d0 + u < F ? cnt[d0 + u] : 0u;
        x += c[u];
    }
    // two digits per thread (F even): one 64-bit atomic reserves both runs
    // (the two 32-bit cursors sit in one aligned word; a cursor stays far
    // below 2^32, so the low add never carries into the high one)
    constexpr bool kPair = DPT == 2 && DPG_SCAT_RSV_PAIR;
    uint32_t o[DPT];
    if constexpr (kPair && DPG_SCAT_RSV_PAIR_EARLY) {
        if (goff && d0 < F) {
            const unsigned long long old = atomicAdd(
                reinterpret_cast<unsigned long long *>(&goff[d0]),
                (unsigned long long)c[0] | ((unsigned long long)c[1] << 32));
            o[0] = (uint32_t)old;
            o[1] = (uint32_t)(old >> 32);
        }
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t wt;
    uint32_t e = wave_excl_scan(x, wt);
    if (lane == 63) sh16[w] = wt;
    __syncthreads();
    uint32_t total = 0;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
        const uint32_t y = sh16[k];
        if (k < w) e += y;
        total += y;
    }
    if constexpr (kPair && !DPG_SCAT_RSV_PAIR_EARLY) {
        if (goff && d0 < F) {
            const unsigned long long old = atomicAdd(
                reinterpret_cast<unsigned long long *>(&goff[d0]),
                (unsigned long long)c[0] | ((unsigned long long)c[1] << 32));
            o[0] = (uint32_t)old;
            o[1] = (uint32_t)(old >> 32);
        }
    }
#pragma unroll
    for (int u = 0; u < DPT; ++u) {
        if (d0 + u < F) {
            dstart[d0 + u] = e;
            if constexpr (kCap) {
                if (c[u]) {
                    const uint32_t ou = kPair ? o[u] : atomicAdd(&goff[d0 + u], c[u]);
                    if (ou + c[u] <= cap) {
                        // lb (piece mode): the region bases in LDS, so cur
                        // needs no reset between sub-tiles
                        cur[d0 + u] = (lb ? lb[d0 + u] : cur[d0 + u]) + ou + c[u];
                    } else {
                        cur[d0 + u] = dump + e + c[u];
                        atomicOr(err, 16u);
                    }
                }
            } else if (goff) {
                if (c[u]) cur[d0 + u] += (kPair ? o[u] : atomicAdd(&goff[d0 + u], c[u])) + c[u];
            } else {
                cur[d0 + u] += c[u];
            }
            cnt[d0 + u] = 0;
        }
        e += c[u];
    }
    if (threadIdx.x == 0) dstart[F] = total;
    __syncthreads();
    return total;
}

// Piece mode's digit scan with the run reservations consumed late: the
// two runs of a thread's digit pair are reserved by one 64-bit atomic issued
// before the scan's barrier, as in scatter_scan_update, but the returned
// cursors are only needed at the write-out, so the caller stages first and
// then calls scatter_rsv_finish; the atomic's round trip (and, being younger
// in the vmcnt order, the drain of the previous write-out's stores) overlaps
// the staging instead of stalling the scan.
template <int DPT>
struct PcRsv {
    uint32_t c[DPT];  // the thread's digit counts
    uint32_t e0;      // local start of its first digit
    unsigned long long old[DPT / 2];
};
// NT threads, DPT (even) consecutive digits per thread: DPT / 2 64-bit
// reservations per thread
template <int NT, int DPT>
__device__ __forceinline__ uint32_t scatter_scan_pc(uint32_t *cnt, uint32_t *dstart, uint32_t F,
                                                    uint32_t *sh16, uint32_t *goff, PcRsv<DPT> &r) {
    const uint32_t d0 = DPT * threadIdx.x;
    uint32_t x = 0;
#pragma unroll
    for (int u = 0; u < DPT; ++u) {
        r.c[u] = d0 + u < F ? cnt[d0 + u] : 0u;
        x += r.c[u];
    }
    // unconditional (threads past F add 0 to a pair of cursors d mod F: a
    // result that is waited for on one path only is waited for again, with
    // vmcnt(0), when its register is next overwritten -- after the prefetch
    // loads).  Not one fixed dummy pair: with F < DPT NT its same-address
    // atomics serialised in L2 (a 1024-digit level 1 ran 17x slower)
#pragma unroll
    for (int q = 0; q < DPT / 2; ++q)
        r.old[q] = atomicAdd(reinterpret_cast<unsigned long long *>(&goff[(d0 + 2 * q) % F]),
                             (unsigned long long)r.c[2 * q] | ((unsigned long long)r.c[2 * q + 1] << 32));
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t wt;
    uint32_t e = wave_excl_scan(x, wt);
    if (lane == 63) sh16[w] = wt;
    __syncthreads();
    uint32_t total = 0;
#pragma unroll
    for (int k = 0; k < NT / 64; ++k) {
        const uint32_t y = sh16[k];
        if (k < w) e += y;
        total += y;
    }
    r.e0 = e;
#pragma unroll
    for (int u = 0; u < DPT; ++u) {
        if (d0 + u < F) {
            dstart[d0 + u] = e;
            cnt[d0 + u] = 0;
        }
        e += r.c[u];
    }
    if (threadIdx.x == 0) dstart[F] = total;
    __syncthreads();
    return total;
}
// cur[d] of the thread's digits from the reservations (lb: the regions'
// bases); a run past the region's capacity goes to the dump area and raises
// err bit 16.  The caller's next barrier publishes cur.
template <int DPT>
__device__ __forceinline__ void scatter_rsv_finish(const PcRsv<DPT> &r, uint32_t *cur,
                                                   const uint32_t *lb, uint32_t F, uint32_t cap,
                                                   uint32_t dump, uint32_t *err) {
    const uint32_t d0 = DPT * threadIdx.x;
    // the returned cursors are consumed on every path (see scatter_scan_pc)
    uint32_t o[DPT];
#pragma unroll
    for (int q = 0; q < DPT / 2; ++q) {
        o[2 * q] = (uint32_t)r.old[q];
        o[2 * q + 1] = (uint32_t)(r.old[q] >> 32);
    }
    uint32_t e = r.e0;
    bool over = false;
#pragma unroll
    for (int u = 0; u < DPT; ++u) {
        const bool fits = o[u] + r.c[u] <= cap;
        const uint32_t v = fits ? (lb[d0 + u < F ? d0 + u : 0u] + o[u] + r.c[u]) : dump + e + r.c[u];
        if (d0 + u < F && r.c[u]) {
            cur[d0 + u] = v;
            over = over || !fits;
        }
        e += r.c[u];
    }
    if (over) atomicOr(err, 16u);
}

// grid S: base[s][d] = seg_start[s] + exclusive_prefix_d(tot[s][.])  (F <= 4096)
__global__ __launch_bounds__(1024) void k_digit_base(const int64_t *seg_start, uint32_t F,
                                                     const uint32_t *tot, int64_t *base) {
    __shared__ uint32_t sh[16];
    const uint32_t s = blockIdx.x;
    const uint32_t d0 = 4 * threadIdx.x;
    uint32_t c[4], x = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        c[u] = d0 + u < F ? tot[(size_t)s * F + d0 + u] : 0u;
        x += c[u];
    }
    uint32_t total;
    uint32_t e = block_excl_scan_1024(x, sh, total);
    const int64_t st = seg_start ? seg_start[s] : 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        if (d0 + u < F) base[(size_t)s * F + d0 + u] = st + e;
        e += c[u];
    }
}

// ---------------------------------------------------------------- scatter
// Returns the rank of this lane's element among all elements of the block
// with the same digit (arbitrary order), via one LDS atomic per distinct
// digit per wave.
__device__ __forceinline__ uint32_t wave_agg_rank(uint32_t *cnt, uint32_t d, bool ok,
                                                  uint32_t bits) {
    uint64_t peers = __ballot(ok);
    for (uint32_t b = 0; b < bits; ++b) {
        uint64_t bal = __ballot((d >> b) & 1u);
        peers &= ((d >> b) & 1u) ? bal : ~bal;
    }
    const int lane = __lane_id();
    const int leader = peers ? __ffsll((long long)peers) - 1 : lane;
    const uint32_t below = __popcll(peers & ((1ull << lane) - 1ull));
    uint32_t basev = 0;
    if (ok && lane == leader) basev = atomicAdd(&cnt[d], (uint32_t)__popcll(peers));
    basev = __shfl(basev, leader, 64);
    return basev + below;
}

// Records travel through registers and LDS as raw 16-, 8- or 4-byte words
// (struct copies would be demoted to scratch by the compiler).
template <class T, int kW = (sizeof(T) % 16 == 0 ? 16 : sizeof(T) % 8 == 0 ? 8 : 4)>
struct Words {
    static constexpr int N = sizeof(T) / 16;
    uint4 w[N];
};
template <class T>
struct Words<T, 8> {
    static constexpr int N = sizeof(T) / 8;
    uint2 w[N];
};
template <class T>
struct Words<T, 4> {
    static constexpr int N = sizeof(T) / 4;
    uint32_t w[N];
};
template <class T>
__device__ __forceinline__ Words<T> to_words(const T &r) {
    Words<T> x;
    __builtin_memcpy(&x, &r, sizeof(T));
    return x;
}
template <class T>
__device__ __forceinline__ T from_words(const Words<T> &x) {
    T r;
    __builtin_memcpy(&r, &x, sizeof(T));
    return r;
}

// LDS bytes of one k_scatter instantiation (one dummy staging slot past the
// sub-tile for records that are dropped).
template <class Src, class Rec, int IPT, int FMAX, int NT = kScatThreads>
constexpr size_t scatter_lds_core() {
    return (size_t)sizeof(Rec) * (NT * IPT + 1) +
           (Src::kDigitFromRec ? 0 : a16((size_t)2 * (NT * IPT + 1))) +
           (size_t)FMAX * 12 + 80;
}
// Grouped / piece modes keep the current segment's digit bases in LDS
// (lbase, FMAX u32) when they fit beside the staging area: every tile of a
// grouped level then starts its runs from LDS instead of FMAX global loads
// whose vmcnt wait also drained the previous write-out's stores and the
// next sub-tile's prefetched loads (level 1 has one sub-tile per tile).
#ifndef DPG_SCAT_LBASE
#define DPG_SCAT_LBASE 1
#endif
#ifndef DPG_PC_NORESET
#define DPG_PC_NORESET 1
#endif
#ifndef DPG_PC_LATE_RSV
#define DPG_PC_LATE_RSV 1
#endif
template <class Src, class Rec, int IPT, int FMAX, int NT = kScatThreads>
constexpr bool scatter_lbase() {
    return scatter_lds_core<Src, Rec, IPT, FMAX, NT>() + (size_t)FMAX * 4 <= 160 * 1024;
}
template <class Src, class Rec, int IPT, int FMAX, int NT = kScatThreads>
constexpr size_t scatter_lds() {
    return scatter_lds_core<Src, Rec, IPT, FMAX, NT>() +
           (scatter_lbase<Src, Rec, IPT, FMAX, NT>() ? (size_t)FMAX * 4 : 0);
}

// Phase clock of k_scatter (timing build only, -DDPG_PHASE_TIMING): wave 0
// of every workgroup stamps s_memtime at the phase boundaries of each
// sub-tile and adds its totals to g_scat_cyc at exit: [0] loop top ->
// ranked (load waits + decode + LDS ranking + barrier), [1] digit scan
// and run reservations, [2] staging + barrier,
// [3] next loads issued + write-out, [4] tile transitions, [5] sub-tiles.
#ifdef DPG_PHASE_TIMING
__device__ unsigned long long g_scat_cyc[8];
#define DPG_SCAT_MARK(k)                                         \
    do {                                                         \
        if (threadIdx.x == 0) {                                  \
            const uint64_t now_ = __builtin_amdgcn_s_memtime();  \
            scyc[k] += now_ - slast;                             \
            slast = now_;                                        \
        }                                                        \
    } while (0)
#else
#define DPG_SCAT_MARK(k) \
    do {                 \
    } while (0)
#endif

// A pointer made provably uniform (scalar-load operands: dpg_team.h
// sload_desc; a pointer the compiler keeps in vector registers is not one).
template <class T>
__device__ __forceinline__ const T *uniform_ptr(const T *p) {
    const uint64_t v = (uint64_t)(uintptr_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return reinterpret_cast<const T *>((uintptr_t)(((uint64_t)hi << 32) | lo));
}

// kAgg: wave-aggregated ranking (few digits) instead of one LDS atomic per
// record; a template parameter so that each kernel holds one ranking path
// (both paths in one kernel cost the hot one its registers)
template <class Src, class Rec, int IPT, int FMAX, bool kAgg, int NT = kScatThreads>
__global__ __launch_bounds__(NT, 4) void k_scatter(Src src_in, const TileDesc *tiles,
                                                          const uint32_t *ntiles, uint32_t F,
                                                          uint32_t bits, const uint32_t *off,
                                                          const int64_t *base, Rec *out,
                                                          XcdQueues xq = XcdQueues{},
                                                          const uint32_t *cbase = nullptr,
                                                          const uint32_t *seg_tile_base = nullptr,
                                                          const uint32_t *seg_ntiles = nullptr,
                                                          uint32_t C = 1, uint32_t *goff = nullptr,
                                                          uint32_t pcap = 0, uint32_t pdump = 0,
                                                          uint32_t *perr = nullptr) {
    constexpr int SUB = NT * IPT;
    // piece mode (histogram-free level 1): one-sub-tile tiles on a static
    // schedule; workgroup b appends its runs of digit d to region (b % 8, d)
    // -- base[(b % 8) F + d], cursor goff[(b % 8) F + d], pcap records -- so
    // the runs of one XCD's workgroups are adjacent and merge in its L2
    constexpr bool kPc = HasPieces<Src>::value;
    constexpr bool kSD = !Src::kDigitFromRec;
    constexpr bool kP = HasFetchPairs<Src>::value && IPT % 2 == 0;
    using W = Words<Rec>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    W *stage = reinterpret_cast<W *>(smem);  // [SUB + 1]: slot SUB takes dropped records
    uint16_t *sdig = reinterpret_cast<uint16_t *>(smem + sizeof(Rec) * (SUB + 1));
    const size_t o = sizeof(Rec) * (SUB + 1) + (kSD ? a16((size_t)2 * (SUB + 1)) : 0);
    uint32_t *cnt = reinterpret_cast<uint32_t *>(smem + o);
    uint32_t *dstart = cnt + FMAX;
    uint32_t *cur = dstart + FMAX + 1;  // output positions (n < 2^32 per device)
    uint32_t *sh16 = cur + FMAX;
    constexpr bool kLB = DPG_SCAT_LBASE && scatter_lbase<Src, Rec, IPT, FMAX, NT>();
    uint32_t *lbase = reinterpret_cast<uint32_t *>(smem + scatter_lds_core<Src, Rec, IPT, FMAX, NT>());
    uint32_t lseg = 0xFFFFFFFFu;  // segment whose bases lbase holds

    // persistent over the tiles.  XCD-local mode (xq.q): workgroup b serves
    // the queue of XCD b % 8 (round-robin placement), taking the next tile id
    // by one atomic per tile, so an XCD's workgroups work on the same
    // segments at the same time and their runs meet in that XCD's L2
    const uint32_t nt = __builtin_amdgcn_readfirstlane(*ntiles);
    const int tid = threadIdx.x;
    // sub-tile position of this thread's element j
    auto elem = [tid](int j) -> uint32_t {
        return kP ? (uint32_t)((j >> 1) * 2 * NT + 2 * tid + (j & 1))
                  : (uint32_t)(j * NT + tid);
    };
    __shared__ uint32_t sh_next;
    const uint32_t xq_id = blockIdx.x & 7u;
    // (uniform: the loop over the tiles holds barriers, so its exits must
    // be visibly wave-uniform -- tools/check_barrier_loops.py)
    const uint32_t xq_len = xq.q ? __builtin_amdgcn_readfirstlane(xq.n[xq_id]) : 0u;
    constexpr uint32_t kNone = 0xFFFFFFFFu;
    Src src = src_in;  // per-thread copy (sources may cache lookup state)
    // software pipeline: the raw loads of the next sub-tile -- of this tile,
    // or the first one of the next tile -- are issued right after the
    // current sub-tile is staged in LDS, so they are in flight during its
    // write-out.  (Grouped XCD-local levels have one sub-tile per tile: the
    // next tile's id is dequeued at the start of the current one.)
    // Loads are unconditional with the index clamped into the sub-tile (a
    // guarded load becomes a branch with its own vmcnt(0) wait, serialising
    // the sub-tile's loads); lanes past the end re-read the last record.
    // Every LDS step below is likewise branch-free: a predicated LDS access
    // whose result is used becomes a branch with an lgkmcnt(0) wait inside,
    // which serialises the IPT accesses of a thread.
    // Pair sources: element j of a thread is sub-tile position
    // (j / 2) * 2T + 2 tid + j % 2, so elements 2m, 2m + 1 load as one
    // 16-byte load (clamped to the last two records; a one-record sub-tile
    // loads singly)
    typename Src::Raw raw[IPT];
    auto load_sub = [&](int64_t b0, uint32_t lim) {
        if constexpr (kP) {
            if (lim >= 2) {
#pragma unroll
                for (int m = 0; m < IPT / 2; ++m) {
                    const uint32_t o = m * 2 * NT + 2 * tid;
                    const uint32_t a = min(o, lim - 2);
                    typename Src::Raw x0, x1;
                    src.fetch2(b0 + a, x0, x1);
                    raw[2 * m] = a == o ? x0 : x1;
                    raw[2 * m + 1] = x1;
                }
                return;
            }
        }
#pragma unroll
        for (int j = 0; j < IPT; ++j) raw[j] = src.fetch(b0 + min(elem(j), lim - 1));
    };
    // the first tile (tiles are never empty: the tile builders cut
    // ceil(n / tile) tiles of n > 0 records)
    uint32_t it = blockIdx.x;  // static schedule: it, it + gridDim.x, ...
    uint32_t t = kNone;
    if (xq.q) {
        if (tid == 0) sh_next = atomicAdd(&xq.next[xq_id], 1u);
        __syncthreads();
        const uint32_t w = __builtin_amdgcn_readfirstlane(sh_next);
        if (w < xq_len) t = __builtin_amdgcn_readfirstlane(xq.q[(size_t)xq_id * xq.stride + w]);
    } else if (it < nt) {
        t = it;
    }
    if (t == kNone) return;
#ifdef DPG_PHASE_TIMING
    uint64_t scyc[6] = {0, 0, 0, 0, 0, 0};
    uint64_t slast = __builtin_amdgcn_s_memtime();
#endif
    TileDesc td = uniform_tile(tiles, t);
    // piece mode: the end of the input (the last tile's end)
    const int64_t n_end = kPc ? uniform_tile(tiles, nt - 1).end : 0;
    load_sub(td.begin, (uint32_t)min<int64_t>(SUB, td.end - td.begin));
    // piece mode with the region bases in LDS: cur is assigned (not
    // accumulated) by the digit scan and cnt is zeroed there, so the tiles
    // need no reset between them -- one setup here.  The per-tile reset was
    // a loop whose spilled LDS address (scratch reload, s_waitcnt vmcnt(0))
    // drained the previous write-out's stores and the prefetched loads at
    // every tile transition.
    constexpr bool kPcLB = kPc && kLB && DPG_PC_NORESET;
    if constexpr (kPcLB) {
        for (uint32_t d = tid; d < F; d += NT) {
            lbase[d] = (uint32_t)base[(size_t)(blockIdx.x & 7u) * F + d];
            cnt[d] = 0;
        }
        __syncthreads();
    }
    for (;;) {
    // the next tile's queue slot: one atomic by thread 0, issued now,
    // published in LDS with the first ranking barrier below
    uint32_t nq = 0;
    const uint32_t *cb = nullptr;
    uint32_t *gof = goff ? goff + (size_t)(kPc ? (blockIdx.x & 7u) : td.pad) * F : nullptr;
    if constexpr (!kPcLB) {
    if (xq.q && tid == 0) nq = atomicAdd(&xq.next[xq_id], 1u);
    __syncthreads();   // the previous tile's write-out has read cur / dstart / sh_next
    // chunked tile scan: the tile's offset is relative to its chunk
    if (cbase) {
        const uint32_t nta = seg_ntiles[td.seg], per = (nta + C - 1) / C;
        cb = cbase + ((size_t)td.seg * C + (t - seg_tile_base[td.seg]) / per) * F;
    }
    // grouped mode: the work item is one sub-tile of group td.pad, whose runs
    // are reserved at the digit scan
    const uint32_t bsel = kPc ? (blockIdx.x & 7u) : td.seg;
    if (kLB && goff) {
        // a thread reads back only the lbase entries it wrote itself
        if (bsel != lseg) {
            for (uint32_t d = tid; d < F; d += NT) lbase[d] = (uint32_t)base[(size_t)bsel * F + d];
            lseg = bsel;
        }
        for (uint32_t d = tid; d < F; d += NT) {
            cur[d] = lbase[d];
            cnt[d] = 0;
        }
    } else {
        for (uint32_t d = tid; d < F; d += NT) {
            cur[d] = (uint32_t)(base[(size_t)bsel * F + d] +
                                (goff ? 0u : off[(size_t)t * F + d] + (cb ? cb[d] : 0u)));
            cnt[d] = 0;
        }
    }
    __syncthreads();
    }  // !kPcLB
    uint32_t tn = kNone;
    TileDesc tdn = td;
    DPG_SCAT_MARK(4);
    for (int64_t sb = td.begin; sb < td.end; sb += SUB) {
        const uint32_t lim = (uint32_t)min<int64_t>(SUB, td.end - sb);  // uniform
        Rec rec[IPT];
        uint32_t dr[IPT];  // digit | rank << 12, or ~0 for a dropped record
        if constexpr (!kAgg) {
            // wide fan-out: one LDS atomic per record ranks it (order inside
            // a digit is free); all IPT atomics are in flight together, a
            // dropped record adds 0 to digit 0
            uint32_t dg[IPT];
            bool okv[IPT];
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                const uint32_t o = elem(j);
                uint32_t d = 0;
                okv[j] = o < lim && src.decode(raw[j], sb + o, rec[j], d);
                dg[j] = okv[j] ? d : 0u;
            }
            uint32_t rk[IPT];
#pragma unroll
            for (int j = 0; j < IPT; ++j) rk[j] = atomicAdd(&cnt[dg[j]], okv[j] ? 1u : 0u);
#pragma unroll
            for (int j = 0; j < IPT; ++j) dr[j] = okv[j] ? (dg[j] | (rk[j] << 12)) : ~0u;
        } else {
            // few digits: wave-aggregated ranking avoids same-address
            // serialisation
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                const uint32_t o = elem(j);
                uint32_t d = 0;
                const bool ok = o < lim && src.decode(raw[j], sb + o, rec[j], d);
                const uint32_t rk = wave_agg_rank(cnt, ok ? d : 0u, ok, bits);
                dr[j] = ok ? (d | (rk << 12)) : ~0u;
            }
        }
        if (xq.q && tid == 0 && sb == td.begin) sh_next = nq;
        __syncthreads();
        DPG_SCAT_MARK(0);
        constexpr int kDPT = FMAX / NT;
        constexpr bool kLate = kPcLB && (kDPT == 2 || kDPT == 4) && FMAX == kDPT * NT && DPG_PC_LATE_RSV;
        PcRsv<(kDPT >= 2 ? kDPT : 2)> rsv;
        uint32_t total;
        if constexpr (kLate)
            total = scatter_scan_pc<NT, kDPT>(cnt, dstart, F, sh16, gof, rsv);
        else
            total = scatter_scan_update<NT, FMAX / NT, kPc>(
                cnt, dstart, cur, F, sh16, gof, pcap, pdump, perr, kPcLB ? lbase : nullptr);
        DPG_SCAT_MARK(1);
        {
            uint32_t ds[IPT];
#pragma unroll
            for (int j = 0; j < IPT; ++j) ds[j] = dstart[dr[j] != ~0u ? (dr[j] & 0xFFFu) : 0u];
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                const uint32_t pos = dr[j] != ~0u ? ds[j] + (dr[j] >> 12) : (uint32_t)SUB;
                stage[pos] = to_words(rec[j]);
                if constexpr (kSD) sdig[pos] = (uint16_t)(dr[j] & 0xFFFu);
            }
        }
        if constexpr (kLate) scatter_rsv_finish(rsv, cur, lbase, F, pcap, pdump, perr);
        __syncthreads();
        DPG_SCAT_MARK(2);
        const int64_t nb = sb + SUB;
        const uint32_t nlim = (uint32_t)max<int64_t>(0, min<int64_t>(SUB, td.end - nb));
        {
            // the next sub-tile of this tile or, after the last one of an
            // XCD-local tile, the next tile's first (one load site)
            int64_t lb = nb;
            uint32_t ll = nlim;
            if constexpr (HasTilePrefetch<Src>::value && kPc) {
                if (nlim == 0 && it + gridDim.x < nt) {
                    tn = it + gridDim.x;
                    // one-sub-tile tiles cut evenly (k_build_tiles_single):
                    // computed, not loaded (a descriptor load here waited
                    // with vmcnt(0) on the critical path of every sub-tile)
                    tdn.begin = (int64_t)tn * SUB;
                    tdn.end = min(tdn.begin + SUB, n_end);
                    lb = tdn.begin;
                    ll = (uint32_t)min<int64_t>(SUB, tdn.end - tdn.begin);
                }
            } else if constexpr (HasTilePrefetch<Src>::value) {
                if (nlim == 0 && xq.q) {
                    const uint32_t w = __builtin_amdgcn_readfirstlane(sh_next);
                    if (w < xq_len) {
                        tn = __builtin_amdgcn_readfirstlane(xq.q[(size_t)xq_id * xq.stride + w]);
                        tdn = uniform_tile(tiles, tn);
                        lb = tdn.begin;
                        ll = (uint32_t)min<int64_t>(SUB, tdn.end - tdn.begin);
                    }
                }
            }
            if (ll > 0) load_sub(lb, ll);
        }
        // write-out in batches of WB staged records per thread, branch-free:
        // slots past the end repeat the last staged record, whose store they
        // duplicate (same value, same address)
        constexpr int WB = IPT < DPG_SCAT_WB ? IPT : DPG_SCAT_WB;
        // piece mode: a fixed trip count, fully unrolled -- as a loop, the
        // compiler's loop-preheader vmcnt flush (a loop with stores, no loads,
        // using a register it still counts as loaded outside) waited for the
        // prefetched loads just issued before the first store
        constexpr int kWbIter = (IPT + WB - 1) / WB;
        auto write_batch = [&](uint32_t k0) {
            W x[WB];
            uint32_t dd[WB], kc[WB];
#pragma unroll
            for (int u = 0; u < WB; ++u) {
                kc[u] = min(k0 + u * NT + tid, total - 1);
                x[u] = stage[kc[u]];
                if constexpr (kSD) dd[u] = sdig[kc[u]];
            }
            if constexpr (!kSD) {
#pragma unroll
                for (int u = 0; u < WB; ++u) dd[u] = src.digit(from_words<Rec>(x[u]));
            }
            uint32_t c1[WB], c2[WB];
#pragma unroll
            for (int u = 0; u < WB; ++u) {
                c1[u] = cur[dd[u]];
                c2[u] = dstart[dd[u] + 1];
            }
            // cur already includes this sub-tile: its run ends at cur[d]
            // (non-temporal loads / stores measured slower: the partial
            // lines of the runs merge in L2)
#if DPG_EXP_SCAT_NOSTORE  // diagnostic only (wrong results): the scatter without its stores
#pragma unroll
            for (int u = 0; u < WB; ++u) {
                uint32_t w0;
                __builtin_memcpy(&w0, &x[u], 4);
                if (w0 == 0x12345u && c1[u] == 0x777u)  // (never)
                    *reinterpret_cast<W *>(&out[c1[u] - c2[u] + kc[u]]) = x[u];
            }
#else
#pragma unroll
            for (int u = 0; u < WB; ++u) *reinterpret_cast<W *>(&out[c1[u] - c2[u] + kc[u]]) = x[u];
#endif
        };
        if constexpr (kPc) {
#pragma unroll
            for (int b = 0; b < kWbIter; ++b) {
                if ((uint32_t)b * WB * NT >= total) break;
                write_batch((uint32_t)b * WB * NT);
            }
        } else {
            for (uint32_t k0 = 0; k0 < total; k0 += WB * NT) write_batch(k0);
        }
        // the next sub-tile's first barrier (after its ranking) orders this
        // write-out's LDS reads before the next scan and staging
        DPG_SCAT_MARK(3);
#ifdef DPG_PHASE_TIMING
        if (tid == 0) ++scyc[5];
#endif
    }
    if (!HasTilePrefetch<Src>::value && xq.q) {
        // XCD-local without the prefetch: dequeued now, loaded unoverlapped
        const uint32_t w = __builtin_amdgcn_readfirstlane(sh_next);
        if (w >= xq_len) break;
        tn = __builtin_amdgcn_readfirstlane(xq.q[(size_t)xq_id * xq.stride + w]);
        tdn = uniform_tile(tiles, tn);
        load_sub(tdn.begin, (uint32_t)min<int64_t>(SUB, tdn.end - tdn.begin));
    } else if (kPc && HasTilePrefetch<Src>::value) {
        it += gridDim.x;  // tn / tdn set and loaded by the prefetch
    } else if (!xq.q) {
        it += gridDim.x;
        if (it >= nt) break;
        tn = it;
        tdn = uniform_tile(tiles, tn);
        load_sub(tdn.begin, (uint32_t)min<int64_t>(SUB, tdn.end - tdn.begin));
    }
    if (tn == kNone) break;
    t = tn;
    td = tdn;
    }
#ifdef DPG_PHASE_TIMING
    if (tid == 0)
        for (int k = 0; k < 6; ++k) atomicAdd(&g_scat_cyc[k], (unsigned long long)scyc[k]);
#endif
}

}  // namespace dpg
