// dpg_partition.h -- MSD radix partitioning of records by privacy-id hash
// (and of kept pairs by partition-key range) for gfx950.
//
// One level = hist -> scan -> digit-base -> scatter.  A level splits every
// segment of its input into F <= 1024 digit buckets.  The scatter stages a
// sub-tile of 8192 records through LDS, ranked per digit with wave-
// aggregated LDS atomics, so each digit leaves as one contiguous run per
// sub-tile (8 records = 128 B per digit on average at F = 1024): coalesced
// writes without per-record global atomics.  Order inside a digit is not
// preserved (nothing downstream depends on it: the sampler keys on record
// contents, see DESIGN.md "Randomness").
#pragma once

#include "dpg_common.h"

namespace dpg {

constexpr int kPartThreads = 1024;          // 16 waves
constexpr int kItemsPerThread = 8;          // 8192 records per sub-tile
constexpr int kSubTile = kPartThreads * kItemsPerThread;

struct TileDesc {
    int64_t begin, end;
    uint32_t seg;
    uint32_t pad;
};

// ---------------------------------------------------------------- sources
// Level 1: the caller's structure-of-arrays input (int64 pid, int64 pk,
// double value) -> Rec16.  Drops records of non-public partitions.  Keys
// outside the supported range raise err bit 1 (the call then fails); such a
// record is still kept, so the scatter agrees with the histogram, which only
// reads pid (and pk when there is a public-partition filter).
struct SrcSoA {
    static constexpr bool kPlainFetch = false;
    const int64_t *pid;
    const int64_t *pk;
    const double *v;
    const uint8_t *pub;  // public-partition bitmap or null
    int64_t P;
    uint32_t *err;
    __device__ __forceinline__ bool load(int64_t i, Rec16 &r) const {
        const int64_t a = pid[i], b = pk[i];
        r.v = v ? v[i] : 0.0;
        r.pid = (uint32_t)a;
        r.pk = (uint32_t)b;
        const bool in_range = (uint64_t)a < 0xFFFFFFFFull && (uint64_t)b < (uint64_t)P;
        if (!in_range) atomicOr(err, 1u);
        return !(pub && in_range && !((pub[b >> 3] >> (b & 7)) & 1));
    }
};

// The level-1 histogram's view of SrcSoA: the same keep decision, reading
// only what it needs.
struct SrcSoAHist {
    const int64_t *pid;
    const int64_t *pk;
    const uint8_t *pub;
    int64_t P;
    __device__ __forceinline__ bool load(int64_t i, Rec16 &r) const {
        const int64_t a = pid[i];
        r.pid = (uint32_t)a;
        if (!pub) return true;
        const int64_t b = pk[i];
        const bool in_range = (uint64_t)a < 0xFFFFFFFFull && (uint64_t)b < (uint64_t)P;
        return !(in_range && !((pub[b >> 3] >> (b & 7)) & 1));
    }
};

template <class Src>
__host__ __device__ inline Src hist_view(const Src &s) {
    return s;
}
__host__ __device__ inline SrcSoAHist hist_view(const SrcSoA &s) {
    return SrcSoAHist{s.pid, s.pk, s.pub, s.P};
}

template <class T>
struct SrcAoS {
    static constexpr bool kPlainFetch = true;
    const T *a;
    __device__ __forceinline__ bool load(int64_t i, T &r) const {
        r = a[i];
        return true;
    }
};

// Items of S per-workgroup regions read as one sequence: element i lives in
// region s with pre[s] <= i < pre[s + 1], at a[off[s] + i - pre[s]].  Each
// thread walks increasing i, so the region found last is cached in
// registers and the binary search runs only when i leaves it.
template <class T>
struct SrcSeg {
    static constexpr bool kPlainFetch = false;
    const T *a;
    const int64_t *pre;  // [S + 1]
    const int64_t *off;  // [S]
    uint32_t S;
    int64_t lo = 0, hi = 0, base = 0;  // cached region [lo, hi), a index = base + i
    __device__ __forceinline__ bool load(int64_t i, T &r) {
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
        r = a[base + i];
        return true;
    }
};

// ----------------------------------------------------------------- digits
struct DigPid {
    uint32_t shift, mask;
    __device__ __forceinline__ uint32_t operator()(const Rec16 &r) const {
        return (fmix32(r.pid) >> shift) & mask;
    }
};

template <class T>
struct DigPk {
    uint32_t shift;
    __device__ __forceinline__ uint32_t operator()(const T &r) const { return r.pk >> shift; }
};

// ------------------------------------------------------------ tile table
// One thread per segment: allocate ceil(n / tile) tiles.
__global__ void k_build_tiles(const int64_t *seg_start, const uint32_t *seg_cnt,
                              const int64_t *seg_cnt64, uint32_t S, int64_t tile,
                              TileDesc *tiles, uint32_t *seg_tile_base, uint32_t *seg_ntiles,
                              uint32_t *ntiles_total) {
    uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    int64_t st = seg_start ? seg_start[s] : 0;
    int64_t n = seg_cnt64 ? seg_cnt64[s] : (int64_t)seg_cnt[s];
    uint32_t nt = (uint32_t)((n + tile - 1) / tile);
    uint32_t b = nt ? atomicAdd(ntiles_total, nt) : 0;
    seg_tile_base[s] = b;
    seg_ntiles[s] = nt;
    for (uint32_t j = 0; j < nt; ++j) {
        TileDesc d;
        d.begin = st + (int64_t)j * tile;
        d.end = st + min((int64_t)(j + 1) * tile, n);
        d.seg = s;
        d.pad = 0;
        tiles[b + j] = d;
    }
}

// ---------------------------------------------------------------- hist
template <class Src, class Rec, class Dig>
__global__ __launch_bounds__(kPartThreads) void k_hist(Src src_in, Dig dig, const TileDesc *tiles,
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
    int64_t i = td.begin + tid;
    for (; i + 3 * kPartThreads < td.end; i += 4 * kPartThreads) {
        Rec r[4];
        bool ok[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) ok[u] = src.load(i + u * kPartThreads, r[u]);
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (ok[u]) atomicAdd(&my[dig(r[u])], 1u);
    }
    for (; i < td.end; i += kPartThreads) {
        Rec r;
        if (src.load(i, r)) atomicAdd(&my[dig(r)], 1u);
    }
    __syncthreads();
    for (uint32_t d = tid; d < F; d += kPartThreads)
        hist[(size_t)t * F + d] = lh[d] + lh[F + d] + lh[2 * F + d] + lh[3 * F + d];
}

// ---------------------------------------------------------------- scan
// grid (S, ceil(F/64)); 16 waves split a segment's tiles, lane = digit.
// hist[t][d] <- exclusive prefix over the segment's tiles; tot[s][d] = total.
__global__ __launch_bounds__(1024) void k_scan_tiles(const uint32_t *seg_tile_base,
                                                     const uint32_t *seg_ntiles, uint32_t F,
                                                     uint32_t *hist, uint32_t *tot) {
    __shared__ uint32_t part[16][64];
    const uint32_t s = blockIdx.x;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t d = blockIdx.y * 64 + lane;
    const uint32_t nt = seg_ntiles[s], tb = seg_tile_base[s];
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
        if (w == 0) tot[(size_t)s * F + d] = total;
    }
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

// grid S: base[s][d] = seg_start[s] + exclusive_prefix_d(tot[s][.])
__global__ __launch_bounds__(1024) void k_digit_base(const int64_t *seg_start, uint32_t F,
                                                     const uint32_t *tot, int64_t *base,
                                                     int64_t *seg_total_out) {
    __shared__ uint32_t sh[16];
    const uint32_t s = blockIdx.x;
    const uint32_t d = threadIdx.x;
    uint32_t x = d < F ? tot[(size_t)s * F + d] : 0u;
    uint32_t total;
    uint32_t e = block_excl_scan_1024(x, sh, total);
    int64_t st = seg_start ? seg_start[s] : 0;
    if (d < F) base[(size_t)s * F + d] = st + e;
    if (d == 0 && seg_total_out) seg_total_out[s] = total;
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

// Records travel through registers and LDS as raw 16-byte words (struct
// copies of Rec would be demoted to scratch by the compiler).
template <class Rec>
struct Words {
    static constexpr int N = sizeof(Rec) / 16;
    uint4 w[N];
};
template <class Rec>
__device__ __forceinline__ Words<Rec> to_words(const Rec &r) {
    Words<Rec> x;
    __builtin_memcpy(&x, &r, sizeof(Rec));
    return x;
}
template <class Rec>
__device__ __forceinline__ Rec from_words(const Words<Rec> &x) {
    Rec r;
    __builtin_memcpy(&r, &x, sizeof(Rec));
    return r;
}

template <class Src, class Rec, class Dig, int IPT>
__global__ __launch_bounds__(kPartThreads) void k_scatter(Src src_in, Dig dig, const TileDesc *tiles,
                                                          const uint32_t *ntiles, uint32_t F,
                                                          uint32_t bits, const uint32_t *off,
                                                          const int64_t *base, Rec *out) {
    constexpr int sub_items = IPT;
    // LDS: staging Rec[sub], cnt[F], dstart[F], cur int64[F], sh16
    extern __shared__ __attribute__((aligned(16))) char smem[];
    Words<Rec> *stage = reinterpret_cast<Words<Rec> *>(smem);
    const int sub = kPartThreads * sub_items;
    uint32_t *cnt = reinterpret_cast<uint32_t *>(smem + sizeof(Rec) * sub);
    uint32_t *dstart = cnt + 1024;
    int64_t *cur = reinterpret_cast<int64_t *>(dstart + 1024);
    uint32_t *sh16 = reinterpret_cast<uint32_t *>(cur + 1024);

    const uint32_t t = blockIdx.x;
    if (t >= *ntiles) return;
    const TileDesc td = tiles[t];
    const int tid = threadIdx.x;
    Src src = src_in;  // per-thread copy (sources may cache lookup state)
    for (uint32_t d = tid; d < F; d += kPartThreads) {
        cur[d] = base[(size_t)td.seg * F + d] + off[(size_t)t * F + d];
        cnt[d] = 0;
    }
    __syncthreads();
    if constexpr (Src::kPlainFetch) {
        // Software pipeline: the records of sub-tile j + 1 are fetched into
        // the (then dead) registers right after sub-tile j is staged in LDS,
        // so the loads are in flight during j's write-out.
        Words<Rec> r[IPT];
        bool inb[IPT];
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            const int64_t i = td.begin + (int64_t)j * kPartThreads + tid;
            inb[j] = i < td.end;
            if (inb[j]) r[j] = to_words(src.a[i]);
        }
        for (int64_t sb = td.begin; sb < td.end; sb += sub) {
            uint32_t dg[IPT], rk[IPT];
#pragma unroll
            for (int j = 0; j < IPT; ++j) dg[j] = inb[j] ? dig(from_words<Rec>(r[j])) : 0u;
#pragma unroll
            for (int j = 0; j < IPT; ++j) rk[j] = wave_agg_rank(cnt, dg[j], inb[j], bits);
            __syncthreads();
            uint32_t c = tid < (int)F ? cnt[tid] : 0u;
            uint32_t total;
            uint32_t e = block_excl_scan_1024(c, sh16, total);
            if (tid < (int)F) dstart[tid] = e;
            __syncthreads();
#pragma unroll
            for (int j = 0; j < IPT; ++j)
                if (inb[j]) stage[dstart[dg[j]] + rk[j]] = r[j];
            __syncthreads();
            const int64_t nb = sb + sub;
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                const int64_t i = nb + (int64_t)j * kPartThreads + tid;
                inb[j] = i < td.end;
                if (inb[j]) r[j] = to_words(src.a[i]);
            }
            for (uint32_t k = tid; k < total; k += kPartThreads) {
                Words<Rec> x = stage[k];
                uint32_t dd = dig(from_words<Rec>(x));
                *reinterpret_cast<Words<Rec> *>(&out[cur[dd] + (int64_t)(k - dstart[dd])]) = x;
            }
            __syncthreads();
            if (tid < (int)F) {
                cur[tid] += cnt[tid];
                cnt[tid] = 0;
            }
            __syncthreads();
        }
        return;
    }
    for (int64_t sb = td.begin; sb < td.end; sb += sub) {
        Words<Rec> r[IPT];
        uint32_t dg[IPT];
        uint32_t rk[IPT];
        bool ok[IPT];
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            int64_t i = sb + (int64_t)j * kPartThreads + tid;
            Rec x;
            ok[j] = i < td.end && src.load(i, x);
            dg[j] = ok[j] ? dig(x) : 0u;
            r[j] = to_words(x);
        }
#pragma unroll
        for (int j = 0; j < IPT; ++j) rk[j] = wave_agg_rank(cnt, dg[j], ok[j], bits);
        __syncthreads();
        uint32_t c = tid < (int)F ? cnt[tid] : 0u;
        uint32_t total;
        uint32_t e = block_excl_scan_1024(c, sh16, total);
        if (tid < (int)F) dstart[tid] = e;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < IPT; ++j)
            if (ok[j]) stage[dstart[dg[j]] + rk[j]] = r[j];
        __syncthreads();
        for (uint32_t k = tid; k < total; k += kPartThreads) {
            Words<Rec> x = stage[k];
            uint32_t dd = dig(from_words<Rec>(x));
            *reinterpret_cast<Words<Rec> *>(&out[cur[dd] + (int64_t)(k - dstart[dd])]) = x;
        }
        __syncthreads();
        if (tid < (int)F) {
            cur[tid] += cnt[tid];
            cnt[tid] = 0;
        }
        __syncthreads();
    }
}

}  // namespace dpg
