// dpg_common.h -- device helpers shared by the gfx950 kernels of libdpg.
//
// Keyed counter-based randomness (Philox4x32-10), the granular noise
// samplers, the privacy-id hash and the bucketed record formats.  The same
// definitions are restated on the CPU in oracle/dp_oracle.c; GPU and oracle
// must agree bit for bit on every priority and selection uniform, and to
// within one granule on noise.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dpg.h"

#define DPG_WAVE 64

namespace dpg {

// ------------------------------------------------------------ record formats
// A bucketed record carries a key and the record's index in the caller's
// input (values are gathered by index, only for records that survive
// bounding).  key = (h << pkbits) | pk with h = hk(pid - pid_min) on kbits
// bits; the stored key drops the level-1 digit (the top b1 bits of h), which
// the bucket position implies.
//   R8 : one word, stored_key << ib | idx    (when it fits 64 bits)
//   R12: stored_key (two words), idx          (always fits; 12 bytes, so
//        the wide format moves 3/4 of the bytes a padded 16-byte record would)
struct alignas(8) R8 {
    uint64_t w;
};
struct alignas(4) R12 {
    uint32_t lo, hi, idx;
};
//   R16: an R8 word and the record's value (the utility pre-aggregate, which
//        sums the value of every record: carrying it through the partition
//        levels moves 8 more bytes per record per pass where a gather by index
//        would fetch a whole 128-byte line per record)
struct alignas(16) R16 {
    uint64_t w;
    double v;
};

struct Fmt {
    uint32_t ib;      // R8: bits of the record index
    uint32_t pkbits;  // bits of the partition key
    uint32_t kbits;   // bits of the privacy-id hash
    uint32_t b1;      // level-1 digit bits (dropped from the stored key)
};

template <class R>
struct RecOps;
template <>
struct RecOps<R8> {
    static __host__ __device__ __forceinline__ uint64_t key(const R8 &r, const Fmt &f) {
        return r.w >> f.ib;
    }
    static __host__ __device__ __forceinline__ uint32_t idx(const R8 &r, const Fmt &f) {
        return (uint32_t)(r.w & ((1ull << f.ib) - 1ull));
    }
    static __host__ __device__ __forceinline__ R8 make(uint64_t key, uint32_t idx, const Fmt &f) {
        return R8{(key << f.ib) | idx};
    }
};
template <>
struct RecOps<R16> {
    static __host__ __device__ __forceinline__ uint64_t key(const R16 &r, const Fmt &f) {
        return r.w >> f.ib;
    }
    static __host__ __device__ __forceinline__ uint32_t idx(const R16 &r, const Fmt &f) {
        return (uint32_t)(r.w & ((1ull << f.ib) - 1ull));
    }
    static __host__ __device__ __forceinline__ R16 make(uint64_t key, uint32_t idx, const Fmt &f) {
        return R16{(key << f.ib) | idx, 0.0};
    }
};
template <>
struct RecOps<R12> {
    static __host__ __device__ __forceinline__ uint64_t key(const R12 &r, const Fmt &) {
        return ((uint64_t)r.hi << 32) | r.lo;
    }
    static __host__ __device__ __forceinline__ uint32_t idx(const R12 &r, const Fmt &) {
        return r.idx;
    }
    static __host__ __device__ __forceinline__ R12 make(uint64_t key, uint32_t idx, const Fmt &) {
        return R12{(uint32_t)key, (uint32_t)(key >> 32), idx};
    }
};

// One value gathered by record index (the sort kernels' gathers).
template <class I>
__device__ __forceinline__ double gather_value(const double *value, I idx) {
#if DPG_EXP_NO_GATHER  // experiment: what the gathers cost (values read as 0)
    (void)value;
    (void)idx;
    return 0.0;
#else
    return value[idx];
#endif
}

// The value of a record: carried in an R16, else gathered from the input
// column by the record's index.
template <class R>
__device__ __forceinline__ double rec_value(const R &r, const double *value, const Fmt &f) {
#if DPG_EXP_NO_GATHER  // experiment: what the gathers cost (values read as 0)
    return 0.0;
#else
    if constexpr (sizeof(R) == 16) return r.v;
    else return value[RecOps<R>::idx(r, f)];
#endif
}

struct alignas(16) Item16 {  // one kept (pid, pk) pair: COUNT / SUM / PID
    uint32_t pk;
    uint32_t cnt;
    double sum;
};

struct alignas(16) Item32 {  // one kept pair with MEAN / VARIANCE moments
    uint32_t pk;
    uint32_t cnt;
    double sum;
    double nsum;
    double nsq;
};

struct alignas(8) ItemV {  // one kept pair with MEAN / VARIANCE moments, no SUM requested
    uint32_t pk;
    uint32_t cnt;
    double nsum;
    double nsq;
};

// 24 bytes: the utility sweep streams the pairs three times (two partition
// levels and the accumulate), so the leader flag rides in the top bit of the
// privacy id's record count (n < 2^31 per dpg_preaggregate call)
struct alignas(8) ItemPA {  // one (pid, pk) pair of the utility-analysis pre-aggregate
    uint32_t pk;
    uint32_t cnt;    // records of the pair
    double sum;      // sum of their values (unclipped)
    uint32_t npart;  // partitions the privacy id contributes to
    uint32_t nl;     // records of the privacy id | leader << 31
    __host__ __device__ uint32_t ncontrib() const { return nl & 0x7FFFFFFFu; }
    __host__ __device__ bool leader() const { return (nl >> 31) != 0; }
    __host__ __device__ static uint32_t pack_nl(uint32_t nc, bool lead) {
        return (nc & 0x7FFFFFFFu) | (lead ? 0x80000000u : 0u);
    }
};

// ------------------------------------------------------------ privacy-id hash
// A bijection on [0, 2^bits): xorshift / odd-multiply rounds (the Murmur3
// finaliser's shape, shifts scaled to the width).  The top bits pick the
// bucket; the bound kernels invert it to recover the privacy id.
struct HashK {
    uint32_t bits, mask, s1, s2, s3, m1, m2, i1, i2;
};

__host__ __device__ __forceinline__ uint32_t hk(uint32_t x, const HashK &H) {
    x &= H.mask;
    x ^= x >> H.s1;
    x = (x * H.m1) & H.mask;
    x ^= x >> H.s2;
    x = (x * H.m2) & H.mask;
    x ^= x >> H.s3;
    return x;
}

__host__ __device__ __forceinline__ uint32_t unxorshift(uint32_t y, uint32_t s, uint32_t bits) {
    uint32_t x = y;
    for (uint32_t k = s; k < bits; k += s) x = y ^ (x >> s);
    return x;
}

__host__ __device__ __forceinline__ uint32_t hk_inv(uint32_t y, const HashK &H) {
    uint32_t x = unxorshift(y & H.mask, H.s3, H.bits);
    x = (x * H.i2) & H.mask;
    x = unxorshift(x, H.s2, H.bits);
    x = (x * H.i1) & H.mask;
    return unxorshift(x, H.s1, H.bits);
}

inline uint32_t inv_odd32(uint32_t m) {
    uint32_t x = m;  // Newton: x <- x (2 - m x), 5 steps reach 32 bits
    for (int k = 0; k < 5; ++k) x *= 2u - m * x;
    return x;
}

inline HashK make_hash(uint32_t bits) {
    HashK H;
    H.bits = bits;
    H.mask = bits >= 32 ? 0xFFFFFFFFu : ((1u << bits) - 1u);
    H.s1 = (bits + 1) / 2;
    H.s2 = (bits * 13) / 32 > 0 ? (bits * 13) / 32 : 1;
    H.s3 = (bits + 1) / 2;
    H.m1 = 0x85EBCA6Bu;
    H.m2 = 0xC2B2AE35u;
    H.i1 = inv_odd32(H.m1);
    H.i2 = inv_odd32(H.m2);
    return H;
}

// ------------------------------------------------------------------ Philox
__host__ __device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0,
                                                       uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        // full 32x32->64 products: one v_mad_u64_u32 each on gfx950
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
        const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
        uint32_t n0 = hi1 ^ c[1] ^ k0;
        uint32_t n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0;
        c[1] = lo1;
        c[2] = n2;
        c[3] = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

// SplitMix64 finaliser and the per-release stream seed (dpg.h
// dpg_stream_seed; restated in oracle/dp_oracle.c).
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z ^= z >> 30;
    z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27;
    z *= 0x94D049BB133111EBull;
    z ^= z >> 31;
    return z;
}
__host__ __device__ __forceinline__ uint64_t stream_seed(uint64_t seed, uint64_t nonce) {
    return mix64(seed ^ mix64(nonce + 0x9E3779B97F4A7C15ull));
}

// Murmur3 finaliser (hash-table slots).
__host__ __device__ __forceinline__ uint32_t fmix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return h;
}

// Sampling priorities (DESIGN.md "Randomness"): keyed chains of the murmur3
// finalizer.  Sampling only has to be uniform without replacement -- the
// privacy guarantee holds for any choice of kept records -- so a cheap mixer
// replaces Philox here (noise keeps Philox).  pid_hash is the per-privacy-id
// state (computed once per pid in the bound kernels); pair_prio_h orders the
// pid's partitions (mpc), rec_prio_h the records of a pair or pid (mcpp, L)
// with the low 32 bits of the global record id as tie-break.
__host__ __device__ __forceinline__ uint32_t pid_hash(uint64_t seed, uint64_t pid) {
    const uint32_t h = fmix32((uint32_t)seed ^ DPG_TAG_PAIR ^ (uint32_t)pid);
    return fmix32(h ^ (uint32_t)(pid >> 32) ^ (uint32_t)(seed >> 32));
}
#ifndef DPG_PRIO_PHILOX
#define DPG_PRIO_PHILOX 0
#endif
#if DPG_PRIO_PHILOX
// Cost experiment only: the same
// priorities drawn from Philox4x32-10 keyed by the per-pid state, as a
// counter-based RNG would draw them.  Not the shipped sampler: the oracle
// restates the fmix32 chains below, so parity tests fail against this build.
__host__ __device__ __forceinline__ uint32_t pair_prio_h(uint32_t hp, uint32_t pk) {
    uint32_t c[4] = {hp, pk, DPG_TAG_PAIR, 0u};
    philox4x32_10(c, hp, DPG_TAG_PAIR);
    return c[0];
}
__host__ __device__ __forceinline__ uint64_t rec_prio_h(uint32_t hp, uint32_t pk, uint64_t gidx) {
    uint32_t c[4] = {pk, (uint32_t)gidx, (uint32_t)(gidx >> 32), DPG_TAG_REC};
    philox4x32_10(c, hp, DPG_TAG_REC);
    return ((uint64_t)c[0] << 32) | (uint32_t)gidx;
}
#else
__host__ __device__ __forceinline__ uint32_t pair_prio_h(uint32_t hp, uint32_t pk) {
    return fmix32(hp ^ pk);
}
__host__ __device__ __forceinline__ uint64_t rec_prio_h(uint32_t hp, uint32_t pk, uint64_t gidx) {
    uint32_t h = fmix32(hp ^ DPG_TAG_REC);
    h = fmix32(h ^ pk);
    h = fmix32(h + (uint32_t)gidx);
    h = fmix32(h ^ (uint32_t)(gidx >> 32));
    return ((uint64_t)h << 32) | (uint32_t)gidx;
}
#endif
__device__ __forceinline__ uint32_t pair_prio(uint64_t seed, uint64_t pid, uint32_t pk) {
    return pair_prio_h(pid_hash(seed, pid), pk);
}
__device__ __forceinline__ uint64_t rec_prio(uint64_t seed, uint64_t pid, uint32_t pk,
                                             uint64_t gidx) {
    return rec_prio_h(pid_hash(seed, pid), pk, gidx);
}

__device__ __forceinline__ double u53(uint32_t a, uint32_t b) {
    uint64_t u = (((uint64_t)a << 32) | b) >> 11;
    return ((double)u + 0.5) * 0x1.0p-53;
}

__device__ __forceinline__ double granularity(double scale) {
    return exp2(ceil(log2(scale * 0x1.0p-40)));
}

// The lattice of a noise scale: g = granularity(scale) and its exact
// reciprocal (g is a power of two, so x * ig == x / g bit for bit).  The
// select / noise kernel computes it once per scale and thread instead of a
// log2 / exp2 pair per partition.
struct Gran {
    double g, ig;
};
__device__ __forceinline__ Gran gran_of(double scale) {
    if (!(scale > 0)) return Gran{0.0, 0.0};
    const double g = granularity(scale);
    return Gran{g, 1.0 / g};
}

// x + Laplace(b), snapped to the granularity lattice (see oracle dpo_laplace)
__device__ __forceinline__ double laplace_noise(double x, double b, const uint32_t u[4],
                                                const Gran &G) {
    if (!(b > 0)) return x;
    const double bg = b * G.ig;
    double e1 = -log(u53(u[0], u[1]));
    double e2 = -log(u53(u[2], u[3]));
    double k = floor(e1 * bg) - floor(e2 * bg);
    return rint(x * G.ig) * G.g + k * G.g;
}

__device__ __forceinline__ double gaussian_noise(double x, double sigma, const uint32_t u[4],
                                                 const Gran &G) {
    if (!(sigma > 0)) return x;
    double r = sqrt(-2.0 * log(u53(u[0], u[1])));
    double z = r * cos(6.283185307179586476925286766559 * u53(u[2], u[3]));
    return rint(x * G.ig) * G.g + rint(sigma * z * G.ig) * G.g;
}

__device__ __forceinline__ double add_noise(int kind, double x, double scale, const Gran &G,
                                            uint64_t seed, uint64_t pk, uint32_t slot) {
    if (kind == DPG_NOISE_NONE) return x;
    uint32_t c[4] = {(uint32_t)pk, (uint32_t)(pk >> 32), slot, 0u};
    philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32) ^ DPG_TAG_NOISE);
    return kind == DPG_NOISE_GAUSSIAN ? gaussian_noise(x, scale, c, G)
                                      : laplace_noise(x, scale, c, G);
}

__device__ __forceinline__ void select_uniforms(uint64_t seed, uint64_t pk, uint32_t c[4]) {
    c[0] = (uint32_t)pk;
    c[1] = (uint32_t)(pk >> 32);
    c[2] = 0u;
    c[3] = 0u;
    philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32) ^ DPG_TAG_SELECT);
}

__device__ __forceinline__ double clampd(double x, double lo, double hi) {
    return x < lo ? lo : (x > hi ? hi : x);
}

// Exclusive prefix sum over the 64 lanes of a wave (all lanes active) in
// registers: DPP row shifts 1/2/4/8 scan each row of 16 lanes, then row
// broadcasts of lanes 15 and 31 carry the row totals (gfx9 DPP).
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t x, uint32_t &total) {
    int v = (int)x;
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    total = (uint32_t)__builtin_amdgcn_readlane(v, 63);
    return (uint32_t)v - x;
}

}  // namespace dpg
