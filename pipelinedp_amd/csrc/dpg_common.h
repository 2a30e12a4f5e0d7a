// dpg_common.h -- device helpers shared by the gfx950 kernels of libdpg.
//
// Keyed counter-based randomness (Philox4x32-10) and the granular noise
// samplers.  The same definitions are restated on the CPU in
// oracle/dp_oracle.c; GPU and oracle must agree bit for bit on every
// priority and selection uniform, and to within one granule on noise.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dpg.h"

#define DPG_WAVE 64

namespace dpg {

struct alignas(16) Rec16 {  // one bucketed record (AoS, one dwordx4)
    uint32_t pid;
    uint32_t pk;
    double v;
};

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

// Murmur3 finaliser: a bijection on 32-bit ints; its top bits pick the
// privacy-id bucket.
__host__ __device__ __forceinline__ uint32_t fmix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return h;
}

__device__ __forceinline__ uint32_t pair_prio(uint64_t seed, uint32_t pid, uint32_t pk) {
    uint32_t c[4] = {pid, pk, 0u, 0u};
    philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32) ^ DPG_TAG_PAIR);
    return c[0];
}

__device__ __forceinline__ uint64_t rec_prio(uint64_t seed, uint32_t pid, uint32_t pk,
                                             uint64_t vbits, uint32_t occ) {
    uint32_t c[4] = {pid, pk, (uint32_t)vbits, (uint32_t)(vbits >> 32)};
    philox4x32_10(c, (uint32_t)seed ^ (occ * 0x9E3779B9u),
                  (uint32_t)(seed >> 32) ^ DPG_TAG_REC);
    return ((uint64_t)c[0] << 32) | c[1];
}

__device__ __forceinline__ double u53(uint32_t a, uint32_t b) {
    uint64_t u = (((uint64_t)a << 32) | b) >> 11;
    return ((double)u + 0.5) * 0x1.0p-53;
}

__device__ __forceinline__ double granularity(double scale) {
    return exp2(ceil(log2(scale * 0x1.0p-40)));
}

// x + Laplace(b), snapped to the granularity lattice (see oracle dpo_laplace)
__device__ __forceinline__ double laplace_noise(double x, double b, const uint32_t u[4]) {
    if (!(b > 0)) return x;
    double g = granularity(b);
    double e1 = -log(u53(u[0], u[1]));
    double e2 = -log(u53(u[2], u[3]));
    double k = floor(e1 * (b / g)) - floor(e2 * (b / g));
    return rint(x / g) * g + k * g;
}

__device__ __forceinline__ double gaussian_noise(double x, double sigma, const uint32_t u[4]) {
    if (!(sigma > 0)) return x;
    double g = granularity(sigma);
    double r = sqrt(-2.0 * log(u53(u[0], u[1])));
    double z = r * cos(6.283185307179586476925286766559 * u53(u[2], u[3]));
    return rint(x / g) * g + rint(sigma * z / g) * g;
}

__device__ __forceinline__ double add_noise(int kind, double x, double scale, uint64_t seed,
                                            uint64_t pk, uint32_t slot) {
    if (kind == DPG_NOISE_NONE) return x;
    uint32_t c[4] = {(uint32_t)pk, (uint32_t)(pk >> 32), slot, 0u};
    philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32) ^ DPG_TAG_NOISE);
    return kind == DPG_NOISE_GAUSSIAN ? gaussian_noise(x, scale, c) : laplace_noise(x, scale, c);
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

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// Wave-level exclusive prefix of a per-lane count; returns the wave total.
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t x, uint32_t &total) {
    uint32_t v = x;
    const int lane = __lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(v, o, 64);
        if (lane >= o) v += y;
    }
    total = __shfl(v, 63, 64);
    return v - x;
}

}  // namespace dpg
