// dpg_utility.h -- utility analysis of many contribution-bound configurations
// in one pass over the per-(privacy id, partition) pre-aggregate (gfx950).
//
// Reference: analysis/per_partition_combiners.py (PartitionSelectionCombiner
// :195-240, SumCombiner :243-297, CountCombiner :300-318,
// PrivacyIdCountCombiner :321-339, RawStatisticsCombiner :342-356) and
// analysis/poisson_binomial.py:39-83.
//
// Layout: the pairs are sorted by partition key (dpg_preaggregate), so every
// partition is one contiguous run.  Lane c of a wave is configuration c
// (<= 64 configurations: one wave covers a whole sweep), so per-pair work is
// a broadcast of the pair and 64 independent evaluations, and every per-
// partition output row [field][config] is one contiguous 512-byte store.
//   k_ua_accumulate: one wave per run of kUaRun pairs; per partition segment
//     the additive accumulators (SUM / COUNT / PRIVACY_ID_COUNT error terms,
//     Poisson-binomial moments of the keep probabilities, raw statistics);
//     a segment wholly inside the run is stored, a segment split between
//     runs is added atomically (the output is zeroed first).
//   k_ua_public: public partitions get the empty accumulator every public
//     partition carries in the reference (dp_engine.py:288-303).
//   k_ua_select: one wave per partition: the exact Poisson-binomial PMF of
//     the privacy-id count (<= 100 pairs; LDS column per lane) or its refined
//     normal approximation from the moments, dotted with the keep
//     probability of the configuration's selection strategy.
#pragma once

#include "dpg_common.h"

namespace dpg {

constexpr int kUaRun = 1024;          // pairs per accumulate wave
constexpr int kUaMaxExact = 100;      // MAX_PROBABILITIES_IN_ACCUMULATOR
constexpr int kUaMom = 3;             // sum p, sum p(1-p), sum p(1-p)(1-2p)

struct UaConfig {                     // device copy of dpg_ua_config
    double mpc, mcpp, lo, hi;         // l0, linf, SUM clipping bounds
    int32_t strategy, pre_threshold;
    int64_t table_offset, table_len;
    double threshold, scale;
};

struct UaArgs {
    int32_t n_configs;
    int32_t has_sum, has_count, has_pid;  // metric blocks present (in this order)
    int32_t n_metrics;
    int64_t P;
    const UaConfig *cfg;              // device [n_configs]
    const double *tables;             // device keep tables
    const uint8_t *sample_mask;       // partitions kept by partitions_sampling_prob (or null)
    const uint8_t *public_mask;       // public partitions (public mode) or null
    double *raw;                      // [P][2]: privacy id count, count
    double *err;                      // [P][n_metrics][5][C]
    double *mom;                      // [P][3][C]
    double *keep;                     // [P][C]
};

__device__ __forceinline__ bool bit_of(const uint8_t *m, int64_t k) {
    return (m[k >> 3] >> (k & 7)) & 1;
}

// SumCombiner.create_accumulator for one pair (per_partition_combiners.py
// :262-287): clip to [lo, hi], clipping errors, l0 bounding moments
struct ErrAcc {
    double tot, cmin, cmax, el0, vl0;
    __device__ void clear() { tot = cmin = cmax = el0 = vl0 = 0.0; }
    __device__ __forceinline__ void add(double x, double lo, double hi, double p, double q) {
        const double pc = x < lo ? lo : (x > hi ? hi : x);
        const double d = pc - x;
        tot += x;
        cmin += x < lo ? d : 0.0;
        cmax += x > hi ? d : 0.0;
        el0 -= pc * (1.0 - p);
        vl0 += pc * pc * q;
    }
};

__device__ __forceinline__ void ua_put(double *dst, double v, bool atomic) {
    if (atomic) atomicAdd(dst, v);
    else *dst = v;
}

__global__ __launch_bounds__(64) void k_ua_accumulate(const ItemPA *pairs,
                                                      const int64_t *pstart, int64_t n,
                                                      UaArgs a) {
    const int64_t lo = (int64_t)blockIdx.x * kUaRun;
    if (lo >= n) return;
    const int64_t hi = lo + kUaRun < n ? lo + kUaRun : n;
    const int c = (int)__lane_id();
    const int C = a.n_configs;
    const bool lane_on = c < C;
    const UaConfig cf = a.cfg[lane_on ? c : 0];
    double e = 0, v = 0, t = 0, rn = 0, rc = 0;
    ErrAcc es, ec, ep;
    es.clear();
    ec.clear();
    ep.clear();
    uint32_t cur = pairs[lo].pk;
    bool skip = a.sample_mask && !bit_of(a.sample_mask, cur);
    auto flush = [&](uint32_t pk) {
        if (skip) return;
        const bool atomic = !(pstart[pk] >= lo && pstart[pk + 1] <= hi);
        const int64_t C64 = C;
        if (c == 0) {
            ua_put(&a.raw[2 * (int64_t)pk], rn, atomic);
            ua_put(&a.raw[2 * (int64_t)pk + 1], rc, atomic);
        }
        if (!lane_on) return;
        double *m = a.mom + (int64_t)pk * kUaMom * C64 + c;
        ua_put(m, e, atomic);
        ua_put(m + C64, v, atomic);
        ua_put(m + 2 * C64, t, atomic);
        double *o = a.err + (int64_t)pk * a.n_metrics * 5 * C64 + c;
        auto put5 = [&](const ErrAcc &x) {
            ua_put(o, x.tot, atomic);
            ua_put(o + C64, x.cmin, atomic);
            ua_put(o + 2 * C64, x.cmax, atomic);
            ua_put(o + 3 * C64, x.el0, atomic);
            ua_put(o + 4 * C64, x.vl0, atomic);
            o += 5 * C64;
        };
        if (a.has_sum) put5(es);
        if (a.has_count) put5(ec);
        if (a.has_pid) put5(ep);
    };
    for (int64_t b = lo; b < hi; b += 64) {
        const int64_t i = b + c < hi ? b + c : hi - 1;
        const ItemPA mine = pairs[i];
        const int m = (int)(hi - b < 64 ? hi - b : 64);
        for (int j = 0; j < m; ++j) {
            const uint32_t pk = __builtin_amdgcn_readlane(mine.pk, j);
            if (pk != cur) {
                flush(cur);
                e = v = t = rn = rc = 0.0;
                es.clear();
                ec.clear();
                ep.clear();
                cur = pk;
                skip = a.sample_mask && !bit_of(a.sample_mask, cur);
            }
            if (skip) continue;
            const uint32_t cnt = __builtin_amdgcn_readlane(mine.cnt, j);
            const uint32_t np = __builtin_amdgcn_readlane(mine.npart, j);
            const uint32_t slo = __builtin_amdgcn_readlane((uint32_t)__double_as_longlong(mine.sum), j);
            const uint32_t shi =
                __builtin_amdgcn_readlane((uint32_t)(__double_as_longlong(mine.sum) >> 32), j);
            const double s = __longlong_as_double((long long)(((uint64_t)shi << 32) | slo));
            // l0 keep probability of this pair (per_partition_combiners.py:203-205)
            const double p = np > 0 ? fmin(1.0, cf.mpc / (double)np) : 0.0;
            const double q = p * (1.0 - p);
            e += p;
            v += q;
            t += q * (1.0 - 2.0 * p);
            rn += 1.0;
            rc += (double)cnt;
            if (a.has_sum) es.add(s, cf.lo, cf.hi, p, q);
            if (a.has_count) ec.add((double)cnt, 0.0, cf.mcpp, p, q);
            if (a.has_pid) ep.add(cnt > 0 ? 1.0 : 0.0, 0.0, 1.0, p, q);
        }
    }
    flush(cur);
}

// The empty accumulator every public partition carries (count 0, sum 0, 0
// partitions): one more privacy id in the raw statistics, and the SUM
// clipping of a zero contribution.  Runs after k_ua_accumulate.
__global__ __launch_bounds__(64) void k_ua_public(UaArgs a) {
    const int c = (int)__lane_id();
    const int64_t C64 = a.n_configs;
    for (int64_t k = blockIdx.x; k < a.P; k += gridDim.x) {
        if (!bit_of(a.public_mask, k)) continue;
        if (c == 0) a.raw[2 * k] += 1.0;
        if (!a.has_sum || c >= a.n_configs) continue;
        const UaConfig cf = a.cfg[c];
        ErrAcc z;
        z.clear();
        z.add(0.0, cf.lo, cf.hi, 0.0, 0.0);
        double *o = a.err + k * a.n_metrics * 5 * C64 + c;
        o[C64] += z.cmin;
        o[2 * C64] += z.cmax;
        o[3 * C64] += z.el0;
    }
}

// Keep probability of a partition whose privacy-id count is i
// (partition_selection.probability_of_keep restated; 0 for i <= 0).
__device__ __forceinline__ double ua_pi(const UaConfig &cf, const double *tables, int64_t i) {
    if (i <= 0) return 0.0;
    if (cf.pre_threshold > 0) {
        if (i < cf.pre_threshold) return 0.0;
        i = i - cf.pre_threshold + 1;
    }
    if (cf.strategy == DPG_SELECT_TRUNCATED_GEOMETRIC)
        return i < cf.table_len ? tables[cf.table_offset + i] : 1.0;
    if (cf.strategy == DPG_SELECT_LAPLACE_THRESHOLD) {
        const double x = ((double)i - cf.threshold) / cf.scale;
        return x >= 0 ? 1.0 - 0.5 * exp(-x) : 0.5 * exp(x);
    }
    const double z = ((double)i - cf.threshold) / cf.scale;
    return 0.5 * erfc(-z * 0.70710678118654752440);
}

// refined normal approximation (poisson_binomial.py:61-83)
__device__ __forceinline__ double ua_G(double x, double skew) {
    const double phi = 0.39894228040143267794 * exp(-0.5 * x * x);
    return 0.5 * erfc(-x * 0.70710678118654752440) + skew * (1.0 - x * x) * phi / 6.0;
}

__global__ __launch_bounds__(64) void k_ua_select(const ItemPA *pairs, const int64_t *pstart,
                                                  UaArgs a) {
    extern __shared__ __attribute__((aligned(16))) double s_pgf[];  // [kUaMaxExact + 1][64]
    const int c = (int)__lane_id();
    const int64_t C64 = a.n_configs;
    const bool lane_on = c < a.n_configs;
    const UaConfig cf = a.cfg[lane_on ? c : 0];
    double *col = s_pgf + c;  // lane-private column, stride 64
    for (int64_t k = blockIdx.x; k < a.P; k += gridDim.x) {
        const int64_t b = pstart[k], n = pstart[k + 1] - b;
        if (n == 0 || (a.sample_mask && !bit_of(a.sample_mask, k))) continue;
        double keep = 0.0;
        if (n <= kUaMaxExact) {
            // exact PMF: coefficients of prod_j (1 - p_j + p_j x)
            col[0] = 1.0;
            for (int64_t j = 0; j < n; ++j) {
                const uint32_t np = pairs[b + j].npart;
                const double p = np > 0 ? fmin(1.0, cf.mpc / (double)np) : 0.0;
                col[64 * (j + 1)] = 0.0;
                for (int64_t i = j + 1; i >= 1; --i)
                    col[64 * i] = col[64 * i] * (1.0 - p) + col[64 * (i - 1)] * p;
                col[0] *= 1.0 - p;
            }
            for (int64_t i = 0; i <= n; ++i) keep += col[64 * i] * ua_pi(cf, a.tables, i);
        } else {
            const double *mm = a.mom + k * kUaMom * C64 + (lane_on ? c : 0);
            const double mean = mm[0], sd = sqrt(mm[C64]);
            if (sd == 0.0) {
                keep = ua_pi(cf, a.tables, (int64_t)rint(mean));
            } else {
                const double skew = mm[2 * C64] / (sd * sd * sd);
                const int64_t st = (int64_t)fmax(0.0, floor(mean - 8.0 * sd));
                const int64_t en = (int64_t)fmin((double)n, rint(mean + 8.0 * sd));
                double prev = fmin(1.0, fmax(0.0, ua_G(((double)(st - 1) + 0.5 - mean) / sd, skew)));
                for (int64_t i = st; i <= en; ++i) {
                    const double cur =
                        fmin(1.0, fmax(0.0, ua_G(((double)i + 0.5 - mean) / sd, skew)));
                    keep += (cur - prev) * ua_pi(cf, a.tables, i);
                    prev = cur;
                }
            }
        }
        if (lane_on) a.keep[k * C64 + c] = keep;
    }
}

}  // namespace dpg
