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
//     the privacy-id count (<= 100 pairs; coefficients in registers) or its refined
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

constexpr int kUaBuckets = 29;        // utility_analysis.py:29-39 bucket bounds
constexpr int kUaRepRun = 512;        // partitions per report wave
constexpr int kUaMaxF = 4 + 24 * 3;   // report fields per configuration

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
    // cross-partition report (k_ua_bucket / k_ua_order / k_ua_report)
    const double *std;                // [n_metrics][C] noise std of each metric
    int32_t *bucket;                  // [P] size bucket of an output partition, -1 else
    uint32_t *bcount;                 // [kUaBuckets] partitions per bucket, then cursors
    int64_t *order;                   // partitions of the output, bucket by bucket
    double *rep;                      // [kUaBuckets][F][C] summed report fields
    // selection classes: configurations with the same l0 and keep function
    // (strategy, pre-threshold, keep table / threshold / scale) share one
    // column of the LDS keep-probability table of k_ua_select and one
    // normal-approximation pass (the moments depend on l0 only)
    const int32_t *cls;               // [C] class of each configuration
    const int32_t *cls_rep;           // [n_cls] a configuration of each class
    int32_t n_cls;
    int32_t npi;                      // keep probabilities pi(0 .. npi - 1) in LDS
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

// min(max(x, lo), hi) as two bare VALU instructions.  fmin / fmax lower to
// the same v_max_f64 / v_min_f64 but, in the kernels' IEEE mode, first
// canonicalise every operand the compiler cannot prove canonical (here x,
// lo and hi: three more FP64 instructions per pair and configuration in
// k_ua_accumulate).  The operands are never signalling NaNs (values and
// bounds come from finite host data), for which the result is the same.
__device__ __forceinline__ double clamp_f64(double x, double lo, double hi) {
    double r;
    asm("v_max_f64 %0, %1, %2\n\tv_min_f64 %0, %0, %3" : "=&v"(r) : "v"(x), "v"(lo), "v"(hi));
    return r;
}

// min(a, b) as one bare v_min_f64 (see clamp_f64: fmin would canonicalise
// both operands first)
__device__ __forceinline__ double min_f64(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// clamp_f64 of a wave-uniform value held in scalar registers (one scalar
// operand per VOP3 instruction)
__device__ __forceinline__ double clamp_f64_s(double x, double lo, double hi) {
    double r;
    asm("v_max_f64 %0, %1, %2\n\tv_min_f64 %0, %0, %3" : "=&v"(r) : "s"(x), "v"(lo), "v"(hi));
    return r;
}

// pk, cnt and sum of one pair by a scalar load: the pair is the same for
// every configuration lane, so the accumulate loop reads them as scalar
// operands (no LDS broadcast and no v_readfirstlane per pair).  Loads only:
// nothing is written through the scalar cache.
struct PairHead {
    uint32_t pk, cnt;
    double sum;
};
__device__ __forceinline__ PairHead sload_head(const ItemPA *p) {
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    u4 r;
    asm volatile("s_load_dwordx4 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r) : "s"(p));
    PairHead h;
    h.pk = r.x;
    h.cnt = r.y;
    h.sum = __hiloint2double((int)r.w, (int)r.z);
    return h;
}

__device__ __forceinline__ void ua_put(double *dst, double v, bool atomic) {
    if (atomic) atomicAdd(dst, v);
    else *dst = v;
}

// kSum / kCount / kPid: the metrics of the sweep (a.has_*), as template
// flags so that the loop holds neither their branches nor the selects the
// compiler if-converts them into.
template <bool kSum, bool kCount, bool kPid>
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
    // Per pair and configuration only the terms that depend on both remain
    // in the loop: COUNT's error terms are those of x = count >= 0 (its
    // total is the raw count, its clip-to-min error 0), and
    // PRIVACY_ID_COUNT's (x = 1 for count > 0) follow from the moments at the
    // flush: total rn - nz, l0 terms -(sum of 1 - p) = e - rn and sum of q =
    // v, corrected by the pairs of count 0 (pre-aggregated input only).
    // The loop is VALU-issue bound (config 5: ~7e8 pairs, one wave64
    // instruction per term for all 64 configurations; ~37 instructions per
    // pair), so every term costs instructions, not bytes: the pair and
    // record counts stay wave-uniform scalars, COUNT's clip-to-max error is
    // the exact double sum of the clipped counts less the record count, and
    // the float terms use min / max / fma forms (same values, fewer
    // instructions than compare-and-select chains).
    double e = 0, v = 0, t = 0;
    uint32_t rn = 0;                   // pairs of the partition (wave-uniform)
    uint64_t rc = 0;                   // records of the partition (wave-uniform)
    ErrAcc es;
    double spci = 0;                   // COUNT: sum of the clipped counts (exact: < 2^53)
    double cel = 0, cvl = 0;           // COUNT: l0 mean, l0 variance
    double nz = 0, zel = 0, zvl = 0;   // pairs of count 0: number, sum 1 - p, sum q
    const double mcpp_d = cf.mcpp;
    const double clo = cf.lo, chi = cf.hi;
    es.clear();
    uint32_t cur = pairs[lo].pk;
    bool skip = a.sample_mask && !bit_of(a.sample_mask, cur);
    // only the run's first and last partitions can be split with the
    // neighbouring runs (added atomically); decided here, so that a flush
    // loads nothing (a load in the flush waited for the previous flush's
    // stores)
    const uint32_t pk_first = pairs[lo].pk, pk_last = pairs[hi - 1].pk;
    const bool split_first = lo > 0 && pairs[lo - 1].pk == pk_first;
    const bool split_last = hi < n && pairs[hi].pk == pk_last;
    auto flush = [&](uint32_t pk) {
        if (skip) return;
        const bool atomic = (pk == pk_first && split_first) || (pk == pk_last && split_last);
        const int64_t C64 = C;
        const double rnd = (double)rn, rcd = (double)rc;
        if (c == 0) {
            ua_put(&a.raw[2 * (int64_t)pk], rnd, atomic);
            ua_put(&a.raw[2 * (int64_t)pk + 1], rcd, atomic);
        }
        if (!lane_on) return;
        double *m = a.mom + (int64_t)pk * kUaMom * C64 + c;
        ua_put(m, e, atomic);
        ua_put(m + C64, v, atomic);
        ua_put(m + 2 * C64, t, atomic);
        double *o = a.err + (int64_t)pk * a.n_metrics * 5 * C64 + c;
        auto put5 = [&](double tot, double cmin, double cmax, double el0, double vl0) {
            ua_put(o, tot, atomic);
            ua_put(o + C64, cmin, atomic);
            ua_put(o + 2 * C64, cmax, atomic);
            ua_put(o + 3 * C64, el0, atomic);
            ua_put(o + 4 * C64, vl0, atomic);
            o += 5 * C64;
        };
        if (kSum) put5(es.tot, es.cmin, es.cmax, es.el0, es.vl0);
        // clip-to-max error sum(min(cnt, mcpp) - cnt) = spci - rc, exact
        if (kCount) put5(rcd, 0.0, spci - rcd, cel, cvl);
        if (kPid) put5(rnd - nz, 0.0, 0.0, (e - rnd) + zel, v - zvl);
    };
    // Per block of 64 pairs each lane computes one pair's 1 / n_partitions
    // into LDS (one division per pair, not per (pair, configuration)); the
    // pair's key, count and sum come by scalar loads (sload_head).  (Round 3
    // loaded the pair into registers per lane and broadcast it by readlane:
    // with the loaded registers live in the loop, every iteration waited for
    // all vector memory operations -- s_waitcnt vmcnt(0) at the loop head --
    // i.e. for the stores of every partition flush.  Round 4 broadcast key,
    // count, sum and inverse through LDS: 31 VALU instructions per pair,
    // 4 of them v_readfirstlane / address moves.)
    // (1 / n_partitions, count) per pair as doubles, read by one LDS load
    __shared__ double2 s_pair[64];
    for (int64_t b = lo; b < hi; b += 64) {
        const int64_t i = b + c < hi ? b + c : hi - 1;
        const uint32_t np = pairs[i].npart;
        s_pair[c] = make_double2(np > 0 ? 1.0 / (double)np : 0.0, (double)pairs[i].cnt);
        __syncthreads();
        // the trip count as a scalar: a vector loop counter costs one VALU
        // instruction per pair
        const int m = __builtin_amdgcn_readfirstlane((int)(hi - b < 64 ? hi - b : 64));
        for (int j = 0; j < m; ++j) {
            const PairHead h = sload_head(pairs + b + j);
            const uint32_t pk = h.pk;
            if (pk != cur) {
                flush(cur);
                e = v = t = 0.0;
                rn = 0;
                rc = 0;
                es.clear();
                spci = 0.0;
                cel = cvl = 0.0;
                nz = zel = zvl = 0.0;
                cur = pk;
                skip = a.sample_mask && !bit_of(a.sample_mask, cur);
            }
            if (skip) continue;
            const uint32_t cnt = h.cnt;
            const double2 ic = s_pair[j];
            const double inv = ic.x;
            // l0 keep probability of this pair (per_partition_combiners.py:203-205)
            const double p = fmin(1.0, cf.mpc * inv);
            const double omp = 1.0 - p;
            const double q = p * omp;
            e += p;
            v += q;
            t = fma(q, fma(-2.0, p, 1.0), t);
            rn += 1;
            rc += cnt;
            if constexpr (kSum) {
                const double x = h.sum;
                const double pc = clamp_f64_s(x, clo, chi);
                // pc - x: lo - x where x < lo, hi - x where x > hi, else 0
                const double d = pc - x;
                es.tot += x;
                es.cmin += fmax(d, 0.0);
                es.cmax += fmin(d, 0.0);
                es.el0 = fma(-pc, omp, es.el0);
                es.vl0 = fma(pc * pc, q, es.vl0);
            }
            if constexpr (kCount) {
                // min(count, mcpp) on the staged double count (exact: < 2^53)
                const double pc = min_f64(ic.y, mcpp_d);
                spci += pc;
                cel = fma(-pc, omp, cel);
                cvl = fma(pc * pc, q, cvl);
            }
            if (kPid && cnt == 0) {  // wave-uniform
                nz += 1.0;
                zel += omp;
                zvl += q;
            }
        }
        __syncthreads();  // the next block rewrites s_pair
    }
    flush(cur);
}

// Private partitions: the rows k_ua_accumulate adds atomically -- those of
// partitions split between runs of kUaRun pairs -- start from zero.  Every
// other row of a partition with pairs is written by plain stores, and rows
// of partitions without pairs are never read (the output is the partitions
// with pairs), so the ~9.7 GB of per-partition outputs of a 64-configuration
// sweep over 1e6 partitions need no zero fill.  One wave per partition;
// vector stores only.
__global__ __launch_bounds__(256) void k_ua_zero_split(const int64_t *pstart, UaArgs a) {
    const int lane = (int)__lane_id();
    const int64_t C64 = a.n_configs;
    const int64_t E = (int64_t)a.n_metrics * 5 * C64;  // error row
    const int64_t M = (int64_t)kUaMom * C64;            // moments row
    const int64_t w0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t k = w0; k < a.P; k += nw) {
        const int64_t b = pstart[k], e = pstart[k + 1];  // wave-uniform
        if (e <= b || b / kUaRun == (e - 1) / kUaRun) continue;
        if (lane < 2) a.raw[2 * k + lane] = 0.0;
        for (int64_t i = lane; i < E; i += 64) a.err[k * E + i] = 0.0;
        for (int64_t i = lane; i < M; i += 64) a.mom[k * M + i] = 0.0;
    }
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

constexpr int kPgfB = 8;                                  // coefficients per block
constexpr int kPgfNB = (kUaMaxExact + kPgfB) / kPgfB;     // 13 blocks: 104 >= 101

// Range [i0, i1] of privacy-id counts whose keep probability is strictly
// between 0 and 1 (below i0 it is 0, above i1 exactly 1.0 in double).
__device__ __forceinline__ void ua_pi_range(const UaConfig &cf, int64_t &i0, int64_t &i1) {
    i0 = cf.pre_threshold > 0 ? cf.pre_threshold : 1;
    const int64_t sh = cf.pre_threshold > 0 ? cf.pre_threshold - 1 : 0;  // i -> i - pre + 1
    if (cf.strategy == DPG_SELECT_TRUNCATED_GEOMETRIC) {
        i1 = cf.table_len - 1 + sh;  // pi = 1.0 beyond the table
    } else if (cf.strategy == DPG_SELECT_LAPLACE_THRESHOLD) {
        // 0.5 exp(-x) < 2^-54 for x > 37.5
        i1 = (int64_t)ceil(cf.threshold + 37.5 * cf.scale) + sh;
    } else {
        // 0.5 erfc(-z / sqrt 2) rounds to 1.0 for z > 8.5
        i1 = (int64_t)ceil(cf.threshold + 8.5 * cf.scale) + sh;
    }
}

// The keep probability pi(i) of every selection class for i < npi, built in
// LDS once per wave ([i][class]): the dot products below read it instead of
// one dependent global table load per count (those loads bounded the
// kernel: 61 ms for 64 configurations over 1e6 partitions).
//
// LPC > 1 (at most 64 / LPC selection classes): the exact PMF depends on the
// class only (p = min(1, l0 / n_partitions)), so the wave computes one PMF
// per class, not per configuration: lane (class k, block l) holds
// coefficients [l CPL, (l + 1) CPL) of class k's PMF (the carry from the
// block below by one lane shuffle per pair), the dot with pi is summed over
// the class's LPC lanes and every configuration lane reads its class's
// value.  (Per configuration, the 104 coefficients held 208 VGPRs, one wave
// per SIMD.)
//
// kPart: 0 every partition; 1 the exact-PMF partitions only (<= 100 pairs,
// LPC > 1), with pi tabled for the 104 counts the PMF can reach (6.5 KB of
// LDS per wave at 8 classes instead of up to 32 KB: one partition per wave
// is latency-bound, so resident waves count); 2 the others (normal
// approximation, the full table).
template <int LPC, int kPart = 0>
__global__ __launch_bounds__(64) void k_ua_select(const ItemPA *pairs, const int64_t *pstart,
                                                  UaArgs a) {
    extern __shared__ __attribute__((aligned(16))) double spi[];
    constexpr int NCO = kPgfB * kPgfNB;
    constexpr int CPL = (NCO + LPC - 1) / LPC;
    static_assert(kPart != 1 || LPC > 1, "exact-only pass needs the class-shared PMF");
    __shared__ double s_inv[kUaMaxExact + 28];
    const int c = (int)__lane_id();
    const int64_t C64 = a.n_configs;
    const bool lane_on = c < a.n_configs;
    const UaConfig cf = a.cfg[lane_on ? c : 0];
    const int K = a.n_cls, NPI = kPart == 1 ? NCO : a.npi;
    for (int x = c; x < NPI * K; x += 64) {
        const int i = x / K, kc = x - i * K;
        spi[x] = ua_pi(a.cfg[a.cls_rep[kc]], a.tables, i);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int my_cls = a.cls[lane_on ? c : 0];
    const int my_sel = lane_on ? my_cls : -1;
    for (int64_t k = blockIdx.x; k < a.P; k += gridDim.x) {
        const int64_t b = pstart[k], n = pstart[k + 1] - b;
        if (n == 0 || (a.sample_mask && !bit_of(a.sample_mask, k))) continue;
        if constexpr (kPart == 1) if (n > kUaMaxExact) continue;
        if constexpr (kPart == 2) if (n <= kUaMaxExact) continue;
        double keep = 0.0;
        if constexpr (LPC > 1 && kPart != 2) if (n <= kUaMaxExact) {
            const int kc = c / LPC, l = c % LPC;
            const int kcs = kc < K ? kc : 0;
            const double mpc_k = a.cfg[a.cls_rep[kcs]].mpc;
            for (int x = c; x < n; x += 64) {
                const uint32_t np = pairs[b + x].npart;
                s_inv[x] = np > 0 ? 1.0 / (double)np : 0.0;
            }
            __syncthreads();
            double co[CPL];
#pragma unroll
            for (int t = 0; t < CPL; ++t) co[t] = (l == 0 && t == 0) ? 1.0 : 0.0;
            for (int64_t j = 0; j < n; ++j) {
                const double inv = s_inv[j];
                const double p = fmin(1.0, mpc_k * inv);
                const double q = 1.0 - p;
                double below = __shfl_up(co[CPL - 1], 1, 64);
                below = l == 0 ? 0.0 : below;
#pragma unroll
                for (int t = CPL - 1; t >= 1; --t) co[t] = co[t] * q + co[t - 1] * p;
                co[0] = co[0] * q + below * p;
            }
            double part = 0.0;
#pragma unroll
            for (int t = 0; t < CPL; ++t) {
                const int i = l * CPL + t;
                if (i <= n) part += co[t] * spi[i * K + kcs];
            }
#pragma unroll
            for (int o = LPC / 2; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
            keep = __shfl(part, (my_sel >= 0 ? my_sel : 0) * LPC, 64);
            __syncthreads();  // s_inv is rewritten by the next partition
            if (lane_on) a.keep[k * C64 + c] = keep;
            continue;
        }
        if constexpr (kPart == 1) continue;
        if (LPC == 1 && n <= kUaMaxExact) {
            // 1 / n_partitions of pairs lane and lane + 64, broadcast below
            const uint32_t n0 = pairs[b + min((int64_t)c, n - 1)].npart;
            const uint32_t n1 = pairs[b + min((int64_t)c + 64, n - 1)].npart;
            const long long r0 = __double_as_longlong(n0 > 0 ? 1.0 / (double)n0 : 0.0);
            const long long r1 = __double_as_longlong(n1 > 0 ? 1.0 / (double)n1 : 0.0);
            // exact PMF: coefficients of prod_j (1 - p_j + p_j x) in registers;
            // pair j touches coefficients 0..j+1 only, so blocks above that
            // are skipped (j is wave-uniform: uniform branches)
            double co[kPgfB * kPgfNB];
#pragma unroll
            for (int i = 0; i < kPgfB * kPgfNB; ++i) co[i] = i == 0 ? 1.0 : 0.0;
            for (int64_t j = 0; j < n; ++j) {
                const long long rb = j < 64 ? r0 : r1;
                const int jl = (int)(j & 63);
                const uint32_t lo32 = __builtin_amdgcn_readlane((uint32_t)rb, jl);
                const uint32_t hi32 = __builtin_amdgcn_readlane((uint32_t)(rb >> 32), jl);
                const double inv = __longlong_as_double((long long)(((uint64_t)hi32 << 32) | lo32));
                const double p = fmin(1.0, cf.mpc * inv);
                const double q = 1.0 - p;
                const int top = (int)j + 1;
#pragma unroll
                for (int bb = kPgfNB - 1; bb >= 0; --bb) {
                    if (bb * kPgfB > top) continue;
#pragma unroll
                    for (int t = kPgfB - 1; t >= 0; --t) {
                        const int i = bb * kPgfB + t;
                        if (i == 0) co[0] *= q;
                        else co[i] = co[i] * q + co[i - 1] * p;
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < kPgfB * kPgfNB; ++i)
                if (i <= n) keep += co[i] * spi[i * K + my_cls];
        } else {
            // refined normal approximation (poisson_binomial.py:61-83): its
            // PMF over [st, en] dotted with pi.  The moments and pi depend on
            // the selection class only, so each class is evaluated once with
            // the wave's lanes over the counts (lane = count, 64 at a time)
            // instead of once per configuration lane; counts with 0 < pi < 1
            // are evaluated one by one (below i0 pi is 0, above i1 it is 1
            // and the remaining mass telescopes to G(en) - G(i1)).
            // the moments of every class in one round of loads, lane kc
            // holding class kc's (one dependent load round per class before:
            // the pass is latency-bound, one partition per wave)
            double m0 = 0.0, m1 = 0.0, m2 = 0.0;
            if (c < K) {
                const double *mm = a.mom + k * kUaMom * C64 + a.cls_rep[c];
                m0 = mm[0];
                m1 = mm[C64];
                m2 = mm[2 * C64];
            }
            for (int kc = 0; kc < K; ++kc) {
                const int rc = a.cls_rep[kc];
                const UaConfig cr = a.cfg[rc];
                const double mean = __shfl(m0, kc, 64), sd = sqrt(__shfl(m1, kc, 64));
                const double m2k = __shfl(m2, kc, 64);
                double kp;
                auto pi_k = [&](int64_t i) {
                    return i < NPI ? spi[i * K + kc] : ua_pi(cr, a.tables, i);
                };
                if (sd == 0.0) {
                    kp = pi_k((int64_t)rint(mean));
                } else {
                    const double skew = m2k / (sd * sd * sd);
                    const int64_t st = (int64_t)fmax(0.0, floor(mean - 8.0 * sd));
                    const int64_t en = (int64_t)fmin((double)n, rint(mean + 8.0 * sd));
                    auto Gc = [&](int64_t i) {
                        return fmin(1.0, fmax(0.0, ua_G(((double)i + 0.5 - mean) / sd, skew)));
                    };
                    int64_t r0, r1;
                    ua_pi_range(cr, r0, r1);
                    const int64_t a0 = st > r0 ? st : r0;
                    const int64_t a1 = en < r1 ? en : r1;
                    double part = 0.0, carry = 0.0;
                    // points j = a0 - 1 .. a1: G(j); count j >= a0 adds
                    // (G(j) - G(j - 1)) pi(j)
                    for (int64_t j0 = a0 - 1; j0 <= a1; j0 += 64) {
                        const int64_t j = j0 + c;
                        const double g = j <= a1 ? Gc(j) : 0.0;
                        double gp = __shfl_up(g, 1, 64);
                        if (c == 0) gp = carry;
                        if (j >= a0 && j <= a1) part += (g - gp) * pi_k(j);
                        carry = __shfl(g, 63, 64);
                    }
#pragma unroll
                    for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
                    kp = a0 <= a1 ? part : 0.0;
                    if (en > r1) kp += Gc(en) - Gc(st > r1 ? st - 1 : r1);
                }
                if (my_sel == kc) keep = kp;
            }
        }
        if (lane_on) a.keep[k * C64 + c] = keep;
    }
}

// ---------------------------------------------------------------- report
// Cross-partition combine (cross_partition_combiners.py:264-343 and the
// size histogram of utility_analysis.py:182-251): per (size bucket,
// configuration) the sums of the CrossPartitionCombiner accumulator fields
//   [0] partitions, [1] weight (= keep probability), [2..3] partition info
//   (kept mean / variance, or non-empty / empty public partitions), then per
//   metric: sum, 3 data-drop terms, 10 absolute and 10 relative error terms
//   (weighted); the host divides by the weight and the metric sums.
__device__ __forceinline__ int ua_bucket_of(double n) {
    // index of the largest bound <= n (bounds 0, 1, 10, 20, 50, 100, ...)
    if (!(n >= 1.0)) return 0;
    int b = 1;
    double base = 10.0;
    for (int i = 0; i < 9; ++i, base *= 10.0) {
        if (n >= base) b = 2 + 3 * i;
        if (n >= 2.0 * base) b = 3 + 3 * i;
        if (n >= 5.0 * base) b = 4 + 3 * i;
    }
    return b;
}

__device__ __forceinline__ bool ua_in_output(const UaArgs &a, const int64_t *pstart, int64_t k) {
    if (a.public_mask) return bit_of(a.public_mask, k);
    return pstart[k + 1] > pstart[k] && !(a.sample_mask && !bit_of(a.sample_mask, k));
}

__global__ __launch_bounds__(256) void k_ua_bucket(const int64_t *pstart, UaArgs a) {
    __shared__ uint32_t h[kUaBuckets];
    if (threadIdx.x < kUaBuckets) h[threadIdx.x] = 0;
    __syncthreads();
    const int64_t C64 = a.n_configs;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < a.P;
         k += (int64_t)gridDim.x * blockDim.x) {
        int b = -1;
        if (ua_in_output(a, pstart, k)) {
            const double size = a.n_metrics ? a.err[k * a.n_metrics * 5 * C64] : a.raw[2 * k];
            b = ua_bucket_of(size);
            atomicAdd(&h[b], 1u);
        }
        a.bucket[k] = b;
    }
    __syncthreads();
    if (threadIdx.x < kUaBuckets && h[threadIdx.x]) atomicAdd(&a.bcount[threadIdx.x], h[threadIdx.x]);
}

// bcount holds each bucket's start: every output partition takes a slot of
// its bucket (one atomic per distinct bucket of a wave)
// Output partitions grouped by size bucket (k_ua_report sums each bucket's
// partitions): per block of kUaOrderPer x 256 partitions, bucket counts in
// LDS, one reservation per bucket per block, then the partitions written at
// their LDS-local offsets.  (One reservation per bucket per wave made ~16K
// waves contend for the few hot bucket counters: 1.2 ms at config 5.)
constexpr int kUaOrderPer = 8;
__global__ __launch_bounds__(256) void k_ua_order(UaArgs a) {
    __shared__ uint32_t cnt[kUaBuckets], base[kUaBuckets];
    const int64_t step = (int64_t)blockDim.x * kUaOrderPer;
    for (int64_t k0 = (int64_t)blockIdx.x * step; k0 < a.P; k0 += (int64_t)gridDim.x * step) {
        if (threadIdx.x < kUaBuckets) cnt[threadIdx.x] = 0;
        __syncthreads();
        int bk[kUaOrderPer];
        uint32_t rk[kUaOrderPer];
#pragma unroll
        for (int u = 0; u < kUaOrderPer; ++u) {
            const int64_t k = k0 + (int64_t)u * blockDim.x + threadIdx.x;
            bk[u] = k < a.P ? a.bucket[k] : -1;
            rk[u] = bk[u] >= 0 ? atomicAdd(&cnt[bk[u]], 1u) : 0u;
        }
        __syncthreads();
        if (threadIdx.x < kUaBuckets && cnt[threadIdx.x])
            base[threadIdx.x] = atomicAdd(&a.bcount[threadIdx.x], cnt[threadIdx.x]);
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kUaOrderPer; ++u)
            if (bk[u] >= 0) a.order[base[bk[u]] + rk[u]] = k0 + (int64_t)u * blockDim.x + threadIdx.x;
        __syncthreads();  // cnt / base are rewritten by the next round
    }
}

__global__ __launch_bounds__(64) void k_ua_report(int64_t K, UaArgs a) {
    const int64_t lo = (int64_t)blockIdx.x * kUaRepRun;
    if (lo >= K) return;
    const int64_t hi = lo + kUaRepRun < K ? lo + kUaRepRun : K;
    const int c = (int)__lane_id();
    const int C = a.n_configs;
    const int64_t C64 = C;
    const bool on = c < C;
    const int cc = on ? c : 0;
    const int M = a.n_metrics;
    const int F = 4 + 24 * M;
    double acc[kUaMaxF];
#pragma unroll
    for (int f = 0; f < kUaMaxF; ++f) acc[f] = 0.0;
    double s2[3];
#pragma unroll
    for (int m = 0; m < 3; ++m) s2[m] = m < M ? a.std[m * C64 + cc] * a.std[m * C64 + cc] : 0.0;
    int cur = a.bucket[a.order[lo]];
    auto flush = [&](int b) {
        if (!on) return;
        double *o = a.rep + (int64_t)b * F * C64 + c;
#pragma unroll
        for (int f = 0; f < kUaMaxF; ++f)
            if (f < F) atomicAdd(o + f * C64, acc[f]);
    };
    for (int64_t i = lo; i < hi; ++i) {
        const int64_t k = a.order[i];
        const int b = a.bucket[k];
        if (b != cur) {
            flush(cur);
#pragma unroll
            for (int f = 0; f < kUaMaxF; ++f) acc[f] = 0.0;
            cur = b;
        }
        const double p = a.public_mask ? 1.0 : a.keep[k * C64 + cc];
        acc[0] += 1.0;
        acc[1] += p;
        if (a.public_mask) {
            const double empty = a.raw[2 * k + 1] == 0.0 ? 1.0 : 0.0;
            acc[2] += 1.0 - empty;
            acc[3] += empty;
        } else {
            acc[2] += p;
            acc[3] += p * (1.0 - p);
        }
#pragma unroll
        for (int m = 0; m < 3; ++m) {
            if (m >= M) break;
            const double *e = a.err + (k * M + m) * 5 * C64 + cc;
            const double tot = e[0], cmin = e[C64], cmax = e[2 * C64], el0 = e[3 * C64],
                         vl0 = e[4 * C64];
            const double w = p;
            const double dl0 = -el0, dlinf = cmin - cmax;
            const double mean = el0 + cmin + cmax, var = vl0 + s2[m];
            const double rmse = sqrt(mean * mean + var);
            const double rwdp = p * rmse + (1.0 - p) * fabs(tot);
            const double ab[8] = {el0 * w, vl0 * w, cmin * w, cmax * w, mean * w, var * w,
                                  rmse * w, rwdp * w};
            const double inv = tot != 0.0 ? 1.0 / tot : 0.0;
            const double sc[8] = {inv, inv * inv, inv, inv, inv, inv * inv, inv, inv};
            double *q = acc + 4 + 24 * m;
            q[0] += tot;
            q[1] += dl0;
            q[2] += dlinf;
            q[3] += (tot - dl0 - dlinf) * (1.0 - p);
            // absolute errors (l1 terms stay 0), then relative ones
            const int ia[8] = {0, 1, 2, 3, 4, 5, 6, 8};
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                q[4 + ia[t]] += ab[t];
                q[14 + ia[t]] += ab[t] * sc[t];
            }
        }
    }
    flush(cur);
}

}  // namespace dpg
