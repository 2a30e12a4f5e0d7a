// dpg_hist.h -- dataset contribution histograms over the per-(privacy id,
// partition) pre-aggregate (gfx950).
//
// Reference: pipeline_dp/dataset_histograms/computing_histograms.py
//   compute_dataset_histograms (:420-474) and its helpers (:237-417):
//   L0 (partitions per privacy id), L1 (records per privacy id), LINF
//   (records per pair), LINF_SUM (value sum per pair, 10^4 equal bins between
//   the min and max sum, :314-362), COUNT_PER_PARTITION (records per
//   partition), PRIVACY_ID_PER_PARTITION (pairs per partition); integer bins
//   keep 3 significant digits (_to_bin_lower_upper_logarithmic, :28-47);
//   compute_dataset_histograms_on_preaggregated_data (:482-684) weights L0 /
//   L1 by 1 / n_partitions and rounds per value (:81-102).
//
// Input: the pre-aggregate of dpg_preaggregate, sorted by partition key, one
// entry per pair: (pk, count, sum, n_partitions, n_contributions, leader)
// where `leader` (bit 31 of the record count) marks one pair per privacy id -- so the per-pid
// histograms count every privacy id once without a pass keyed by pid.
//
// Integer bins: index v for v < 1000 (width 1), else 1000 + 900 e + (m - 100)
// for v = m.xxx * 10^(e+1), m in [100, 999] (3 significant digits).  Values
// < 1000 (almost all of them) are counted in LDS per workgroup -- a width-1
// bin's sum and max follow from its count -- the rest go to global atomics.
// All of it is HBM-bound streaming over 32-byte pairs.
#pragma once

#include "dpg_common.h"

namespace dpg {

constexpr int kHiExact = 1000;                  // width-1 bins
constexpr int kHiBins = kHiExact + 17 * 900;    // every uint64 value (<= 20 digits)
constexpr int kHsBins = 10000;                  // NUMBER_OF_BUCKETS_IN_LINF_SUM_...
constexpr int kHiTypes = 5;                     // L0, L1, LINF, COUNT_PP, PID_PP
constexpr int kHistThreads = 256;

struct HistArgs {
    unsigned long long *ib;       // [kHiTypes][kHiBins][3]: count, sum, max
    unsigned int *pcount;         // [P] records per partition
    unsigned long long *minmax;   // [2] ordered keys of the min / max pair sum
    double *lowers;               // [kHsBins + 1]
    unsigned long long *scount;   // [kHsBins]
    double *ssum;                 // [kHsBins]
    unsigned long long *smax;     // [kHsBins] ordered keys
    double *w0, *w1;              // pre-aggregated mode: weight per exact value
    int64_t wlen0, wlen1;
};

__device__ __forceinline__ uint32_t int_bin(uint64_t v) {
    if (v < (uint64_t)kHiExact) return (uint32_t)v;
    uint64_t p = 10;  // v in [100 p, 1000 p)
    uint32_t e = 0;
    while (e < 16 && v / p >= 1000) p *= 10, ++e;
    return (uint32_t)kHiExact + 900u * e + (uint32_t)(v / p) - 100u;
}

// order-preserving key of a double (unsigned comparison = numeric order)
__device__ __forceinline__ unsigned long long dkey(double x) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(x);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double dkey_inv(unsigned long long k) {
    const unsigned long long b = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
    return __longlong_as_double((long long)b);
}

// one value of integer histogram t: LDS counter when < 1000, else global
__device__ __forceinline__ void hi_add(unsigned int *small, const HistArgs &a, int t, uint64_t v,
                                       uint64_t times = 1) {
    if (v < (uint64_t)kHiExact) {
        atomicAdd(&small[v], (unsigned int)times);
        return;
    }
    unsigned long long *g = a.ib + ((size_t)t * kHiBins + int_bin(v)) * 3;
    atomicAdd(&g[0], (unsigned long long)times);
    atomicAdd(&g[1], (unsigned long long)(v * times));
    if (g[2] < v) atomicMax(&g[2], (unsigned long long)v);
}

__device__ __forceinline__ void hi_flush(const unsigned int *small, const HistArgs &a, int t) {
    for (int v = threadIdx.x; v < kHiExact; v += blockDim.x) {
        const unsigned int c = small[v];
        if (!c) continue;
        unsigned long long *g = a.ib + ((size_t)t * kHiBins + v) * 3;
        atomicAdd(&g[0], (unsigned long long)c);
        atomicAdd(&g[1], (unsigned long long)c * (unsigned long long)v);
        if (g[2] < (unsigned long long)v) atomicMax(&g[2], (unsigned long long)v);
    }
}

// Pass over the pairs: LINF per pair, L0 / L1 per leader pair, min / max of
// the pair sums, records per partition (a segmented wave scan over the
// pk-sorted pairs: one atomic per partition run of a wave).
template <bool kWeighted>
__global__ __launch_bounds__(kHistThreads) void k_hist_pairs(const ItemPA *pairs, int64_t n,
                                                             HistArgs a) {
    __shared__ unsigned int small[3][kHiExact];
    for (int i = threadIdx.x; i < 3 * kHiExact; i += kHistThreads) (&small[0][0])[i] = 0;
    __syncthreads();
    const uint32_t lane = __lane_id();
    double lo = HUGE_VAL, hi = -HUGE_VAL;
    const int64_t stride = (int64_t)gridDim.x * kHistThreads;
    for (int64_t b = (int64_t)blockIdx.x * kHistThreads; b < n; b += stride) {
        const int64_t i = b + threadIdx.x;
        const bool on = i < n;
        ItemPA e;
        if (on) e = pairs[i];
        const uint32_t pk = on ? e.pk : 0xFFFFFFFFu;
        uint32_t s = on ? e.cnt : 0u;
        if (on) {
            hi_add(small[2], a, 2, e.cnt);
            if constexpr (kWeighted) {
                // per exact value: sum of 1 / n_partitions (rounded later)
                if (e.npart > 0) {
                    const double w = 1.0 / (double)e.npart;
                    atomicAdd(&a.w0[e.npart], w);
                    atomicAdd(&a.w1[e.ncontrib()], w);
                }
            } else if (e.leader()) {
                hi_add(small[0], a, 0, e.npart);
                hi_add(small[1], a, 1, e.ncontrib());
            }
            lo = fmin(lo, e.sum);
            hi = fmax(hi, e.sum);
        }
        // segmented inclusive scan of the counts by partition (sorted: equal
        // pk at lane - d means the whole span is one partition)
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = __shfl_up(s, d);
            const uint32_t opk = __shfl_up(pk, d);
            if ((int)lane >= d && opk == pk) s += o;
        }
        const uint32_t npk = __shfl_down(pk, 1);
        if (on && (lane == 63 || npk != pk)) atomicAdd(&a.pcount[pk], s);
    }
    // block min / max of the pair sums, then one atomic each
    __shared__ unsigned long long red[2];
    if (threadIdx.x == 0) red[0] = ~0ull, red[1] = 0ull;
    __syncthreads();
    if (lo <= hi) {
        atomicMin(&red[0], dkey(lo));
        atomicMax(&red[1], dkey(hi));
    }
    __syncthreads();
    if (threadIdx.x == 0 && red[0] != ~0ull) {
        atomicMin(&a.minmax[0], red[0]);
        atomicMax(&a.minmax[1], red[1]);
    }
    if constexpr (!kWeighted) {
        hi_flush(small[0], a, 0);
        hi_flush(small[1], a, 1);
    }
    hi_flush(small[2], a, 2);
}

// largest n_partitions / n_contributions of the pairs (pre-aggregated mode)
__global__ __launch_bounds__(kHistThreads) void k_pa_max(const ItemPA *pairs, int64_t n,
                                                         uint32_t *mx) {
    uint32_t a = 0, b = 0;
    for (int64_t i = (int64_t)blockIdx.x * kHistThreads + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * kHistThreads) {
        a = max(a, pairs[i].npart);
        b = max(b, pairs[i].ncontrib());
    }
    if (a) atomicMax(&mx[0], a);
    if (b) atomicMax(&mx[1], b);
}

// Pre-aggregated mode: the rounded weight of every exact value is its
// frequency; a value whose weight rounds to 0 still opens its bin (max).
__global__ __launch_bounds__(kHistThreads) void k_hist_weights(HistArgs a) {
    __shared__ unsigned int small[2][kHiExact];
    for (int i = threadIdx.x; i < 2 * kHiExact; i += kHistThreads) (&small[0][0])[i] = 0;
    __syncthreads();
    for (int t = 0; t < 2; ++t) {
        const double *w = t ? a.w1 : a.w0;
        const int64_t len = t ? a.wlen1 : a.wlen0;
        for (int64_t v = (int64_t)blockIdx.x * kHistThreads + threadIdx.x; v < len;
             v += (int64_t)gridDim.x * kHistThreads) {
            const double x = w[v];
            if (!(x > 0.0)) continue;
            const uint64_t c = (uint64_t)rint(x);  // Python round(): half to even
            unsigned long long *g = a.ib + ((size_t)t * kHiBins + int_bin((uint64_t)v)) * 3;
            if (c) {
                if (v < kHiExact) atomicAdd(&small[t][v], (unsigned int)c);
                else {
                    atomicAdd(&g[0], (unsigned long long)c);
                    atomicAdd(&g[1], (unsigned long long)(c * (uint64_t)v));
                }
            }
            atomicMax(&g[2], (unsigned long long)v);
        }
    }
    __syncthreads();
    for (int t = 0; t < 2; ++t)
        for (int v = threadIdx.x; v < kHiExact; v += kHistThreads) {
            const unsigned int c = small[t][v];
            if (!c) continue;
            unsigned long long *g = a.ib + ((size_t)t * kHiBins + v) * 3;
            atomicAdd(&g[0], (unsigned long long)c);
            atomicAdd(&g[1], (unsigned long long)c * (unsigned long long)v);
        }
}

// Pass over the partitions: COUNT_PER_PARTITION (records) and
// PRIVACY_ID_PER_PARTITION (pairs) of every partition with pairs.
__global__ __launch_bounds__(kHistThreads) void k_hist_parts(const int64_t *pstart, int64_t P,
                                                             HistArgs a) {
    __shared__ unsigned int small[2][kHiExact];
    for (int i = threadIdx.x; i < 2 * kHiExact; i += kHistThreads) (&small[0][0])[i] = 0;
    __syncthreads();
    for (int64_t k = (int64_t)blockIdx.x * kHistThreads + threadIdx.x; k < P;
         k += (int64_t)gridDim.x * kHistThreads) {
        const int64_t np = pstart[k + 1] - pstart[k];
        if (np <= 0) continue;
        hi_add(small[0], a, 3, a.pcount[k]);
        hi_add(small[1], a, 4, (uint64_t)np);
    }
    __syncthreads();
    hi_flush(small[0], a, 3);
    hi_flush(small[1], a, 4);
}

// np.linspace(min, max, kHsBins + 1) bit for bit: y = i * step + start in two
// roundings (no contraction), the zero-step branch (i / div) * delta, and the
// last entry = stop (numpy/_core/function_base.py).
__global__ __launch_bounds__(kHistThreads) void k_hist_lowers(HistArgs a) {
    // HIP contracts x * y + z into one FMA by default (one rounding, not
    // numpy's two); plain operators under contract(off) -- the __d*_rn
    // intrinsics carry the header's contraction flags into this function
#pragma clang fp contract(off)
    const double start = dkey_inv(a.minmax[0]), stop = dkey_inv(a.minmax[1]);
    const double div = (double)kHsBins;
    const double delta = stop - start;
    const double step = delta / div;
    for (int i = blockIdx.x * kHistThreads + threadIdx.x; i <= kHsBins;
         i += gridDim.x * kHistThreads) {
        double y;
        if (i == kHsBins) {
            y = stop;
        } else if (step == 0.0) {
            const double t = (double)i / div;
            y = t * delta;
            y = y + start;
        } else {
            y = (double)i * step;
            y = y + start;
        }
        a.lowers[i] = y;
    }
}

// LINF_SUM: bisect_right(lowers, v) - 1, v == lowers[-1] in the last bin
// (_bin_lower_index, computing_histograms.py:50-59): a guess from the step,
// corrected against the exact lowers; counts and sums in LDS (120 KB), the
// max by a filtered global atomic.
__global__ __launch_bounds__(1024) void k_hist_sums(const ItemPA *pairs, int64_t n, HistArgs a) {
    extern __shared__ char hs_smem[];
    unsigned int *cnt = reinterpret_cast<unsigned int *>(hs_smem);
    double *sum = reinterpret_cast<double *>(hs_smem + 4 * kHsBins);
    for (int i = threadIdx.x; i < kHsBins; i += 1024) cnt[i] = 0, sum[i] = 0.0;
    __syncthreads();
    const double lo = a.lowers[0], top = a.lowers[kHsBins];
    const double step = (top - lo) / (double)kHsBins;
    for (int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * 1024) {
        const double v = pairs[i].sum;
        int b;
        if (v == top) {
            b = kHsBins - 1;
        } else {
            const double g = step > 0.0 ? (v - lo) / step : 0.0;
            b = g <= 0.0 ? 0 : (g >= (double)(kHsBins - 1) ? kHsBins - 1 : (int)g);
            while (b < kHsBins - 1 && a.lowers[b + 1] <= v) ++b;
            while (b > 0 && a.lowers[b] > v) --b;
        }
        atomicAdd(&cnt[b], 1u);
        atomicAdd(&sum[b], v);
        const unsigned long long k = dkey(v);
        if (a.smax[b] < k) atomicMax(&a.smax[b], k);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kHsBins; i += 1024) {
        if (!cnt[i]) continue;
        atomicAdd(&a.scount[i], (unsigned long long)cnt[i]);
        atomicAdd(&a.ssum[i], sum[i]);
    }
}

// ordered max keys -> doubles (in place)
__global__ __launch_bounds__(kHistThreads) void k_hist_finish(HistArgs a) {
    for (int i = blockIdx.x * kHistThreads + threadIdx.x; i < kHsBins; i += gridDim.x * kHistThreads) {
        const unsigned long long k = a.smax[i];
        reinterpret_cast<double *>(a.smax)[i] = k ? dkey_inv(k) : 0.0;
    }
}

}  // namespace dpg
