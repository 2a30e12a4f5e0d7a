// dpg_select.h -- per-partition merge, private partition selection + noise,
// and compaction of the kept partitions (gfx950).
#pragma once

#include "dpg_common.h"
#include "dpg_partition.h"
#include "dpg_bound.h"

namespace dpg {

constexpr int kRangeBits = 12;  // 4096 partitions per LDS-resident range
constexpr int kRange = 1 << kRangeBits;

struct Partials {
    int64_t *rows;
    int64_t *count;
    double *sum;
    double *nsum;
    double *nsq;
};

// combine_accumulators_per_key (pipeline_backend.py:555-565): the kept pairs
// of one partition-key range are summed in LDS, then written to the dense
// partials: by plain coalesced stores of the whole range when this tile is
// the range's only one (full-line writes, no read of the zero-filled
// partials), by coalesced global atomics when a hot range spans several.
template <class Item>
__global__ __launch_bounds__(1024) void k_reduce_items(const Item *items, const TileDesc *tiles,
                                                       const uint32_t *ntiles,
                                                       const uint32_t *seg_ntiles, int64_t P,
                                                       Partials out) {
    constexpr bool kVar = ItemTraits<Item>::var;
    constexpr bool kSum = ItemTraits<Item>::sum;
    constexpr int kArr = kVar ? (kSum ? 3 : 2) : 1;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double *s_sum = reinterpret_cast<double *>(smem);
    double *s_nsum = s_sum + (kSum ? kRange : 0);
    double *s_nsq = s_nsum + kRange;
    // rows in the high word, records in the low one: one LDS atomic for both
    // (a device holds < 2^32 records, so neither word overflows)
    unsigned long long *s_rc = reinterpret_cast<unsigned long long *>(smem + kArr * kRange * 8);
    const uint32_t t = blockIdx.x;
    if (t >= *ntiles) return;
    const TileDesc td = tiles[t];
    const bool sole = seg_ntiles[td.seg] == 1;
    const int tid = threadIdx.x;
    for (int k = tid; k < kRange; k += 1024) {
        if (kSum) s_sum[k] = 0.0;
        if (kVar) {
            s_nsum[k] = 0.0;
            s_nsq[k] = 0.0;
        }
        s_rc[k] = 0;
    }
    __syncthreads();
    // kRU item loads per thread in flight before their LDS atomics (one
    // outstanding load per thread left the kernel latency-bound); items past
    // the tile end add nothing
    constexpr int kRU = sizeof(Item) <= 16 ? 8 : 4;
    for (int64_t i0 = td.begin; i0 < td.end; i0 += (int64_t)kRU * 1024) {
        Item it[kRU];
#pragma unroll
        for (int u = 0; u < kRU; ++u) it[u] = items[min(i0 + u * 1024 + tid, td.end - 1)];
#pragma unroll
        for (int u = 0; u < kRU; ++u) {
            if (i0 + u * 1024 + tid >= td.end) continue;
            const uint32_t k = it[u].pk & (kRange - 1);
            atomicAdd(&s_rc[k], (1ull << 32) | (unsigned long long)it[u].cnt);
            if constexpr (kSum)
                if (it[u].sum != 0.0) atomicAdd(&s_sum[k], it[u].sum);
            if constexpr (kVar) {
                if (it[u].nsum != 0.0) atomicAdd(&s_nsum[k], it[u].nsum);
                if (it[u].nsq != 0.0) atomicAdd(&s_nsq[k], it[u].nsq);
            }
        }
    }
    __syncthreads();
    const int64_t pk0 = (int64_t)td.seg << kRangeBits;
    for (int k = tid; k < kRange; k += 1024) {
        const int64_t pk = pk0 + k;
        if (pk >= P) break;
        const unsigned long long rc = s_rc[k];
        const int64_t rows = (int64_t)(rc >> 32), cnt = (int64_t)(rc & 0xFFFFFFFFull);
        if (sole) {
            out.rows[pk] = rows;
            out.count[pk] = cnt;
            if (kSum && out.sum) out.sum[pk] = s_sum[k];
            if constexpr (kVar) {
                if (out.nsum) out.nsum[pk] = s_nsum[k];
                if (out.nsq) out.nsq[pk] = s_nsq[k];
            }
            continue;
        }
        if (rows == 0) continue;
        atomicAdd((unsigned long long *)&out.rows[pk], (unsigned long long)rows);
        atomicAdd((unsigned long long *)&out.count[pk], (unsigned long long)cnt);
        if (kSum && out.sum) atomicAdd(&out.sum[pk], s_sum[k]);
        if constexpr (kVar) {
            if (out.nsum) atomicAdd(&out.nsum[pk], s_nsum[k]);
            if (out.nsq) atomicAdd(&out.nsq[pk], s_nsq[k]);
        }
    }
}

// Fallback merge for very large partition spaces: one global atomic per item.
template <class Item, class Src>
__global__ void k_reduce_items_direct(Src items, const uint32_t *n_items, Partials out) {
    constexpr bool kVar = ItemTraits<Item>::var;
    const uint32_t n = *n_items;
    Src src = items;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const Item it = src.fetch(i);
        atomicAdd((unsigned long long *)&out.rows[it.pk], 1ull);
        atomicAdd((unsigned long long *)&out.count[it.pk], (unsigned long long)it.cnt);
        if constexpr (ItemTraits<Item>::sum)
            if (out.sum) atomicAdd(&out.sum[it.pk], it.sum);
        if constexpr (kVar) {
            if (out.nsum) atomicAdd(&out.nsum[it.pk], it.nsum);
            if (out.nsq) atomicAdd(&out.nsq[it.pk], it.nsq);
        }
    }
}

struct SelectArgs {
    int strategy;
    int table_len;
    const double *table;  // device copy of the keep table (or null)
    double threshold, noise_scale;
    int64_t pre_threshold, max_rows;
    int64_t pk_offset, pk_stride;  // global pk of local partition k: pk_offset + k * pk_stride
    const uint8_t *public_mask;
};

struct NoiseArgs {
    int kind, family;
    uint32_t slot_mask;
    int n_out;
    int out_src[8];
    double scale[4];
    double mid;
    int mean_const, msq_const;
    double mean_const_value, msq_const_value;
};

__device__ __forceinline__ bool keep_partition(const SelectArgs &s, uint64_t seed, uint64_t gk,
                                               int64_t local, int64_t rows, const double *tab,
                                               const Gran &sg) {
    if (s.strategy == DPG_SELECT_NONE)
        return s.public_mask ? ((s.public_mask[local >> 3] >> (local & 7)) & 1) : true;
    if (rows <= 0) return false;  // partitions absent from the data
    int64_t n = (rows + s.max_rows - 1) / s.max_rows;  // dp_engine.py:334-343
    if (s.pre_threshold > 0) {
        if (n < s.pre_threshold) return false;
        n = n - s.pre_threshold + 1;
    }
    uint32_t u[4];
    select_uniforms(seed, gk, u);
    if (s.strategy == DPG_SELECT_TRUNCATED_GEOMETRIC) {
        double pr = n < s.table_len ? tab[n] : 1.0;
        return u53(u[0], u[1]) < pr;
    }
    if (s.strategy == DPG_SELECT_LAPLACE_THRESHOLD)
        return laplace_noise((double)n, s.noise_scale, u, sg) > s.threshold;
    return gaussian_noise((double)n, s.noise_scale, u, sg) > s.threshold;
}

// _select_private_partitions_internal (dp_engine.py:305-361) fused with
// CompoundCombiner.compute_metrics (combiners.py:708-730).
__global__ __launch_bounds__(256) void k_select_noise(const int64_t *rows, const int64_t *count,
                                                      const double *sum, const double *nsum,
                                                      const double *nsq, int64_t P,
                                                      SelectArgs s, NoiseArgs z, uint64_t seed,
                                                      uint8_t *keep, double *out) {
    extern __shared__ __attribute__((aligned(16))) double s_tab[];
    const bool lds_tab = s.table != nullptr && s.table_len <= 4096;
    if (lds_tab) {
        for (int i = threadIdx.x; i < s.table_len; i += blockDim.x) s_tab[i] = s.table[i];
        __syncthreads();
    }
    const double *tab = lds_tab ? s_tab : s.table;
    // lattices of the selection noise and of each metric slot, per thread
    const Gran sg = gran_of(s.noise_scale);
    Gran G[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) G[q] = gran_of(z.scale[q]);
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < P;
         k += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t gk = (uint64_t)(s.pk_offset + k * s.pk_stride);
        const int64_t r = rows[k];
        const bool kp = keep_partition(s, seed, gk, k, r, tab, sg);
        keep[k] = kp ? 1 : 0;
        double *o = out + k * z.n_out;
        if (!kp) {
            for (int j = 0; j < z.n_out; ++j) o[j] = 0.0;
            continue;
        }
        const double cnt = (double)count[k];
        double V[5] = {0, 0, 0, 0, 0};
        const int kind = z.kind;
        if (z.family == DPG_FAMILY_VARIANCE) {
            // dp_computations.py:307-366
            double dc = add_noise(kind, cnt, z.scale[DPG_SLOT_COUNT], G[DPG_SLOT_COUNT], seed, gk,
                                  DPG_SLOT_COUNT);
            double den = dc > 1.0 ? dc : 1.0;
            double mean = z.mean_const ? z.mean_const_value
                                       : add_noise(kind, nsum ? nsum[k] : 0.0,
                                                   z.scale[DPG_SLOT_SUM], G[DPG_SLOT_SUM], seed, gk,
                                                   DPG_SLOT_SUM) / den;
            double msq = z.msq_const ? z.msq_const_value
                                     : add_noise(kind, nsq ? nsq[k] : 0.0, z.scale[DPG_SLOT_NSQ],
                                                 G[DPG_SLOT_NSQ], seed, gk, DPG_SLOT_NSQ) / den;
            double var = msq - mean * mean;
            if (!z.mean_const) mean += z.mid;
            V[DPG_V_VARIANCE] = var;
            V[DPG_V_COUNT] = dc;
            V[DPG_V_SUM] = mean * dc;
            V[DPG_V_MEAN] = mean;
        } else if (z.family == DPG_FAMILY_MEAN) {
            // dp_computations.py:563-569
            double dc = add_noise(kind, cnt, z.scale[DPG_SLOT_COUNT], G[DPG_SLOT_COUNT], seed, gk,
                                  DPG_SLOT_COUNT);
            double dn = add_noise(kind, nsum ? nsum[k] : 0.0, z.scale[DPG_SLOT_SUM], G[DPG_SLOT_SUM],
                                  seed, gk, DPG_SLOT_SUM);
            double mean = z.mid + dn / (dc > 1.0 ? dc : 1.0);
            V[DPG_V_COUNT] = dc;
            V[DPG_V_SUM] = mean * dc;
            V[DPG_V_MEAN] = mean;
        } else {
            if (z.slot_mask & (1u << DPG_SLOT_COUNT))
                V[DPG_V_COUNT] =
                    add_noise(kind, cnt, z.scale[DPG_SLOT_COUNT], G[DPG_SLOT_COUNT], seed, gk,
                              DPG_SLOT_COUNT);
            if (z.slot_mask & (1u << DPG_SLOT_SUM))
                V[DPG_V_SUM] = add_noise(kind, sum ? sum[k] : 0.0, z.scale[DPG_SLOT_SUM],
                                         G[DPG_SLOT_SUM], seed, gk, DPG_SLOT_SUM);
        }
        if (z.slot_mask & (1u << DPG_SLOT_PID))
            V[DPG_V_PRIVACY_ID_COUNT] =
                add_noise(kind, (double)r, z.scale[DPG_SLOT_PID], G[DPG_SLOT_PID], seed, gk,
                          DPG_SLOT_PID);
        for (int j = 0; j < z.n_out; ++j) o[j] = V[z.out_src[j]];
    }
}

// --------------------------------------------------------- compaction
constexpr int kCompactThreads = 1024;
constexpr int kCompactPerBlock = 8192;

__global__ __launch_bounds__(kCompactThreads) void k_compact_count(const uint8_t *keep, int64_t P,
                                                                   uint32_t *block_cnt) {
    __shared__ uint32_t sh[16];
    const int64_t b0 = (int64_t)blockIdx.x * kCompactPerBlock;
    uint32_t c = 0;
    for (int j = 0; j < kCompactPerBlock / kCompactThreads; ++j) {
        int64_t k = b0 + j * kCompactThreads + threadIdx.x;
        if (k < P) c += keep[k];
    }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int k = 0; k < 16; ++k) t += sh[k];
        block_cnt[blockIdx.x] = t;
    }
}

// single block: exclusive scan of block counts (nb may exceed 1024)
__global__ __launch_bounds__(1024) void k_compact_scan(uint32_t *block_cnt, uint32_t nb,
                                                       int64_t *total) {
    __shared__ uint32_t sh[16];
    uint32_t carry = 0;
    for (uint32_t b = 0; b < nb; b += 1024) {
        uint32_t i = b + threadIdx.x;
        uint32_t x = i < nb ? block_cnt[i] : 0u;
        uint32_t tot;
        uint32_t e = block_excl_scan_1024(x, sh, tot);
        if (i < nb) block_cnt[i] = carry + e;
        carry += tot;
    }
    if (threadIdx.x == 0) *total = carry;
}

__global__ __launch_bounds__(kCompactThreads) void k_compact_write(
    const uint8_t *keep, const double *out, int64_t P, int n_out, const uint32_t *block_off,
    int64_t *kept_ids, double *kept_out) {
    __shared__ uint32_t sh[16];
    const int64_t b0 = (int64_t)blockIdx.x * kCompactPerBlock;
    uint32_t run = block_off[blockIdx.x];
    for (int j = 0; j < kCompactPerBlock / kCompactThreads; ++j) {
        int64_t k = b0 + j * kCompactThreads + threadIdx.x;
        uint32_t f = k < P ? keep[k] : 0u;
        uint32_t tot;
        uint32_t e = block_excl_scan_1024(f, sh, tot);
        if (f) {
            int64_t dst = run + e;
            kept_ids[dst] = k;
            for (int c = 0; c < n_out; ++c) kept_out[dst * n_out + c] = out[k * n_out + c];
        }
        run += tot;
    }
}

}  // namespace dpg
