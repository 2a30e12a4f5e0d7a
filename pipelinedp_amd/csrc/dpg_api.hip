// dpg_api.hip -- C ABI + host orchestration of the MI355X DPEngine.aggregate
// hot path.  Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC.
//
// Pipeline of dpg_bound_aggregate (DESIGN.md "Kernels"):
//   [pid range reduction when the caller does not declare it]
//   level 1: SoA (pid, pk) -> packed records (key residual, record index),
//            bucketed by the top b1 <= 11 bits of hk(pid)
//   level 2: records -> buckets by the next b2 <= 11 hash bits (~512 records)
//   -> k_make_chunks (greedy packing of fine buckets into <= 1024-record
//      chunks), refine level for oversize buckets -> k_bound_chunks
//      (+ k_bound_big for single buckets still over the chunk capacity)
//   -> one partition-key-range level over the kept pairs -> k_reduce_items
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // types and enums only: the functions are resolved by dlsym

#include <algorithm>
#include <cstddef>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

// Occupancy and the dynamic-LDS attribute are fixed per (device, kernel,
// block size, LDS): looked up and set once per process.  A release makes
// ~10 of these calls, several right after a host synchronisation, where
// host time is GPU idle time.
static hipError_t occ_query(int *blocks, const void *kern, int threads, size_t lds) {
    static std::mutex mu;
    static std::map<std::tuple<int, const void *, int, size_t>, int> cache;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> g(mu);
    const auto key = std::make_tuple(dev, kern, threads, lds);
    const auto it = cache.find(key);
    if (it != cache.end()) {
        *blocks = it->second;
        return hipSuccess;
    }
    const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, kern, threads, lds);
    if (e == hipSuccess) cache[key] = *blocks;
    return e;
}
static hipError_t set_func_attr(const void *kern, hipFuncAttribute attr, int value) {
    if (attr != hipFuncAttributeMaxDynamicSharedMemorySize) return hipFuncSetAttribute(kern, attr, value);
    static std::mutex mu;
    static std::map<std::pair<int, const void *>, int> done;  // largest value set
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> g(mu);
    const auto key = std::make_pair(dev, kern);
    const auto it = done.find(key);
    if (it != done.end() && it->second >= value) return hipSuccess;
    const hipError_t e = hipFuncSetAttribute(kern, attr, value);
    if (e == hipSuccess) done[key] = value;
    return e;
}

#include "dpg_bound.h"
#include "dpg_chunk.h"
#include "dpg_common.h"
#include "dpg_hist.h"
#include "dpg_partition.h"
#include "dpg_select.h"
#include "dpg_sortb.h"
#include "dpg_sortmw.h"
#include "dpg_team.h"
#include "dpg_utility.h"
#include "dpg_wave.h"

using namespace dpg;

namespace {

constexpr uint32_t kBucketTarget = 256;  // average records per fine bucket
// level 2 (records) may take 12 bits (4096 digits: its scatter stages fewer
// records per sub-tile); refine and item levels keep <= 11
constexpr uint32_t kMaxB1 = 11, kMaxB2 = 12, kMaxBR = 11;
// 23-bit plans of 8-byte records (N > 2^30): level 1 takes 12 bits so that
// level 2 (11 bits) runs by teams (dpg_team.h handles <= 2048 digits); the
// record then also drops one more stored hash bit, which keeps N up to 2^31
// in 8-byte records (config 3's 2e9-record shards)
constexpr uint32_t kMaxB1W = 12;
// records per thread of the 4096-digit level-1 scatters (LDS: the digit
// arrays take 48 KB + 16 KB of bases)
constexpr int kIptL1W = 8;
// pinned host words: up to 4096 level-1 bucket totals, then the error word
constexpr uint32_t kPinErr = 4096;
constexpr uint32_t kChunkGroup = 32;     // fine buckets per packing thread
// Status of bound_and_reduce when a team level-2 barrier timed out (err bit
// 8): the caller redoes level 2 with the histogram path.
constexpr int kRedoLevel2 = -100;
#ifndef DPG_PC_HALF
#define DPG_PC_HALF 0
#endif
#ifndef DPG_IPT_PC
// records per thread of the histogram-free level 1: an even count, so that
// the key columns load two records per 16-byte load (SrcSoAKey::fetch2);
// same-box A/B at config 2: 9 records by 8-byte loads 6.38-6.40 ms, 8 by
// pairs 5.97-5.99 (profiles/r6/r6w_pairs/); 10 exceeds the scatter's LDS
#define DPG_IPT_PC 8
#endif

struct Buf {
    void *p = nullptr;
    size_t bytes = 0;
};

struct Control {  // device-side counters, zeroed per call
    uint32_t err;
    uint32_t item_cursor;
    uint32_t ntiles[8];
    int64_t n_scalar;
    uint32_t n_chunks;
    uint32_t n_over;   // fine buckets over the chunk capacity
    uint32_t n_over2;  // refined buckets still over it
    uint32_t n_mchunks;  // single-bucket chunks above the small-chunk capacity
    uint32_t heavy_nfb;  // heavy buckets handed back to k_bound_big
    uint32_t pad_;
    unsigned long long over_records;
    unsigned long long over2_records;
    unsigned long long pid_lo, pid_hi;  // order-preserving (x ^ 2^63) min / max
};

}  // namespace

struct dpg_ctx {
    int device = 0;
    uint64_t seed = 0;
    int n_cu = 256;
    std::string err;
    std::map<std::string, Buf> bufs;
    std::vector<std::string> stage_names;
    std::vector<hipEvent_t> events;
    int n_events_used = 0;
    hipStream_t last_stream = nullptr;
    uint32_t bucket_target = 0;  // 0: kBucketTarget
    uint32_t bucket_cap = kBCap;
    void *comm = nullptr;        // ncclComm_t (dpg_ctx_create_comm)
    // device flags of the last dpg_bound_aggregate (its internal-error bit is
    // read at the next synchronising call, dpg_compact_kept)
    const uint32_t *last_err = nullptr;
    int rank = 0, nranks = 1;
    // pinned staging arena for host -> device uploads (see upload()): one
    // completion event per stream that has uploaded through it
    char *stage_buf = nullptr;
    size_t stage_cap = 0, stage_head = 0;
    std::map<hipStream_t, hipEvent_t> stage_done;
    // level-1 bucket counts copied to the host while the level-1 scatter
    // runs (the team level-2 decision, see pipeline())
    uint32_t *pin_tot = nullptr;
    hipEvent_t tot_ev = nullptr;
    // a team level-2 barrier timed out on this context (workgroups not
    // co-resident: other work shares the GPU): the next team_backoff calls
    // take the histogram level 2 directly instead of paying the timeout
    // again (stage "team_backoff" marks them); then the team path is tried
    // again.  Each further timeout doubles the back-off (64 .. 4096 calls).
    uint32_t team_backoff = 0;
    uint32_t team_backoff_next = 64;
};

namespace {

// Debug watchdog (env DPG_WATCHDOG_S=<seconds>): instead of blocking, poll
// the stream; on timeout print each workgroup's last phase and abort.
// Debug builds only (-DDPG_WATCHDOG or the timing build): the product
// kernels do not record their phases.
int watchdog_seconds() {
#if defined(DPG_WATCHDOG) || defined(DPG_PHASE_TIMING)
    const char *e = std::getenv("DPG_WATCHDOG_S");
    return e ? std::atoi(e) : 0;
#else
    return 0;
#endif
}

uint32_t *watchdog_buffer(size_t n) {
    static uint32_t *buf = nullptr;
    static size_t cap = 0;
    if (n > cap) {
        if (buf) (void)hipHostFree(buf);
        if (hipHostMalloc((void **)&buf, n * 4, hipHostMallocCoherent) != hipSuccess) return nullptr;
        cap = n;
    }
    std::memset(buf, 0, n * 4);
    return buf;
}

void watchdog_wait(hipStream_t s, const uint32_t *prog, size_t n, const char *what) {
    int secs = watchdog_seconds();
    for (int i = 0; i < secs * 100; ++i) {
        if (hipStreamQuery(s) == hipSuccess) return;
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
    std::fprintf(stderr, "[dpg watchdog] %s did not finish in %d s; phases:", what, secs);
    for (size_t i = 0; i < n; ++i) std::fprintf(stderr, " %u", prog[i]);
    std::fprintf(stderr, "\n");
    std::fflush(stderr);
    std::abort();
}

int fail(dpg_ctx *c, int code, const std::string &msg) {
    if (c) c->err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                     \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess)                                                             \
            return fail(ctx, DPG_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

#define LAUNCH_CHECK()                                                                        \
    do {                                                                                      \
        hipError_t e_ = hipGetLastError();                                                    \
        if (e_ != hipSuccess)                                                                 \
            return fail(ctx, DPG_ERR_HIP, std::string("kernel launch: ") + hipGetErrorString(e_)); \
    } while (0)

void *ws(dpg_ctx *ctx, const char *name, size_t bytes, int *status) {
    Buf &b = ctx->bufs[name];
    if (b.bytes >= bytes && b.p) return b.p;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
    size_t want = std::max<size_t>(bytes, 256);
    if (hipMalloc(&b.p, want) != hipSuccess) {
        (void)hipGetLastError();
        *status = fail(ctx, DPG_ERR_OOM, std::string("out of device memory allocating ") + name +
                                             " (" + std::to_string(want) + " bytes)");
        return nullptr;
    }
    b.bytes = want;
    return b.p;
}

// Host -> device upload of `bytes` from any host memory (stack arrays,
// temporaries, caller buffers): the bytes are copied into a pinned arena
// owned by the context and DMA'd from there, stream-ordered, so the source
// may die as soon as this returns and the copy never stages pageable memory.
// The arena is reused round-robin; when it wraps, the host waits for the
// uploads already queued on EVERY stream that has used it (rare: 4 MB, grown
// on demand), so a copy still queued on another stream never reads bytes
// that are being overwritten.
int upload(dpg_ctx *ctx, void *dst, const void *src, size_t bytes, hipStream_t s) {
    if (bytes == 0) return DPG_OK;
    const size_t need = (bytes + 255) & ~(size_t)255;
    hipEvent_t &done = ctx->stage_done[s];
    if (!done && hipEventCreateWithFlags(&done, hipEventDisableTiming) != hipSuccess) {
        ctx->stage_done.erase(s);
        return fail(ctx, DPG_ERR_HIP, "hipEventCreate (upload arena)");
    }
    if (need > ctx->stage_cap || ctx->stage_head + need > ctx->stage_cap) {
        // every queued upload must have left the arena before it is reused
        if (ctx->stage_buf)
            for (auto &kv : ctx->stage_done)
                if (hipEventSynchronize(kv.second) != hipSuccess)
                    return fail(ctx, DPG_ERR_HIP, "hipEventSynchronize (upload arena)");
        ctx->stage_head = 0;
        if (need > ctx->stage_cap) {
            if (ctx->stage_buf) (void)hipHostFree(ctx->stage_buf);
            ctx->stage_buf = nullptr;
            const size_t cap = std::max<size_t>(need, (size_t)4 << 20);
            if (hipHostMalloc((void **)&ctx->stage_buf, cap, hipHostMallocDefault) != hipSuccess) {
                ctx->stage_cap = 0;
                return fail(ctx, DPG_ERR_OOM, "pinned upload arena");
            }
            ctx->stage_cap = cap;
        }
    }
    char *p = ctx->stage_buf + ctx->stage_head;
    std::memcpy(p, src, bytes);
    ctx->stage_head += need;
    if (hipMemcpyAsync(dst, p, bytes, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipEventRecord(done, s) != hipSuccess)
        return fail(ctx, DPG_ERR_HIP, "upload");
    return DPG_OK;
}

#define UPLOAD(dst, src, bytes)                                  \
    do {                                                          \
        const int r_ = upload(ctx, (dst), (src), (bytes), s);    \
        if (r_) return r_;                                        \
    } while (0)

#define WS(ptr, T, name, count)                                           \
    T *ptr = reinterpret_cast<T *>(ws(ctx, name, sizeof(T) * (size_t)(count), &st)); \
    if (!ptr) return st;

void stage(dpg_ctx *ctx, hipStream_t s, const std::string &name) {
    if (ctx->n_events_used >= (int)ctx->events.size()) {
        hipEvent_t e;
        (void)hipEventCreate(&e);
        ctx->events.push_back(e);
    }
    (void)hipEventRecord(ctx->events[ctx->n_events_used++], s);
    ctx->stage_names.push_back(name);
}

// bits needed to index `count` distinct values (0 for count <= 1)
uint32_t bits_for(uint64_t count) {
    uint32_t b = 0;
    while (b < 64 && (count - 1) >> b) ++b;
    return count <= 1 ? 0 : b;
}

uint64_t low_mask(uint32_t bits) { return bits >= 64 ? ~0ull : ((1ull << bits) - 1ull); }

// pid range of the input (order-preserving unsigned atomics)
__global__ void k_pid_minmax(const int64_t *pid, int64_t n, unsigned long long *lo,
                             unsigned long long *hi) {
    unsigned long long a = ~0ull, b = 0ull;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const unsigned long long x = (unsigned long long)pid[i] ^ 0x8000000000000000ull;
        a = x < a ? x : a;
        b = x > b ? x : b;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long c = __shfl_xor(a, o, 64), d = __shfl_xor(b, o, 64);
        a = c < a ? c : a;
        b = d > b ? d : b;
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMin(lo, a);
        atomicMax(hi, b);
    }
}

// Levels of at most this many digit bits rank with wave-aggregated LDS
// atomics (one per distinct digit per wave) instead of one per record;
// DPG_AGG_BITS overrides it for experiments.
int agg_bits() {
    static const int v = [] {
        const char *e = std::getenv("DPG_AGG_BITS");
        return e ? std::atoi(e) : 4;
    }();
    return v;
}

// One partition level in grouped XCD-local mode: digit histograms per group
// (level 1: G consecutive sub-tiles of the input, G = the CUs of one XCD;
// later levels: one group per segment), every group's sub-tiles scattered
// by the workgroups of one XCD at the same time (their adjacent runs meet in
// that XCD's L2), each sub-tile reserving its runs inside the group by one
// atomic add per digit.  No per-sub-tile histograms: at level 1 the
// per-tile histograms of the plain XCD-local mode cost 667 MB of traffic and
// scans per 1e9 records.  Order inside a digit is arrival order (nothing
// downstream depends on it, DESIGN.md "Randomness").
// Timing build (DPG_PHASE_TIMING=1 at run time): k_scatter's phase clock
// (dpg_partition.h g_scat_cyc) around one launch, printed per workgroup.
int scat_phase_begin(dpg_ctx *ctx, hipStream_t s) {
#ifdef DPG_PHASE_TIMING
    if (std::getenv("DPG_PHASE_TIMING")) {
        unsigned long long z[8] = {};
        if (hipMemcpyToSymbolAsync(HIP_SYMBOL(g_scat_cyc), z, sizeof(z), 0, hipMemcpyHostToDevice,
                                   s) != hipSuccess)
            return fail(ctx, DPG_ERR_HIP, "scatter phase clock");
    }
#else
    (void)ctx;
    (void)s;
#endif
    return DPG_OK;
}
int scat_phase_end(dpg_ctx *ctx, hipStream_t s, const char *tag, uint32_t gs) {
#ifdef DPG_PHASE_TIMING
    if (std::getenv("DPG_PHASE_TIMING")) {
        unsigned long long h[8];
        if (hipMemcpyFromSymbolAsync(h, HIP_SYMBOL(g_scat_cyc), sizeof(h), 0, hipMemcpyDeviceToHost,
                                     s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return fail(ctx, DPG_ERR_HIP, "scatter phase clock");
        static const char *nm[5] = {"rank", "scan", "stage", "write", "tile"};
        std::fprintf(stderr, "[dpg] %s scatter phases (wave-0 cycles per workgroup, %u WGs, "
                             "%.1f sub-tiles each):", tag, gs, (double)h[5] / gs);
        for (int k = 0; k < 5; ++k) std::fprintf(stderr, " %s %.0f", nm[k], (double)h[k] / gs);
        std::fprintf(stderr, "\n");
    }
#else
    (void)ctx;
    (void)s;
    (void)tag;
    (void)gs;
#endif
    return DPG_OK;
}

template <class Src, class Rec, int IPT, int FMAX>
int run_level_grouped(dpg_ctx *ctx, hipStream_t s, const Src &src, uint32_t S,
                      const int64_t *seg_start, const uint32_t *seg_cnt, const int64_t *seg_cnt64,
                      int64_t n_upper, uint32_t F, uint32_t bits, Rec *out, const char *tag,
                      int64_t **base_out, uint32_t **tot_out, uint32_t *ntiles_dev,
                      const int64_t *out_start, uint32_t *host_tot = nullptr) {
    int st = DPG_OK;
    const int64_t sub = (int64_t)kScatThreads * IPT;
    const bool single = S == 1 && !seg_start && !seg_cnt;  // level 1: all n records
#ifndef DPG_L1_GROUP
#define DPG_L1_GROUP 1
#endif
    // later levels: one group per segment, or (DPG_SEG_GROUP, experiments)
    // groups of that many records, rounded to whole sub-tiles
    static const int64_t seg_group = [] {
        const char *e = std::getenv("DPG_SEG_GROUP");
        return e ? std::max<int64_t>(0, std::atoll(e)) : (int64_t)0;
    }();
    const int64_t gsz = single ? sub * std::max<int64_t>(1, DPG_L1_GROUP * ctx->n_cu / 8)
                        : seg_group > 0 ? std::max<int64_t>(1, seg_group / sub) * sub
                                        : ((int64_t)1 << 40);
    const uint32_t max_groups = (uint32_t)(n_upper / std::min<int64_t>(gsz, n_upper + 1) + S + 1);
    const uint32_t max_subs = (uint32_t)(n_upper / sub + max_groups + 1);
    std::string t(tag);
    WS(groups, TileDesc, (t + ".groups").c_str(), max_groups);
    WS(stb, uint32_t, (t + ".stb").c_str(), S);
    WS(snt, uint32_t, (t + ".snt").c_str(), S);
    WS(hist, uint32_t, (t + ".hist").c_str(), (size_t)max_groups * F);
    WS(tot, uint32_t, (t + ".tot").c_str(), (size_t)S * F);
    WS(base, int64_t, (t + ".base").c_str(), (size_t)S * F);
    WS(tiles, TileDesc, (t + ".tiles").c_str(), max_subs);
    WS(ngrp, uint32_t, (t + ".ngroups").c_str(), 1);
    WS(xqq, uint32_t, (t + ".xq").c_str(), (size_t)8 * max_subs);
    WS(xqn, uint32_t, (t + ".xqn").c_str(), 16);
    HIP_TRY(hipMemsetAsync(xqn, 0, 16 * 4, s));
    HIP_TRY(hipMemsetAsync(ngrp, 0, 4, s));
    HIP_TRY(hipMemsetAsync(ntiles_dev, 0, 4, s));
    const XcdQueues xq{xqq, xqn, xqn + 8, max_subs};
    stage(ctx, s, (t + ":hist").c_str());
    if (single) {
        const uint32_t ng = (uint32_t)((n_upper + gsz - 1) / gsz);
        k_build_tiles_single<<<(ng + 255) / 256, 256, 0, s>>>(n_upper, gsz, 1u, groups, stb, snt,
                                                             ngrp, XcdQueues{});
    } else {
        k_build_tiles<<<build_tiles_blocks(S), 256, 0, s>>>(seg_start, seg_cnt, seg_cnt64, S, gsz,
                                                      groups, stb, snt, ngrp, XcdQueues{});
    }
    LAUNCH_CHECK();
    k_build_subtiles<<<(max_groups + 255) / 256, 256, 0, s>>>(groups, ngrp, sub, tiles, ntiles_dev,
                                                             xq);
    LAUNCH_CHECK();
    if (F > 2048)
        (void)set_func_attr((const void *)k_hist<Src>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)(4 * F * sizeof(uint32_t)));
    k_hist<Src><<<max_groups, kPartThreads, 4 * F * sizeof(uint32_t), s>>>(src, groups, ngrp, F, hist);
    LAUNCH_CHECK();
    // hist[g][d] <- the group's exclusive digit offset inside its segment
    k_scan_tiles<<<dim3(S, (F + 63) / 64, 1), 1024, 0, s>>>(stb, snt, F, hist, tot);
    LAUNCH_CHECK();
    k_digit_base<<<S, 1024, 0, s>>>(out_start ? out_start : seg_start, F, tot, base);
    LAUNCH_CHECK();
    if (host_tot) {
        // the segment totals reach the host while the scatter runs
        if (!ctx->tot_ev && hipEventCreateWithFlags(&ctx->tot_ev, hipEventDisableTiming) != hipSuccess)
            return fail(ctx, DPG_ERR_HIP, "hipEventCreate (totals)");
        HIP_TRY(hipMemcpyAsync(host_tot, tot, (size_t)S * F * 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipEventRecord(ctx->tot_ev, s));
    }
    constexpr size_t lds = scatter_lds<Src, Rec, IPT, FMAX>();
    static_assert(lds <= 160 * 1024, "scatter LDS");
    auto kern = bits > agg_bits() ? k_scatter<Src, Rec, IPT, FMAX, false> : k_scatter<Src, Rec, IPT, FMAX, true>;
    (void)set_func_attr((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    stage(ctx, s, (t + ":scatter").c_str());
    const uint32_t gs = std::min<uint32_t>(max_subs, (uint32_t)ctx->n_cu);  // one per CU
    if (int r = scat_phase_begin(ctx, s)) return r;
    kern<<<gs, kScatThreads, lds, s>>>(src, tiles, ntiles_dev, F, bits, nullptr, base, out, xq,
                                       nullptr, nullptr, nullptr, 1u, hist, 0u, 0u, nullptr);
    LAUNCH_CHECK();
    if (int r = scat_phase_end(ctx, s, tag, gs)) return r;
    *base_out = base;
    *tot_out = tot;
    return DPG_OK;
}

// One partition level over `S` segments of the source.
template <class Src, class Rec, int IPT, int FMAX>
int run_level(dpg_ctx *ctx, hipStream_t s, const Src &src, uint32_t S, const int64_t *seg_start,
              const uint32_t *seg_cnt, const int64_t *seg_cnt64, int64_t n_upper, uint32_t F,
              uint32_t bits, Rec *out, const char *tag, int64_t **base_out, uint32_t **tot_out,
              uint32_t *ntiles_dev, const int64_t *out_start = nullptr, bool xcd_local = false,
              int subs = 1, bool grouped = false, uint32_t *host_tot = nullptr) {
    int st = DPG_OK;
    if (F > (uint32_t)FMAX) return fail(ctx, DPG_ERR_HIP, "internal: digit fan-out too large");
    const int64_t sub = (int64_t)kScatThreads * IPT;
    if (grouped) return run_level_grouped<Src, Rec, IPT, FMAX>(ctx, s, src, S, seg_start, seg_cnt,
                                                               seg_cnt64, n_upper, F, bits, out, tag,
                                                               base_out, tot_out, ntiles_dev, out_start,
                                                               host_tot);
    // XCD-local mode: `subs` sub-tiles per tile, tiles of a segment on one
    // XCD (every tile carries a digit histogram: tiny tiles cost histogram
    // traffic and scan time)
    const int64_t tile = xcd_local ? sub * std::max(1, subs)
                                   : std::max<int64_t>(sub, ((n_upper / 3072 + sub - 1) / sub) * sub);
    const uint32_t max_tiles = (uint32_t)(n_upper / tile + S + 1);
    XcdQueues xq{};
    if (xcd_local) {
        WS(xqq, uint32_t, (std::string(tag) + ".xq").c_str(), (size_t)8 * max_tiles);
        WS(xqn, uint32_t, (std::string(tag) + ".xqn").c_str(), 16);
        HIP_TRY(hipMemsetAsync(xqn, 0, 16 * 4, s));
        xq = XcdQueues{xqq, xqn, xqn + 8, max_tiles};
    }
    // one segment cut into many tiles: the tile scan runs in C chunks
    const bool single = xcd_local && S == 1 && !seg_start && !seg_cnt;  // level 1: all n records
    const uint32_t C = single ? std::max<uint32_t>(1, std::min<uint32_t>(256, max_tiles / 256)) : 1u;
    std::string t(tag);
    WS(tiles, TileDesc, (t + ".tiles").c_str(), max_tiles);
    WS(stb, uint32_t, (t + ".stb").c_str(), S);
    WS(snt, uint32_t, (t + ".snt").c_str(), S);
    WS(hist, uint32_t, (t + ".hist").c_str(), (size_t)max_tiles * F);
    WS(tot, uint32_t, (t + ".tot").c_str(), (size_t)S * F);
    WS(base, int64_t, (t + ".base").c_str(), (size_t)S * F);
    uint32_t *ctot = tot;
    if (C > 1) {
        WS(ct, uint32_t, (t + ".ctot").c_str(), (size_t)S * C * F);
        ctot = ct;
    }
    stage(ctx, s, (t + ":hist").c_str());
    if (single) {
        const uint32_t nt = (uint32_t)((n_upper + tile - 1) / tile);
#ifndef DPG_L1_GROUP
#define DPG_L1_GROUP 1
#endif
        k_build_tiles_single<<<(nt + 255) / 256, 256, 0, s>>>(n_upper, tile,
                                                             (uint32_t)(DPG_L1_GROUP * ctx->n_cu / 8),
                                                             tiles, stb, snt, ntiles_dev, xq);
    } else {
        k_build_tiles<<<build_tiles_blocks(S), 256, 0, s>>>(seg_start, seg_cnt, seg_cnt64, S, tile, tiles,
                                                      stb, snt, ntiles_dev, xq);
    }
    LAUNCH_CHECK();
    if (F > 2048)
        (void)set_func_attr((const void *)k_hist<Src>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)(4 * F * sizeof(uint32_t)));
    k_hist<Src><<<max_tiles, kPartThreads, 4 * F * sizeof(uint32_t), s>>>(src, tiles, ntiles_dev,
                                                                          F, hist);
    LAUNCH_CHECK();
    k_scan_tiles<<<dim3(S, (F + 63) / 64, C), 1024, 0, s>>>(stb, snt, F, hist, ctot);
    LAUNCH_CHECK();
    if (C > 1) {
        k_scan_chunks<<<(S * F + 255) / 256, 256, 0, s>>>(S, C, F, ctot, tot);
        LAUNCH_CHECK();
    }
    k_digit_base<<<S, 1024, 0, s>>>(out_start ? out_start : seg_start, F, tot, base);
    LAUNCH_CHECK();
    constexpr size_t lds = scatter_lds<Src, Rec, IPT, FMAX>();
    static_assert(lds <= 160 * 1024, "scatter LDS");
    // few digits: wave-aggregated ranking; otherwise one LDS atomic per record
    auto kern = bits > agg_bits() ? k_scatter<Src, Rec, IPT, FMAX, false> : k_scatter<Src, Rec, IPT, FMAX, true>;
    (void)set_func_attr((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    stage(ctx, s, (t + ":scatter").c_str());
#ifndef DPG_SCAT_WGS
#define DPG_SCAT_WGS 0  // 0: one workgroup per tile
#endif
    uint32_t gs = DPG_SCAT_WGS > 0 ? std::min<uint32_t>(max_tiles, (uint32_t)DPG_SCAT_WGS)
                                   : max_tiles;
    if (xcd_local) gs = std::min<uint32_t>(max_tiles, (uint32_t)ctx->n_cu);  // one per CU
    kern<<<gs, kScatThreads, lds, s>>>(src, tiles, ntiles_dev, F, bits, hist, base, out, xq,
                                       C > 1 ? ctot : nullptr, stb, snt, C, nullptr, 0u, 0u,
                                       nullptr);
    LAUNCH_CHECK();
    *base_out = base;
    *tot_out = tot;
    return DPG_OK;
}

// sub-tile sizes per record size: level 1 stages a 2-byte digit beside the
// record; later levels recompute it
template <class R>
struct Ipt {
#ifndef DPG_IPT_L1
#define DPG_IPT_L1 11  // same-box A/B config 2: 12 -> 11 level-1 scatter 7.88 -> 7.25 ms (spills)
#endif
#ifndef DPG_IPT_L1_R16
#define DPG_IPT_L1_R16 7  // the utility pre-aggregate's 16-byte records
#endif
    static constexpr int L1 = sizeof(R) == 8 ? DPG_IPT_L1 : sizeof(R) == 16 ? DPG_IPT_L1_R16 : 8;
#ifndef DPG_IPT_LN
#define DPG_IPT_LN 12  // same-box A/B config 2: 16 -> 12 level-2 scatter 5.97 -> 4.37 ms (spills)
#endif
#ifndef DPG_IPT_LN_R16
#define DPG_IPT_LN_R16 8
#endif
    static constexpr int LN = sizeof(R) == 8 ? DPG_IPT_LN : sizeof(R) == 16 ? DPG_IPT_LN_R16 : 10;
    // the refine level has few digits (wave-aggregated ranking, which holds
    // more registers per record: at LN records per thread it spilled)
    static constexpr int LR = sizeof(R) == 8 ? 8 : 6;
    // level 2 with 4096 digits: the digit arrays take 48 KB of LDS
    static constexpr int LW = sizeof(R) == 8 ? 12 : sizeof(R) == 16 ? 6 : 8;
};

BoundParams to_bound(const dpg_bound_params *p, uint64_t seed) {
    BoundParams b{};
    b.mode = p->mode;
    b.sum_mode = p->sum_mode;
    b.mask = p->metric_mask;
    b.need_values = (p->metric_mask & (DPG_M_SUM | DPG_M_MEAN | DPG_M_VARIANCE)) != 0;
    b.mpc = (uint32_t)std::min<int64_t>(p->max_partitions_contributed, 0x7FFFFFFF);
    b.mcpp = (uint32_t)std::min<int64_t>(p->max_contributions_per_partition, 0x7FFFFFFF);
    b.L = (uint32_t)std::min<int64_t>(p->max_contributions, 0x7FFFFFFF);
    b.lo = p->min_value;
    b.hi = p->max_value;
    b.lo_pp = p->min_sum_per_partition;
    b.hi_pp = p->max_sum_per_partition;
    b.mid = p->min_value + (p->max_value - p->min_value) / 2;
    b.seed = seed;
    b.rec_base = p->rec_id_offset;
    // candidate records per filtered pid in the sort kernel: DPG_SORT_CAND_C
    // x (mpc + 2 sqrt(mpc) + 2); DPG_SORT_CAND_C overrides it for experiments
    float cc = kSortCandC;
    if (const char *e = std::getenv("DPG_SORT_CAND_C")) cc = (float)std::atof(e);
    b.cand_mul = cc * ((float)b.mpc + 2.0f * std::sqrt((float)b.mpc) + 2.0f);
    // expected candidates past which the narrow / streamed passes defer a
    // chunk before drawing its pair priorities (1.25 x their 256-candidate
    // working set; DPG_EARLY_DEFER=0: off)
    const char *ed = std::getenv("DPG_EARLY_DEFER");
    b.defer_est = (ed && std::atoi(ed) == 0) ? 0.0f : 1.25f * 256.0f;
    return b;
}

struct Plan {
    uint32_t b1, b2, kbits, pkbits;
    uint32_t plb;  // pid hash bits left below the fine buckets (<= 7)
    int64_t P;
};

// Pre-aggregate output (dpg_preaggregate): pairs sorted by partition key.
struct PaOut {
    ItemPA *pairs;
    int64_t capacity;
    int64_t *partition_start;  // [P + 1]
    int64_t n_pairs;
};

__global__ void k_set_i64(int64_t *p, int64_t v) { *p = v; }
__global__ void k_set_bits(uint32_t *p, uint32_t bits) { atomicOr(p, bits); }

// Bounding of the fine buckets + merge of the kept pairs per partition (or,
// for the pre-aggregate, the pairs sorted by partition key).
template <class R, class KeyT, class Item>
int bound_and_reduce(dpg_ctx *ctx, hipStream_t s, const Plan &pl, const R *recs,
                     const int64_t *bstart, const uint32_t *bcnt, uint32_t B,
                     const BoundParams &bp, int64_t n, const dpg_partials *out, Control *ctl,
                     PaOut *pa) {
    int st = DPG_OK;
    using CL = ChunkLayout<KeyT, Item>;
    using WL = WaveLayout<KeyT, Item>;
    uint32_t capM = std::min<uint32_t>(ctx->bucket_cap, (uint32_t)kBCap);
    if (const char *e = std::getenv("DPG_DEBUG_CAP"))  // debug: medium-chunk experiments
        capM = std::max<uint32_t>(1, std::min<uint32_t>(capM, (uint32_t)std::atoi(e)));
    // small chunks need <= 7 pid hash bits below a bucket (kWCq = 128 slots)
    uint32_t capS = (uint32_t)kWCap;
    if (const char *e = std::getenv("DPG_DEBUG_CAPS"))  // debug: small-chunk packing experiments
        capS = std::max<uint32_t>(64, std::min<uint32_t>(capS, (uint32_t)std::atoi(e)));
    auto cap_small = [&](uint32_t plb) {
        return plb <= 7 ? std::min<uint32_t>(capM, capS) : 0u;
    };
    const Fmt f = bp.fmt;
    // ---- pack fine buckets into chunks (groups never span level-1 buckets)
    stage(ctx, s, "chunks");
    WS(chunks, uint4, "chunks", B);
    WS(mchunks, uint4, "mchunks", B);
    WS(ostart, int64_t, "over.start", B);
    WS(ocnt, uint32_t, "over.cnt", B);
    WS(od1, uint32_t, "over.d1", B);
    WS(ohb, uint32_t, "over.hb", B);
    const uint32_t group = std::min<uint32_t>(kChunkGroup, 1u << pl.b2);
    const uint32_t ngroups = (B + group - 1) / group;
    k_make_chunks<<<(ngroups + 255) / 256, 256, 0, s>>>(
        bstart, bcnt, B, group, cap_small(pl.plb), capM, 0u, pl.b2, nullptr, nullptr, pl.plb,
        chunks, &ctl->n_chunks, mchunks, &ctl->n_mchunks, ostart, ocnt, od1, ohb, &ctl->n_over,
        &ctl->over_records);
    LAUNCH_CHECK();
    Control hctl;
    HIP_TRY(hipMemcpyAsync(&hctl, ctl, sizeof(Control), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (hctl.err & 1u)
        return fail(ctx, DPG_ERR_KEY_RANGE,
                    "privacy id outside its declared range or partition key outside [0, P)");
    if (hctl.err & 8u) return kRedoLevel2;
    uint4 *chunk_list = chunks;
    size_t chunk_cap = B;  // entries of chunk_list
    uint4 *mchunk_list = mchunks;
    const R *refined = recs;
    // global-memory leftovers: (buffer, starts, counts, level-1 buckets, number)
    const R *g_base = recs;
    const int64_t *g_start = ostart;
    const uint32_t *g_cnt = ocnt;
    const uint32_t *g_d1 = od1;
    const uint32_t *g_hb = ohb;
    unsigned long long g_records = hctl.over_records;
    uint32_t g_plb = pl.plb;  // pid hash bits below an oversize bucket
    uint32_t n_global = 0;
    if (hctl.n_over > 0) {
        const uint32_t rbits = std::min<uint32_t>(kMaxBR, pl.plb);  // hash bits not yet used
        if (rbits == 0) {
            n_global = hctl.n_over;
        } else {
            // ---- refine oversize buckets by further privacy-id hash bits
            const uint32_t no = hctl.n_over, F2 = 1u << rbits;
            std::vector<uint32_t> hc(no);
            HIP_TRY(hipMemcpy(hc.data(), ocnt, no * 4, hipMemcpyDeviceToHost));
            std::vector<int64_t> hout(no);
            int64_t acc = 0;
            for (uint32_t i = 0; i < no; ++i) hout[i] = acc, acc += hc[i];
            WS(oout, int64_t, "over.out", no);
            UPLOAD(oout, hout.data(), no * 8);
            WS(rbuf, R, "refined", std::max<int64_t>(acc, 1));
            int64_t *base2;
            uint32_t *tot2;
            const uint32_t shift = pl.pkbits + (pl.kbits - pl.b1) - pl.b2 - rbits;
            SrcAoS<R> src{recs, f, shift, F2 - 1};
            int r = run_level<SrcAoS<R>, R, Ipt<R>::LR, 2048>(ctx, s, src, no, ostart, ocnt,
                                                               nullptr, acc, F2, rbits, rbuf,
                                                               "refine", &base2, &tot2,
                                                               &ctl->ntiles[3], oout);
            if (r) return r;
            const uint32_t B2 = no * F2;
            WS(chunks2, uint4, "chunks.r", (size_t)hctl.n_chunks + B2);
            WS(mchunks2, uint4, "mchunks.r", (size_t)hctl.n_mchunks + B2);
            if (hctl.n_chunks)
                HIP_TRY(hipMemcpyAsync(chunks2, chunks, (size_t)hctl.n_chunks * sizeof(uint4),
                                       hipMemcpyDeviceToDevice, s));
            if (hctl.n_mchunks)
                HIP_TRY(hipMemcpyAsync(mchunks2, mchunks, (size_t)hctl.n_mchunks * sizeof(uint4),
                                       hipMemcpyDeviceToDevice, s));
            WS(o2start, int64_t, "over2.start", B2);
            WS(o2cnt, uint32_t, "over2.cnt", B2);
            WS(o2d1, uint32_t, "over2.d1", B2);
            WS(o2hb, uint32_t, "over2.hb", B2);
            const uint32_t plb2 = pl.plb - rbits;
            k_make_chunks<<<(no + 255) / 256, 256, 0, s>>>(
                base2, tot2, B2, F2, cap_small(plb2), capM, 1u, rbits, od1, ohb, plb2, chunks2,
                &ctl->n_chunks, mchunks2, &ctl->n_mchunks, o2start, o2cnt, o2d1, o2hb,
                &ctl->n_over2, &ctl->over2_records);
            LAUNCH_CHECK();
            HIP_TRY(hipMemcpyAsync(&hctl, ctl, sizeof(Control), hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
            chunk_list = chunks2;
            chunk_cap = (size_t)hctl.n_chunks + B2;
            mchunk_list = mchunks2;
            refined = rbuf;
            g_base = rbuf;
            g_start = o2start;
            g_cnt = o2cnt;
            g_d1 = o2d1;
            g_hb = o2hb;
            g_records = hctl.over2_records;
            g_plb = plb2;
            n_global = hctl.n_over2;
        }
    }
    // ---- heavy buckets (single privacy ids over every chunk, cross-partition
    // modes): candidate records into heavy chunks of the small-chunk list
    // (dpg_wave.h); the rest, and buckets the wave kernel hands back, stay on
    // the global-memory path.  mpc <= 128: ~mpc pairs below a 512-record cut.
    const bool per_pid = bp.mode == DPG_MODE_PER_PRIVACY_ID;
    const bool heavy = n_global > 0 && !per_pid && !ItemTraits<Item>::preagg && bp.mpc <= 128 &&
                       std::getenv("DPG_NO_HEAVY") == nullptr;
    // the cross-partition modes sort (dpg_sortb.h) when the partition key
    // fits the sort key; PER_PRIVACY_ID, the pre-aggregate and wider keys
    // take the hash-table kernel (dpg_wave.h).  DPG_BOUND_HASH: force it.
    bool use_sort = false;
    if constexpr (!ItemTraits<Item>::preagg)
        use_sort = !per_pid && std::getenv("DPG_BOUND_HASH") == nullptr &&
                   (pl.pkbits <= kSkPkBits || (sizeof(R) == 12 && pl.pkbits <= 32));
    // medium chunks: streamed by single waves of the sort kernel (tier 3,
    // the narrow pass's working set), the chunks it defers by the hash-table
    // kernel; DPG_MEDIUM_STREAM=0 (or DPG_MW_MEDIUM): the workgroup kernels
    // alone.  Pid slots need <= 7 hash bits below a bucket.
    const char *ms_env = std::getenv("DPG_MEDIUM_STREAM");
    const bool stream_ok = use_sort && pl.plb <= 7 && !(ms_env && std::atoi(ms_env) == 0) &&
                           std::getenv("DPG_MW_MEDIUM") == nullptr;
    // ... and the oversize buckets join the medium list instead of the heavy
    // filter: the streamed pass holds candidates, never a chunk, so size does
    // not matter; an oversize chunk it cannot bound goes back to the
    // global-memory kernel (heavy_fb, as the heavy chunks' do).
    // Only while the pass aims at its full kStreamMul x cand_mul candidates
    // per big privacy id (mpc <= ~13): with a capped aim (config 4, mpc 50)
    // the kept pairs often include a Zipf-heavy pair of more records than
    // the working set holds, and a handed-back bucket costs the global-memory
    // kernel (same-box A/B: config 4 75.6 -> 92.6 ms, bound.tail 18 ms;
    // (1e9, 1e6), mpc 8: 21.7 -> 18.5 ms).  DPG_STREAM_OVER=0: the heavy
    // filter always, =1: the streamed pass always.
    const char *so_env = std::getenv("DPG_STREAM_OVER");
    const bool so_aim = bp.cand_mul * kStreamMul <= 0.5f * (float)kNarrowCand<R>;
    const bool stream_over = heavy && stream_ok &&
                             (so_env ? std::atoi(so_env) != 0 : so_aim);
    uint32_t n_m0 = 0xFFFFFFFFu;  // first oversize entry of the medium list (none)
    const R *hrec = recs;
    uint32_t *hfb = nullptr;
    if (stream_over) {
        WS(hf, uint32_t, "heavy.fb", n_global);
        hfb = hf;
        n_m0 = hctl.n_mchunks;
        k_over_to_medium<<<(n_global + 255) / 256, 256, 0, s>>>(
            g_start, g_cnt, g_d1, g_hb, n_global, g_base == recs ? 0u : 1u, mchunk_list,
            &ctl->n_mchunks, n_m0);
        LAUNCH_CHECK();
        hctl.n_mchunks += n_global;
    } else if (heavy) {
        stage(ctx, s, "heavy");
        WS(hr, R, "heavy.recs", (size_t)n_global * kWCap);
        WS(hf, uint32_t, "heavy.fb", n_global);
        BoundParams bph = bp;
        bph.heavy_fb = hf;
        bph.heavy_nfb = &ctl->heavy_nfb;
        k_heavy_filter<R><<<n_global, kHvThreads, 0, s>>>(g_base, g_start, g_cnt, g_d1, bph, hr,
                                                          chunk_list, &ctl->n_chunks);
        LAUNCH_CHECK();
        hrec = hr;
        hfb = hf;
    }
    // ---- bounding in LDS: Gw single-wave workgroups over the small chunks,
    // Gm 256-thread workgroups over the medium ones (launched only if there
    // are any), the global-memory path last; workgroup g of the Gw + Gm + 1
    // writes its items to items[wg_off[g], ...)
    // one kernel per bounding family (PER_PRIVACY_ID or cross-partition), so
    // that the hot one holds one path only
    auto wave_kern = per_pid ? k_bound_waves<KeyT, Item, R, true> : k_bound_waves<KeyT, Item, R, false>;
    size_t wave_lds = WL::TOTAL;
    // partition keys wider than the sort key's 24 bits: the wide-key kernels
    // (their low bits ride in the sort payload; 12-byte records only)
    const bool wpk = pl.pkbits > kSkPkBits;
    // resident single-wave workgroups per CU of a kernel: the LDS share or
    // the register file, whichever binds, rounded down to a multiple of the
    // 4 SIMDs: the static schedule gives every wave the same share of
    // chunks, so two waves sharing a SIMD next to SIMDs with one would finish
    // last (same-box A/B, config 4 with 32-KB working sets: 5 waves per CU
    // 42 ms, 4 per CU 29.7 ms)
    auto waves_per_cu = [&](const void *kern, size_t lds, int cap = 16) {
        int wpc = 0;
        if (occ_query(&wpc, kern, 64, lds) != hipSuccess ||
            wpc <= 0)
            wpc = 1;
        int pc = std::min(wpc, (int)std::min<size_t>((size_t)cap, (160 * 1024) / lds));
        if (pc > 4) pc &= ~3;
        if (const char *e = std::getenv("DPG_DEBUG_WPC"))  // debug: occupancy experiments
            pc = std::max(1, std::min(pc, std::atoi(e)));
        return pc;
    };
    // multi-wave sort kernels (dpg_sortmw.h) for the wide and the medium
    // chunks; DPG_MW_OFF: the single-wave wide kernel and the hash-table
    // medium kernel.  Their pid slots need <= 7 hash bits below a bucket.
    const bool use_mw = use_sort && pl.plb <= 7 && std::getenv("DPG_MW_OFF") == nullptr;
    auto blocks_per_cu = [&](const void *kern, int threads, size_t lds) {
        int b = 0;
        if (occ_query(&b, kern, threads, lds) != hipSuccess ||
            b <= 0)
            b = 1;
        return b;
    };
    const void *narrow = nullptr, *mid = nullptr, *wide = nullptr, *medium = nullptr;
    size_t mid_lds = wave_lds, wide_lds = wave_lds;
    constexpr bool kMid = kHasMid<R>;
    if constexpr (!ItemTraits<Item>::preagg) {
        if (use_sort && !wpk) {
            narrow = (const void *)k_bound_sorted<Item, R, 0, false>;
            if constexpr (kMid) mid = (const void *)k_bound_sorted<Item, R, 1, false>;
            wide = (const void *)k_bound_sorted<Item, R, 2, false>;
            medium = (const void *)k_bound_sorted<Item, R, 3, false>;
            wave_lds = SortLayout<Item, R, false, kTierCand<R, 0>>::TOTAL;
            mid_lds = SortLayout<Item, R, false, kTierCand<R, 1>>::TOTAL;
            wide_lds = SortLayout<Item, R, false, kTierCand<R, 2>>::TOTAL;
        }
        if constexpr (sizeof(R) == 12) {
            if (use_sort && wpk) {
                narrow = (const void *)k_bound_sorted<Item, R, 0, true>;
                if constexpr (kMid) mid = (const void *)k_bound_sorted<Item, R, 1, true>;
                wide = (const void *)k_bound_sorted<Item, R, 2, true>;
                medium = (const void *)k_bound_sorted<Item, R, 3, true>;
                wave_lds = SortLayout<Item, R, true, kTierCand<R, 0>>::TOTAL;
                mid_lds = SortLayout<Item, R, true, kTierCand<R, 1>>::TOTAL;
                wide_lds = SortLayout<Item, R, true, kTierCand<R, 2>>::TOTAL;
            }
        }
    }
    const int per_cu = use_sort ? waves_per_cu(narrow, wave_lds, 4 * kNarrowWPS<R>)
                                : waves_per_cu((const void *)wave_kern, wave_lds);
    const uint32_t Gw = (uint32_t)(ctx->n_cu * per_cu);
    const bool stream_med = medium != nullptr && hctl.n_mchunks > 0 && stream_ok;
    const uint32_t Gm =
        !hctl.n_mchunks ? 0u
        : stream_med    ? (uint32_t)std::min<uint32_t>(
                           ctx->n_cu * waves_per_cu(medium, wave_lds, 4 * kNarrowWPS<R>),
                           hctl.n_mchunks)
                        : (uint32_t)std::min<uint32_t>(ctx->n_cu * CL::PER_CU, hctl.n_mchunks);
    const uint32_t G = Gw + Gm;
    // heavy buckets handed back are counted twice (candidates + bucket)
    // streamed oversize buckets handed back emit behind the regions of the
    // chunk lists: <= mpc items per privacy id (one per bucket when no hash
    // bits are left below it), else <= its records
    const int64_t hv_extra =
        !heavy        ? 0
        : stream_over ? (g_plb == 0 ? (int64_t)n_global * bp.mpc : (int64_t)g_records)
                      : (int64_t)n_global * kWCap;
    const int64_t items_cap = std::max<int64_t>(n + hv_extra, 1);
    WS(items, Item, "items", items_cap);
    WS(wg_rec, uint32_t, "wg.rec", G + 1);
    WS(wg_off, int64_t, "wg.off", G + 2);
    WS(wg_cnt, uint32_t, "wg.cnt", G + 1);
    WS(wg_pre, int64_t, "wg.pre", G + 2);
    k_wg_records<<<Gw, 256, 0, s>>>(chunk_list, &ctl->n_chunks, Gw, wg_rec);
    LAUNCH_CHECK();
    if (Gm) {
        k_wg_records<<<Gm, 256, 0, s>>>(mchunk_list, &ctl->n_mchunks, Gm, wg_rec + Gw);
        LAUNCH_CHECK();
    }
    k_scan_small<<<1, 1024, 0, s>>>(wg_rec, G, wg_off, nullptr);
    LAUNCH_CHECK();
    HIP_TRY(hipMemsetAsync(wg_cnt + G, 0, 4, s));
    BoundParams bpl = bp;
    uint32_t *prog = watchdog_seconds() ? watchdog_buffer(G) : nullptr;
    bpl.progress = prog;
    const bool timing = std::getenv("DPG_PHASE_TIMING") != nullptr;
    bpl.phase_cyc = nullptr;
    bpl.heavy_fb = hfb;
    bpl.heavy_nfb = &ctl->heavy_nfb;
    if (timing) {
        WS(pc, unsigned long long, "bound.phase_cyc", 64);
        HIP_TRY(hipMemsetAsync(pc, 0, 64 * 8, s));
        bpl.phase_cyc = pc;
    }
    // zero-length marker stage: which small-chunk kernel bounded this call
    stage(ctx, s, use_sort ? "bound.kernel=sort" : "bound.kernel=hash");
    if (use_mw) stage(ctx, s, "bound.multiwave");  // marker: wide / medium chunks in dpg_sortmw.h
    stage(ctx, s, "bound");
    if constexpr (!ItemTraits<Item>::preagg) if (use_sort) {
        WS(defer, uint8_t, "bound.defer", std::max<size_t>(chunk_cap, 1));
        (void)set_func_attr(narrow, hipFuncAttributeMaxDynamicSharedMemorySize, (int)wave_lds);
        if (mid) (void)set_func_attr(mid, hipFuncAttributeMaxDynamicSharedMemorySize, (int)mid_lds);
        (void)set_func_attr(wide, hipFuncAttributeMaxDynamicSharedMemorySize, (int)wide_lds);
        auto launch = [&](auto wpk_tag) {
            constexpr bool W = decltype(wpk_tag)::value;
            k_bound_sorted<Item, R, 0, W><<<Gw, 64, wave_lds, s>>>(
                recs, refined, hrec, chunk_list, &ctl->n_chunks, bpl, items, wg_off, wg_cnt, defer,
                Gw);
            BoundParams bpx = bpl;
            bpx.phase_cyc = nullptr;
            if constexpr (kMid) {
                // chunks of 129-256 candidates: 4 waves per SIMD
                stage(ctx, s, "bound.mid");
                const uint32_t Gx = std::min<uint32_t>(
                    Gw, (uint32_t)(ctx->n_cu * waves_per_cu(mid, mid_lds)));
                k_bound_sorted<Item, R, 1, W><<<Gx, 64, mid_lds, s>>>(
                    recs, refined, hrec, chunk_list, &ctl->n_chunks, bpx, items, wg_off, wg_cnt,
                    defer, Gw);
            }
            // chunks with more candidates than the narrow / mid passes sort:
            // two waves per chunk (4 waves per SIMD) or, DPG_MW_OFF, the
            // single-wave 8-element kernel (2 waves per SIMD)
            stage(ctx, s, "bound.wide");
            if (use_mw) {
                if (timing) bpx.phase_cyc = bpl.phase_cyc + 48;
                using LW = SortLayoutMW<Item, R, W, 2>;
                const void *k2 = (const void *)k_bound_sorted_w2<Item, R, W>;
                (void)set_func_attr(k2, hipFuncAttributeMaxDynamicSharedMemorySize,
                                          (int)LW::TOTAL);
                const uint32_t Gx = std::min<uint32_t>(
                    Gw, (uint32_t)(ctx->n_cu * blocks_per_cu(k2, LW::T, LW::TOTAL)));
                k_bound_sorted_w2<Item, R, W><<<Gx, LW::T, LW::TOTAL, s>>>(
                    recs, refined, hrec, chunk_list, &ctl->n_chunks, bpx, items, wg_off, wg_cnt,
                    defer, Gw);
            } else {
                const uint32_t Gx = std::min<uint32_t>(
                    Gw, (uint32_t)(ctx->n_cu * waves_per_cu(wide, wide_lds)));
                k_bound_sorted<Item, R, 2, W><<<Gx, 64, wide_lds, s>>>(
                    recs, refined, hrec, chunk_list, &ctl->n_chunks, bpx, items, wg_off, wg_cnt,
                    defer, Gw);
            }
        };
        if (!wpk) {
            launch(std::false_type{});
        } else if constexpr (sizeof(R) == 12) {
            launch(std::true_type{});
        }
        LAUNCH_CHECK();
    }
    if (!use_sort) {
        (void)set_func_attr((const void *)wave_kern,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)wave_lds);
        wave_kern<<<Gw, 64, wave_lds, s>>>(recs, refined, hrec, chunk_list, &ctl->n_chunks, bpl,
                                           items, wg_off, wg_cnt);
        LAUNCH_CHECK();
    }
    if (prog) watchdog_wait(s, prog, Gw, "k_bound_waves");
    stage(ctx, s, "bound.medium");
    bool medium_done = false;
    uint8_t *mdefer = nullptr;
    if constexpr (!ItemTraits<Item>::preagg) {
        if (stream_med) {
            WS(mdef, uint8_t, "bound.mdefer", hctl.n_mchunks);
            mdefer = mdef;
            // tier 3 shares the narrow pass's working set (kTierCand)
            (void)set_func_attr(medium, hipFuncAttributeMaxDynamicSharedMemorySize, (int)wave_lds);
            BoundParams bpm = bpl;
            if (timing) bpm.phase_cyc = bpl.phase_cyc + 16;
            auto launch_s = [&](auto wpk_tag) {
                constexpr bool W = decltype(wpk_tag)::value;
                k_bound_sorted<Item, R, 3, W><<<Gm, 64, wave_lds, s>>>(
                    recs, refined, recs, mchunk_list, &ctl->n_mchunks, bpm, items, wg_off + Gw,
                    wg_cnt + Gw, mdefer, n_m0);
            };
            if (!wpk) {
                launch_s(std::false_type{});
            } else if constexpr (sizeof(R) == 12) {
                launch_s(std::true_type{});
            }
            LAUNCH_CHECK();
            stage(ctx, s, "bound.medium_deferred");
            BoundParams bpd = bpl;
            bpd.phase_cyc = nullptr;
            (void)set_func_attr((const void *)k_bound_chunks_deferred<KeyT, Item, R>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)CL::TOTAL);
            k_bound_chunks_deferred<KeyT, Item, R>
                <<<std::min<uint32_t>(Gm, ctx->n_cu * CL::PER_CU), kBT, CL::TOTAL, s>>>(
                    recs, refined, mchunk_list, &ctl->n_mchunks, bpd, items, wg_off + Gw,
                    wg_cnt + Gw, mdefer, Gm);
            LAUNCH_CHECK();
            medium_done = true;
        }
        // the 4-wave medium kernel measured slower than the hash-table one
        // (config 4 medium 9.8 vs 7.6 ms: a 1024-element sort for ~300
        // candidates): opt-in
        if (Gm && !medium_done && use_mw && std::getenv("DPG_MW_MEDIUM") != nullptr) {
            auto launch_m = [&](auto wpk_tag) {
                constexpr bool W = decltype(wpk_tag)::value;
                using LM = SortLayoutMW<Item, R, W, 4>;
                (void)set_func_attr((const void *)k_bound_sorted_m4<Item, R, W>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)LM::TOTAL);
                BoundParams bpm = bpl;
                if (timing) bpm.phase_cyc = bpl.phase_cyc + 16;
                k_bound_sorted_m4<Item, R, W><<<Gm, LM::T, LM::TOTAL, s>>>(
                    recs, refined, mchunk_list, &ctl->n_mchunks, bpm, items, wg_off + Gw,
                    wg_cnt + Gw);
            };
            if (!wpk) {
                launch_m(std::false_type{});
                medium_done = true;
            } else if constexpr (sizeof(R) == 12) {
                launch_m(std::true_type{});
                medium_done = true;
            }
            LAUNCH_CHECK();
        }
    }
    if (Gm && !medium_done) {
        BoundParams bpm = bpl;
        if (timing) bpm.phase_cyc = bpl.phase_cyc + 16;
        if (prog) bpm.progress = prog + Gw;
        (void)set_func_attr((const void *)k_bound_chunks<KeyT, Item, R>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)CL::TOTAL);
        k_bound_chunks<KeyT, Item, R><<<Gm, kBT, CL::TOTAL, s>>>(
            recs, refined, mchunk_list, &ctl->n_mchunks, bpm, items, wg_off + Gw, wg_cnt + Gw);
        LAUNCH_CHECK();
        if (prog) watchdog_wait(s, prog + Gw, Gm, "k_bound_chunks");
    }
    stage(ctx, s, "bound.tail");
    if (timing) {
        unsigned long long h[64];
        HIP_TRY(hipMemcpy(h, bpl.phase_cyc, sizeof(h), hipMemcpyDeviceToHost));
        static const char *nmh[12] = {"A0.cas", "A1.count", "B.slots", "C1.cand", "C2.rank",
                                      "D.state", "E.mcpp", "F.acc", "G.emit", "A.probe",
                                      "Am.pidc", "Am.cand"};
        static const char *nms[12] = {"A.pids+cand", "S.sort", "P.pairs", "M.mcpp", "F.emit",
                                      "end", "-", "-", "-", "-", "-", "-"};
        static const char *nmc[9] = {"A0.cas", "A1.count", "A2.barrier", "B.slots", "C.mpc",
                                     "D.state", "E.mcpp", "F.acc", "G.emit"};
        for (int part = 0; part < 3; ++part) {
            // small chunks, medium chunks, wide chunks (multi-wave kernel);
            // totals per workgroup of the kernel's own grid size
            const unsigned long long *hp = h + (part == 2 ? 48 : 16 * part);
            if (part == 2 && !use_mw) continue;
            const uint32_t gg = part == 1 ? Gm : Gw;
            if (!gg) continue;
            unsigned long long tot = 0;
            const bool sortnames =
                part == 0 ? use_sort
                : part == 1 && stream_med
                    ? true
                    : use_mw && (part == 2 || std::getenv("DPG_MW_MEDIUM") != nullptr);
            const int np = sortnames ? 6 : part ? 9 : 12;
            for (int i = 0; i < np; ++i) tot += hp[i];
            std::fprintf(stderr, "[dpg phase] %s chunks=%u over=%u over2=%u per-WG Mcycles:",
                         part == 2 ? "wide(mw)" : part ? "medium" : "small",
                         part == 1 ? hctl.n_mchunks : hctl.n_chunks, hctl.n_over, hctl.n_over2);
            const char *const *nm = sortnames ? nms : part ? nmc : nmh;
            for (int i = 0; i < np; ++i)
                std::fprintf(stderr, " %s=%.3f(%.0f%%)", nm[i], hp[i] / 1e6 / gg,
                             100.0 * hp[i] / (tot ? tot : 1));
            std::fprintf(stderr, "\n");
        }
        if (mdefer) {
            std::vector<uint8_t> hd(hctl.n_mchunks);
            HIP_TRY(hipMemcpy(hd.data(), mdefer, hd.size(), hipMemcpyDeviceToHost));
            size_t nd = 0;
            for (uint8_t x : hd) nd += x;
            std::fprintf(stderr, "[dpg phase] medium chunks streamed=%u deferred=%zu\n",
                         hctl.n_mchunks, nd);
        }
    }
    // ---- single buckets beyond the chunk capacity: global-memory working sets
    if (heavy) {
        HIP_TRY(hipMemcpyAsync(&hctl, ctl, sizeof(Control), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        const uint32_t nfb = hctl.heavy_nfb;
        if (nfb > 0) {
            WS(fst, int64_t, "heavy.fb.start", nfb);
            WS(fcnt, uint32_t, "heavy.fb.cnt", nfb);
            WS(fd1, uint32_t, "heavy.fb.d1", nfb);
            k_gather_heavy<<<(nfb + 255) / 256, 256, 0, s>>>(hfb, &ctl->heavy_nfb, g_start, g_cnt,
                                                             g_d1, fst, fcnt, fd1);
            LAUNCH_CHECK();
            g_start = fst;
            g_cnt = fcnt;
            g_d1 = fd1;
        }
        if (timing) std::fprintf(stderr, "[dpg phase] heavy buckets=%u handed back=%u\n", n_global, nfb);
        n_global = nfb;
    }
    if (n_global > 0) {
        std::vector<uint32_t> cnt(n_global);
        HIP_TRY(hipMemcpy(cnt.data(), g_cnt, n_global * 4, hipMemcpyDeviceToHost));
        std::vector<size_t> off(n_global);
        size_t total = 0;
        for (uint32_t i = 0; i < n_global; ++i) {
            off[i] = total;
            total += align16(BigLayout::make(cnt[i], ItemTraits<Item>::var).total);
        }
        WS(scratch, char, "bound.scratch", total);
        WS(doff, size_t, "bound.scratch_off", n_global);
        UPLOAD(doff, off.data(), n_global * sizeof(size_t));
        BoundParams bpg = bp;
        uint32_t *gprog = watchdog_seconds() ? watchdog_buffer(n_global) : nullptr;
        bpg.progress = gprog;
        bpg.phase_cyc = timing ? bpl.phase_cyc + 32 : nullptr;
        if (watchdog_seconds())
            std::fprintf(stderr, "[dpg] %u oversize buckets, scratch %zu bytes\n", n_global, total);
        k_bound_big<Item, R><<<n_global, kBigThreads, 0, s>>>(g_base, g_start, g_cnt, g_d1, doff,
                                                              scratch, bpg, items, wg_off + G,
                                                              wg_cnt + G);
        LAUNCH_CHECK();
        if (gprog) watchdog_wait(s, gprog, n_global, "k_bound_big");
        if (timing) {
            unsigned long long h[8];
            HIP_TRY(hipMemcpy(h, bpl.phase_cyc + 32, sizeof(h), hipMemcpyDeviceToHost));
            static const char *nmb[8] = {"clear", "A.insert", "B.slots", "C.mpc", "D.state",
                                         "E.mcpp", "F.acc", "G.emit"};
            unsigned long long tot = 0;
            for (int i = 0; i < 8; ++i) tot += h[i];
            size_t recs_big = 0;
            uint32_t nmax = 0;
            for (uint32_t i = 0; i < n_global; ++i) recs_big += cnt[i], nmax = std::max(nmax, cnt[i]);
            std::fprintf(stderr, "[dpg phase] big buckets=%u records=%zu max=%u per-WG Mcycles:",
                         n_global, recs_big, nmax);
            for (int i = 0; i < 8; ++i)
                std::fprintf(stderr, " %s=%.3f(%.0f%%)", nmb[i], h[i] / 1e6 / n_global,
                             100.0 * h[i] / (tot ? tot : 1));
            std::fprintf(stderr, "\n");
        }
    }
    k_scan_small<<<1, 1024, 0, s>>>(wg_cnt, G + 1, wg_pre, &ctl->item_cursor);
    LAUNCH_CHECK();
    constexpr bool kPA = ItemTraits<Item>::preagg;
    int64_t n_items;
    if constexpr (kPA) {
        // the caller needs the pair count on return
        HIP_TRY(hipMemcpyAsync(&hctl, ctl, sizeof(Control), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (hctl.err & 2u) return fail(ctx, DPG_ERR_HIP, "internal hash-table error in bounding");
        n_items = hctl.item_cursor;
    } else {
        // no host round trip: the item levels and the merge size their grids
        // and buffers by an upper bound (a privacy id keeps at most mpc
        // pairs, or L records under PER_PRIVACY_ID) and read the count on the
        // device; the internal-error flag is checked by dpg_compact_kept
        const uint64_t pairs_per_id = std::max<uint32_t>(1u, per_pid ? bp.L : bp.mpc);
        n_items = (int64_t)std::min<uint64_t>((uint64_t)items_cap,
                                              ((uint64_t)1 << pl.kbits) * pairs_per_id);
    }
    const int64_t P = pl.P;
#ifndef DPG_ITEM_IPT_WIDE
#define DPG_ITEM_IPT_WIDE 4  // 24-byte items per thread per sub-tile (LDS caps it at 5)
#endif
    constexpr int kItemIpt = sizeof(Item) == 16 ? 8 : sizeof(Item) == 24 ? DPG_ITEM_IPT_WIDE : 4;
    // the items are partitioned by partition-key range: one level up to 1024
    // ranges, else two (pk >> (rbits + b2), then (pk >> rbits) mod 2^b2) --
    // the final segment index is the range id either way
#ifndef DPG_PA_RB
#define DPG_PA_RB 11  // pre-aggregate: low partition-key bits sorted by the last (pairs) level
#endif
    constexpr uint32_t kRB = kPA ? (uint32_t)DPG_PA_RB : (uint32_t)kRangeBits;
    const int64_t nranges = (P + (1ll << kRB) - 1) >> kRB;
    int64_t *baseR = nullptr;
    uint32_t *totR = nullptr;
    const Item *sorted = items;
    uint32_t F = 1;
    if (n_items > 0) {
        const uint32_t rb = std::max<uint32_t>(1, bits_for((uint64_t)std::max<int64_t>(1, nranges)));
        // two levels split the bits evenly: a sub-tile of 4096-8192 items
        // writes runs of 16-64 items per digit at both levels (a 4 + 11 split
        // at config 4's 24 415 ranges wrote runs of ~2 items at level 2)
        const uint32_t b2 = rb > 10 ? std::min<uint32_t>(kMaxBR, rb / 2) : 0u;
        const uint32_t b1 = rb - b2;
        const uint32_t F1 = nranges <= 1024 ? (uint32_t)std::max<int64_t>(1, nranges) : 1u << b1;
        WS(items2, Item, "items2", n_items);
        const SrcSeg<Item> src1{items, wg_pre, wg_off, G + 1, kRB + b2};
        int r = run_level<SrcSeg<Item>, Item, kItemIpt, 1024>(
            ctx, s, src1, 1u, nullptr, &ctl->item_cursor, nullptr, n_items, F1, b1, items2,
            "items", &baseR, &totR, &ctl->ntiles[4]);
        if (r) return r;
        sorted = items2;
        F = F1;
        if (b2 > 0) {
            const SrcItems<Item> src2{items2, kRB, (1u << b2) - 1u};
            int64_t *base2;
            uint32_t *tot2;
            r = run_level<SrcItems<Item>, Item, kItemIpt, 2048>(ctx, s, src2, F1, baseR, totR,
                                                                 nullptr, n_items, 1u << b2, b2,
                                                                 items, "items2", &base2, &tot2,
                                                                 &ctl->ntiles[6]);
            if (r) return r;
            baseR = base2;
            totR = tot2;
            sorted = items;
            F = F1 << b2;
        }
    }
    if constexpr (kPA) {
        // ---- pre-aggregate: one more level on the low 11 key bits sorts the
        // pairs by partition key, straight into the caller's array; the
        // digit offsets of that level are the partition starts
        pa->n_pairs = n_items;
        if (n_items > pa->capacity)
            return fail(ctx, DPG_ERR_INVALID_ARG,
                        "pairs capacity " + std::to_string(pa->capacity) + " < " +
                            std::to_string(n_items) + " pairs");
        if (n_items == 0) {
            HIP_TRY(hipMemsetAsync(pa->partition_start, 0, (P + 1) * 8, s));
            stage(ctx, s, "end");
            return DPG_OK;
        }
        const SrcItems<Item> src3{sorted, 0u, (1u << kRB) - 1u};
        int64_t *base3;
        uint32_t *tot3;
        int r = run_level<SrcItems<Item>, Item, kItemIpt, 2048>(
            ctx, s, src3, F, baseR, totR, nullptr, n_items, 1u << kRB, kRB, pa->pairs, "pairs",
            &base3, &tot3, &ctl->ntiles[7]);
        if (r) return r;
        HIP_TRY(hipMemcpyAsync(pa->partition_start, base3, P * 8, hipMemcpyDeviceToDevice, s));
        k_set_i64<<<1, 1, 0, s>>>(pa->partition_start + P, n_items);
        LAUNCH_CHECK();
    } else if (n_items > 0) {
        // ---- merge kept pairs per partition
        Partials po{out->rows, out->count, out->sum, out->nsum, out->nsq};
        stage(ctx, s, "reduce");
        const int64_t rtile = 65536;
        uint32_t max_tiles = (uint32_t)(n_items / rtile + F + 1);
        WS(rt, TileDesc, "reduce.tiles", max_tiles);
        WS(rstb, uint32_t, "reduce.stb", F);
        WS(rsnt, uint32_t, "reduce.snt", F);
        k_build_tiles<<<build_tiles_blocks(F), 256, 0, s>>>(baseR, totR, nullptr, F, rtile, rt, rstb,
                                                      rsnt, &ctl->ntiles[5]);
        LAUNCH_CHECK();
        size_t lds_r = (size_t)kRange * 8 * (ItemTraits<Item>::var ? (ItemTraits<Item>::sum ? 3 : 2) : 1) +
                       kRange * 8;
        k_reduce_items<Item><<<max_tiles, 1024, lds_r, s>>>(sorted, rt, &ctl->ntiles[5], rsnt, P,
                                                         po);
        LAUNCH_CHECK();
    }
    stage(ctx, s, "end");
    return DPG_OK;
}

// Histogram-free level 1 (k_scatter's piece mode): region (x, d) of C
// records starts at (8 d + x) C, so a bucket's 8 pieces are neighbours.
__global__ void k_region_base(int64_t *rbase, uint32_t F, uint32_t C) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 8 * F) return;
    const uint32_t x = i / F, d = i % F;
    rbase[i] = ((int64_t)d * 8 + x) * C;
}

// Bucket totals of the pieces and the buckets' starts in the compact level-2
// output (one workgroup; F <= 2048).
// desc[d]: the bucket's pieces in one record for the team level 2's scalar
// loads (dpg_team.h PieceDesc).
__global__ __launch_bounds__(1024) void k_piece_totals(const uint32_t *cum, const int64_t *rbase,
                                                       uint32_t F, uint32_t *tot, uint32_t *ptot,
                                                       int64_t *ostart, PieceDesc *desc) {
    __shared__ uint32_t sh[16];
    constexpr int DPT = 4;  // F <= 4096
    const uint32_t d0 = DPT * threadIdx.x;
    uint32_t c[DPT], x = 0;
#pragma unroll
    for (int u = 0; u < DPT; ++u) {
        c[u] = 0;
        uint32_t cp = 0;  // padded: each piece rounded up to even (team pair loads)
        if (d0 + u < F) {
            const uint32_t d = d0 + u;
            const int64_t b0 = rbase[d];
            PieceDesc &pd = desc[d];
            for (int r = 0; r < 8; ++r) {
                const uint32_t y = cum[(size_t)r * F + d];
                pd.ppre[r] = cp;
                pd.dl[r] = (uint32_t)(rbase[(size_t)r * F + d] - b0) - cp;
                pd.cend[r] = cp + y;
                c[u] += y;
                cp += (y + 1u) & ~1u;
            }
            pd.n = cp;
            pd.base0 = b0;
            ptot[d] = cp;
        }
        x += c[u];
    }
    uint32_t total;
    uint32_t e = block_excl_scan_1024(x, sh, total);
#pragma unroll
    for (int u = 0; u < DPT; ++u) {
        if (d0 + u < F) {
            tot[d0 + u] = c[u];
            ostart[d0 + u] = e;
            desc[d0 + u].ostart = e;
        }
        e += c[u];
    }
}

// Capacity C of one region, or 0 when the piece layout does not apply (the
// record positions of all 8 F regions plus the dump area must stay below
// 2^32).  Hashed privacy ids spread a level-1 digit's records evenly over
// the XCDs' static tile shares; 25 % + 4096 records of slack, an overflow
// redoes the level with the histogram path (DPG_DEBUG_PIECE_CAP: a test
// hook forcing a smaller capacity).
uint32_t piece_capacity(int64_t n, uint32_t F, int64_t sub) {
    double c = 1.25 * (double)n / (8.0 * F) + 4096.0;
    if (const char *e = std::getenv("DPG_DEBUG_PIECE_CAP")) c = std::max(2.0, std::atof(e));
    const double slots = c * 8.0 * F + (double)sub;
    if (slots >= 4294967295.0) return 0;
    return (uint32_t)c & ~1u;  // even: the team reads pieces by 16-byte pairs
}

template <class R, int IPT, int FMAX, int NT = kScatThreads>
int run_level1_pieces(dpg_ctx *ctx, hipStream_t s, const SrcSoAKey<R, true> &src, int64_t n,
                      uint32_t F, uint32_t bits, uint32_t C, R *out, Control *ctl,
                      PieceTab *pt, uint32_t *host_tot) {
    int st = DPG_OK;
    const int64_t sub = (int64_t)NT * IPT;
    const uint32_t nt = (uint32_t)((n + sub - 1) / sub);
    WS(tiles, TileDesc, "pieces.tiles", nt);
    WS(stb, uint32_t, "pieces.stb", 1);
    WS(snt, uint32_t, "pieces.snt", 1);
    WS(rbase, int64_t, "pieces.rbase", (size_t)8 * F);
    WS(cum, uint32_t, "pieces.cum", (size_t)8 * F);
    WS(tot, uint32_t, "pieces.tot", F);
    WS(ptot, uint32_t, "pieces.ptot", F);
    WS(ostart, int64_t, "pieces.ostart", F);
    WS(pdesc, PieceDesc, "pieces.desc", F);
    HIP_TRY(hipMemsetAsync(cum, 0, (size_t)8 * F * 4, s));
    HIP_TRY(hipMemsetAsync(&ctl->ntiles[0], 0, 4, s));
    stage(ctx, s, "partition1:pieces");
    k_region_base<<<(8 * F + 255) / 256, 256, 0, s>>>(rbase, F, C);
    LAUNCH_CHECK();
    k_build_tiles_single<<<(nt + 255) / 256, 256, 0, s>>>(n, sub, 1u, tiles, stb, snt,
                                                         &ctl->ntiles[0], XcdQueues{});
    LAUNCH_CHECK();
    using Src = SrcSoAKey<R, true>;
    constexpr size_t lds = scatter_lds<Src, R, IPT, FMAX, NT>();
    // (kScatThreads / NT) workgroups per CU
    static_assert(lds <= (size_t)160 * 1024 * NT / kScatThreads - 512, "scatter LDS");
    if (F > (uint32_t)FMAX) return fail(ctx, DPG_ERR_HIP, "internal: piece level fan-out too large");
    auto kern = k_scatter<Src, R, IPT, FMAX, false, NT>;
    if (bits <= (uint32_t)agg_bits()) return fail(ctx, DPG_ERR_HIP, "internal: piece level fan-out");
    (void)set_func_attr((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    // one 1024-thread workgroup per CU, or two of 512 (whose load, ranking
    // and write-out phases interleave)
    const uint32_t gs = std::min<uint32_t>(nt, (uint32_t)ctx->n_cu * (kScatThreads / NT));
    if (int r = scat_phase_begin(ctx, s)) return r;
    kern<<<gs, NT, lds, s>>>(src, tiles, &ctl->ntiles[0], F, bits, nullptr, rbase, out,
                             XcdQueues{}, nullptr, nullptr, nullptr, 1u, cum, C,
                             (uint32_t)((uint64_t)8 * F * C), &ctl->err);
    LAUNCH_CHECK();
    if (int r = scat_phase_end(ctx, s, "partition1:pieces", gs)) return r;
    k_piece_totals<<<1, 1024, 0, s>>>(cum, rbase, F, tot, ptot, ostart, pdesc);
    LAUNCH_CHECK();
    // totals and the error word reach the host for the overflow / team checks
    if (!ctx->tot_ev && hipEventCreateWithFlags(&ctx->tot_ev, hipEventDisableTiming) != hipSuccess)
        return fail(ctx, DPG_ERR_HIP, "hipEventCreate (totals)");
    HIP_TRY(hipMemcpyAsync(host_tot, tot, (size_t)F * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(host_tot + kPinErr, &ctl->err, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipEventRecord(ctx->tot_ev, s));
    *pt = PieceTab{rbase, cum, tot, ptot, ostart, F, pdesc};
    return DPG_OK;
}

// Level 2 by teams of workgroups (dpg_team.h): S level-1 buckets; pt: the
// buckets are the pieces of the histogram-free level 1.  Buckets whose
// member share exceeds sub_cap records are skipped by the single-round
// launch and done by a second, multi-round launch (k_part2_team kMulti), run
// only when the host's level-1 totals (max_bucket) say one may exist.
template <class R>
int run_team_level2(dpg_ctx *ctx, hipStream_t s, const SrcAoS<R> &src, uint32_t S, uint32_t F2,
                    const int64_t *seg_start, const uint32_t *seg_cnt, R *out, Control *ctl,
                    int64_t **base_out, uint32_t **tot_out, const PieceTab *pt,
                    uint64_t max_bucket) {
    int st = DPG_OK;
    const uint32_t F = kTeamF;
    const size_t words = (size_t)8 * 3 * F + 8 * kTeamArriveStride + 32;
    WS(tw, uint32_t, "team.sync", words);
    WS(base, int64_t, "partition2.base", (size_t)S * F2);
    WS(tot, uint32_t, "partition2.tot", (size_t)S * F2);
    HIP_TRY(hipMemsetAsync(tw, 0, words * 4, s));
    uint32_t *abort_flag = tw + (size_t)8 * 3 * F + 8 * kTeamArriveStride;
    const TeamSync ts{tw, tw + (size_t)8 * 3 * F, abort_flag, &ctl->err};
    if (std::getenv("DPG_DEBUG_TEAM_ABORT")) {
        // test hook: the team gives up at its first barrier, as after a
        // timeout (abort flag and err bit 8), so the host redoes level 2
        const uint32_t one = 1;
        UPLOAD(abort_flag, &one, 4);
        k_set_bits<<<1, 1, 0, s>>>(&ctl->err, 8u);
        LAUNCH_CHECK();
    }
    // records per member per round (test hook DPG_DEBUG_TEAM_SUB: a smaller,
    // even cap, so that small inputs take the multi-round path)
    uint32_t sub_cap = (uint32_t)kTeamSub;
    if (const char *e = std::getenv("DPG_DEBUG_TEAM_SUB"))
        sub_cap = std::min<uint32_t>(sub_cap, std::max<uint32_t>(2, (uint32_t)std::atoi(e)) & ~1u);
    const uint32_t T = (uint32_t)ctx->n_cu / 8;
    // a member's share: ceil(n / T) (+ 1, even, with up to 8 slots of piece padding)
    const bool multi = (max_bucket + 8 + T - 1) / T + 2 > sub_cap;
    const void *k = pt ? (const void *)k_part2_team<R, true> : (const void *)k_part2_team<R, false>;
    (void)set_func_attr(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)team_lds<R>());
    stage(ctx, s, "partition2:team");
    if (pt)
        k_part2_team<R, true><<<(unsigned)ctx->n_cu, kScatThreads, team_lds<R>(), s>>>(
            src, seg_start, seg_cnt, S, F2, out, base, tot, ts, *pt, sub_cap);
    else
        k_part2_team<R, false><<<(unsigned)ctx->n_cu, kScatThreads, team_lds<R>(), s>>>(
            src, seg_start, seg_cnt, S, F2, out, base, tot, ts, PieceTab{}, sub_cap);
    LAUNCH_CHECK();
    if (multi) {
        // the oversized buckets, in rounds; fresh team counters (the
        // abort flag keeps its value: a timed-out first launch is redone
        // anyway, err bit 8)
        stage(ctx, s, "partition2:team_multi");
        HIP_TRY(hipMemsetAsync(tw, 0, ((size_t)8 * 3 * F + 8 * kTeamArriveStride) * 4, s));
        const void *km = pt ? (const void *)k_part2_team<R, true, true>
                            : (const void *)k_part2_team<R, false, true>;
        (void)set_func_attr(km, hipFuncAttributeMaxDynamicSharedMemorySize, (int)team_lds<R>());
        if (pt)
            k_part2_team<R, true, true><<<(unsigned)ctx->n_cu, kScatThreads, team_lds<R>(), s>>>(
                src, seg_start, seg_cnt, S, F2, out, base, tot, ts, *pt, sub_cap);
        else
            k_part2_team<R, false, true><<<(unsigned)ctx->n_cu, kScatThreads, team_lds<R>(), s>>>(
                src, seg_start, seg_cnt, S, F2, out, base, tot, ts, PieceTab{}, sub_cap);
        LAUNCH_CHECK();
    }
    *base_out = base;
    *tot_out = tot;
    return DPG_OK;
}

template <class R>
int pipeline(dpg_ctx *ctx, hipStream_t s, const int64_t *pid, const int64_t *pk,
             const double *value, int64_t n, const dpg_bound_params *p, const dpg_partials *out,
             Control *ctl, const Plan &pl, int64_t pid_min, uint64_t U, uint32_t ib, PaOut *pa) {
    int st = DPG_OK;
    const bool var = (p->metric_mask & (DPG_M_MEAN | DPG_M_VARIANCE)) != 0;
    const Fmt f{ib, pl.pkbits, pl.kbits, pl.b1};
    const HashK H = make_hash(pl.kbits);
    // ---- level 1: SoA -> records bucketed by the top b1 hash bits
    const uint32_t F1 = 1u << pl.b1;
    SrcSoAKey<R> s1{pid, pk, p->public_mask, pl.P, pid_min, U, H, f,
                    low_mask(pl.kbits - pl.b1 + pl.pkbits), pl.kbits - pl.b1, &ctl->err};
    s1.value = value;  // read by R16 sources only
    int64_t *bstart = nullptr;
    uint32_t *bcnt = nullptr;
#ifndef DPG_L1_XCD
#define DPG_L1_XCD 0
#endif
#ifndef DPG_L1_SUBS
#define DPG_L1_SUBS 1
#endif
#ifndef DPG_L2_SUBS
#define DPG_L2_SUBS 1
#endif
    // debug knobs for same-box experiments: XCD-local level 1, sub-tiles per
    // XCD-local tile
    auto env_int = [](const char *name, int dflt) {
        const char *e = std::getenv(name);
        return e ? std::atoi(e) : dflt;
    };
    const bool l1_xcd = env_int("DPG_L1_XCD", DPG_L1_XCD) != 0;
    const int l1_subs = env_int("DPG_L1_SUBS", DPG_L1_SUBS);
    const int l2_subs = env_int("DPG_L2_SUBS", DPG_L2_SUBS);
// grouped XCD-local levels (run_level_grouped; same-box A/B, config 2:
// level-1 hist + scatter 1.60 + 9.35 -> 1.43 + 7.8 ms, level-2 hist 2.03 ->
// 1.69 ms, level-2 scatter unchanged)
#ifndef DPG_L1_GRP
#define DPG_L1_GRP 1
#endif
#ifndef DPG_L2_GRP
#define DPG_L2_GRP 1
#endif
    const bool l1_grp = env_int("DPG_L1_GRP", DPG_L1_GRP) != 0;
    const bool l2_grp = env_int("DPG_L2_GRP", DPG_L2_GRP) != 0;
    const uint32_t shift2 = pl.pkbits + (pl.kbits - pl.b1) - pl.b2;
    // level 2 by teams of workgroups (dpg_team.h, no histogram pass): 8-byte
    // records, an 11-bit level 2, every workgroup of a one-per-CU launch
    // resident, and -- checked on the level-1 totals, which reach the host
    // while the level-1 scatter runs -- every level-1 bucket within a team's
    // registers.  DPG_TEAM_L2=0: the grouped histogram path.
    const uint32_t team_T = (uint32_t)ctx->n_cu / 8;
    const bool backoff = ctx->team_backoff > 0;
    if (backoff) {
        --ctx->team_backoff;
        stage(ctx, s, "team_backoff");  // visible in the stage times (bench lines)
    }
    bool team = sizeof(R) == 8 && pl.b2 >= 6 && pl.b2 <= kMaxB1 && ctx->n_cu % 8 == 0 && team_T > 0 && l1_grp &&
                env_int("DPG_TEAM_L2", 1) != 0 && !backoff;
    if constexpr (sizeof(R) != 8) team = false;
    if constexpr (sizeof(R) == 8) if (team) {
        int occ = 0;
        const void *tk = (const void *)k_part2_team<R>;
        (void)set_func_attr(tk, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)team_lds<R>());
        team = occ_query(&occ, tk, kScatThreads,
                                                            team_lds<R>()) == hipSuccess &&
               occ >= 1;
    }
    if (team && !ctx->pin_tot &&
        hipHostMalloc((void **)&ctx->pin_tot, (size_t)4 * (kPinErr + 64), hipHostMallocDefault) != hipSuccess) {
        ctx->pin_tot = nullptr;
        team = false;
    }
    // level 1 without a histogram pass (k_scatter's piece mode, dpg_team.h
    // PieceTab): 8-byte records whose level 2 runs by teams; every XCD
    // appends to fixed-capacity regions, so recA holds 8 F1 regions of
    // `pcap` records (+ a dump area).  The default since round 5
    // (DPG_L1_PIECES=0: the histogram path): with the team level 2 loading
    // the next bucket's pieces during its barrier and write-out, same-box
    // A/B at config 2 22.07-22.26 -> 21.42-21.44 ms per step (level 1 1.46 +
    // 7.08 -> 7.35 ms, team 4.42-4.49 -> 4.93 ms; profiles/r5/r5d_ab.txt).
    // Round 4, without that prefetch, measured it a net loss (team 5.1 ->
    // 6.8 ms).
    constexpr int kIptPc = DPG_IPT_PC;
    // two 512-thread workgroups per CU for the 2048-digit piece level
    // (DPG_PC_HALF=1)
    const bool pc_half = F1 <= 2048 && env_int("DPG_PC_HALF", DPG_PC_HALF) != 0;
    const int64_t subPc = (int64_t)(pc_half ? kScatThreads / 2 : kScatThreads) *
                          (F1 > 2048 ? kIptL1W : kIptPc);
    uint32_t pcap = 0;
    bool pieces = false;
    if constexpr (sizeof(R) == 8) {
        if (team && env_int("DPG_L1_PIECES", 1) != 0 && n >= ((int64_t)1 << 22) &&
            pl.b1 > (uint32_t)agg_bits()) {
            pcap = piece_capacity(n, F1, subPc);
            pieces = pcap > 0;
        }
    }
    // (the histogram path may redo level 1 into the same buffer: >= n)
    WS(recA, R, "recA", pieces ? std::max<int64_t>(n, (int64_t)8 * F1 * pcap + subPc) : n);
    WS(recB, R, "recB", n);
    int64_t *bstart1 = nullptr;
    uint32_t *bcnt1 = nullptr;
    auto level1_std = [&](bool with_tot) -> int {
        if constexpr (sizeof(R) == 8) {
            if (F1 > 2048)  // a 12-bit level 1 (kMaxB1W)
                return run_level<SrcSoAKey<R>, R, kIptL1W, 4096>(
                    ctx, s, s1, 1u, nullptr, nullptr, &ctl->n_scalar, n, F1, pl.b1, recA,
                    "partition1", &bstart1, &bcnt1, &ctl->ntiles[0], nullptr, l1_xcd, l1_subs,
                    l1_grp, with_tot ? ctx->pin_tot : nullptr);
        }
        return run_level<SrcSoAKey<R>, R, Ipt<R>::L1, 2048>(
            ctx, s, s1, 1u, nullptr, nullptr, &ctl->n_scalar, n, F1, pl.b1, recA, "partition1",
            &bstart1, &bcnt1, &ctl->ntiles[0], nullptr, l1_xcd, l1_subs, l1_grp,
            with_tot ? ctx->pin_tot : nullptr);
    };
    PieceTab ptab{};
    uint64_t max_bucket = 0;  // the largest level-1 bucket (team launches)
    int r = DPG_OK;
    if constexpr (sizeof(R) == 8) {
        if (pieces) {
            SrcSoAKey<R, true> sp{pid, pk, p->public_mask, pl.P, pid_min, U, H, f,
                                  low_mask(pl.kbits - pl.b1 + pl.pkbits), pl.kbits - pl.b1,
                                  &ctl->err};
            r = F1 > 2048 ? run_level1_pieces<R, kIptL1W, 4096>(ctx, s, sp, n, F1, pl.b1, pcap, recA,
                                                               ctl, &ptab, ctx->pin_tot)
                : pc_half ? run_level1_pieces<R, kIptPc, 2048, kScatThreads / 2>(
                                ctx, s, sp, n, F1, pl.b1, pcap, recA, ctl, &ptab, ctx->pin_tot)
                          : run_level1_pieces<R, kIptPc, 2048>(ctx, s, sp, n, F1, pl.b1, pcap, recA,
                                                               ctl, &ptab, ctx->pin_tot);
            if (r) return r;
            HIP_TRY(hipEventSynchronize(ctx->tot_ev));
            for (uint32_t d = 0; d < F1; ++d) max_bucket = std::max<uint64_t>(max_bucket, ctx->pin_tot[d]);
            const bool over = (ctx->pin_tot[kPinErr] & 16u) != 0;
            // (a bucket over the team's single-round capacity takes the
            // multi-round team launch, run_team_level2)
            if (over) {
                std::fprintf(stderr, "[dpg] histogram-free level 1: a region overflowed; redone "
                                     "with the histogram path\n");
                HIP_TRY(hipMemsetAsync(&ctl->err, 0, 4, s));
                pieces = false;
                max_bucket = 0;
            }
        }
    }
    if (!pieces) {
        r = level1_std(team);
        if (r) return r;
        if (team) {
            HIP_TRY(hipEventSynchronize(ctx->tot_ev));
            for (uint32_t d = 0; d < F1; ++d) max_bucket = std::max<uint64_t>(max_bucket, ctx->pin_tot[d]);
        }
    }
    bstart = bstart1;
    bcnt = bcnt1;
    const R *cur = recA;
    uint32_t B = F1;
    auto level2_grouped = [&]() -> int {
        // ---- level 2: next b2 hash bits inside every level-1 bucket
        const uint32_t F2 = 1u << pl.b2;
        SrcAoS<R> s2{recA, f, shift2, F2 - 1};
// Level 2 in XCD-local mode: one-sub-tile tiles, all tiles of a level-1
// bucket served by one XCD's workgroups at the same time, so the partial
// lines of their adjacent runs merge in that XCD's L2 before write-back
// (same-box A/B, config 2: level-2 scatter 7.0-7.4 -> 4.4-4.8 ms, hist +0.25
// ms).  Level 1 in the same mode (tile groups per XCD) measured a net loss:
// scatter -1.0 ms, hist +1.35 ms for 81K tiles.
#ifndef DPG_L2_XCD
#define DPG_L2_XCD 1
#endif
        int r = pl.b2 > 11
                ? run_level<SrcAoS<R>, R, Ipt<R>::LW, 4096>(ctx, s, s2, F1, bstart1, bcnt1, nullptr, n,
                                                             F2, pl.b2, recB, "partition2", &bstart,
                                                             &bcnt, &ctl->ntiles[1], nullptr,
                                                             DPG_L2_XCD != 0, l2_subs, l2_grp)
                : run_level<SrcAoS<R>, R, Ipt<R>::LN, 2048>(ctx, s, s2, F1, bstart1, bcnt1, nullptr, n,
                                                             F2, pl.b2, recB, "partition2", &bstart,
                                                             &bcnt, &ctl->ntiles[1], nullptr,
                                                             DPG_L2_XCD != 0, l2_subs, l2_grp);
        return r;
    };
    if (pl.b2 > 0) {
        const uint32_t F2 = 1u << pl.b2;
        if constexpr (sizeof(R) == 8) {
            if (team) {
                SrcAoS<R> s2{recA, f, shift2, F2 - 1};
                r = run_team_level2<R>(ctx, s, s2, F1, F2, bstart1, bcnt1, recB, ctl, &bstart, &bcnt,
                                       pieces ? &ptab : nullptr, max_bucket);
            }
        }
        if (!team) {
            r = level2_grouped();
        }
        if (r) return r;
        cur = recB;
        B = F1 * F2;
    }
    BoundParams bp = to_bound(p, stream_seed(ctx->seed, p->nonce));
    bp.fmt = f;
    bp.hash = H;
    bp.pid_min = pid_min;
    bp.value = value;
    bp.err = &ctl->err;
    const bool key32 = pl.pkbits <= 21;  // (pid slot < 2^10) << pkbits | pk < 2^31
    auto bound = [&]() -> int {
        if (pa)
            return key32 ? bound_and_reduce<R, uint32_t, ItemPA>(ctx, s, pl, cur, bstart, bcnt, B, bp,
                                                                 n, out, ctl, pa)
                         : bound_and_reduce<R, uint64_t, ItemPA>(ctx, s, pl, cur, bstart, bcnt, B, bp,
                                                                 n, out, ctl, pa);
        if constexpr (sizeof(R) == 16) {
            return fail(ctx, DPG_ERR_HIP, "internal: R16 outside the pre-aggregate");
        } else {
            // MEAN / VARIANCE without SUM (and without per-partition sum
            // clipping): 24-byte items with the normalised moments only
            if (var && !(p->metric_mask & DPG_M_SUM) && p->sum_mode != DPG_SUM_CLIP_PARTITION)
                return key32 ? bound_and_reduce<R, uint32_t, ItemV>(ctx, s, pl, cur, bstart, bcnt, B,
                                                                    bp, n, out, ctl, nullptr)
                             : bound_and_reduce<R, uint64_t, ItemV>(ctx, s, pl, cur, bstart, bcnt, B,
                                                                    bp, n, out, ctl, nullptr);
            if (var)
                return key32 ? bound_and_reduce<R, uint32_t, Item32>(ctx, s, pl, cur, bstart, bcnt, B,
                                                                     bp, n, out, ctl, nullptr)
                             : bound_and_reduce<R, uint64_t, Item32>(ctx, s, pl, cur, bstart, bcnt, B,
                                                                     bp, n, out, ctl, nullptr);
            return key32 ? bound_and_reduce<R, uint32_t, Item16>(ctx, s, pl, cur, bstart, bcnt, B, bp,
                                                                 n, out, ctl, nullptr)
                         : bound_and_reduce<R, uint64_t, Item16>(ctx, s, pl, cur, bstart, bcnt, B, bp,
                                                                 n, out, ctl, nullptr);
        }
    };
    r = bound();
    if (r == kRedoLevel2) {
        // a team barrier timed out (workgroups not co-resident): level 2 again
        // with the histogram path, the chunk counters reset
        std::fprintf(stderr, "[dpg] team level 2 timed out; redone with the histogram path "
                             "(and on this context for the next %u calls)\n",
                     ctx->team_backoff_next);
        ctx->team_backoff = ctx->team_backoff_next;
        if (const char *e = std::getenv("DPG_DEBUG_TEAM_BACKOFF"))  // test hook
            ctx->team_backoff = (uint32_t)std::max(0, std::atoi(e));
        ctx->team_backoff_next = std::min<uint32_t>(2 * ctx->team_backoff_next, 4096);
        // a stage of its own, so that stage times (bench lines) show the redo
        stage(ctx, s, "partition2:team_redo");
        HIP_TRY(hipMemsetAsync(&ctl->err, 0, 4, s));
        HIP_TRY(hipMemsetAsync(&ctl->n_chunks, 0,
                               offsetof(Control, pid_lo) - offsetof(Control, n_chunks), s));
        if (pieces) {
            // the grouped level 2 reads a contiguous level 1
            r = level1_std(false);
            if (r) return r;
            pieces = false;
        }
        r = level2_grouped();
        if (r) return r;
        r = bound();
        if (r == kRedoLevel2) return fail(ctx, DPG_ERR_HIP, "internal: level-2 redo flagged again");
    }
    return r;
}

// dpg_bound_aggregate / dpg_preaggregate after argument checks: pid range,
// level plan, record format.
int aggregate_impl(dpg_ctx *ctx, const int64_t *pid, const int64_t *pk, const double *value,
                   int64_t n, const dpg_bound_params *p, dpg_partials *out, PaOut *pa,
                   hipStream_t s) {
    int st = DPG_OK;
    const int64_t P = p->n_partitions;
    WS(ctl, Control, "control", 1);
    ctx->last_err = &ctl->err;
    HIP_TRY(hipMemsetAsync(ctl, 0, sizeof(Control), s));
    k_set_i64<<<1, 1, 0, s>>>(&ctl->n_scalar, n);
    LAUNCH_CHECK();
    // ---- privacy-id range
    int64_t pid_min = p->pid_min;
    uint64_t U = (uint64_t)p->pid_count;
    if (U == 0) {
        stage(ctx, s, "pidrange");
        const unsigned long long init[2] = {~0ull, 0ull};
        UPLOAD(&ctl->pid_lo, init, 16);
        const int64_t blocks = std::min<int64_t>((n + 255) / 256, (int64_t)ctx->n_cu * 8);
        k_pid_minmax<<<(unsigned)blocks, 256, 0, s>>>(pid, n, &ctl->pid_lo, &ctl->pid_hi);
        LAUNCH_CHECK();
        unsigned long long h[2];
        HIP_TRY(hipMemcpyAsync(h, &ctl->pid_lo, 16, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        const int64_t lo = (int64_t)(h[0] ^ 0x8000000000000000ull);
        const int64_t hi = (int64_t)(h[1] ^ 0x8000000000000000ull);
        const uint64_t span = (uint64_t)hi - (uint64_t)lo;
        if (span >= (1ull << 32))
            return fail(ctx, DPG_ERR_KEY_RANGE, "privacy ids span more than 2^32 values");
        pid_min = lo;
        U = span + 1;
    }
    // ---- level plan: hash bits so that fine buckets average ~target records
    Plan pl;
    pl.P = P;
    pl.kbits = std::max<uint32_t>(1, bits_for(U));
    pl.pkbits = std::max<uint32_t>(1, bits_for((uint64_t)P));
    uint32_t target = ctx->bucket_target ? ctx->bucket_target : kBucketTarget;
    if (const char *e = std::getenv("DPG_DEBUG_TARGET")) target = (uint32_t)std::max(1, std::atoi(e));
    // at most 7 pid hash bits may stay below a fine bucket (direct pid slots
    // of a small chunk: kWCq = 128), hence the lower bound kbits - 7
    uint32_t bits_total = bits_for((uint64_t)((n + target - 1) / target));
    bits_total = std::max<uint32_t>(bits_total, pl.kbits > 7 ? pl.kbits - 7 : 0);
    bits_total = std::max<uint32_t>(1, std::min<uint32_t>(bits_total, kMaxB1 + kMaxB2));
    bits_total = std::min<uint32_t>(bits_total, pl.kbits);
    // one level up to 11 bits; beyond, the smaller half first (level 1 reads
    // 16 B per record, so its runs should be the longer ones)
    pl.b1 = bits_total <= kMaxB1 ? bits_total : bits_total / 2;
    // level-1 buckets within the team level 2's single round (T members x
    // kTeamSub records, 5 % slack): e.g. N = 1e9 with 2^20 privacy-id hash
    // values (20 bits: 10 + 10 by halves) takes 11 + 9, whose ~490K-record
    // buckets fit, instead of 1024 buckets of ~980K that all need the
    // multi-round team launch (applies when level 2 keeps >= 6 bits)
    if (bits_total > kMaxB1 && ctx->n_cu >= 8) {
        const double cap = 0.95 * (double)(ctx->n_cu / 8) * (double)kTeamSub;
        uint32_t need = 0;
        while (need < kMaxB1 && (double)n / (double)(1u << need) > cap) ++need;
        const uint32_t b1 = std::min<uint32_t>(std::max<uint32_t>(pl.b1, need), bits_total - 6);
        if (b1 <= kMaxB1 && b1 > pl.b1) pl.b1 = b1;
    }
    pl.b2 = bits_total - pl.b1;
    if (const char *e = std::getenv("DPG_DEBUG_B1")) {  // debug: level split experiments
        const uint32_t b1 = (uint32_t)std::atoi(e);
        if (b1 >= 1 && b1 <= kMaxB1 && b1 <= bits_total && bits_total - b1 <= kMaxB2) {
            pl.b1 = b1;
            pl.b2 = bits_total - b1;
        }
    }
    pl.plb = pl.kbits - bits_total;
    const uint32_t ib = std::max<uint32_t>(1, bits_for((uint64_t)n));
    // 23-bit plans (N > 2^30): 12 + 11 bits instead of 11 + 12 when the
    // records are then 8 bytes (not for the utility pre-aggregate's R16
    // records), so that level 1 runs without a histogram pass and level 2
    // by teams, as at smaller N
    const char *b1w = std::getenv("DPG_B1W");  // "0": keep 11 + 12 (A/B)
    if (!pa && bits_total == kMaxB1 + 12 && std::getenv("DPG_DEBUG_B1") == nullptr &&
        !(b1w && std::atoi(b1w) == 0) &&
        (pl.kbits - kMaxB1W) + pl.pkbits + ib <= 64) {
        pl.b1 = kMaxB1W;
        pl.b2 = bits_total - kMaxB1W;
    }
    const bool r8 = (pl.kbits - pl.b1) + pl.pkbits + ib <= 64;
    // the utility pre-aggregate sums every record's value: R16 records carry
    // it (DPG_PA_GATHER=1: gather by index as the bounded paths do)
    if (r8 && pa && value && std::getenv("DPG_PA_GATHER") == nullptr)
        return pipeline<R16>(ctx, s, pid, pk, value, n, p, out, ctl, pl, pid_min, U, ib, pa);
    if (r8) return pipeline<R8>(ctx, s, pid, pk, value, n, p, out, ctl, pl, pid_min, U, ib, pa);
    return pipeline<R12>(ctx, s, pid, pk, value, n, p, out, ctl, pl, pid_min, U, ib, pa);
}

}  // namespace

namespace {

// ---------------------------------------------------------------- RCCL
// Resolved at first use from the librccl already in the process (a host
// such as PyTorch loads its own) or from the ROCm install; libdpg.so does
// not link it.
struct Rccl {
    bool tried = false, ok = false;
    ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*reduce_scatter)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t,
                                   ncclComm_t, hipStream_t) = nullptr;
    const char *(*error_string)(ncclResult_t) = nullptr;
};

Rccl &rccl() {
    static Rccl r;
    if (r.tried) return r;
    r.tried = true;
    void *h = nullptr;
    for (const char *name : {"librccl.so.1", "librccl.so"})
        if (!h) h = dlopen(name, RTLD_NOW | RTLD_NOLOAD);
    for (const char *name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
        if (!h) h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
    if (!h) return r;
    r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
    r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(h, "ncclCommInitRank");
    r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
    r.reduce_scatter = (decltype(r.reduce_scatter))dlsym(h, "ncclReduceScatter");
    r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
    r.ok = r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.reduce_scatter;
    return r;
}

std::string rccl_msg(ncclResult_t e) {
    const Rccl &r = rccl();
    return r.error_string ? std::string(r.error_string(e)) : "RCCL error " + std::to_string((int)e);
}

// Partials to the reduce-scatter layout and back.  Partition pk is owned by
// rank pk mod R at local index pk / R (interleaved ownership: hot low ids,
// e.g. an unpermuted Zipf key space, spread over every rank).  Rank r's block
// is B = A * S + 1 doubles: [array][S] for its partitions, zero padded past
// P, then the sender's internal-error flag, so that the sum over ranks
// delivers every rank the flags of all of them.  Integer arrays are exact in
// float64 below 2^53.
struct PackArrays {
    const void *a[5];
    int is_int[5];
    int n;
};

__global__ void k_pack_partials(PackArrays src, int64_t P, int64_t S, int nranks,
                                const uint32_t *err, double *pack) {
    const int64_t B = (int64_t)src.n * S + 1;
    const int64_t total = S * nranks;
    // k enumerates partition ids: the reads are coalesced, each wave's
    // stores form nranks runs
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < total;
         k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = k / nranks, r = k - i * nranks;
        for (int j = 0; j < src.n; ++j) {
            double v = 0.0;
            if (k < P)
                v = src.is_int[j] ? (double)static_cast<const int64_t *>(src.a[j])[k]
                                  : static_cast<const double *>(src.a[j])[k];
            pack[r * B + j * S + i] = v;
        }
    }
    if (blockIdx.x == 0)
        for (int r = threadIdx.x; r < nranks; r += blockDim.x)
            pack[r * B + (int64_t)src.n * S] = (err && (*err & 2u)) ? 1.0 : 0.0;
}

struct UnpackArrays {
    void *a[5];
    int is_int[5];
    int n;
};

// part: this rank's summed block; latches a nonzero error sum into `err`
// (the internal-error bit dpg_compact_kept checks)
__global__ void k_unpack_partials(const double *part, int64_t S, int64_t n_local,
                                  UnpackArrays dst, uint32_t *err) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && err && part[(int64_t)dst.n * S] != 0.0)
        atomicOr(err, 2u);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_local;
         i += (int64_t)gridDim.x * blockDim.x) {
        for (int j = 0; j < dst.n; ++j) {
            const double v = part[j * S + i];
            if (dst.is_int[j]) static_cast<int64_t *>(dst.a[j])[i] = (int64_t)llrint(v);
            else static_cast<double *>(dst.a[j])[i] = v;
        }
    }
}

__global__ void k_export_error(const uint32_t *err, double *dst) {
    *dst = (err && (*err & 2u)) ? 1.0 : 0.0;
}

__global__ void k_import_error(const double *src, int64_t n, uint32_t *err) {
    bool bad = false;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) bad |= src[i] != 0.0;
    if (bad) atomicOr(err, 2u);
}

// the word the next dpg_compact_kept checks: the last bounding's control
// word, or (a context that has not bounded yet) a word of its own
uint32_t *latch_word(dpg_ctx *ctx, hipStream_t s, int *status) {
    if (ctx->last_err) return const_cast<uint32_t *>(ctx->last_err);
    uint32_t *w = reinterpret_cast<uint32_t *>(ws(ctx, "comm.err", 4, status));
    if (!w) return nullptr;
    if (hipMemsetAsync(w, 0, 4, s) != hipSuccess) {
        *status = fail(ctx, DPG_ERR_HIP, "hipMemsetAsync (error word)");
        return nullptr;
    }
    ctx->last_err = w;
    return w;
}

}  // namespace

extern "C" {

dpg_ctx *dpg_ctx_create(int device, uint64_t seed) {
    if (hipSetDevice(device) != hipSuccess) return nullptr;
    dpg_ctx *c = new dpg_ctx();
    c->device = device;
    c->seed = seed;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->n_cu = prop.multiProcessorCount;
    return c;
}

void dpg_ctx_destroy(dpg_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->comm && rccl().ok) (void)rccl().comm_destroy(static_cast<ncclComm_t>(c->comm));
    for (auto &kv : c->bufs)
        if (kv.second.p) (void)hipFree(kv.second.p);
    for (auto e : c->events) (void)hipEventDestroy(e);
    for (auto &kv : c->stage_done) {
        (void)hipEventSynchronize(kv.second);
        (void)hipEventDestroy(kv.second);
    }
    if (c->stage_buf) (void)hipHostFree(c->stage_buf);
    if (c->tot_ev) (void)hipEventDestroy(c->tot_ev);
    if (c->pin_tot) (void)hipHostFree(c->pin_tot);
    delete c;
}

int dpg_last_error(dpg_ctx *c, char *buf, size_t len) {
    if (!c || !buf || len == 0) return DPG_ERR_INVALID_ARG;
    std::snprintf(buf, len, "%s", c->err.c_str());
    return DPG_OK;
}

int dpg_set_seed(dpg_ctx *c, uint64_t seed) {
    if (!c) return DPG_ERR_INVALID_ARG;
    c->seed = seed;
    return DPG_OK;
}

uint64_t dpg_stream_seed(uint64_t seed, uint64_t nonce) { return stream_seed(seed, nonce); }

int dpg_set_tuning(dpg_ctx *ctx, int32_t bucket_target, int32_t bucket_cap) {
    if (!ctx) return DPG_ERR_INVALID_ARG;
    if (bucket_target > 0) ctx->bucket_target = (uint32_t)bucket_target;
    if (bucket_cap > 0) ctx->bucket_cap = std::min<uint32_t>((uint32_t)bucket_cap, kBCap);
    return DPG_OK;
}

int dpg_bound_aggregate(dpg_ctx *ctx, const int64_t *pid, const int64_t *pk, const double *value,
                        int64_t n, const dpg_bound_params *p, dpg_partials *out, void *stream) {
    if (!ctx) return DPG_ERR_INVALID_ARG;
    if (!p || !out || n < 0 || (n > 0 && (!pid || !pk)))
        return fail(ctx, DPG_ERR_INVALID_ARG, "null argument");
    if (p->n_partitions <= 0 || p->n_partitions >= 0xFFFFFFFFll)
        return fail(ctx, DPG_ERR_INVALID_ARG, "n_partitions must be in [1, 2^32-1)");
    if (out->n_partitions != p->n_partitions || !out->rows || !out->count)
        return fail(ctx, DPG_ERR_INVALID_ARG, "partials must cover n_partitions");
    if (p->mode < 0 || p->mode > 2) return fail(ctx, DPG_ERR_INVALID_ARG, "bad mode");
    const bool per_pid = p->mode == DPG_MODE_PER_PRIVACY_ID;
    if (per_pid ? p->max_contributions <= 0
                : (p->max_partitions_contributed <= 0 || p->max_contributions_per_partition <= 0))
        return fail(ctx, DPG_ERR_INVALID_ARG, "contribution bounds must be positive");
    if (n >= 0xFFFFFFFFll) return fail(ctx, DPG_ERR_UNSUPPORTED, "n must be < 2^32 per device");
    if (p->pid_count < 0 || p->pid_count > (1ll << 32))
        return fail(ctx, DPG_ERR_INVALID_ARG, "pid_count must be in [0, 2^32]");
    const bool var = (p->metric_mask & (DPG_M_MEAN | DPG_M_VARIANCE)) != 0;
    const bool need_values = (p->metric_mask & (DPG_M_SUM | DPG_M_MEAN | DPG_M_VARIANCE)) != 0;
    if (need_values && n > 0 && !value)
        return fail(ctx, DPG_ERR_INVALID_ARG, "value array required for SUM/MEAN/VARIANCE");
    if (var && out->nsum == nullptr)
        return fail(ctx, DPG_ERR_INVALID_ARG, "MEAN/VARIANCE need nsum/nsq partials");
    if (need_values && !var && out->sum == nullptr)
        return fail(ctx, DPG_ERR_INVALID_ARG, "SUM needs sum partials");
    (void)hipSetDevice(ctx->device);
    hipStream_t s = (hipStream_t)stream;
    ctx->stage_names.clear();
    ctx->n_events_used = 0;
    ctx->last_stream = s;
    int st = DPG_OK;
    const int64_t P = p->n_partitions;
    stage(ctx, s, "begin");
    HIP_TRY(hipMemsetAsync(out->rows, 0, P * 8, s));
    HIP_TRY(hipMemsetAsync(out->count, 0, P * 8, s));
    if (out->sum) HIP_TRY(hipMemsetAsync(out->sum, 0, P * 8, s));
    if (out->nsum) HIP_TRY(hipMemsetAsync(out->nsum, 0, P * 8, s));
    if (out->nsq) HIP_TRY(hipMemsetAsync(out->nsq, 0, P * 8, s));
    if (n == 0) return DPG_OK;
    return aggregate_impl(ctx, pid, pk, value, n, p, out, nullptr, s);
}

int dpg_preaggregate(dpg_ctx *ctx, const int64_t *pid, const int64_t *pk, const double *value,
                     int64_t n, const dpg_bound_params *p, dpg_pair_entry *pairs,
                     int64_t capacity, int64_t *partition_start, int64_t *n_pairs, void *stream) {
    static_assert(sizeof(dpg_pair_entry) == sizeof(ItemPA), "dpg_pair_entry layout");
    if (!ctx) return DPG_ERR_INVALID_ARG;
    if (!p || !partition_start || !n_pairs || n < 0 || (n > 0 && (!pid || !pk || !pairs)))
        return fail(ctx, DPG_ERR_INVALID_ARG, "null argument");
    if (p->n_partitions <= 0 || p->n_partitions >= 0xFFFFFFFFll)
        return fail(ctx, DPG_ERR_INVALID_ARG, "n_partitions must be in [1, 2^32-1)");
    if (n >= 0x7FFFFFFFll)  // n_contributions shares a word with the leader bit
        return fail(ctx, DPG_ERR_UNSUPPORTED, "n must be < 2^31 per device");
    if (p->pid_count < 0 || p->pid_count > (1ll << 32))
        return fail(ctx, DPG_ERR_INVALID_ARG, "pid_count must be in [0, 2^32]");
    (void)hipSetDevice(ctx->device);
    hipStream_t s = (hipStream_t)stream;
    ctx->stage_names.clear();
    ctx->n_events_used = 0;
    ctx->last_stream = s;
    int st = DPG_OK;
    stage(ctx, s, "begin");
    *n_pairs = 0;
    if (n == 0) {
        HIP_TRY(hipMemsetAsync(partition_start, 0, (p->n_partitions + 1) * 8, s));
        return DPG_OK;
    }
    // no bounding: every pair kept, values summed unclipped
    dpg_bound_params q = *p;
    q.mode = DPG_MODE_CROSS_PARTITION;
    q.sum_mode = value ? DPG_SUM_CLIP_PARTITION : DPG_SUM_NONE;
    q.metric_mask = value ? (DPG_M_COUNT | DPG_M_SUM) : DPG_M_COUNT;
    q.max_partitions_contributed = 0x7FFFFFFF;
    q.max_contributions_per_partition = 0x7FFFFFFF;
    q.max_contributions = 0;
    q.min_sum_per_partition = -HUGE_VAL;
    q.max_sum_per_partition = HUGE_VAL;
    PaOut pa{reinterpret_cast<ItemPA *>(pairs), capacity, partition_start, 0};
    dpg_partials none{};
    const int rc = aggregate_impl(ctx, pid, pk, value, n, &q, &none, &pa, s);
    *n_pairs = pa.n_pairs;
    return rc;
}

int dpg_select_and_noise(dpg_ctx *ctx, const dpg_partials *in, const dpg_select_params *sel,
                         const dpg_noise_params *z, uint8_t *keep, double *out, void *stream) {
    if (!ctx) return DPG_ERR_INVALID_ARG;
    if (!in || !sel || !z || !keep || (!out && z->n_outputs > 0))
        return fail(ctx, DPG_ERR_INVALID_ARG, "null argument");
    if (z->n_outputs < 0 || z->n_outputs > 8)
        return fail(ctx, DPG_ERR_INVALID_ARG, "n_outputs must be in [0, 8]");
    if (sel->strategy != DPG_SELECT_NONE && sel->max_rows_per_privacy_id <= 0)
        return fail(ctx, DPG_ERR_INVALID_ARG, "max_rows_per_privacy_id must be positive");
    (void)hipSetDevice(ctx->device);
    hipStream_t s = (hipStream_t)stream;
    int st = DPG_OK;
    const int64_t P = in->n_partitions;
    if (P <= 0) return DPG_OK;
    SelectArgs a{};
    a.strategy = sel->strategy;
    a.table_len = sel->table_len;
    a.threshold = sel->threshold;
    a.noise_scale = sel->noise_scale;
    a.pre_threshold = sel->pre_threshold;
    a.max_rows = std::max<int64_t>(1, sel->max_rows_per_privacy_id);
    a.pk_offset = sel->pk_offset;
    a.pk_stride = sel->pk_stride > 0 ? sel->pk_stride : 1;
    a.public_mask = sel->public_mask;
    a.table = nullptr;
    if (sel->strategy == DPG_SELECT_TRUNCATED_GEOMETRIC) {
        if (sel->table_len <= 0 || !sel->keep_table)
            return fail(ctx, DPG_ERR_INVALID_ARG, "truncated geometric needs keep_table");
        WS(tab, double, "select.table", sel->table_len);
        UPLOAD(tab, sel->keep_table, sizeof(double) * sel->table_len);
        a.table = tab;
    }
    NoiseArgs na{};
    na.kind = z->noise_kind;
    na.family = z->family;
    na.slot_mask = z->slot_mask;
    na.n_out = z->n_outputs;
    for (int j = 0; j < 8; ++j) na.out_src[j] = std::min(4, std::max(0, z->out_src[j]));
    for (int j = 0; j < 4; ++j) na.scale[j] = z->scale[j];
    na.mid = z->mid;
    na.mean_const = z->mean_const;
    na.msq_const = z->msq_const;
    na.mean_const_value = z->mean_const_value;
    na.msq_const_value = z->msq_const_value;
    const int threads = 256;
    int64_t blocks = std::min<int64_t>((P + threads - 1) / threads, (int64_t)ctx->n_cu * 16);
    size_t lds = (a.table && a.table_len <= 4096) ? (size_t)a.table_len * 8 : 0;
    k_select_noise<<<(unsigned)blocks, threads, lds, s>>>(in->rows, in->count, in->sum, in->nsum,
                                                         in->nsq, P, a, na,
                                                         stream_seed(ctx->seed, sel->nonce), keep,
                                                         out);
    LAUNCH_CHECK();
    return DPG_OK;
}

int dpg_compact_kept(dpg_ctx *ctx, const uint8_t *keep, const double *out, int64_t P,
                     int32_t n_out, int64_t *kept_ids, double *kept_out, int64_t *n_kept,
                     void *stream) {
    if (!ctx) return DPG_ERR_INVALID_ARG;
    if (!keep || !kept_ids || !n_kept || (n_out > 0 && (!out || !kept_out)))
        return fail(ctx, DPG_ERR_INVALID_ARG, "null argument");
    (void)hipSetDevice(ctx->device);
    hipStream_t s = (hipStream_t)stream;
    int st = DPG_OK;
    if (P <= 0) {
        *n_kept = 0;
        return DPG_OK;
    }
    uint32_t nb = (uint32_t)((P + kCompactPerBlock - 1) / kCompactPerBlock);
    WS(bc, uint32_t, "compact.blocks", nb);
    WS(tot, int64_t, "compact.total", 1);
    k_compact_count<<<nb, kCompactThreads, 0, s>>>(keep, P, bc);
    LAUNCH_CHECK();
    k_compact_scan<<<1, 1024, 0, s>>>(bc, nb, tot);
    LAUNCH_CHECK();
    k_compact_write<<<nb, kCompactThreads, 0, s>>>(keep, out, P, n_out, bc, kept_ids, kept_out);
    LAUNCH_CHECK();
    HIP_TRY(hipMemcpyAsync(n_kept, tot, 8, hipMemcpyDeviceToHost, s));
    uint32_t err = 0;
    if (ctx->last_err) HIP_TRY(hipMemcpyAsync(&err, ctx->last_err, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (err & 2u) return fail(ctx, DPG_ERR_HIP, "internal hash-table error in bounding");
    return DPG_OK;
}

int dpg_compact_kept_async(dpg_ctx *ctx, const uint8_t *keep, const double *out, int64_t P,
                           int32_t n_out, int64_t *kept_ids, double *kept_out, int64_t *info,
                           void *stream) {
    if (!ctx) return DPG_ERR_INVALID_ARG;
    if (!keep || !kept_ids || !info || (n_out > 0 && (!out || !kept_out)))
        return fail(ctx, DPG_ERR_INVALID_ARG, "null argument");
    (void)hipSetDevice(ctx->device);
    hipStream_t s = (hipStream_t)stream;
    int st = DPG_OK;
    HIP_TRY(hipMemsetAsync(info, 0, 16, s));
    if (P > 0) {
        uint32_t nb = (uint32_t)((P + kCompactPerBlock - 1) / kCompactPerBlock);
        WS(bc, uint32_t, "compact.blocks", nb);
        k_compact_count<<<nb, kCompactThreads, 0, s>>>(keep, P, bc);
        LAUNCH_CHECK();
        k_compact_scan<<<1, 1024, 0, s>>>(bc, nb, info);
        LAUNCH_CHECK();
        k_compact_write<<<nb, kCompactThreads, 0, s>>>(keep, out, P, n_out, bc, kept_ids, kept_out);
        LAUNCH_CHECK();
    }
    // the error word as it stands now in stream order (the next bounding on
    // this context reuses it)
    if (ctx->last_err)
        HIP_TRY(hipMemcpyAsync(info + 1, ctx->last_err, 4, hipMemcpyDeviceToDevice, s));
    return DPG_OK;
}

int dpg_utility_analysis(dpg_ctx *ctx, const dpg_pair_entry *pairs,
                         const int64_t *partition_start, int64_t P, const dpg_ua_params *u,
                         double *raw, double *errors, double *keep, double *report,
                         int64_t *n_out, void *stream) {
    if (!ctx) return DPG_ERR_INVALID_ARG;
    if (!u || !partition_start || !raw || !errors || !u->configs || P <= 0)
        return fail(ctx, DPG_ERR_INVALID_ARG, "null argument");
    if (u->n_configs < 1 || u->n_configs > 64)
        return fail(ctx, DPG_ERR_INVALID_ARG, "n_configs must be in [1, 64]");
    if (!u->public_partitions && !keep)
        return fail(ctx, DPG_ERR_INVALID_ARG, "private partitions need the keep output");
    if (u->public_partitions && !u->public_mask)
        return fail(ctx, DPG_ERR_INVALID_ARG, "public partitions need public_mask");
    (void)hipSetDevice(ctx->device);
    hipStream_t s = (hipStream_t)stream;
    int st = DPG_OK;
    const int C = u->n_configs;
    UaArgs a{};
    a.n_configs = C;
    a.has_sum = (u->metric_mask & DPG_M_SUM) != 0;
    a.has_count = (u->metric_mask & DPG_M_COUNT) != 0;
    a.has_pid = (u->metric_mask & DPG_M_PRIVACY_ID_COUNT) != 0;
    a.n_metrics = a.has_sum + a.has_count + a.has_pid;
    a.P = P;
    // configurations and keep tables to the device
    std::vector<UaConfig> hc(C);
    std::vector<double> tabs;
    for (int i = 0; i < C; ++i) {
        const dpg_ua_config &x = u->configs[i];
        if (x.max_partitions_contributed <= 0 || x.max_contributions_per_partition <= 0)
            return fail(ctx, DPG_ERR_INVALID_ARG, "contribution bounds must be positive");
        UaConfig &y = hc[i];
        y.mpc = (double)x.max_partitions_contributed;
        y.mcpp = (double)x.max_contributions_per_partition;
        y.lo = x.min_sum_per_partition;
        y.hi = x.max_sum_per_partition;
        y.strategy = x.selection_strategy;
        y.pre_threshold = (int32_t)x.pre_threshold;
        y.threshold = x.threshold;
        y.scale = x.noise_scale;
        y.table_offset = 0;
        y.table_len = 0;
        if (!u->public_partitions && x.selection_strategy == DPG_SELECT_TRUNCATED_GEOMETRIC) {
            if (!x.keep_table || x.table_len <= 0)
                return fail(ctx, DPG_ERR_INVALID_ARG, "truncated geometric needs keep_table");
            // one copy of equal tables (a sweep repeats each l0's table)
            int64_t off = -1;
            for (int j = 0; j < i && off < 0; ++j)
                if (hc[j].table_len == x.table_len &&
                    std::equal(x.keep_table, x.keep_table + x.table_len,
                               tabs.begin() + hc[j].table_offset))
                    off = hc[j].table_offset;
            if (off < 0) {
                off = (int64_t)tabs.size();
                tabs.insert(tabs.end(), x.keep_table, x.keep_table + x.table_len);
            }
            y.table_offset = off;
            y.table_len = x.table_len;
        }
    }
    // selection classes: configurations with equal l0 and keep function share
    // the LDS keep-probability column and the normal-approximation pass of
    // k_ua_select
    std::vector<int32_t> cls(C), cls_rep;
    for (int i = 0; i < C; ++i) {
        int k = 0;
        for (; k < (int)cls_rep.size(); ++k) {
            const UaConfig &r = hc[cls_rep[k]], &y = hc[i];
            if (r.mpc == y.mpc && r.strategy == y.strategy && r.pre_threshold == y.pre_threshold &&
                r.table_offset == y.table_offset && r.table_len == y.table_len &&
                r.threshold == y.threshold && r.scale == y.scale)
                break;
        }
        if (k == (int)cls_rep.size()) cls_rep.push_back(i);
        cls[i] = k;
    }
    a.n_cls = (int32_t)cls_rep.size();
    // pi(0 .. npi - 1) per class in LDS: at least the exact PMF's 104
    // counts, at most 16 KB, and no further than the last count whose keep
    // probability is below 1 (ua_pi_range; beyond it the normal
    // approximation telescopes without reading pi): the smaller the table,
    // the more waves of k_ua_select share a CU
    int64_t top = 0;
    for (int k = 0; k < a.n_cls; ++k) {
        const UaConfig &r = hc[cls_rep[k]];
        const int64_t sh = r.pre_threshold > 0 ? r.pre_threshold - 1 : 0;
        // the bound is clamped in double before the conversion (an extreme
        // epsilon / delta gives a huge or non-finite threshold or scale, whose
        // conversion to int64 would be undefined): past the table cap, any
        // value gives the same npi
        auto cap_count = [](double x) -> int64_t {
            return std::isfinite(x) ? (int64_t)std::min(std::max(x, 0.0), (double)INT32_MAX)
                                    : (int64_t)INT32_MAX;
        };
        int64_t i1;
        if (r.strategy == DPG_SELECT_TRUNCATED_GEOMETRIC)
            i1 = r.table_len - 1 + sh;
        else if (r.strategy == DPG_SELECT_LAPLACE_THRESHOLD)
            i1 = cap_count(std::ceil(r.threshold + 37.5 * r.scale)) + sh;
        else
            i1 = cap_count(std::ceil(r.threshold + 8.5 * r.scale)) + sh;
        top = std::max(top, std::min<int64_t>(i1, INT32_MAX) + 1);
    }
    // (16 KB: the normal-approximation pass is latency-bound, and a table of
    // 32 KB held it at 5 waves per CU; counts past the table read pi from
    // the keep table in global memory)
    a.npi = (int32_t)std::max<int64_t>(
        kPgfB * kPgfNB, std::min<int64_t>(top, (16 * 1024 / 8) / a.n_cls));
    WS(dcls, int32_t, "ua.cls", C + cls_rep.size());
    std::vector<int32_t> hcls(cls);
    hcls.insert(hcls.end(), cls_rep.begin(), cls_rep.end());
    UPLOAD(dcls, hcls.data(), 4 * hcls.size());
    a.cls = dcls;
    a.cls_rep = dcls + C;
    WS(dcfg, UaConfig, "ua.cfg", C);
    UPLOAD(dcfg, hc.data(), sizeof(UaConfig) * C);
    a.cfg = dcfg;
    if (!tabs.empty()) {
        WS(dtab, double, "ua.tables", tabs.size());
        UPLOAD(dtab, tabs.data(), 8 * tabs.size());
        a.tables = dtab;
    }
    a.sample_mask = u->sample_mask;
    a.public_mask = u->public_partitions ? u->public_mask : nullptr;
    WS(mom, double, "ua.mom", (size_t)P * kUaMom * C);
    a.raw = raw;
    a.err = errors;
    a.mom = mom;
    a.keep = keep;
    // public partitions: every public row is added to (k_ua_public), so all
    // start from zero; private: only the rows of partitions split between
    // accumulate runs (k_ua_zero_split; DPG_UA_FULL_ZERO=1: the full fill,
    // for A/B runs)
    static const bool full_zero = std::getenv("DPG_UA_FULL_ZERO") != nullptr;
    if (u->public_partitions || full_zero) {
        HIP_TRY(hipMemsetAsync(raw, 0, (size_t)P * 2 * 8, s));
        HIP_TRY(hipMemsetAsync(errors, 0, (size_t)P * a.n_metrics * 5 * C * 8, s));
        HIP_TRY(hipMemsetAsync(mom, 0, (size_t)P * kUaMom * C * 8, s));
        if (keep) HIP_TRY(hipMemsetAsync(keep, 0, (size_t)P * C * 8, s));
    } else {
        const unsigned g = (unsigned)std::min<int64_t>((P + 3) / 4, (int64_t)ctx->n_cu * 8);
        k_ua_zero_split<<<g, 256, 0, s>>>(partition_start, a);
        LAUNCH_CHECK();
    }
    int64_t n = 0;
    HIP_TRY(hipMemcpyAsync(&n, partition_start + P, 8, hipMemcpyDeviceToHost, s));
    if (n_out) *n_out = 0;
    HIP_TRY(hipStreamSynchronize(s));
    stage(ctx, s, "ua.accumulate");
    if (n > 0) {
        const int64_t runs = (n + kUaRun - 1) / kUaRun;
        if (runs >= 0x7FFFFFFF) return fail(ctx, DPG_ERR_UNSUPPORTED, "too many pairs");
        using AccK = void (*)(const ItemPA *, const int64_t *, int64_t, UaArgs);
        static const AccK acc_k[8] = {
            k_ua_accumulate<false, false, false>, k_ua_accumulate<false, false, true>,
            k_ua_accumulate<false, true, false>,  k_ua_accumulate<false, true, true>,
            k_ua_accumulate<true, false, false>,  k_ua_accumulate<true, false, true>,
            k_ua_accumulate<true, true, false>,   k_ua_accumulate<true, true, true>};
        const AccK kern = acc_k[(a.has_sum ? 4 : 0) | (a.has_count ? 2 : 0) | (a.has_pid ? 1 : 0)];
        kern<<<(unsigned)runs, 64, 0, s>>>(reinterpret_cast<const ItemPA *>(pairs),
                                           partition_start, n, a);
        LAUNCH_CHECK();
    }
    if (u->public_partitions) {
        const unsigned g = (unsigned)std::min<int64_t>(P, (int64_t)ctx->n_cu * 16);
        k_ua_public<<<g, 64, 0, s>>>(a);
        LAUNCH_CHECK();
    } else if (n > 0) {
        stage(ctx, s, "ua.select");
        const size_t lds = (size_t)a.npi * a.n_cls * 8;
        // the exact-PMF partitions (<= 100 pairs) in a pass of their own
        // with a 104-count pi table (its LDS share allows several times the
        // resident waves of the full table), then the others
        const size_t lds_x = (size_t)kPgfB * kPgfNB * a.n_cls * 8;
        auto launch = [&](auto kern, size_t l) {
            (void)set_func_attr((const void *)kern,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)l);
            int occ = 0;
            if (occ_query(&occ, (const void *)kern, 64, l) !=
                    hipSuccess || occ < 1)
                occ = 4;
            const unsigned g = (unsigned)std::min<int64_t>(P, (int64_t)ctx->n_cu * occ);
            kern<<<g, 64, l, s>>>(reinterpret_cast<const ItemPA *>(pairs), partition_start, a);
        };
        // lanes per selection class of the exact PMF (dpg_utility.h)
        if (a.n_cls <= 8) launch(k_ua_select<8, 1>, lds_x), launch(k_ua_select<8, 2>, lds);
        else if (a.n_cls <= 16) launch(k_ua_select<4, 1>, lds_x), launch(k_ua_select<4, 2>, lds);
        else if (a.n_cls <= 32) launch(k_ua_select<2, 1>, lds_x), launch(k_ua_select<2, 2>, lds);
        else launch(k_ua_select<1>, lds);
        LAUNCH_CHECK();
    }
    if (report) {
        // ---- cross-partition report sums per (size bucket, configuration)
        stage(ctx, s, "ua.report");
        std::vector<double> hs((size_t)std::max(1, a.n_metrics) * C, 0.0);
        int mi = 0;
        for (int bit : {DPG_M_SUM, DPG_M_COUNT, DPG_M_PRIVACY_ID_COUNT}) {
            if (!(u->metric_mask & bit)) continue;
            const int slot = bit == DPG_M_SUM ? 0 : (bit == DPG_M_COUNT ? 1 : 2);
            for (int i = 0; i < C; ++i) hs[(size_t)mi * C + i] = u->configs[i].noise_std[slot];
            ++mi;
        }
        WS(dstd, double, "ua.std", hs.size());
        UPLOAD(dstd, hs.data(), 8 * hs.size());
        WS(bucket, int32_t, "ua.bucket", P);
        WS(bcount, uint32_t, "ua.bcount", kUaBuckets);
        WS(order, int64_t, "ua.order", P);
        a.std = dstd;
        a.bucket = bucket;
        a.bcount = bcount;
        a.order = order;
        a.rep = report;
        const int F = 4 + 24 * a.n_metrics;
        HIP_TRY(hipMemsetAsync(bcount, 0, 4 * kUaBuckets, s));
        HIP_TRY(hipMemsetAsync(report, 0, (size_t)kUaBuckets * F * C * 8, s));
        const unsigned gb = (unsigned)std::min<int64_t>((P + 255) / 256, (int64_t)ctx->n_cu * 8);
        k_ua_bucket<<<gb, 256, 0, s>>>(partition_start, a);
        LAUNCH_CHECK();
        uint32_t hc[kUaBuckets];
        HIP_TRY(hipMemcpyAsync(hc, bcount, sizeof(hc), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        uint32_t run = 0, start[kUaBuckets];
        for (int b = 0; b < kUaBuckets; ++b) start[b] = run, run += hc[b];
        UPLOAD(bcount, start, sizeof(start));
        const unsigned go = (unsigned)std::min<int64_t>((P + 256 * kUaOrderPer - 1) / (256 * kUaOrderPer),
                                                       (int64_t)ctx->n_cu * 8);
        k_ua_order<<<go, 256, 0, s>>>(a);
        LAUNCH_CHECK();
        if (run > 0) {
            k_ua_report<<<(unsigned)((run + kUaRepRun - 1) / kUaRepRun), 64, 0, s>>>((int64_t)run, a);
            LAUNCH_CHECK();
        }
        if (n_out) *n_out = run;
    }
    stage(ctx, s, "ua.end");
    return DPG_OK;
}

int dpg_dataset_histograms(dpg_ctx *ctx, const dpg_pair_entry *pairs, int64_t n_pairs,
                           const int64_t *partition_start, int64_t P, int32_t pre_aggregated,
                           const dpg_hist_out *out, void *stream) {
    static_assert(DPG_HIST_INT_BINS == kHiBins && DPG_HIST_SUM_BINS == kHsBins, "hist bins");
    if (!ctx) return DPG_ERR_INVALID_ARG;
    if (!out || !out->int_bins || !out->sum_count || !out->sum_sum || !out->sum_max ||
        !out->lowers || !partition_start || P <= 0 || n_pairs < 0 || (n_pairs > 0 && !pairs))
        return fail(ctx, DPG_ERR_INVALID_ARG, "null argument");
    if (P >= 0xFFFFFFFFll) return fail(ctx, DPG_ERR_INVALID_ARG, "n_partitions must be < 2^32-1");
    (void)hipSetDevice(ctx->device);
    hipStream_t s = (hipStream_t)stream;
    ctx->stage_names.clear();
    ctx->n_events_used = 0;
    ctx->last_stream = s;
    int st = DPG_OK;
    stage(ctx, s, "hist.begin");
    const ItemPA *pa = reinterpret_cast<const ItemPA *>(pairs);
    HistArgs a{};
    a.ib = reinterpret_cast<unsigned long long *>(out->int_bins);
    a.scount = reinterpret_cast<unsigned long long *>(out->sum_count);
    a.ssum = out->sum_sum;
    a.smax = reinterpret_cast<unsigned long long *>(out->sum_max);
    a.lowers = out->lowers;
    WS(pcount, unsigned int, "hist.pcount", P);
    WS(minmax, unsigned long long, "hist.minmax", 2);
    a.pcount = pcount;
    a.minmax = minmax;
    HIP_TRY(hipMemsetAsync(a.ib, 0, sizeof(unsigned long long) * kHiTypes * kHiBins * 3, s));
    HIP_TRY(hipMemsetAsync(a.scount, 0, 8 * kHsBins, s));
    HIP_TRY(hipMemsetAsync(a.ssum, 0, 8 * kHsBins, s));
    HIP_TRY(hipMemsetAsync(a.smax, 0, 8 * kHsBins, s));
    HIP_TRY(hipMemsetAsync(a.lowers, 0, 8 * (kHsBins + 1), s));
    HIP_TRY(hipMemsetAsync(pcount, 0, 4 * (size_t)P, s));
    const unsigned long long mm0[2] = {~0ull, 0ull};
    UPLOAD(minmax, mm0, sizeof(mm0));
    if (n_pairs == 0) {
        stage(ctx, s, "hist.end");
        return DPG_OK;
    }
    const unsigned gp = (unsigned)std::min<int64_t>((n_pairs + kHistThreads - 1) / kHistThreads,
                                                    (int64_t)ctx->n_cu * 8);
    if (pre_aggregated) {
        // weights per exact n_partitions / n_contributions value: dense
        // tables sized by the largest value present
        uint32_t mx[2] = {0u, 0u};
        WS(dmx, uint32_t, "hist.wmax", 2);
        HIP_TRY(hipMemsetAsync(dmx, 0, 8, s));
        k_pa_max<<<gp, kHistThreads, 0, s>>>(pa, n_pairs, dmx);
        LAUNCH_CHECK();
        HIP_TRY(hipMemcpyAsync(mx, dmx, 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (mx[0] >= (1u << 30) || mx[1] >= (1u << 30))
            return fail(ctx, DPG_ERR_UNSUPPORTED, "n_partitions / n_contributions >= 2^30");
        a.wlen0 = (int64_t)mx[0] + 1;
        a.wlen1 = (int64_t)mx[1] + 1;
        WS(w0, double, "hist.w0", a.wlen0);
        WS(w1, double, "hist.w1", a.wlen1);
        HIP_TRY(hipMemsetAsync(w0, 0, 8 * a.wlen0, s));
        HIP_TRY(hipMemsetAsync(w1, 0, 8 * a.wlen1, s));
        a.w0 = w0;
        a.w1 = w1;
    }
    stage(ctx, s, "hist.pairs");
    if (pre_aggregated) k_hist_pairs<true><<<gp, kHistThreads, 0, s>>>(pa, n_pairs, a);
    else k_hist_pairs<false><<<gp, kHistThreads, 0, s>>>(pa, n_pairs, a);
    LAUNCH_CHECK();
    if (pre_aggregated) {
        const int64_t wl = std::max(a.wlen0, a.wlen1);
        k_hist_weights<<<(unsigned)std::min<int64_t>((wl + kHistThreads - 1) / kHistThreads,
                                                     (int64_t)ctx->n_cu * 4),
                         kHistThreads, 0, s>>>(a);
        LAUNCH_CHECK();
    }
    stage(ctx, s, "hist.partitions");
    k_hist_parts<<<(unsigned)std::min<int64_t>((P + kHistThreads - 1) / kHistThreads,
                                               (int64_t)ctx->n_cu * 8),
                   kHistThreads, 0, s>>>(partition_start, P, a);
    LAUNCH_CHECK();
    stage(ctx, s, "hist.sums");
    k_hist_lowers<<<(kHsBins + kHistThreads) / kHistThreads, kHistThreads, 0, s>>>(a);
    LAUNCH_CHECK();
    const size_t lds = (size_t)kHsBins * (4 + 8);
    (void)set_func_attr((const void *)k_hist_sums, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    k_hist_sums<<<(unsigned)std::min<int64_t>((n_pairs + 1023) / 1024, (int64_t)ctx->n_cu), 1024,
                  lds, s>>>(pa, n_pairs, a);
    LAUNCH_CHECK();
    k_hist_finish<<<(kHsBins + kHistThreads - 1) / kHistThreads, kHistThreads, 0, s>>>(a);
    LAUNCH_CHECK();
    stage(ctx, s, "hist.end");
    return DPG_OK;
}

int dpg_last_stage_times(dpg_ctx *ctx, char *names, size_t names_len, double *ms,
                         int32_t max_stages, int32_t *n_stages) {
    if (!ctx || !n_stages) return DPG_ERR_INVALID_ARG;
    int ns = ctx->n_events_used - 1;
    if (ns < 0) ns = 0;
    if (ns > max_stages) ns = max_stages;
    *n_stages = ns;
    if (ns == 0) return DPG_OK;
    (void)hipEventSynchronize(ctx->events[ctx->n_events_used - 1]);
    std::string joined;
    for (int i = 0; i < ns; ++i) {
        float t = 0.f;
        (void)hipEventElapsedTime(&t, ctx->events[i], ctx->events[i + 1]);
        if (ms) ms[i] = t;
        if (i) joined += ",";
        joined += ctx->stage_names[i];
    }
    if (names && names_len) std::snprintf(names, names_len, "%s", joined.c_str());
    return DPG_OK;
}

int dpg_comm_unique_id(uint8_t *id) {
    if (!id) return DPG_ERR_INVALID_ARG;
    Rccl &r = rccl();
    if (!r.ok) return DPG_ERR_UNSUPPORTED;
    ncclUniqueId u;
    if (r.get_unique_id(&u) != ncclSuccess) return DPG_ERR_HIP;
    static_assert(sizeof(u) == DPG_COMM_ID_BYTES, "unique id size");
    std::memcpy(id, &u, DPG_COMM_ID_BYTES);
    return DPG_OK;
}

int dpg_ctx_create_comm(dpg_ctx *ctx, const uint8_t *id, int rank, int nranks) {
    if (!ctx || !id || nranks < 1 || rank < 0 || rank >= nranks) return DPG_ERR_INVALID_ARG;
    Rccl &r = rccl();
    if (!r.ok) return fail(ctx, DPG_ERR_UNSUPPORTED, "librccl could not be loaded");
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, DPG_ERR_HIP, "hipSetDevice");
    if (ctx->comm) {
        (void)r.comm_destroy(static_cast<ncclComm_t>(ctx->comm));
        ctx->comm = nullptr;
    }
    ncclUniqueId u;
    std::memcpy(&u, id, DPG_COMM_ID_BYTES);
    ncclComm_t c = nullptr;
    const ncclResult_t e = r.comm_init_rank(&c, nranks, u, rank);
    if (e != ncclSuccess) return fail(ctx, DPG_ERR_HIP, "ncclCommInitRank: " + rccl_msg(e));
    ctx->comm = c;
    ctx->rank = rank;
    ctx->nranks = nranks;
    return DPG_OK;
}

namespace {
// The non-null arrays of `full` (and their counterparts in `slice`, when
// given) in the pack order rows, count, sum, nsum, nsq.
int pack_arrays(dpg_ctx *ctx, const dpg_partials *full, const dpg_partials *slice,
                PackArrays &pa, UnpackArrays &ua) {
    const void *src[5] = {full->rows, full->count, full->sum, full->nsum, full->nsq};
    void *dst[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    if (slice) {
        dst[0] = slice->rows, dst[1] = slice->count, dst[2] = slice->sum;
        dst[3] = slice->nsum, dst[4] = slice->nsq;
    }
    pa = PackArrays{};
    ua = UnpackArrays{};
    for (int k = 0; k < 5; ++k) {
        if (!src[k]) continue;
        if (slice && !dst[k]) return fail(ctx, DPG_ERR_INVALID_ARG, "slice lacks an array the partials have");
        pa.a[pa.n] = src[k];
        pa.is_int[pa.n] = k < 2;
        ua.a[ua.n] = dst[k];
        ua.is_int[ua.n] = k < 2;
        ++pa.n;
        ++ua.n;
    }
    if (pa.n == 0) return fail(ctx, DPG_ERR_INVALID_ARG, "no partial arrays");
    return DPG_OK;
}

int launch_pack(dpg_ctx *ctx, const PackArrays &pa, int64_t P, int R, double *pack, hipStream_t s) {
    int st = DPG_OK;
    const int64_t S = (P + R - 1) / R;
    const int64_t total = S * R;
    const unsigned blocks = (unsigned)std::min<int64_t>((total + 255) / 256, (int64_t)ctx->n_cu * 16);
    k_pack_partials<<<blocks, 256, 0, s>>>(pa, P, S, R, ctx->last_err, pack);
    LAUNCH_CHECK();
    return st;
}

int launch_unpack(dpg_ctx *ctx, const UnpackArrays &ua, const double *part, int64_t P, int R,
                  int rank, dpg_partials *slice, int64_t *lo, int64_t *n, hipStream_t s) {
    int st = DPG_OK;
    const int64_t S = (P + R - 1) / R;
    // partitions rank, rank + R, rank + 2R, ... below P
    const int64_t nl = rank < P ? (P - rank + R - 1) / R : 0;
    uint32_t *err = latch_word(ctx, s, &st);
    if (!err) return st;
    const unsigned ub = (unsigned)std::max<int64_t>(1, std::min<int64_t>((nl + 255) / 256,
                                                                         (int64_t)ctx->n_cu * 16));
    k_unpack_partials<<<ub, 256, 0, s>>>(part, S, nl, ua, err);
    LAUNCH_CHECK();
    *lo = rank;
    *n = nl;
    slice->n_partitions = nl;
    return st;
}
}  // namespace

int dpg_pack_partials(dpg_ctx *ctx, const dpg_partials *full, int nranks, double *pack,
                      void *stream) {
    if (!ctx || !full || !pack || nranks < 1) return DPG_ERR_INVALID_ARG;
    const int64_t P = full->n_partitions;
    if (P <= 0) return fail(ctx, DPG_ERR_INVALID_ARG, "n_partitions must be positive");
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, DPG_ERR_HIP, "hipSetDevice");
    PackArrays pa;
    UnpackArrays ua;
    if (int r = pack_arrays(ctx, full, nullptr, pa, ua)) return r;
    return launch_pack(ctx, pa, P, nranks, pack, static_cast<hipStream_t>(stream));
}

int dpg_unpack_partials(dpg_ctx *ctx, const double *part, int64_t n_partitions, int nranks,
                        int rank, dpg_partials *slice, int64_t *lo, int64_t *n, void *stream) {
    if (!ctx || !part || !slice || !lo || !n || nranks < 1 || rank < 0 || rank >= nranks)
        return DPG_ERR_INVALID_ARG;
    if (n_partitions <= 0) return fail(ctx, DPG_ERR_INVALID_ARG, "n_partitions must be positive");
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, DPG_ERR_HIP, "hipSetDevice");
    // the slice's non-null arrays name the packed arrays (same order)
    PackArrays pa;
    UnpackArrays ua;
    dpg_partials like = *slice;
    like.n_partitions = n_partitions;
    if (int r = pack_arrays(ctx, &like, slice, pa, ua)) return r;
    return launch_unpack(ctx, ua, part, n_partitions, nranks, rank, slice, lo, n,
                         static_cast<hipStream_t>(stream));
}

int dpg_reduce_scatter_partials(dpg_ctx *ctx, const dpg_partials *full, dpg_partials *slice,
                                int64_t *lo, int64_t *n, void *stream) {
    if (!ctx || !full || !slice || !lo || !n) return DPG_ERR_INVALID_ARG;
    if (!ctx->comm) return fail(ctx, DPG_ERR_INVALID_ARG, "no communicator: dpg_ctx_create_comm");
    const int64_t P = full->n_partitions;
    if (P <= 0) return fail(ctx, DPG_ERR_INVALID_ARG, "n_partitions must be positive");
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, DPG_ERR_HIP, "hipSetDevice");
    hipStream_t s = static_cast<hipStream_t>(stream);
    int st = DPG_OK;
    const int R = ctx->nranks;
    const int64_t S = (P + R - 1) / R;
    PackArrays pa;
    UnpackArrays ua;
    if (int r = pack_arrays(ctx, full, slice, pa, ua)) return r;
    WS(pack, double, "comm.pack", (size_t)R * (pa.n * S + 1));
    WS(part, double, "comm.part", (size_t)pa.n * S + 1);
    if (int r = launch_pack(ctx, pa, P, R, pack, s)) return r;
    const ncclResult_t e = rccl().reduce_scatter(pack, part, (size_t)pa.n * S + 1, ncclFloat64, ncclSum,
                                                 static_cast<ncclComm_t>(ctx->comm), s);
    if (e != ncclSuccess) return fail(ctx, DPG_ERR_HIP, "ncclReduceScatter: " + rccl_msg(e));
    return launch_unpack(ctx, ua, part, P, R, ctx->rank, slice, lo, n, s);
}

int dpg_export_error(dpg_ctx *ctx, double *dst, void *stream) {
    if (!ctx || !dst) return DPG_ERR_INVALID_ARG;
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, DPG_ERR_HIP, "hipSetDevice");
    hipStream_t s = static_cast<hipStream_t>(stream);
    int st = DPG_OK;
    k_export_error<<<1, 1, 0, s>>>(ctx->last_err, dst);
    LAUNCH_CHECK();
    return st;
}

int dpg_import_error(dpg_ctx *ctx, const double *src, int64_t n, void *stream) {
    if (!ctx || !src || n < 0) return DPG_ERR_INVALID_ARG;
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, DPG_ERR_HIP, "hipSetDevice");
    hipStream_t s = static_cast<hipStream_t>(stream);
    int st = DPG_OK;
    uint32_t *err = latch_word(ctx, s, &st);
    if (!err) return st;
    if (n > 0) {
        k_import_error<<<1, 64, 0, s>>>(src, n, err);
        LAUNCH_CHECK();
    }
    return st;
}

}  // extern "C"
