// dpg_team.h -- level-2 partitioning without a histogram pass (gfx950).
//
// The grouped level 2 of dpg_partition.h reads every record twice: once in
// k_hist (the digit counts of its level-1 bucket) and once in k_scatter.
// Here the digit counts come from the records the scatter holds anyway:
//
// * a TEAM is the workgroups w = x, x + 8, x + 16, ... of one persistent
//   launch of one workgroup per CU (round-robin dispatch puts them on XCD x,
//   so the team shares one L2); team x takes the level-1 buckets x, x + 8,
//   ... in order;
// * each member loads its 1/T share of the bucket (<= kTeamSub records)
//   into registers, ranks it by digit in LDS and adds its digit counts to
//   the team's totals with one atomic per digit -- the returned old value is
//   the member's run offset inside the digit (arrival order, as the grouped
//   scatter's reservations);
// * after a team barrier every member reads the totals, scans them into the
//   bucket's digit starts and writes its runs, staged through LDS as in
//   k_scatter (member 0 also writes the fine buckets' starts and counts).
//
// The records therefore cross HBM once in and once out; the barrier replaces
// the histogram pass.  Totals are triple-buffered per team (a member zeroes
// the buffer of the bucket after next once every member has read the one
// before), so one barrier per bucket suffices.  The barrier is bounded: a
// member that waits longer than kTeamTimeout (co-residency lost) raises
// err bit 8 and the abort flag, every member leaves, and the host redoes
// the level with the histogram path.
#pragma once

#include "dpg_partition.h"

namespace dpg {

constexpr int kTeamIPT = 16;                       // records per thread
#ifndef DPG_TEAM_PF
#define DPG_TEAM_PF 1  // next share loaded during the barrier + write-out (same-box A/B, config 2: 5.09 -> 4.39 ms)
#endif
#ifndef DPG_TEAM_PF_PC
#define DPG_TEAM_PF_PC 1  // the same for the histogram-free level 1's pieces
#endif
#ifndef DPG_TEAM_WB
#define DPG_TEAM_WB 4  // staged records per thread per write-out batch
#endif
constexpr uint32_t kTeamF = 2048;                  // digits (11 bits)
constexpr int kTeamSub = kScatThreads * kTeamIPT;  // records per member per bucket
constexpr uint64_t kTeamTimeout = 50000000ull;     // wall_clock64 ticks (100 MHz): 0.5 s
constexpr uint32_t kTeamArriveStride = 32;         // counters on separate 128-B lines

struct TeamSync {
    uint32_t *tot;     // [8][3][kTeamF] digit totals per team, triple-buffered (zeroed)
    uint32_t *arrive;  // [8 * kTeamArriveStride] arrivals per team (zeroed)
    uint32_t *abort;   // nonzero: a barrier timed out, every member leaves
    uint32_t *err;     // Control::err; bit 8 = team barrier timeout
};

template <class R>
constexpr size_t team_lds() {
    return sizeof(R) * (kTeamSub + 1) + (size_t)kTeamF * 12 + 4 * 4 + 64;
}

__device__ __forceinline__ uint32_t ld_agent(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// All members of `team` have arrived `target` times in total.  Returns false
// when the team gave up (timeout or another member's abort).
//
// Hand-off form (MI355X_MICROARCH.md, inter-workgroup visibility, first row
// of the sc1 table): the only data the members exchange are the digit totals,
// written by agent-scope atomics (adds; the zeroing by atomic stores) and
// read by sc1 loads (ld_agent), so no L2 write-back or L1 invalidate is
// needed -- only that every wave's atomics have completed before one lane
// adds to the arrival counter behind a workgroup barrier, and that the
// poll is an sc1 load.  (Agent-scope fences here -- __threadfence in every
// thread, a release add, an acquire per poll -- wrote back and invalidated
// the XCD L2 that holds the scattered runs: 20.5 ms instead of ~4 ms.)
//
// `between` runs in every thread after the arrival and before the poll: the
// loads it issues (the next bucket's share) are in flight during the wait
// instead of behind the arrival's vmcnt(0).
struct NoOp {
    __device__ __forceinline__ void operator()() const {}
};
template <class F = NoOp>
__device__ __forceinline__ bool team_barrier(const TeamSync &ts, uint32_t team, uint32_t target,
                                             uint32_t *sh_ok, const F &between = F{}) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's reservations / zeroing done
    __syncthreads();
    uint32_t *ctr = ts.arrive + team * kTeamArriveStride;
    // the first poll is issued before `between`: vmcnt counts in issue order,
    // so a poll issued after the prefetch loads would wait for all of them
    // (wave 0 then held the whole workgroup at the closing barrier for the
    // next share's load latency although the team had long arrived)
    uint32_t seen = 0;
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        seen = ld_agent(ctr);
    }
    between();
    if (threadIdx.x == 0) {
        const uint64_t t0 = wall_clock64();
        uint32_t ok = 1;
        for (; seen < target; seen = ld_agent(ctr)) {
            if (ld_agent(ts.abort)) {
                ok = 0;
                break;
            }
            if (wall_clock64() - t0 > kTeamTimeout) {
                atomicOr(ts.abort, 1u);
                atomicOr(ts.err, 8u);
                ok = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        *sh_ok = ok;
    }
    __syncthreads();
    return *sh_ok != 0;
}

// The histogram-free level 1 (k_scatter's piece mode) leaves level-1 bucket
// s as 8 pieces, one per XCD region: records [rbase[x F1 + s], + cum[x F1 +
// s]) for x < 8; tot[s] = their sum, ostart[s] = the bucket's start in the
// (compact) level-2 output.  Region starts are even (C even).
// One bucket's pieces in one 128-byte record (k_piece_totals), read by two
// scalar loads: a team member's next share then costs one round trip of
// descriptor reads instead of ten dependent ones (bucket size, start, first
// region, and each piece's region offset and count).
struct PieceDesc {
    uint32_t n;        // padded records (each piece rounded up to even)
    uint32_t pad0;
    int64_t ostart;    // the bucket's start in the compact level-2 output
    int64_t base0;     // the bucket's first region (rbase[s])
    uint32_t ppre[8];  // padded exclusive prefix of the pieces
    uint32_t dl[8];    // index i of piece p sits at base0 + i + dl[p] (mod 2^32)
    uint32_t cend[8];  // end of piece p's records in the padded index space
    uint32_t pad1[2];
};
static_assert(sizeof(PieceDesc) == 128, "PieceDesc is two 64-byte scalar loads");

struct PieceTab {
    const int64_t *rbase;
    const uint32_t *cum;
    const uint32_t *tot;
    const uint32_t *ptot;  // the pieces' counts each rounded up to even, summed
    const int64_t *ostart;
    uint32_t F1;
    const PieceDesc *desc = nullptr;  // [F1]
};

typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
// 128 bytes at a uniform, 64-byte aligned address into scalar registers
// (loads only: nothing is written through the scalar cache)
__device__ __forceinline__ void sload_desc(const PieceDesc *p, u32x16 &a, u32x16 &b) {
    p = uniform_ptr(p);
    asm volatile("s_load_dwordx16 %0, %2, 0x0\n\ts_load_dwordx16 %1, %2, 0x40\n\ts_waitcnt lgkmcnt(0)"
                 : "=s"(a), "=s"(b)
                 : "s"(p)
                 : "memory");
}

// Level 2 over S level-1 buckets (seg_start / seg_cnt; every count <= T *
// kTeamSub, checked by the host): records of bucket s land in out[seg_start[s],
// + seg_cnt[s]) grouped by digit (F2 <= kTeamF digits; the scans run over
// kTeamF, the digits past F2 count 0); base_out[s][d] / tot_out[s][d] = start
// and count of fine bucket (s, d), d < F2.  gridDim.x = 8 T workgroups, all
// resident.  kPc: the buckets are PieceTab pieces (seg_start / seg_cnt
// unused), read with one 8-byte load per record (a piece may start at an odd
// record), written compactly from ostart[s].
//
// kMulti: a member's share may exceed the kTeamSub records its registers and
// LDS stage hold (heavy privacy ids or N past 2^30 make level-1 buckets
// larger than T kTeamSub).  A bucket whose share exceeds sub_cap (<= kTeamSub,
// even) is done in J = ceil(share / sub_cap) rounds: pass A loads the rounds
// one after another and only counts digits, the member reserves its runs of
// all rounds at once, the team barrier publishes the totals, and pass B
// reloads each round, ranks, stages and writes it at the member's advancing
// run cursors -- one more read of the bucket, the same output layout.
// Buckets that fit take the single-round path unchanged.
template <class R, bool kPc = false, bool kMulti = false>
__global__ __launch_bounds__(kScatThreads) void k_part2_team(SrcAoS<R> src,
                                                             const int64_t *seg_start,
                                                             const uint32_t *seg_cnt, uint32_t S,
                                                             uint32_t F2, R *out, int64_t *base_out,
                                                             uint32_t *tot_out, TeamSync ts,
                                                             PieceTab pt = PieceTab{},
                                                             uint32_t sub_cap = kTeamSub) {
    constexpr int IPT = kTeamIPT;
    constexpr int SUB = kTeamSub;
    constexpr uint32_t F = kTeamF;
    constexpr int DPT = F / kScatThreads;  // digits per thread in the scans
    using W = Words<R>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    W *stage = reinterpret_cast<W *>(smem);  // [SUB + 1]: slot SUB takes the padding
    uint32_t *cnt = reinterpret_cast<uint32_t *>(smem + sizeof(R) * (SUB + 1));
    uint32_t *dstart = cnt + F;     // [F + 1] local digit starts
    uint32_t *cur = dstart + F + 1; // [F] this member's run start inside the bucket
    uint32_t *sh16 = cur + F;       // [16] wave totals
    __shared__ uint32_t sh_ok;
    const uint32_t team = blockIdx.x & 7u;
    const uint32_t T = gridDim.x >> 3;
    const uint32_t m = blockIdx.x >> 3;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6;
    for (uint32_t d = tid; d < F; d += kScatThreads) cnt[d] = 0;
    __syncthreads();
    // element j of a thread: 16-byte pair loads, as k_scatter's pair sources
    auto elem = [tid](int j) -> uint32_t {
        return (uint32_t)((j >> 1) * 2 * kScatThreads + 2 * tid + (j & 1));
    };
    // this member's share of bucket s: [st + b0, + lim).  Piece mode: the
    // share is cut from the bucket's padded index space (every piece rounded
    // up to an even length, see load_pieces) in even lengths; st is the
    // bucket's start in the compact output
    auto share = [&](uint32_t s, int64_t &st, uint32_t &n, uint32_t &b0, uint32_t &lim) {
        n = __builtin_amdgcn_readfirstlane(kPc ? pt.ptot[s] : seg_cnt[s]);
        const int64_t st0 = kPc ? pt.ostart[s] : seg_start[s];
        st = (int64_t)(((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)st0 >> 32)) << 32) |
                       (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)st0));
        const uint32_t q = kPc ? (((n + T - 1) / T + 1) & ~1u) : (n + T - 1) / T;
        b0 = min(n, m * q);
        lim = min(n, b0 + q) - b0;  // <= sub_cap <= SUB, or the bucket is the kMulti launch's
    };
    R rec[IPT];
    uint32_t vmask = ~0u;  // piece mode: bit j = element j is a record (not padding)
    // loads of a share (unconditional, clamped into it: a guarded load would
    // serialise them); a member past the bucket's end loads nothing
    auto load = [&](int64_t base, uint32_t lim) {
        if (lim >= 2) {
#pragma unroll
            for (int mm = 0; mm < IPT / 2; ++mm) {
                const uint32_t o = mm * 2 * kScatThreads + 2 * tid;
                const uint32_t a = min(o, lim - 2);
                R x0, x1;
                src.fetch2(base + a, x0, x1);
                rec[2 * mm] = a == o ? x0 : x1;
                rec[2 * mm + 1] = x1;
            }
        } else {
#pragma unroll
            for (int j = 0; j < IPT; ++j) rec[j] = lim ? src.fetch(base) : R{};
        }
    };
    // piece mode: the bucket's index space lists its 8 pieces in order, each
    // padded to an even length (ppre: padded exclusive prefix), so an even
    // index and its successor lie in one piece at an even offset -- one
    // 16-byte load (region starts are even: C is even); the padding slot
    // after an odd piece is loaded from inside the region and masked out.
    // Offsets are 32-bit from the bucket's first region (the bucket's
    // regions span 8 C records).
    auto load_pieces = [&](uint32_t s, uint32_t b0, uint32_t lim) {
        uint32_t ppre[8], dl[8], pc[8];
        const int64_t rb0 = pt.rbase[s];
        const int64_t base0 = (int64_t)(((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)rb0 >> 32)) << 32) |
                                        (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)rb0));
        uint32_t acc = 0;
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            const uint32_t off = __builtin_amdgcn_readfirstlane(
                (uint32_t)(pt.rbase[(size_t)p * pt.F1 + s] - rb0));
            pc[p] = __builtin_amdgcn_readfirstlane(pt.cum[(size_t)p * pt.F1 + s]);
            ppre[p] = acc;
            dl[p] = off - acc;  // index i of piece p sits at base0 + i + dl[p] (mod 2^32)
            acc += (pc[p] + 1u) & ~1u;
        }
        const char *bp = reinterpret_cast<const char *>(src.a + base0);
        uint32_t vm = 0;
#pragma unroll
        for (int mm = 0; mm < IPT / 2; ++mm) {
            const uint32_t o = mm * 2 * kScatThreads + 2 * tid;
            const uint32_t i = b0 + min(o, lim - 2);  // even (b0, lim even)
            uint32_t d = dl[0], c = pc[0] + ppre[0];
#pragma unroll
            for (int p = 1; p < 8; ++p) {
                const bool in = i >= ppre[p];
                d = in ? dl[p] : d;
                c = in ? pc[p] + ppre[p] : c;  // end of the piece's records
            }
            R x0, x1;
            const uint32_t boff = (i + d) * (uint32_t)sizeof(R);
            static_assert(sizeof(R) == 8, "piece-mode teams read 8-byte records");
            const u64x2 w = *reinterpret_cast<const u64x2 *>(bp + boff);
            const uint64_t w0 = w.x, w1 = w.y;
            __builtin_memcpy(&x0, &w0, sizeof(R));
            __builtin_memcpy(&x1, &w1, sizeof(R));
            rec[2 * mm] = x0;
            rec[2 * mm + 1] = x1;
            vm |= (i < c ? 1u : 0u) << (2 * mm);
            vm |= (i + 1 < c ? 1u : 0u) << (2 * mm + 1);
        }
        vmask = vm;
    };
    // the same from the bucket's PieceDesc, already in scalar registers
    auto load_pieces_desc = [&](const u32x16 &da, const u32x16 &db, uint32_t b0, uint32_t lim) {
        const int64_t base0 = (int64_t)(((uint64_t)da[5] << 32) | da[4]);
        uint32_t ppre[8], dl[8], ce[8];
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            ppre[p] = da[6 + p];
            dl[p] = p < 2 ? da[14 + p] : db[p - 2];
            ce[p] = db[6 + p];
        }
        const char *bp = reinterpret_cast<const char *>(src.a + base0);
        uint32_t vm = 0;
#pragma unroll
        for (int mm = 0; mm < IPT / 2; ++mm) {
            const uint32_t o = mm * 2 * kScatThreads + 2 * tid;
            const uint32_t i = b0 + min(o, lim - 2);  // even (b0, lim even)
            uint32_t d = dl[0], c = ce[0];
#pragma unroll
            for (int p = 1; p < 8; ++p) {
                const bool in = i >= ppre[p];
                d = in ? dl[p] : d;
                c = in ? ce[p] : c;
            }
            R x0, x1;
            const uint32_t boff = (i + d) * (uint32_t)sizeof(R);
            const u64x2 w = *reinterpret_cast<const u64x2 *>(bp + boff);
            const uint64_t w0 = w.x, w1 = w.y;
            __builtin_memcpy(&x0, &w0, sizeof(R));
            __builtin_memcpy(&x1, &w1, sizeof(R));
            rec[2 * mm] = x0;
            rec[2 * mm + 1] = x1;
            vm |= (i < c ? 1u : 0u) << (2 * mm);
            vm |= (i + 1 < c ? 1u : 0u) << (2 * mm + 1);
        }
        vmask = vm;
    };
    uint32_t k = 0;  // buckets done = team barriers passed
    // kPF: the share of this member's next non-empty bucket (piece mode: its
    // piece descriptors too) is loaded during the current bucket's team
    // barrier and write-out (the local staging moves before the barrier,
    // which frees the record registers); pf_s = the bucket those registers
    // hold
    constexpr bool kPF = DPG_TEAM_PF && (!kPc || DPG_TEAM_PF_PC) && !kMulti;
    // a member's share of n records (team-uniform): over sub_cap, the bucket
    // is left to the kMulti launch
    auto share_q = [&](uint32_t n) -> uint32_t {
        return kPc ? (((n + T - 1) / T + 1) & ~1u) : (n + T - 1) / T;
    };
    auto next_nonempty = [&](uint32_t s) -> uint32_t {
        for (; s < S; s += 8) {
            const uint32_t n = __builtin_amdgcn_readfirstlane(kPc ? pt.ptot[s] : seg_cnt[s]);
            if (n != 0 && share_q(n) <= sub_cap) break;
        }
        return s;
    };
    // the loads of one share (piece mode: its 8-piece descriptors first);
    // the share's bounds are kept for the bucket's iteration (kPF), whose
    // loop head then issues no loads: a load there waited with vmcnt(0) for
    // the previous bucket's write-out stores before the ranking could start
    int64_t pf_st = 0;
    uint32_t pf_n = 0, pf_b0 = 0, pf_lim = 0;
    constexpr bool use_desc = kPc && kPF;  // the host always builds pt.desc
    auto load_share = [&](uint32_t s) {
        if constexpr (kPc) {
            if constexpr (use_desc) {
                // branch-free: past the last bucket (s = S) the loads read the
                // last one, a member past the bucket's end reads its tail
                // (inside the regions, masked out): no path without loads,
                // so the barrier's first poll is waited for by count
                u32x16 da, db;
                sload_desc(pt.desc + min(s, S - 1), da, db);
                pf_n = __builtin_amdgcn_readfirstlane(da[0]);
                pf_st = (int64_t)(((uint64_t)da[3] << 32) | da[2]);
                const uint32_t q = ((pf_n + T - 1) / T + 1) & ~1u;
                pf_b0 = min(pf_n, m * q);
                pf_lim = min(pf_n, pf_b0 + q) - pf_b0;
                load_pieces_desc(da, db, pf_b0, max(pf_lim, 2u));
                return;
            }
        }
        share(s, pf_st, pf_n, pf_b0, pf_lim);
        if constexpr (kPc) {
            vmask = 0;
            if (pf_lim > 0) load_pieces(s, pf_b0, pf_lim);
        } else {
            load(pf_st + pf_b0, pf_lim);
        }
    };
    uint32_t pf_s = S;
    if constexpr (kPF) {
        pf_s = next_nonempty(team);
        if (use_desc || pf_s < S) load_share(pf_s);
    }
    // the staged records [0, nv) to their runs: out[st + cur[d] + (k -
    // dstart[d])] for staged position k of digit d
    auto write_out = [&](int64_t st, uint32_t nv) {
        constexpr int WB = DPG_TEAM_WB;
        for (uint32_t k0 = 0; k0 < nv; k0 += WB * kScatThreads) {
            W x[WB];
            uint32_t dd[WB], kc[WB];
#pragma unroll
            for (int u = 0; u < WB; ++u) {
                kc[u] = min(k0 + u * kScatThreads + tid, nv - 1);
                x[u] = stage[kc[u]];
                dd[u] = src.digit(from_words<R>(x[u]));
            }
            uint32_t c1[WB], c2[WB];
#pragma unroll
            for (int u = 0; u < WB; ++u) {
                c1[u] = cur[dd[u]];
                c2[u] = dstart[dd[u]];
            }
#pragma unroll
            for (int u = 0; u < WB; ++u)
                *reinterpret_cast<W *>(&out[st + c1[u] + (kc[u] - c2[u])]) = x[u];
        }
    };
    for (uint32_t s = team; s < S; s += 8) {
        int64_t st;
        uint32_t n, b0, lim;
        if constexpr (kPF) {
            if (s == pf_s) {
                st = pf_st;
                n = pf_n;
                b0 = pf_b0;
                lim = pf_lim;
            } else {
                share(s, st, n, b0, lim);  // an empty bucket (next_nonempty skipped it)
            }
        } else {
            share(s, st, n, b0, lim);
        }
        if constexpr (kMulti) {
            if (n == 0 || share_q(n) <= sub_cap) continue;  // the single-round launch's
        } else {
            if (n == 0) {
                if (m == 0)
                    for (uint32_t d = tid; d < F2; d += kScatThreads) {
                        base_out[(size_t)s * F2 + d] = st;
                        tot_out[(size_t)s * F2 + d] = 0;
                    }
                continue;  // uniform over the team: no barrier
            }
            if (share_q(n) > sub_cap) continue;  // left to the kMulti launch (uniform)
        }
        // ---- the bucket's digit starts from the team totals (after the
        // team barrier): cur += digit start; member 0 writes the fine
        // buckets' starts and counts and zeroes the totals of the bucket
        // after next
        auto team_starts = [&](const uint32_t *tt) {
            const uint32_t d0 = DPT * tid;
            uint32_t c[DPT], x = 0;
#pragma unroll
            for (int u = 0; u < DPT; ++u) {
                c[u] = ld_agent(&tt[d0 + u]);
                x += c[u];
            }
            uint32_t wt;
            uint32_t e = wave_excl_scan(x, wt);
            if (lane == 63) sh16[wv] = wt;
            __syncthreads();
#pragma unroll
            for (int w = 0; w < kScatThreads / 64; ++w)
                if (w < wv) e += sh16[w];
            uint32_t *tz = ts.tot + ((size_t)team * 3 + (k + 1) % 3) * F;  // the bucket after next
#pragma unroll
            for (int u = 0; u < DPT; ++u) {
                cur[d0 + u] += e;
                if (m == 0) {
                    if (d0 + u < F2) {
                        base_out[(size_t)s * F2 + d0 + u] = st + e;
                        tot_out[(size_t)s * F2 + d0 + u] = c[u];
                    }
                    __hip_atomic_store(&tz[d0 + u], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                e += c[u];
            }
        };
        if constexpr (kMulti) {
            const uint32_t q = share_q(n);
            {
                uint32_t *tt = ts.tot + ((size_t)team * 3 + k % 3) * F;
                const uint32_t J = (q + sub_cap - 1) / sub_cap;
                auto load_part = [&](uint32_t j, uint32_t &lj) {
                    const uint32_t bj = b0 + j * sub_cap;
                    lj = lim > j * sub_cap ? min(sub_cap, lim - j * sub_cap) : 0u;
                    if constexpr (kPc) {
                        if constexpr (use_desc) {
                            u32x16 da, db;
                            sload_desc(pt.desc + s, da, db);
                            load_pieces_desc(da, db, bj, max(lj, 2u));
                        } else {
                            vmask = 0;
                            if (lj > 0) load_pieces(s, bj, lj);
                        }
                    } else {
                        load(st + bj, lj);
                    }
                };
                auto ok_elem = [&](int jj, uint32_t lj) {
                    bool ok = elem(jj) < lj;
                    if constexpr (kPc) ok = ok && ((vmask >> jj) & 1u);
                    return ok;
                };
                // ---- pass A: the member's digit counts over all its rounds
                for (uint32_t j = 0; j < J; ++j) {
                    uint32_t lj;
                    load_part(j, lj);
#pragma unroll
                    for (int jj = 0; jj < IPT; ++jj) {
                        const bool ok = ok_elem(jj, lj);
                        atomicAdd(&cnt[ok ? src.digit(rec[jj]) : 0u], ok ? 1u : 0u);
                    }
                }
                __syncthreads();
                {
                    const uint32_t d0 = DPT * tid;
#pragma unroll
                    for (int u = 0; u < DPT; ++u) {
                        cur[d0 + u] = atomicAdd(&tt[d0 + u], cnt[d0 + u]);
                        cnt[d0 + u] = 0;
                    }
                }
                ++k;
                if (!team_barrier(ts, team, T * k, &sh_ok)) return;
                team_starts(tt);
                // ---- pass B: each round ranked, staged and written at the
                // member's run cursors, which then advance by its counts
                for (uint32_t j = 0; j < J; ++j) {
                    __syncthreads();  // the previous round's write-out / cursor updates
                    uint32_t lj;
                    load_part(j, lj);
                    uint32_t drm[IPT];
#pragma unroll
                    for (int jj = 0; jj < IPT; ++jj) {
                        const bool ok = ok_elem(jj, lj);
                        const uint32_t dg = ok ? src.digit(rec[jj]) : 0u;
                        const uint32_t rk = atomicAdd(&cnt[dg], ok ? 1u : 0u);
                        drm[jj] = ok ? (dg | (rk << 12)) : ~0u;
                    }
                    __syncthreads();
                    const uint32_t d0 = DPT * tid;
                    uint32_t c[DPT], x = 0;
#pragma unroll
                    for (int u = 0; u < DPT; ++u) {
                        c[u] = cnt[d0 + u];
                        x += c[u];
                    }
                    uint32_t wt;
                    uint32_t e = wave_excl_scan(x, wt);
                    if (lane == 63) sh16[wv] = wt;
                    __syncthreads();
                    uint32_t nvj = 0;
#pragma unroll
                    for (int w = 0; w < kScatThreads / 64; ++w) {
                        if (w < wv) e += sh16[w];
                        nvj += sh16[w];
                    }
#pragma unroll
                    for (int u = 0; u < DPT; ++u) {
                        dstart[d0 + u] = e;
                        cnt[d0 + u] = 0;
                        e += c[u];
                    }
                    __syncthreads();
#pragma unroll
                    for (int jj = 0; jj < IPT; ++jj) {
                        const uint32_t pos = drm[jj] != ~0u ? dstart[drm[jj] & 0xFFFu] + (drm[jj] >> 12)
                                                            : (uint32_t)SUB;
                        stage[pos] = to_words(rec[jj]);
                    }
                    __syncthreads();
                    write_out(st, nvj);
                    __syncthreads();
#pragma unroll
                    for (int u = 0; u < DPT; ++u) cur[d0 + u] += c[u];
                }
                __syncthreads();
                continue;
            }
        } else {
        uint32_t *tt = ts.tot + ((size_t)team * 3 + k % 3) * F;
        // ---- load + rank
        if constexpr (!kPF) load_share(s);
        uint32_t dr[IPT];
        uint32_t nv = 0;  // records of the share (lim less the padding)
        {
            uint32_t dg[IPT];
            bool okv[IPT];
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                okv[j] = elem(j) < lim;
                if constexpr (kPc) okv[j] = okv[j] && ((vmask >> j) & 1u);
                dg[j] = okv[j] ? src.digit(rec[j]) : 0u;
            }
            uint32_t rk[IPT];
#pragma unroll
            for (int j = 0; j < IPT; ++j) rk[j] = atomicAdd(&cnt[dg[j]], okv[j] ? 1u : 0u);
#pragma unroll
            for (int j = 0; j < IPT; ++j) dr[j] = okv[j] ? (dg[j] | (rk[j] << 12)) : ~0u;
        }
        __syncthreads();
        // ---- local digit starts; runs reserved in the team totals
        {
            const uint32_t d0 = DPT * tid;
            uint32_t c[DPT], x = 0;
#pragma unroll
            for (int u = 0; u < DPT; ++u) {
                c[u] = cnt[d0 + u];
                x += c[u];
            }
            // the reservations, issued before the scan: unconditional (a
            // count of 0 adds 0), so that a thread's atomics are in flight
            // together and overlap the scan, instead of one branch-guarded
            // round trip after another; the team barrier's vmcnt(0) waits
            // for them
            uint32_t o[DPT];
#pragma unroll
            for (int u = 0; u < DPT; ++u) o[u] = atomicAdd(&tt[d0 + u], c[u]);
            uint32_t wt;
            uint32_t e = wave_excl_scan(x, wt);
            if (lane == 63) sh16[wv] = wt;
            __syncthreads();
#pragma unroll
            for (int w = 0; w < kScatThreads / 64; ++w) {
                if (w < wv) e += sh16[w];
                nv += sh16[w];
            }
#pragma unroll
            for (int u = 0; u < DPT; ++u) {
                dstart[d0 + u] = e;
                if constexpr (!kPF) cur[d0 + u] = o[u];
                cnt[d0 + u] = 0;
                e += c[u];
            }
            if (tid == 0) dstart[F] = nv;
            if constexpr (kPF) {
                // ---- stage by local digit now (independent of the team
                // totals); the reservations' round trip overlaps it
                __syncthreads();
#pragma unroll
                for (int j = 0; j < IPT; ++j) {
                    const uint32_t pos = dr[j] != ~0u ? dstart[dr[j] & 0xFFFu] + (dr[j] >> 12) : (uint32_t)SUB;
                    stage[pos] = to_words(rec[j]);
                }
#pragma unroll
                for (int u = 0; u < DPT; ++u) cur[d0 + u] = o[u];
                pf_s = next_nonempty(s + 8);
            }
        }
        ++k;
        auto prefetch = [&]() {
            if constexpr (kPF) {
                if (use_desc || pf_s < S) load_share(pf_s);
            }
        };
        if (!team_barrier(ts, team, T * k, &sh_ok, prefetch)) return;
        // ---- the bucket's digit starts from the team totals (the
        // team_starts code, inline: as a lambda call it cost the single-round
        // path 6 spilled VGPRs)
        {
            const uint32_t d0 = DPT * tid;
            uint32_t c[DPT], x = 0;
#pragma unroll
            for (int u = 0; u < DPT; ++u) {
                c[u] = ld_agent(&tt[d0 + u]);
                x += c[u];
            }
            uint32_t wt;
            uint32_t e = wave_excl_scan(x, wt);
            if (lane == 63) sh16[wv] = wt;
            __syncthreads();
#pragma unroll
            for (int w = 0; w < kScatThreads / 64; ++w)
                if (w < wv) e += sh16[w];
            uint32_t *tz = ts.tot + ((size_t)team * 3 + (k + 1) % 3) * F;  // the bucket after next
#pragma unroll
            for (int u = 0; u < DPT; ++u) {
                cur[d0 + u] += e;
                if (m == 0) {
                    if (d0 + u < F2) {
                        base_out[(size_t)s * F2 + d0 + u] = st + e;
                        tot_out[(size_t)s * F2 + d0 + u] = c[u];
                    }
                    __hip_atomic_store(&tz[d0 + u], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                e += c[u];
            }
        }
        // ---- stage by local digit, write every digit's run contiguously
        if constexpr (!kPF) {
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                const uint32_t pos = dr[j] != ~0u ? dstart[dr[j] & 0xFFFu] + (dr[j] >> 12) : (uint32_t)SUB;
                stage[pos] = to_words(rec[j]);
            }
        }
        __syncthreads();
        // (loading the next bucket's share during the write-out measured
        // slower: 5.2 -> 5.65 ms at config 2, 128 VGPRs with spills)
        {
            constexpr int WB = DPG_TEAM_WB;
            for (uint32_t k0 = 0; k0 < nv; k0 += WB * kScatThreads) {
                W x[WB];
                uint32_t dd[WB], kc[WB];
#pragma unroll
                for (int u = 0; u < WB; ++u) {
                    kc[u] = min(k0 + u * kScatThreads + tid, nv - 1);
                    x[u] = stage[kc[u]];
                    dd[u] = src.digit(from_words<R>(x[u]));
                }
                uint32_t c1[WB], c2[WB];
#pragma unroll
                for (int u = 0; u < WB; ++u) {
                    c1[u] = cur[dd[u]];
                    c2[u] = dstart[dd[u]];
                }
#pragma unroll
                for (int u = 0; u < WB; ++u)
                    *reinterpret_cast<W *>(&out[st + c1[u] + (kc[u] - c2[u])]) = x[u];
            }
        }
        __syncthreads();  // dstart / cur / stage are rewritten by the next bucket
        }  // !kMulti
    }
}

}  // namespace dpg
