// k_closure.h — the single-candidate objective callback as ONE launch.
//
// DirectSearch calls the objective closure once per trial point (SetObjective,
// src/TDM_STATIC_opt.jl:125; AreaMaxObjective :82-100 -> calculateArea
// src/AreaCoverageCalculation.jl:63-78). For that path a batch chain (index, walk, finalize) is
// all latency, so mac_area_f64 runs one kernel instead: wave w of workgroup b = disk 4b + w.
//   1. every workgroup stages the candidate's N disks (x, y, r) in LDS (one coalesced read);
//   2. disk i's lower-index neighbours: the disks j < i that may share a covered entry with it
//      (disks_may_overlap, conservative), their exact thresholds T(r_j) in LDS;
//   3. the entries of disk i's tile span (CSR rows of the tile-sorted list, their offsets loaded
//      in one round trip beside step 2) that disk i covers and
//      no listed neighbour covers — each covered entry is credited to the LOWEST-index disk
//      covering it, so the sum over disks is the reference's first-hit `break` sum over the same
//      multiset of entries — counted (every weight equal: integer, exact in any order) or summed
//      in fp64 in a fixed order;
//   4. counts: one 64-bit atomic add per workgroup of (1 << 40 | count) — the workgroup whose add
//      sees N - 1 earlier arrivals holds the total; weights: the credit goes to part[i]
//      (agent-scope store, then one counter add) and the workgroup whose add arrives last sums
//      part[0 .. N) in disk order. It writes the area to the device word and to the caller's
//      mapped host slot {area bits, 0, seq, check} (k_final.h mirror_check): the host reads it
//      with no copy and no stream synchronisation.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "predicate.h"
#include "k_common.h"
#include "k_final.h"

#pragma clang fp contract(off)

namespace mac {

constexpr int kClosureMaxN = 2048;   // disks staged in LDS: 24 B each (dynamic LDS)
constexpr int kClosureNbr = 64;      // neighbours kept per disk (more: every lower-index disk)

__host__ __device__ inline size_t closure_lds_bytes(int N) { return (size_t)24 * (size_t)N; }

struct ClosureOut {
    unsigned long long* part;   // [N] per-disk credit (double bits), weighted entries
    unsigned long long* total;  // counts: {arrivals << 40 | covered entries}, zero between launches
    unsigned* arrive;           // weights: arrival counter, zero between launches
    double* area;               // the area on the device
    uint64_t* slot;             // mapped host slot {area bits, 0, seq, check}
    uint64_t seq;
};

// Disks per workgroup: one wave per disk (the candidate is staged once per 4 disks).
constexpr int kClosureDisksPerWG = kWavesPerBlock;

__global__ __launch_bounds__(kBlock) void closure_kernel(uint64_t* ts, const double* cand,
                                                         int N, Grid g, const double2* __restrict__ xy,
                                                         const double* __restrict__ w,
                                                         const int32_t* __restrict__ off, int counts,
                                                         double w0, ClosureOut o)
{
    ts_begin(ts);
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    double* sx = (double*)lds_raw;
    double* sy = sx + N;
    double* sr = sy + N;
    __shared__ int nb[kClosureDisksPerWG][kClosureNbr];
    __shared__ double nT[kClosureDisksPerWG][kClosureNbr];
    __shared__ int rs[kClosureDisksPerWG][kWave], rpre[kClosureDisksPerWG][kWave + 1];
    __shared__ unsigned long long wcnt[kClosureDisksPerWG];
    __shared__ int sarr;
    // grid.y: the candidates of a coalesced batch (mac_area_f64 callers arriving together), each
    // with its own counters, credits, device word and slot (ts: null for batches)
    {
        const int b = (int)blockIdx.y;
        cand += (size_t)b * 3 * (size_t)N;
        o.part += (size_t)b * (size_t)N;
        o.total += b;
        o.arrive += b;
        o.area += b;
        if (o.slot) o.slot += 4 * b;
    }
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
    const int i = blockIdx.x * kClosureDisksPerWG + wid;   // this wave's disk
    const bool valid = i < N;                                // (wave-uniform)
    for (int j = tid; j < N; j += kBlock) {
        sx[j] = cand[j];
        sy[j] = cand[N + j];
        sr[j] = cand[2 * N + j];
    }
    __syncthreads();
    double cx = 0.0, cy = 0.0, r = 0.0, T = -1.0;
    int x0 = 0, x1 = -1, y0 = 0, y1 = -1;
    bool any = false;
    if (valid) {
        cx = sx[i];
        cy = sy[i];
        r = sr[i];
        T = cover_threshold(r);
        any = T >= 0.0 && tile_span(cx, r, g.gx0, g.invS, g.nTx, x0, x1) &&
              tile_span(cy, r, g.gy0, g.invS, g.nTy, y0, y1);
    }
    // the span's row runs (a row of tiles is a contiguous run of the sorted list): lane = row,
    // every offset in flight during the neighbour tests, then a wave prefix; spans of more than
    // 64 rows walk row by row below
    const int nrows = any ? y1 - y0 + 1 : 0;
    const bool flat = nrows <= kWave;
    int rs0 = 0, rlen = 0;
    if (any && flat && lane < nrows) {
        const int64_t rb = (int64_t)(y0 + lane) * g.nTx;
        rs0 = off[rb + x0];
        rlen = off[rb + x1 + 1] - rs0;
    }
    // disk i's lower-index neighbours, compacted by ballot (list order is irrelevant: an OR)
    int nc = 0;
    if (any) {
        for (int j0 = 0; j0 < i; j0 += kWave) {
            const int j = j0 + lane;
            const bool hit = j < i && sr[j] > 0.0 && disks_may_overlap(cx, cy, r, sx[j], sy[j], sr[j]);
            const uint64_t bal = __ballot(hit);
            const int q = nc + __popcll(bal & ((1ull << lane) - 1));
            if (hit && q < kClosureNbr) nb[wid][q] = j;
            nc += __popcll(bal);
        }
    }
    if (any && flat) {
        const int incl = wave_incl_scan_i32(rlen, lane);
        if (lane < nrows) rs[wid][lane] = rs0;
        rpre[wid][lane + 1] = incl;
        if (lane == 0) rpre[wid][0] = 0;
    }
    __syncthreads();
    if (any && lane < min(nc, kClosureNbr)) nT[wid][lane] = cover_threshold(sr[nb[wid][lane]]);
    __syncthreads();
    uint64_t cnt = 0;
    double acc = 0.0;
    // entry j: covered by disk i and by none of its listed lower-index neighbours
    auto credit = [&](int j) {
        const double2 p = xy[j];
        if (!(sqdist(p.x, p.y, cx, cy) <= T)) return;
        bool owned = true;
        if (nc <= kClosureNbr) {
            for (int q = 0; q < nc && owned; ++q) {
                const int c2 = nb[wid][q];
                owned = !(sqdist(p.x, p.y, sx[c2], sy[c2]) <= nT[wid][q]);
            }
        } else {   // overflowed list: every lower-index disk
            for (int c2 = 0; c2 < i && owned; ++c2)
                owned = !(sqdist(p.x, p.y, sx[c2], sy[c2]) <= cover_threshold(sr[c2]));
        }
        if (owned) {
            ++cnt;
            if (!counts) acc += w[j];
        }
    };
    if (any && flat) {
        const int total = rpre[wid][nrows];
        for (int f = lane; f < total; f += kWave) {
            int lo = 0, hi = nrows - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (rpre[wid][mid] <= f) lo = mid; else hi = mid - 1;
            }
            credit(rs[wid][lo] + (f - rpre[wid][lo]));
        }
    } else if (any) {
        for (int ty = y0; ty <= y1; ++ty) {
            const int64_t rowbase = (int64_t)ty * g.nTx;
            const int s0 = off[rowbase + x0], e0 = off[rowbase + x1 + 1];
            for (int j = s0 + lane; j < e0; j += kWave) credit(j);
        }
    }
    // the area
    if (counts) {
#pragma unroll
        for (int off2 = 32; off2 >= 1; off2 >>= 1) cnt += __shfl_xor(cnt, off2, kWave);
        if (lane == 0) wcnt[wid] = cnt;
        __syncthreads();
        if (tid == 0) {
            uint64_t mine = 0;
#pragma unroll
            for (int q = 0; q < kClosureDisksPerWG; ++q) mine += wcnt[q];
            const uint64_t old = __hip_atomic_fetch_add(o.total, (1ull << 40) | mine, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
            if ((old >> 40) == (uint64_t)(gridDim.x - 1)) {   // the last arrival: the total
                const double area = (double)((old & ((1ull << 40) - 1)) + mine) * w0;
                __hip_atomic_store(o.total, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                o.area[0] = area;
                if (o.slot) {   // the device word first (ordering as the poll's mirror, k_final.h)
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    const uint64_t b = __builtin_bit_cast(uint64_t, area);
                    o.slot[0] = b;
                    o.slot[1] = 0;
                    o.slot[2] = o.seq;
                    o.slot[3] = mirror_check(b, 0, o.seq);
                }
            }
        }
        ts_end(ts);
        return;
    }
    const double v = wave_sum_f64(acc);   // disk i's credit (fixed butterfly)
    if (valid && lane == 0)
        __hip_atomic_store(o.part + i, __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (tid == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        sarr = (int)__hip_atomic_fetch_add(o.arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if ((unsigned)sarr != gridDim.x - 1) {   // uniform: not the last workgroup
        ts_end(ts);
        return;
    }
    // the last workgroup: the area over every disk's credit, in disk order per thread then in
    // thread order (fixed), from agent-scope loads of the published credits
    __shared__ double dred[kWavesPerBlock];
    double a = 0.0;
    for (int j = tid; j < N; j += kBlock)
        a += __builtin_bit_cast(double, __hip_atomic_load(o.part + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    const double area = block_sum_f64(a, dred);   // valid in thread 0
    if (tid == 0) {
        __hip_atomic_store(o.arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        o.area[0] = area;
        if (o.slot) {   // the device word first (ordering as the poll's mirror, k_final.h)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint64_t b = __builtin_bit_cast(uint64_t, area);
            o.slot[0] = b;
            o.slot[1] = 0;
            o.slot[2] = o.seq;
            o.slot[3] = mirror_check(b, 0, o.seq);
        }
    }
    ts_end(ts);
}

}  // namespace mac
