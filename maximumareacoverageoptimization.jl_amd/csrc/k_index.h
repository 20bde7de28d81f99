// k_index.h — per-poll disk index: one workgroup per UAV disk i, over all K candidates.
//
// Everything the tiled / poll walks need about disk i of candidate k depends only on that disk's
// own (cx, cy, r):
//   * its record {cx, cy, T(r), r};
//   * its objective-penalty term |r - r_max_i| and cons3 mark (pen_term);
//   * its tile span;
//   * in the poll walk, its credit over region i's non-shared entries (no other disk can cover
//     those, k_poll.h "Ownership").
// A MADS poll moves each UAV by small integer steps. LTMADS directions are columns of a
// lower-triangular basis with entries bounded by 2^ell, and about a quarter of them do not move a
// given UAV at all. So the K candidates hold far fewer DISTINCT disks per UAV: about 270 of 3073
// at ell = 2 in the config-4 polls.
//
// disk_index_kernel reads the K candidates' (x_i, y_i, r_i) once, straight from the candidate
// source (the matrix, or the LTMADS generator). It numbers the distinct disks in an LDS hash table
// (exact keys: the bit patterns of the three doubles) and writes per distinct disk u the record
// urec[i*K + u], plus the map umap[i*K + k] = u and the penalty term pen[i*K + k] for every
// candidate (computed once per distinct disk) and the count ucount[i]. It also writes disk i's region (the union of its tile
// spans over the K candidates) and the two walk costs (K * |region|, sum of span areas).
// Consumers read disk i of candidate k as urec[i*K + umap[i*K + k]]: the result is bit-identical
// to per-candidate records (same inputs, same arithmetic), and every candidate is still
// evaluated. Polls larger than kIndexMaxK use the identity map (one position per candidate).
//
// Workgroup b handles disk (b % 8) * ceil(N/8) + b / 8. Workgroups go to the 8 XCDs round-robin,
// so consecutive disks run on one XCD and share its L2 for the candidate matrix's cache lines
// (8 consecutive doubles of a column: 8 consecutive disks).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "predicate.h"
#include "k_common.h"
#include "k_prep.h"

#pragma clang fp contract(off)

namespace mac {

constexpr int kIndexSlots = 4096;            // LDS hash table (int32 slots)
#ifdef MAC_DIAG
__device__ uint64_t g_diag_index[8 * 65536];  // diagnostic build only: per-disk phase stamps
#define MAC_IDX_STAMP(q) if (threadIdx.x == 0 && i < 65536) g_diag_index[8 * i + (q)] = __builtin_amdgcn_s_memrealtime()
#else
#define MAC_IDX_STAMP(q)
#endif
constexpr int kIndexMaxK = 3584;             // larger polls: identity map (load <= 7/8)

__device__ __forceinline__ uint32_t key_hash(uint64_t a, uint64_t b, uint64_t c)
{
    uint64_t z = a * 0x9E3779B97F4A7C15ull;
    z ^= b + 0xBF58476D1CE4E5B9ull + (z << 6) + (z >> 2);
    z ^= c + 0x94D049BB133111EBull + (z << 6) + (z >> 2);
    z = (z ^ (z >> 31)) * 0xD6E8FEB86659FD93ull;
    return (uint32_t)(z ^ (z >> 32));
}

// tile span of disk (x, y, r): the same decision as disk_span(make_disk(x, y, r)) without the
// threshold (T(r) >= 0 exactly when r > 0)
__device__ __forceinline__ bool span_of(double x, double y, double r, const Grid& g, int4& sp)
{
    int x0, x1, y0, y1;
    if (!(r > 0.0)) return false;
    if (!tile_span(x, r, g.gx0, g.invS, g.nTx, x0, x1)) return false;
    if (!tile_span(y, r, g.gy0, g.invS, g.nTy, y0, y1)) return false;
    sp = make_int4(x0, x1, y0, y1);
    return true;
}

constexpr int kIdxThreads = 1024;            // 16 waves: the phases are latency-bound
constexpr int kIdxWaves = kIdxThreads / kWave;

struct IndexOut {
    DiskRec* urec;
    double* pen;     // per candidate: pen[i*K + k] (null: no objective)
    int* umap;
    int* ucount;
    int4* region;
    double2* cost;
    int* dcount;     // the poll walk's disks-with-neighbours counter, cleared here
};

__global__ __launch_bounds__(kIdxThreads) void disk_index_kernel(CandSrc src, int N, int K, Grid g,
                                                            PenArgs pa, int dedup, IndexOut o)
{
    __shared__ double kx[kIndexMaxK], ky[kIndexMaxK], kr[kIndexMaxK];
    __shared__ int table[kIndexSlots];       // owner candidate, then (owner << 12 | id)
    __shared__ uint16_t slot_of[kIndexMaxK];
    __shared__ uint16_t owner_of[kIndexMaxK];
    __shared__ int mult[kIndexMaxK];         // candidates per distinct disk
    __shared__ double s_pen[kIndexMaxK];     // penalty term per distinct disk
    __shared__ int ucnt;
    __shared__ int sred[4][kIdxWaves];
    __shared__ double dred[kIdxWaves];

    const int per_xcd = (N + 7) / 8;
    const int i = (int)(blockIdx.x % 8) * per_xcd + (int)(blockIdx.x / 8);
    if (i >= N) return;                                   // uniform
    MAC_IDX_STAMP(0);
    if (blockIdx.x == 0 && threadIdx.x == 0) *o.dcount = 0;
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
    const int64_t row = (int64_t)i * K;
    const bool hashed = dedup && K <= kIndexMaxK;

    int4 R = make_int4(0x7fffffff, -1, 0x7fffffff, -1);
    double span_area = 0.0;
    auto add_span = [&](double x, double y, double r, double m) {
        int4 sp;
        if (span_of(x, y, r, g, sp)) {
            R.x = min(R.x, sp.x);
            R.y = max(R.y, sp.y);
            R.z = min(R.z, sp.z);
            R.w = max(R.w, sp.w);
            span_area += m * ((double)(sp.y - sp.x + 1) * (double)(sp.w - sp.z + 1));
        }
    };

    if (!hashed) {  // identity: one position per candidate
        for (int k = tid; k < K; k += kIdxThreads) {
            const double x = src.get(k, i, N), y = src.get(k, N + i, N), r = src.get(k, 2 * N + i, N);
            add_span(x, y, r, 1.0);
            o.urec[row + k] = make_disk(x, y, r);
            if (o.pen) o.pen[row + k] = pen_term(x, y, r, i, N, pa);
            o.umap[row + k] = k;
        }
        if (tid == 0) o.ucount[i] = K;
    } else {
        // ---- keys to LDS (batched loads), table cleared
        constexpr int kIdxB = 4;
        const double* tx = src.candsT ? src.candsT + (int64_t)i * src.ldt : nullptr;
        const double* ty = tx ? tx + (int64_t)N * src.ldt : nullptr;
        const double* tr = tx ? ty + (int64_t)N * src.ldt : nullptr;
        for (int k0 = tid; k0 < K; k0 += kIdxThreads * kIdxB) {
            double bx_[kIdxB], by_[kIdxB], br_[kIdxB];
            if (tx) {  // rows of the transposed matrix: coalesced, all loads in flight
#pragma unroll
                for (int b = 0; b < kIdxB; ++b) {
                    const int kc = min(k0 + b * kIdxThreads, K - 1);
                    bx_[b] = tx[kc];
                    by_[b] = ty[kc];
                    br_[b] = tr[kc];
                }
            } else {
#pragma unroll
                for (int b = 0; b < kIdxB; ++b) {
                    const int kc = min(k0 + b * kIdxThreads, K - 1);
                    bx_[b] = src.get(kc, i, N);
                    by_[b] = src.get(kc, N + i, N);
                    br_[b] = src.get(kc, 2 * N + i, N);
                }
            }
#pragma unroll
            for (int b = 0; b < kIdxB; ++b) {
                const int k = k0 + b * kIdxThreads;
                if (k < K) {
                    kx[k] = bx_[b];
                    ky[k] = by_[b];
                    kr[k] = br_[b];
                }
            }
        }
        for (int q = tid; q < kIndexSlots; q += kIdxThreads) table[q] = -1;
        for (int q = tid; q < K; q += kIdxThreads) mult[q] = 0;
        if (tid == 0) ucnt = 0;
        __syncthreads();
        MAC_IDX_STAMP(1);
        // ---- insert (exact keys; linear probing)
        constexpr uint32_t mask = kIndexSlots - 1;
        for (int k = tid; k < K; k += kIdxThreads) {
            const uint64_t bx = __builtin_bit_cast(uint64_t, kx[k]);
            const uint64_t by = __builtin_bit_cast(uint64_t, ky[k]);
            const uint64_t br = __builtin_bit_cast(uint64_t, kr[k]);
            uint32_t s = key_hash(bx, by, br) & mask;
            for (;;) {
                int cur = table[s];
                if (cur < 0) {
                    cur = atomicCAS(&table[s], -1, k);
                    if (cur < 0) break;                      // claimed an empty slot
                }
                if (__builtin_bit_cast(uint64_t, kx[cur]) == bx &&
                    __builtin_bit_cast(uint64_t, ky[cur]) == by &&
                    __builtin_bit_cast(uint64_t, kr[cur]) == br)
                    break;                                   // same disk: share the slot
                s = (s + 1) & mask;                          // another disk: probe on
            }
            slot_of[k] = (uint16_t)s;
        }
        __syncthreads();
        MAC_IDX_STAMP(2);
        // ---- ids for the occupied slots (any order: nothing computed depends on the numbering)
        for (int q = tid; q < kIndexSlots; q += kIdxThreads) {
            const int owner = table[q];
            if (owner >= 0) {
                const int u = atomicAdd(&ucnt, 1);
                owner_of[u] = (uint16_t)owner;
                table[q] = (owner << 12) | u;
            }
        }
        __syncthreads();
        const int U = ucnt;
        // ---- per distinct disk: record and penalty term
        for (int u = tid; u < U; u += kIdxThreads) {
            const int k = owner_of[u];
            const double x = kx[k], y = ky[k], r = kr[k];
            o.urec[row + u] = make_disk(x, y, r);
            if (o.pen) s_pen[u] = pen_term(x, y, r, i, N, pa);
        }
        __syncthreads();
        MAC_IDX_STAMP(3);
        // ---- per candidate: the map, the penalty term, and the multiplicities
        for (int k = tid; k < K; k += kIdxThreads) {
            const int u = table[slot_of[k]] & 0xfff;
            o.umap[row + k] = u;
            if (o.pen) o.pen[row + k] = s_pen[u];
            atomicAdd(&mult[u], 1);
        }
        __syncthreads();
        // ---- spans of the distinct disks, weighted by multiplicity (region and walk costs)
        for (int u = tid; u < U; u += kIdxThreads) {
            const int k = owner_of[u];
            add_span(kx[k], ky[k], kr[k], (double)mult[u]);
        }
        if (tid == 0) o.ucount[i] = U;
    }
    MAC_IDX_STAMP(4);
    // ---- region (block min / max) and costs (block sum: exact, integer-valued)
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        R.x = min(R.x, __shfl_xor(R.x, off, kWave));
        R.y = max(R.y, __shfl_xor(R.y, off, kWave));
        R.z = min(R.z, __shfl_xor(R.z, off, kWave));
        R.w = max(R.w, __shfl_xor(R.w, off, kWave));
    }
    if (lane == 0) {
        sred[0][wid] = R.x;
        sred[1][wid] = R.y;
        sred[2][wid] = R.z;
        sred[3][wid] = R.w;
    }
    const double csum = block_sum_f64<kIdxWaves>(span_area, dred);   // (contains a barrier)
    if (tid == 0) {
        int4 Rg = make_int4(0x7fffffff, -1, 0x7fffffff, -1);
        for (int q = 0; q < kIdxWaves; ++q) {
            Rg.x = min(Rg.x, sred[0][q]);
            Rg.y = max(Rg.y, sred[1][q]);
            Rg.z = min(Rg.z, sred[2][q]);
            Rg.w = max(Rg.w, sred[3][q]);
        }
        if (Rg.x > Rg.y || Rg.z > Rg.w) Rg = make_int4(0x7fffffff, -1, 0x7fffffff, -1);
        o.region[i] = Rg;
        const double rc = Rg.x <= Rg.y ? (double)(Rg.y - Rg.x + 1) * (double)(Rg.w - Rg.z + 1) : 0.0;
        o.cost[i] = make_double2(rc * (double)K, csum);
    }
    MAC_IDX_STAMP(5);
}

// disk i of candidate k through the index
__device__ __forceinline__ DiskRec rec_of(const DiskRec* __restrict__ urec,
                                          const int* __restrict__ umap, int i, int K, int k)
{
    const int64_t row = (int64_t)i * K;
    return urec[row + umap[row + k]];
}

}  // namespace mac
