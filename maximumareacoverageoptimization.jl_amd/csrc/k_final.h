// k_final.h — objective penalty + cons3 mask, partial-sum reduction and the poll argmin.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "predicate.h"
#include "k_common.h"

#pragma clang fp contract(off)

namespace mac {

constexpr int kFinC = 16;   // candidates per finalize block (x 64 slice groups)
constexpr int kFinThreads = 1024;
constexpr int kMaxMaskWords = (65535 + 31) / 32;   // N <= 65535 (mac_* argument check)

// Sequential objective penalty (src/TDM_STATIC_opt.jl:88-92): violation_k = sum over i = 0..N-1
// of pen[i*K + k] (the index's per-candidate term, k_index.h), accumulated IN ORDER from 0.0
// (bit-exact with the reference's loop); vp_k = violation_k * penalty, or +inf when a term is
// negative (cons3 fails, src/TDM_Constraints.jl:54-75: the extreme barrier never evaluates the
// objective).
//
// One workgroup = kChainC candidates x kChainG disk groups. Thread (c, grp) loads its group's
// kChainSeg consecutive disks of candidate k0 + c in one go (rows of 16 consecutive candidates:
// one cache line per row; every load in flight at once), then the running sum is relayed through
// LDS: group 0 adds its terms, then group 1, ... (one barrier per group), so the additions stay
// in order while the loads cost one latency per kChainG * kChainSeg disks instead of one per
// disk. Used by the poll kernel's chain workgroups (overlapping the walk) and by
// penalty_chain_kernel on the other paths. Needs kChainG * kChainC == kBlock threads.
constexpr int kChainC = 16;
constexpr int kChainG = kBlock / kChainC;
constexpr int kChainSeg = 32;
__device__ __forceinline__ void penalty_chain_block(const double* __restrict__ pen, int K, int N,
                                                    int k0, double penalty,
                                                    double* __restrict__ vp)
{
    __shared__ double carry[kChainC];
    __shared__ int bad[kChainC];
    const int t = threadIdx.x, c = t % kChainC, grp = t / kChainC;
    const int k = k0 + c;
    if (t < kChainC) {
        carry[t] = 0.0;
        bad[t] = 0;
    }
    for (int base = 0; base < N; base += kChainG * kChainSeg) {
        const int i0 = base + grp * kChainSeg;
        double v[kChainSeg];
#pragma unroll
        for (int j = 0; j < kChainSeg; ++j) {
            const int ii = i0 + j;
            v[j] = (k < K && ii < N) ? pen[(int64_t)ii * K + k] : 0.0;   // pad: + 0.0, exact
        }
        __syncthreads();
        for (int sgrp = 0; sgrp < kChainG; ++sgrp) {
            if (grp == sgrp) {
                double acc = carry[c];
                bool neg = false;
#pragma unroll
                for (int j = 0; j < kChainSeg; ++j) {
                    neg |= v[j] < 0.0;
                    acc += v[j];
                }
                carry[c] = acc;
                if (neg) bad[c] = 1;
            }
            __syncthreads();
        }
    }
    if (t < kChainC && k < K) vp[k] = bad[t] ? __builtin_inf() : carry[t] * penalty;
}

__global__ __launch_bounds__(kBlock) void penalty_chain_kernel(const double* __restrict__ pen,
                                                               int K, int N, double penalty,
                                                               double* __restrict__ vp)
{
    penalty_chain_block(pen, K, N, blockIdx.x * kChainC, penalty, vp);
}

// Block = 16 candidates x 64 slice groups. area_k = sum over slices g of partial[g*K + k] in a
// fixed order (thread (c, sg) sums g = sg, sg+64, ... in batches of 8, then the 64 groups in
// order): bit-reproducible, loads kept in flight. The slice
// count is n_poll when *mode == poll, else n_other. With spart != null and the poll walk chosen,
// the shared-entry rows spart[i*K + k] of the disks with ncount[i] > 0 are added too (ascending
// i within each slice group: fixed order). obj_k = -area_k + vp_k when obj_out != null.
__global__ __launch_bounds__(kFinThreads) void finalize_kernel(
    const double* __restrict__ partial, const int* __restrict__ mode, int n_poll, int n_other,
    int K, int N, const int* __restrict__ map, const double* __restrict__ spart,
    const int* __restrict__ ncount,
    const double* __restrict__ vp, double* __restrict__ area_out, double* __restrict__ obj_out)
{
    __shared__ double red[kFinThreads / kFinC][kFinC];
    __shared__ uint32_t smask[kMaxMaskWords];   // disks whose shared-entry row exists
    const int t = threadIdx.x, c = t % kFinC, sg = t / kFinC;
    constexpr int SG = kFinThreads / kFinC;
    const int k0 = blockIdx.x * kFinC;
    const int k = k0 + c;
    const int G = (mode && *mode == kModePoll) ? n_poll : n_other;
    const bool rows = spart && mode && *mode == kModePoll;
    if (rows) {
        const int nw = (N + 31) / 32;
        for (int q = t; q < nw; q += kFinThreads) smask[q] = 0u;
        __syncthreads();
        for (int i = t; i < N; i += kFinThreads)
            if (ncount[i] > 0) atomicOr(&smask[i >> 5], 1u << (i & 31));
        __syncthreads();
    }
    // Rows in batches of kFinB per thread, every load of a batch issued before any is used (the
    // map loads, then the gathers they index): latency paid once per batch, not per row. Each
    // batch is added in order to one accumulator: fixed order.
    constexpr int kFinB = 8;
    double acc = 0.0;
    // poll walk with distinct-disk positions: row g's credit for candidate k sits at map[g*K+k]
    const int* mp = (map && rows) ? map : nullptr;
    if (k < K) {
        for (int g = sg; g < G; g += kFinB * SG) {
            int pos[kFinB];
#pragma unroll
            for (int b = 0; b < kFinB; ++b) {
                const int gb = g + b * SG;
                pos[b] = gb < G ? (mp ? mp[(int64_t)gb * K + k] : k) : -1;
            }
            double v[kFinB];
#pragma unroll
            for (int b = 0; b < kFinB; ++b)
                v[b] = pos[b] >= 0 ? partial[(int64_t)(g + b * SG) * K + pos[b]] : 0.0;
            double bs = 0.0;
#pragma unroll
            for (int b = 0; b < kFinB; ++b) bs += v[b];
            acc += bs;
        }
        // poll walk: the shared-entry rows of the disks that have lower-index neighbours (other
        // disks' rows are never written and never read; a batch's idle slots add +0.0, which
        // leaves every sum unchanged)
        if (rows)
            for (int i = sg; i < N; i += kFinB * SG) {
                double v[kFinB];
#pragma unroll
                for (int b = 0; b < kFinB; ++b) {
                    const int ib = i + b * SG;
                    v[b] = (ib < N && (smask[ib >> 5] & (1u << (ib & 31))))
                               ? spart[(int64_t)ib * K + k] : 0.0;
                }
                double bs = 0.0;
#pragma unroll
                for (int b = 0; b < kFinB; ++b) bs += v[b];
                acc += bs;
            }
    }
    red[sg][c] = acc;

    __syncthreads();
    if (sg == 0 && k < K) {
        double area = 0.0;
#pragma unroll
        for (int q = 0; q < SG; ++q) area += red[q][c];
        if (area_out) area_out[k] = area;
        if (obj_out) obj_out[k] = -area + vp[k];
    }
}

// Single block: lexicographic minimum over (obj, index); NaN / +inf never selected.
// best[0] = objective, best[1] = index (int64 bits), index = idx_base + k, -1 if none. With a
// mirror (mapped pinned host memory), the two words are also written there followed by seq in
// mirror[2], so the host reads the result without a copy (mac_best_fetch).
__global__ __launch_bounds__(kBlock) void argmin_kernel(const double* __restrict__ obj, int K,
                                                        int64_t idx_base, double* __restrict__ best,
                                                        double* __restrict__ mirror, uint64_t seq)
{
    __shared__ double sv[kBlock];
    __shared__ int si[kBlock];
    double bv = __builtin_inf();
    int bi = -1;
    for (int k = threadIdx.x; k < K; k += kBlock) {
        const double v = obj[k];
        if (v < bv) { bv = v; bi = k; }  // ascending k per thread: first minimum kept
    }
    sv[threadIdx.x] = bv;
    si[threadIdx.x] = bi;
    __syncthreads();
    for (int s = kBlock / 2; s > 0; s >>= 1) {
        if (threadIdx.x < s) {
            const double v2 = sv[threadIdx.x + s];
            const int i2 = si[threadIdx.x + s];
            const double v1 = sv[threadIdx.x];
            const int i1 = si[threadIdx.x];
            const bool take = (i2 >= 0) && (i1 < 0 || v2 < v1 || (v2 == v1 && i2 < i1));
            if (take) { sv[threadIdx.x] = v2; si[threadIdx.x] = i2; }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const int i = si[0];
        best[0] = i >= 0 ? sv[0] : __builtin_inf();
        const int64_t gidx = i >= 0 ? idx_base + i : (int64_t)-1;
        best[1] = __builtin_bit_cast(double, gidx);
        if (mirror) {  // pinned coherent host words: the result, then (released) its sequence number
            mirror[0] = best[0];
            mirror[1] = best[1];
            __threadfence_system();
            __hip_atomic_store(reinterpret_cast<uint64_t*>(mirror + 2), seq, __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

__global__ void dlim_threshold_kernel(const double* __restrict__ dlim, int N,
                                      double* __restrict__ out)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < N) out[i] = dlim_threshold(dlim[i]);
}

}  // namespace mac
