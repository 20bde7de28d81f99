// k_final.h — objective penalty + cons3 mask, partial-sum reduction and the poll argmin.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "predicate.h"
#include "k_common.h"

#pragma clang fp contract(off)

namespace mac {

constexpr int kFinC = 16;   // candidates per finalize block (x 16 slice groups)
constexpr int kMaxMaskWords = (65535 + 31) / 32;   // N <= 65535 (mac_* argument check)

// Sequential objective penalty of candidate k (src/TDM_STATIC_opt.jl:89-97): violation =
// sum_{i=0..N-1} pen[i*K + umap[i*K + k]] (the disk index, k_index.h; pen[i*K + k] without a
// map) accumulated IN ORDER from 0.0 (bit-exact with the reference's
// loop); vp = violation * penalty, or +inf when a term is negative (cons3 fails,
// src/TDM_Constraints.jl:54-75: the extreme barrier never evaluates the objective). The chain is
// latency-bound (N dependent adds), so loads run kChainB ahead; lanes are consecutive
// candidates (coalesced). Used by the poll kernel's leading workgroups (overlapping the walk)
// and by penalty_chain_kernel on the other paths.
constexpr int kChainB = 32;
__device__ __forceinline__ void penalty_chain(const double* __restrict__ pen,
                                              const int* __restrict__ umap, int K, int N, int k,
                                              double penalty, double* __restrict__ vp)
{
    double violation = 0.0;
    bool infeasible = false;
    int i = 0;
    for (; i + kChainB <= N; i += kChainB) {
        int pos[kChainB];
#pragma unroll
        for (int j = 0; j < kChainB; ++j)
            pos[j] = umap ? umap[(int64_t)(i + j) * K + k] : k;
        double v[kChainB];
#pragma unroll
        for (int j = 0; j < kChainB; ++j) v[j] = pen[(int64_t)(i + j) * K + pos[j]];
#pragma unroll
        for (int j = 0; j < kChainB; ++j) {
            infeasible |= v[j] < 0.0;
            violation += v[j];
        }
    }
    for (; i < N; ++i) {
        const int64_t r = (int64_t)i * K;
        const double v = pen[r + (umap ? umap[r + k] : k)];
        infeasible |= v < 0.0;
        violation += v;
    }
    vp[k] = infeasible ? __builtin_inf() : violation * penalty;
}

__global__ __launch_bounds__(kBlock) void penalty_chain_kernel(const double* __restrict__ pen,
                                                               const int* __restrict__ umap, int K,
                                                               int N, double penalty,
                                                               double* __restrict__ vp)
{
    const int k = blockIdx.x * kBlock + threadIdx.x;
    if (k < K) penalty_chain(pen, umap, K, N, k, penalty, vp);
}

// Block = 16 candidates x 16 slice groups. area_k = sum over slices g of partial[g*K + k] in a
// fixed order (thread (c, sg) sums g = sg, sg+16, ... into 4 interleaved accumulators combined
// in order, then the 16 groups in order): bit-reproducible, loads kept in flight. The slice
// count is n_poll when *mode == poll, else n_other. With spart != null and the poll walk chosen,
// the shared-entry rows spart[i*K + k] of the disks with ncount[i] > 0 are added too (ascending
// i within each slice group: fixed order). obj_k = -area_k + vp_k when obj_out != null.
__global__ __launch_bounds__(kBlock) void finalize_kernel(
    const double* __restrict__ partial, const int* __restrict__ mode, int n_poll, int n_other,
    int K, int N, const int* __restrict__ map, const double* __restrict__ spart,
    const int* __restrict__ ncount,
    const double* __restrict__ vp, double* __restrict__ area_out, double* __restrict__ obj_out)
{
    __shared__ double red[kBlock / kFinC][kFinC];
    __shared__ uint32_t smask[kMaxMaskWords];   // disks whose shared-entry row exists
    const int t = threadIdx.x, c = t % kFinC, sg = t / kFinC;
    constexpr int SG = kBlock / kFinC;
    const int k0 = blockIdx.x * kFinC;
    const int k = k0 + c;
    const int G = (mode && *mode == kModePoll) ? n_poll : n_other;
    const bool rows = spart && mode && *mode == kModePoll;
    if (rows) {
        const int nw = (N + 31) / 32;
        for (int q = t; q < nw; q += kBlock) smask[q] = 0u;
        __syncthreads();
        for (int i = t; i < N; i += kBlock)
            if (ncount[i] > 0) atomicOr(&smask[i >> 5], 1u << (i & 31));
        __syncthreads();
    }
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    // poll walk with distinct-disk positions: row g's credit for candidate k sits at map[g*K+k]
    const int* mp = (map && rows) ? map : nullptr;
    auto at = [&](int g) -> double {
        const int64_t r = (int64_t)g * K;
        return partial[r + (mp ? mp[r + k] : k)];
    };
    if (k < K) {
        int g = sg;
        for (; g + 3 * SG < G; g += 4 * SG) {
            a0 += at(g);
            a1 += at(g + SG);
            a2 += at(g + 2 * SG);
            a3 += at(g + 3 * SG);
        }
        for (; g < G; g += SG) a0 += at(g);
        // poll walk: the shared-entry rows of the disks that have lower-index neighbours
        if (rows)
            for (int i = sg; i < N; i += SG)
                if (smask[i >> 5] & (1u << (i & 31))) a3 += spart[(int64_t)i * K + k];
    }
    red[sg][c] = ((a0 + a1) + a2) + a3;

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
// best[0] = objective, best[1] = index (int64 bits), index = idx_base + k, -1 if none.
__global__ __launch_bounds__(kBlock) void argmin_kernel(const double* __restrict__ obj, int K,
                                                        int64_t idx_base, double* __restrict__ best)
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
    }
}

__global__ void dlim_threshold_kernel(const double* __restrict__ dlim, int N,
                                      double* __restrict__ out)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < N) out[i] = dlim_threshold(dlim[i]);
}

}  // namespace mac
