// k_final.h — objective penalty + cons3 mask, partial-sum reduction and the poll argmin.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "predicate.h"
#include "k_common.h"

#pragma clang fp contract(off)

namespace mac {

constexpr int kPenC = 64;   // candidates per penalty block
constexpr int kPenT = 64;   // UAV indices per LDS tile
constexpr int kFinC = 16;   // candidates per finalize block (x 16 slice groups)

// vp_k = violation_k * penalty with violation_k = sum_{i=0..N-1} |x[2N+i] - rmax[i]| accumulated
// SEQUENTIALLY in i from 0.0 (src/TDM_STATIC_opt.jl:89-97, bit-exact), or +inf when candidate k
// fails cons3 (src/TDM_Constraints.jl:54-75; prev != null; sqrt(s) > d_lim[i] evaluated exactly
// as s > dlimT[i], predicate.h), so -area + vp is the reference objective or +inf (the extreme
// barrier never evaluates it). Block = 64 candidates: their columns are staged through LDS in
// 64 x 64 tiles (coalesced reads); lane k of wave 0 runs the sequential chain over its tile row.
// Independent of the coverage walk: runs on a forked stream beside it.
__global__ __launch_bounds__(kBlock) void penalty_kernel(
    int K, const double* __restrict__ cands, int N, int ldc, const double* __restrict__ rmax,
    double penalty, const double* __restrict__ prev, const double* __restrict__ dlimT,
    double tan_half_fov, double* __restrict__ vp)
{
    __shared__ double tile[kPenC][kPenT + 1];
    __shared__ int infeas[kPenC];
    const int t = threadIdx.x, lane = t & (kWave - 1), grp = t / kWave;
    const int k0 = blockIdx.x * kPenC;
    const int k = k0 + lane;
    if (t < kPenC) infeas[t] = 0;
    double violation = 0.0;
    for (int i0 = 0; i0 < N; i0 += kPenT) {
        const int ni = min(kPenT, N - i0);
        __syncthreads();
        for (int e = t; e < kPenC * kPenT; e += kBlock) {
            const int c = e / kPenT, ii = e % kPenT, kc = k0 + c;
            if (kc >= K || ii >= ni) continue;
            const double* x = cands + (int64_t)kc * ldc;
            const int i = i0 + ii;
            tile[c][ii] = rmax ? __builtin_fabs(x[2 * N + i] - rmax[i]) : 0.0;
            if (prev) {
                const double x1 = prev[i], y1 = prev[N + i], z1 = prev[2 * N + i] / tan_half_fov;
                const double x2 = x[i], y2 = x[N + i], z2 = x[2 * N + i] / tan_half_fov;
                const double ddx = x1 - x2, ddy = y1 - y2, ddz = z1 - z2;
                const double s = ddx * ddx + ddy * ddy + ddz * ddz;
                if (s > dlimT[i]) infeas[c] = 1;  // benign race: every writer stores 1
            }
        }
        __syncthreads();
        if (grp == 0 && k < K)
            for (int ii = 0; ii < ni; ++ii) violation += tile[lane][ii];
    }
    __syncthreads();
    if (grp == 0 && k < K) vp[k] = infeas[lane] ? __builtin_inf() : violation * penalty;
}

// Block = 16 candidates x 16 slice groups. area_k = sum over slices g of partial[g*K + k] in a
// fixed order (thread (c, sg) sums g = sg, sg+16, ... into 4 interleaved accumulators combined
// in order, then the 16 groups in order): bit-reproducible, loads kept in flight. The slice
// count is n_poll when *mode == poll, else n_other. obj_k = -area_k + vp_k when vp != null.
__global__ __launch_bounds__(kBlock) void finalize_kernel(
    const double* __restrict__ partial, const int* __restrict__ mode, int n_poll, int n_other,
    int K, const double* __restrict__ vp, double* __restrict__ area_out,
    double* __restrict__ obj_out)
{
    __shared__ double red[kBlock / kFinC][kFinC];
    const int t = threadIdx.x, c = t % kFinC, sg = t / kFinC;
    constexpr int SG = kBlock / kFinC;
    const int k = blockIdx.x * kFinC + c;
    const int G = (mode && *mode == kModePoll) ? n_poll : n_other;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    if (k < K) {
        int g = sg;
        for (; g + 3 * SG < G; g += 4 * SG) {
            a0 += partial[(int64_t)g * K + k];
            a1 += partial[(int64_t)(g + SG) * K + k];
            a2 += partial[(int64_t)(g + 2 * SG) * K + k];
            a3 += partial[(int64_t)(g + 3 * SG) * K + k];
        }
        for (; g < G; g += SG) a0 += partial[(int64_t)g * K + k];
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
