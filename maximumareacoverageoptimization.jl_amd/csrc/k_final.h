// k_final.h — partial-sum reduction, objective penalty, cons3 mask and the poll argmin.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "predicate.h"
#include "k_common.h"

#pragma clang fp contract(off)

namespace mac {

constexpr int kFinC = 64;  // candidates per finalize block
constexpr int kFinT = 64;  // UAV indices per LDS tile

// Block = 64 candidates x 4 waves.
//  area_k  = sum over slices g of partial[g*K + k]: wave w sums slices g = w (mod 4) in order,
//            then the 4 wave sums are added in wave order (fixed => bit-reproducible). The slice
//            count is n_poll when *mode == poll, else n_other.
//  obj_k   = -area_k + penalty * violation_k, violation_k = sum_{i=0..N-1} |x[2N+i] - rmax[i]|
//            accumulated SEQUENTIALLY in i from 0.0 (src/TDM_STATIC_opt.jl:89-97, bit-exact).
//            The candidate columns are staged through LDS in 64 x 64 tiles (coalesced reads);
//            lane k of wave 0 then runs the sequential chain over its tile row.
//  cons3   (src/TDM_Constraints.jl:54-75) when prev != null: candidate k is infeasible when
//            any UAV has s > dlimT[i] (exact form of sqrt(s) > d_lim[i], predicate.h); its
//            objective becomes +inf (the extreme barrier never evaluates it).
__global__ __launch_bounds__(kBlock) void finalize_kernel(
    const double* __restrict__ partial, const int* __restrict__ mode, int n_poll, int n_other,
    int K, const double* __restrict__ cands, int N, int ldc, const double* __restrict__ rmax,
    double penalty, const double* __restrict__ prev, const double* __restrict__ dlimT,
    double tan_half_fov, double* __restrict__ area_out, double* __restrict__ obj_out)
{
    __shared__ double tile[kFinC][kFinT + 1];
    __shared__ double red[kWavesPerBlock][kFinC];
    __shared__ int infeas[kFinC];
    const int t = threadIdx.x, lane = t & (kWave - 1), grp = t / kWave;
    const int k0 = blockIdx.x * kFinC;
    const int k = k0 + lane;
    const bool valid = k < K;
    const int G = (mode && *mode == kModePoll) ? n_poll : n_other;

    double a = 0.0;
    if (valid)
        for (int g = grp; g < G; g += kWavesPerBlock) a += partial[(int64_t)g * K + k];
    red[grp][lane] = a;
    if (t < kFinC) infeas[t] = 0;
    __syncthreads();
    double area = 0.0;
    if (grp == 0) {
#pragma unroll
        for (int q = 0; q < kWavesPerBlock; ++q) area += red[q][lane];
        if (valid && area_out) area_out[k] = area;
    }
    if (!obj_out) return;  // uniform

    double violation = 0.0;
    for (int i0 = 0; i0 < N; i0 += kFinT) {
        const int ni = min(kFinT, N - i0);
        __syncthreads();
        for (int e = t; e < kFinC * kFinT; e += kBlock) {
            const int c = e / kFinT, ii = e % kFinT, kk = k0 + c;
            if (kk >= K || ii >= ni) continue;
            const double* x = cands + (int64_t)kk * ldc;
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
        if (grp == 0 && valid)
            for (int ii = 0; ii < ni; ++ii) violation += tile[lane][ii];
    }
    __syncthreads();
    if (grp == 0 && valid) {
        const double obj = -area + violation * penalty;
        obj_out[k] = infeas[lane] ? __builtin_inf() : obj;
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
