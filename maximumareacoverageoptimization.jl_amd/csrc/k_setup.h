// k_setup.h — once-per-MPC-step point-list set-up: bbox, tile binning, offsets, flags.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "predicate.h"
#include "k_common.h"

#pragma clang fp contract(off)

namespace mac {

// ------------------------------------------------------------------ set-up kernels

// Per-block min/max of finite x and y: out[blk] = {xmin, xmax, ymin, ymax}.
// Per block: bbox of the finite points, and wmix[b] = 1 when one of its weights differs (bit for
// bit) from w[0] (equal weights let the poll walk credit integer counts, k_poll.h).
__global__ __launch_bounds__(kBlock) void bbox_kernel(const double* __restrict__ x,
                                                      const double* __restrict__ y,
                                                      const double* __restrict__ w, int64_t M,
                                                      double4* __restrict__ out,
                                                      int* __restrict__ wmix)
{
    double xmn = __builtin_inf(), xmx = -__builtin_inf();
    double ymn = __builtin_inf(), ymx = -__builtin_inf();
    const uint64_t w0 = M > 0 ? __builtin_bit_cast(uint64_t, w[0]) : 0;
    bool mixed = false;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < M;
         i += (int64_t)gridDim.x * kBlock) {
        const double a = x[i], b = y[i];
        if (__builtin_isfinite(a)) { xmn = a < xmn ? a : xmn; xmx = a > xmx ? a : xmx; }
        if (__builtin_isfinite(b)) { ymn = b < ymn ? b : ymn; ymx = b > ymx ? b : ymx; }
        mixed |= __builtin_bit_cast(uint64_t, w[i]) != w0;
    }
    const int anym = __syncthreads_or(mixed);
    if (threadIdx.x == 0) wmix[blockIdx.x] = anym;
    __shared__ double4 sh[kBlock];
    sh[threadIdx.x] = make_double4(xmn, xmx, ymn, ymx);
    __syncthreads();
    for (int s = kBlock / 2; s > 0; s >>= 1) {
        if (threadIdx.x < s) {
            double4 a = sh[threadIdx.x], b = sh[threadIdx.x + s];
            a.x = b.x < a.x ? b.x : a.x;
            a.y = b.y > a.y ? b.y : a.y;
            a.z = b.z < a.z ? b.z : a.z;
            a.w = b.w > a.w ? b.w : a.w;
            sh[threadIdx.x] = a;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) out[blockIdx.x] = sh[0];
}

__global__ void tile_key_kernel(const double* __restrict__ x, const double* __restrict__ y,
                                int64_t M, Grid g, uint32_t* __restrict__ key,
                                uint32_t* __restrict__ idx)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M) return;
    const int tx = tile_of(x[i], g.gx0, g.invS, g.nTx);
    const int ty = tile_of(y[i], g.gy0, g.invS, g.nTy);
    key[i] = (uint32_t)ty * (uint32_t)g.nTx + (uint32_t)tx;
    idx[i] = (uint32_t)i;
}

__global__ void gather_sorted_kernel(const double* __restrict__ x, const double* __restrict__ y,
                                     const double* __restrict__ w,
                                     const uint32_t* __restrict__ perm, int64_t M,
                                     double2* __restrict__ xys, double* __restrict__ ws)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M) return;
    const uint32_t p = perm[i];
    xys[i] = make_double2(x[p], y[p]);
    ws[i] = w[p];
}

// off[t] = first sorted position with key >= t (lower bound), t in [0, nTiles].
__global__ void tile_offsets_kernel(const uint32_t* __restrict__ key, int64_t M, int64_t nTiles,
                                    int32_t* __restrict__ off)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t > nTiles) return;
    int64_t lo = 0, hi = M;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if ((int64_t)key[mid] < t) lo = mid + 1; else hi = mid;
    }
    off[t] = (int32_t)lo;
}

// Streaming copy of interleaved xy for the scan path when points are unsorted.
__global__ void pack_xy_kernel(const double* __restrict__ x, const double* __restrict__ y,
                               int64_t M, double2* __restrict__ xy)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < M) xy[i] = make_double2(x[i], y[i]);
}

// Covered flags on the sorted list by the disk-major walk (idempotent byte stores), one
// candidate (the current UAV footprints), used by rmvCoveredPOI.
__global__ __launch_bounds__(kBlock) void covered_flags_tiled_kernel(
    const double2* __restrict__ xy, const int32_t* __restrict__ off, Grid g,
    const DiskRec* __restrict__ disks, int N, uint8_t* __restrict__ flag_sorted)
{
    const int lane = threadIdx.x & (kWave - 1);
    const int gw = (blockIdx.x * kBlock + threadIdx.x) / kWave;
    const int nw = gridDim.x * kWavesPerBlock;
    for (int c = gw; c < N; c += nw) {
        const DiskRec d = disks[c];
        int x0, x1, y0, y1;
        if (!(d.T >= 0.0) || !tile_span(d.cx, d.r, g.gx0, g.invS, g.nTx, x0, x1) ||
            !tile_span(d.cy, d.r, g.gy0, g.invS, g.nTy, y0, y1))
            continue;
        for (int ty = y0; ty <= y1; ++ty) {
            const int64_t rowbase = (int64_t)ty * g.nTx;
            const int s = off[rowbase + x0], e = off[rowbase + x1 + 1];
            for (int j = s + lane; j < e; j += kWave) {
                const double2 p = xy[j];
                if (sqdist(p.x, p.y, d.cx, d.cy) <= d.T) flag_sorted[j] = 1;
            }
        }
    }
}

__global__ void scatter_flags_kernel(const uint8_t* __restrict__ flag_sorted,
                                     const uint32_t* __restrict__ perm, int64_t M,
                                     uint8_t* __restrict__ flag_orig)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < M) flag_orig[perm[i]] = flag_sorted[i];
}

// keep[i] = !covered[i] (for the order-preserving compaction)
__global__ void invert_flags_kernel(const uint8_t* __restrict__ in, int64_t M,
                                    uint8_t* __restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < M) out[i] = in[i] ? 0 : 1;
}

}  // namespace mac
