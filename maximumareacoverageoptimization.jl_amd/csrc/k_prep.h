// k_prep.h — per-poll disk preparation, per-disk regions and the device-side walk choice.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "predicate.h"
#include "k_common.h"

#pragma clang fp contract(off)

namespace mac {

// ------------------------------------------------------------------ per-batch disk prep

// cands: 3N x K column-major (candidate k at cands + k*ldc). Writes disks[k*N + i] (scan walk).
__global__ void disk_prep_kernel(const double* __restrict__ cands, int N, int ldc, int K,
                                 DiskRec* __restrict__ disks)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)N * K) return;
    const int k = (int)(t / N), i = (int)(t % N);
    const double* c = cands + (int64_t)k * ldc;
    disks[t] = make_disk(c[i], c[N + i], c[2 * N + i]);
}

// Transposed prep: disksT[i*K + k] (disk-major, candidates contiguous). 32 x 32 tiles through
// LDS so both the candidate reads and the record writes are coalesced.
__global__ __launch_bounds__(kBlock) void disk_prep_T_kernel(const double* __restrict__ cands,
                                                             int N, int ldc, int K,
                                                             DiskRec* __restrict__ disksT)
{
    __shared__ double sx[32][33], sy[32][33], sr[32][33];
    const int i0 = blockIdx.x * 32, k0 = blockIdx.y * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
    for (int kk = ty; kk < 32; kk += 8) {
        const int k = k0 + kk, i = i0 + tx;
        if (k < K && i < N) {
            const double* c = cands + (int64_t)k * ldc;
            sx[kk][tx] = c[i];
            sy[kk][tx] = c[N + i];
            sr[kk][tx] = c[2 * N + i];
        }
    }
    __syncthreads();
    for (int ii = ty; ii < 32; ii += 8) {
        const int i = i0 + ii, k = k0 + tx;
        if (k < K && i < N) disksT[(int64_t)i * K + k] = make_disk(sx[tx][ii], sy[tx][ii], sr[tx][ii]);
    }
}

// ------------------------------------------------------------------ region + decision

// Block i: union over the K candidates of disk i's tile span (region[i]) and two costs in
// point-visits / ppt: poll walk = K * |region|, per-candidate walk = sum_k |span_k|.
__global__ __launch_bounds__(kBlock) void region_kernel(const DiskRec* __restrict__ disksT,
                                                        int N, int K, Grid g,
                                                        int4* __restrict__ region,
                                                        double2* __restrict__ cost)
{
    const int i = blockIdx.x;
    int x0 = 0x7fffffff, y0 = 0x7fffffff, x1 = -1, y1 = -1;
    double cand = 0.0;
    for (int k = threadIdx.x; k < K; k += kBlock) {
        const DiskRec d = disksT[(int64_t)i * K + k];
        int4 sp;
        if (disk_span(d, g, sp)) {
            x0 = min(x0, sp.x);
            x1 = max(x1, sp.y);
            y0 = min(y0, sp.z);
            y1 = max(y1, sp.w);
            cand += (double)(sp.y - sp.x + 1) * (double)(sp.w - sp.z + 1);
        }
    }
    __shared__ int sh[4][kBlock];
    __shared__ double red[kWavesPerBlock];
    sh[0][threadIdx.x] = x0;
    sh[1][threadIdx.x] = -x1;
    sh[2][threadIdx.x] = y0;
    sh[3][threadIdx.x] = -y1;
    __syncthreads();
    for (int s = kBlock / 2; s > 0; s >>= 1) {
        if (threadIdx.x < s)
            for (int q = 0; q < 4; ++q) sh[q][threadIdx.x] = min(sh[q][threadIdx.x], sh[q][threadIdx.x + s]);
        __syncthreads();
    }
    const double candsum = block_sum_f64(cand, red);
    if (threadIdx.x == 0) {
        const int4 R = make_int4(sh[0][0], -sh[1][0], sh[2][0], -sh[3][0]);
        region[i] = R;
        const double rc = R.x <= R.y ? (double)(R.y - R.x + 1) * (double)(R.w - R.z + 1) : 0.0;
        cost[i] = make_double2(rc * (double)K, candsum);
    }
}

// One block: mode = poll walk when its point-visits stay within `ratio` x the per-candidate
// walk's (its visits are broadcast LDS reads; the other's are scattered global loads).
// mode[1] (the poll walk's disks-with-neighbours counter) is cleared here.
__global__ __launch_bounds__(kBlock) void decide_kernel(const double2* __restrict__ cost, int N,
                                                        double ratio, int forced,
                                                        int* __restrict__ mode)
{
    __shared__ double red[kWavesPerBlock];
    double a = 0.0, b = 0.0;
    for (int i = threadIdx.x; i < N; i += kBlock) {
        a += cost[i].x;
        b += cost[i].y;
    }
    const double A = block_sum_f64(a, red);
    __syncthreads();
    const double B = block_sum_f64(b, red);
    if (threadIdx.x == 0) {
        mode[0] = forced ? forced : (A <= ratio * B ? kModePoll : kModeTiled);
        mode[1] = 0;
    }
}

}  // namespace mac
