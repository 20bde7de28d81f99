// k_prep.h — per-poll disk preparation, per-disk regions and the device-side walk choice.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "predicate.h"
#include "k_common.h"

#pragma clang fp contract(off)

namespace mac {

// ------------------------------------------------------------------ per-batch disk prep

// Objective-penalty inputs (src/TDM_STATIC_opt.jl:89-97) and the cons3 constraint
// (src/TDM_Constraints.jl:54-75). rmax == null: no penalty term; prev == null: no cons3.
struct PenArgs {
    const double* rmax;
    const double* prev;
    const double* dlimT;   // per UAV: cons3 holds iff s <= dlimT[i] (predicate.h dlim_threshold)
    double tan_half_fov;
};

// Term i of candidate (x_i, y_i, R_i): |R_i - rmax_i| (0 without rmax), or -1 when UAV i's move
// violates cons3 (sqrt(dx^2 + dy^2 + dz^2) > d_lim[i], z = R / tan(FOV/2), evaluated exactly as
// s > dlimT[i]). A negative term marks the candidate infeasible; the finalize chain sums the
// others sequentially in i (bit-exact with the reference's loop).
__device__ __forceinline__ double pen_term(double x2, double y2, double R2, int i, int N,
                                           const PenArgs& pa)
{
    if (pa.prev) {
        const double x1 = pa.prev[i], y1 = pa.prev[N + i], z1 = pa.prev[2 * N + i] / pa.tan_half_fov;
        const double z2 = R2 / pa.tan_half_fov;
        const double ddx = x1 - x2, ddy = y1 - y2, ddz = z1 - z2;
        const double s = ddx * ddx + ddy * ddy + ddz * ddz;
        if (s > pa.dlimT[i]) return -1.0;
    }
    return pa.rmax ? __builtin_fabs(R2 - pa.rmax[i]) : 0.0;
}

// ------------------------------------------------------------------ candidate sources

// splitmix64 stream value number `idx` (1-based) after `state` (workloads.SplitMix64).
__host__ __device__ __forceinline__ uint64_t splitmix_at(uint64_t state, uint64_t idx)
{
    uint64_t z = state + idx * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__host__ __device__ __forceinline__ double splitmix_uniform_at(uint64_t state, uint64_t idx)
{
    return (double)(splitmix_at(state, idx) >> 11) * (1.0 / 9007199254740992.0);
}

// Entry (r, c) of the lower-triangular LTMADS matrix L drawn from the stream at `state`
// (workloads.ltmads_basis): diagonal sign(u_{r+1} < 0.5 ? -1 : 1) * 2^ell; strictly lower
// entries uniform integers in [-(2^ell - 1), 2^ell - 1] from stream values n + 1 + r(r-1)/2 + c
// (numpy's tril_indices order); zero above the diagonal.
__host__ __device__ __forceinline__ double ltmads_entry(uint64_t state, int64_t n, int64_t b,
                                                        int64_t r, int64_t c)
{
    if (r < c) return 0.0;
    if (r == c) return (splitmix_uniform_at(state, (uint64_t)r + 1) < 0.5 ? -1.0 : 1.0) * (double)b;
    const int64_t lo = -b + 1, span = 2 * b - 1;
    const double u = splitmix_uniform_at(state, (uint64_t)(n + 1 + r * (r - 1) / 2 + c));
    return (double)(lo + (int64_t)__builtin_floor(u * (double)span));
}

// Where candidate coordinates come from: a 3N x K column-major matrix (the batch APIs), or a
// complete LTMADS poll around an incumbent generated on the fly (the native MADS driver):
// candidate k < n is x + B[:, k], k >= n is x - B[:, k - n], B = L[rp][:, cp] (variable v of a
// candidate = x_i for v = i, y_i for v = N + i, r_i for v = 2N + i).
struct CandSrc {
    const double* cands;   // matrix source when non-null
    int ldc;
    const double* xinc;    // generator: incumbent (3N), row / column permutations (n each)
    const int* rp;
    const int* cp;
    uint64_t state;
    int64_t b;             // 2^ell
    __device__ __forceinline__ double get(int k, int v, int N) const
    {
        if (cands) return cands[(int64_t)k * ldc + v];
        const int n = 3 * N;
        const int kk = k < n ? k : k - n;
        const double d = ltmads_entry(state, n, b, rp[v], cp[kk]);
        return k < n ? xinc[v] + d : xinc[v] - d;
    }
};

// cands: see CandSrc. Writes disks[k*N + i] (scan walk) and, when pen != null,
// pen[i*K + k] = pen_term (disk-major, as penalty_chain reads it).
__global__ void disk_prep_kernel(CandSrc src, int N, int K, DiskRec* __restrict__ disks,
                                 PenArgs pa, double* __restrict__ pen)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)N * K) return;
    const int k = (int)(t / N), i = (int)(t % N);
    const double x = src.get(k, i, N), y = src.get(k, N + i, N), r = src.get(k, 2 * N + i, N);
    disks[t] = make_disk(x, y, r);
    if (pen) pen[(int64_t)i * K + k] = pen_term(x, y, r, i, N, pa);
}

// Transposed prep: disksT[i*K + k] (disk-major, candidates contiguous). 32 x 32 tiles through
// LDS so both the candidate reads (matrix source) and the record writes are coalesced. Also, per tile:
//   penT[i*K + k] = pen_term (when penT != null), and
//   regP[kt*N + i], costP[kt*N + i] (kt = blockIdx.y): the union of disk i's tile spans over the
//   tile's 32 candidates and the sum of their span areas (when regP != null; region_kernel
//   finishes the reduction over kt).
__global__ __launch_bounds__(kBlock) void disk_prep_T_kernel(
    CandSrc src, int N, int K, DiskRec* __restrict__ disksT,
    PenArgs pa, double* __restrict__ penT, Grid g, int4* __restrict__ regP,
    double* __restrict__ costP)
{
    __shared__ double sx[32][33], sy[32][33], sr[32][33];
    const int i0 = blockIdx.x * 32, k0 = blockIdx.y * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
    for (int kk = ty; kk < 32; kk += 8) {
        const int k = k0 + kk, i = i0 + tx;
        if (k < K && i < N) {
            sx[kk][tx] = src.get(k, i, N);
            sy[kk][tx] = src.get(k, N + i, N);
            sr[kk][tx] = src.get(k, 2 * N + i, N);
        }
    }
    __syncthreads();
    for (int ii = ty; ii < 32; ii += 8) {
        const int i = i0 + ii, k = k0 + tx;
        int4 sp = make_int4(0x7fffffff, -1, 0x7fffffff, -1);
        double area = 0.0;
        if (k < K && i < N) {
            const double x = sx[tx][ii], y = sy[tx][ii], r = sr[tx][ii];
            const DiskRec d = make_disk(x, y, r);
            disksT[(int64_t)i * K + k] = d;
            if (penT) penT[(int64_t)i * K + k] = pen_term(x, y, r, i, N, pa);
            int4 s;
            if (regP && disk_span(d, g, s)) {
                sp = s;
                area = (double)(s.y - s.x + 1) * (double)(s.w - s.z + 1);
            }
        }
        if (regP) {
            // the 32 candidates of disk i sit in 32 consecutive lanes: butterfly over them
#pragma unroll
            for (int o = 16; o >= 1; o >>= 1) {
                sp.x = min(sp.x, __shfl_xor(sp.x, o, 32));
                sp.y = max(sp.y, __shfl_xor(sp.y, o, 32));
                sp.z = min(sp.z, __shfl_xor(sp.z, o, 32));
                sp.w = max(sp.w, __shfl_xor(sp.w, o, 32));
                area += __shfl_xor(area, o, 32);
            }
            if (tx == 0 && i < N) {
                regP[(int64_t)blockIdx.y * N + i] = sp;
                costP[(int64_t)blockIdx.y * N + i] = area;
            }
        }
    }
}

// ------------------------------------------------------------------ region + decision

// One wave per disk i: region[i] = union over the KT candidate tiles of regP (the union of
// disk i's tile spans over all K candidates) and cost[i] = (K * |region|, sum of span areas):
// the point visits of the poll walk and of the per-candidate walk, in units of ppt.
// Block 0 also clears the poll walk's disks-with-neighbours counter.
__global__ __launch_bounds__(kWave) void region_kernel(const int4* __restrict__ regP,
                                                       const double* __restrict__ costP, int N,
                                                       int KT, int K, int4* __restrict__ region,
                                                       double2* __restrict__ cost,
                                                       int* __restrict__ dcount)
{
    if (blockIdx.x == 0 && threadIdx.x == 0) *dcount = 0;  // neighbors_kernel appends after us
    const int i = blockIdx.x, lane = threadIdx.x;
    int4 R = make_int4(0x7fffffff, -1, 0x7fffffff, -1);
    double c = 0.0;
    for (int kt = lane; kt < KT; kt += kWave) {
        const int4 p = regP[(int64_t)kt * N + i];
        R.x = min(R.x, p.x);
        R.y = max(R.y, p.y);
        R.z = min(R.z, p.z);
        R.w = max(R.w, p.w);
        c += costP[(int64_t)kt * N + i];
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        R.x = min(R.x, __shfl_xor(R.x, o, kWave));
        R.y = max(R.y, __shfl_xor(R.y, o, kWave));
        R.z = min(R.z, __shfl_xor(R.z, o, kWave));
        R.w = max(R.w, __shfl_xor(R.w, o, kWave));
        c += __shfl_xor(c, o, kWave);
    }
    if (lane == 0) {
        if (R.x > R.y || R.z > R.w) R = make_int4(0x7fffffff, -1, 0x7fffffff, -1);
        region[i] = R;
        const double rc = R.x <= R.y ? (double)(R.y - R.x + 1) * (double)(R.w - R.z + 1) : 0.0;
        cost[i] = make_double2(rc * (double)K, c);
    }
}

}  // namespace mac
