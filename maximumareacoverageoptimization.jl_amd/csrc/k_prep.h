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
    const double* dlim;    // ... or the raw d_lim[i], thresholded where it is read (dlimT == null)
    double tan_half_fov;
};

// UAV i's cons3 threshold: dlimT[i], or dlim_threshold(d_lim[i]) (evaluated once per disk by the
// callers that loop over candidates, so the device API needs no threshold launch of its own)
__device__ __forceinline__ double pen_threshold(const PenArgs& pa, int i)
{
    if (!pa.prev) return 0.0;
    return pa.dlimT ? pa.dlimT[i] : dlim_threshold(pa.dlim[i]);
}

// Term i of candidate (x_i, y_i, R_i): |R_i - rmax_i| (0 without rmax), or -1 when UAV i's move
// violates cons3 (sqrt(dx^2 + dy^2 + dz^2) > d_lim[i], z = R / tan(FOV/2), evaluated exactly as
// s > T3 = pen_threshold(pa, i)). A negative term marks the candidate infeasible; the finalize
// chain sums the others sequentially in i (bit-exact with the reference's loop).
__device__ __forceinline__ double pen_term(double x2, double y2, double R2, int i, int N,
                                           const PenArgs& pa, double T3)
{
    if (pa.prev) {
        const double x1 = pa.prev[i], y1 = pa.prev[N + i], z1 = pa.prev[2 * N + i] / pa.tan_half_fov;
        const double z2 = R2 / pa.tan_half_fov;
        const double ddx = x1 - x2, ddy = y1 - y2, ddz = z1 - z2;
        const double s = ddx * ddx + ddy * ddy + ddz * ddz;
        if (s > T3) return -1.0;
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
    const float* keysT;    // matrix: fp32 keys, variable-major (cands_keys_kernel), when non-null
    const int* kbad;       // matrix: per (variable, 32-candidate tile) "a key is inexact" flags
    int nkt;               // tiles per variable
    const double* xinc;    // generator: incumbent (3N), row / column permutations (n each)
    const int* rp;
    const int* cp;
    uint64_t state;
    int64_t b;             // 2^ell
    int k0;                // generator: candidate k of this source is candidate k0 + k of the poll
                           // (a rank's shard of it)
    __device__ __forceinline__ double get(int kl, int v, int N) const
    {
        if (cands) return cands[(int64_t)kl * ldc + v];
        const int n = 3 * N;
        const int k = kl + k0;
        const int kk = k < n ? k : k - n;
        const double d = ltmads_entry(state, n, b, rp[v], cp[kk]);
        return k < n ? xinc[v] + d : xinc[v] - d;
    }
};

// cands (3N x K column-major) -> keysT (3N x K variable-major: candidates contiguous) of fp32
// keys, key = fl32(x - x0) with x0 = the variable's value in candidate 0, through 32 x 64 LDS
// tiles so that both sides are coalesced. A key is exact when x0 + (double)key reproduces x bit
// for bit (k_index.h "Keys"); kbad[v*nkt + tile] = 1 when some key of variable v in this tile is
// not (every tile writes its flag, so nothing needs clearing). Half the bytes of a transposed
// fp64 copy are written here and read by the index.
constexpr int kKeysK = 128;  // candidates per cands_keys_kernel tile (x 32 variables)

__global__ __launch_bounds__(kBlock) void cands_keys_kernel(uint64_t* ts, const double* __restrict__ cands,
                                                            int n, int K, float* __restrict__ keysT,
                                                            int* __restrict__ kbad, int nkt)
{
    ts_begin(ts);   // profiling only (the chain's first launch: k_common.h)
    constexpr int NB = kKeysK / 32;   // 32-candidate flag tiles per workgroup tile
    __shared__ float t[kKeysK][33];
    __shared__ int sbad[NB][32];
    const int v0 = blockIdx.x * 32, k0 = blockIdx.y * kKeysK;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 32 x 8
    if (threadIdx.x < 32 * NB) sbad[threadIdx.x >> 5][threadIdx.x & 31] = 0;
    const int vr = v0 + tx;
    const double base = vr < n ? cands[vr] : 0.0;
    constexpr int J = kKeysK / 8;
    double x[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {   // every load in flight at once
        const int k = k0 + ty + 8 * j;
        x[j] = (k < K && vr < n) ? cands[(int64_t)k * n + vr] : base;
    }
    bool ok[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) ok[b] = true;
#pragma unroll
    for (int j = 0; j < J; ++j) {   // candidate ty + 8j lies in flag tile (8j) / 32 = j / 4
        const float f = (float)(x[j] - base);
        ok[j / 4] &= __builtin_bit_cast(uint64_t, base + (double)f) == __builtin_bit_cast(uint64_t, x[j]);
        t[ty + 8 * j][tx] = f;
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < NB; ++b)
        if (!ok[b]) atomicOr(&sbad[b][tx], 1);
    // rows of kKeysK keys per variable: 64 consecutive threads write one row (256 B)
    const int kk = threadIdx.x & (kKeysK - 1), vq = threadIdx.x / kKeysK;
#pragma unroll
    for (int j = 0; j < 32 / (kBlock / kKeysK); ++j) {
        const int vv = vq + (kBlock / kKeysK) * j;
        const int v = v0 + vv, k = k0 + kk;
        if (k < K && v < n) keysT[(int64_t)v * K + k] = t[kk][vv];
    }
    __syncthreads();
    if (threadIdx.x < 32 * NB) {
        const int h = threadIdx.x >> 5, vv = threadIdx.x & 31, v = v0 + vv;
        const int tile = NB * blockIdx.y + h;
        if (v < n && tile < nkt) kbad[(int64_t)v * nkt + tile] = sbad[h][vv];
    }
    ts_end(ts);
}

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
    if (pen) pen[(int64_t)i * K + k] = pen_term(x, y, r, i, N, pa, pen_threshold(pa, i));
}

}  // namespace mac
