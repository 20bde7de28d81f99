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
    const int* kbad;       // matrix: per (column-pass block, variable) "a key is inexact" flags
    int nkt;               // column-pass blocks (flags) per variable
    int ldk;               // keysT row pitch (keys_ld(K))
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

// ------------------------------------------------------------------ the column pass
// The first launch of every evaluation: one 16-wave workgroup per kColC = 16 consecutive
// candidates (columns of the 3N x K matrix as Julia hands it over, or of the LTMADS generator);
// wave w owns candidate k0 + w. Per block of kColB UAVs, every lane issues all its loads at once
// (x, y, r of UAVs l, l + 64, ...: contiguous 512-B segments of the column), while the workgroup
// stages what every candidate shares in LDS: candidate 0's values (the key bases) and each
// UAV's prev / r_max / cons3 threshold.
//   objective (vp != null): term_i = |R_i - rmax_i|, or -1 when UAV i's move fails cons3
//     (pen_term's arithmetic). The wave folds its candidate's terms IN ORDER i = 0, 1, ..., N-1
//     from 0.0, as src/TDM_STATIC_opt.jl:88-92 does (bit-exact): term i sits in lane i % 64, so
//     the fold reads it with v_readlane (no LDS round trip per term) into one sequential chain
//     of fp64 adds, identical in every lane. vp[k] = violation * penalty, or +inf when a term is
//     negative (the extreme barrier of src/TDM_Constraints.jl:54-75);
//   keys (kKeys, matrix source, for the disk index): the fp32 key fl32(v - v0) of every value
//     (v0 = candidate 0's value), transposed through LDS into keysT[v*ldk + k] (64-B row
//     segments), and kbad[blockIdx.x * 3N + v] = 1 when some key of variable v in this block
//     does not reproduce v bit for bit (k_index.h "Keys": the disk then takes the identity map).
// The penalty chain thereby costs no buffer (one term per disk and candidate was 12.6 MB written
// and re-read at config 4) and no workgroups of the later launches.
constexpr int kColC = 16;                         // candidates (waves) per workgroup
constexpr int kColThreads = kColC * kWave;
constexpr int kColJ = 8;                          // UAVs per lane per block
constexpr int kColB = kColJ * kWave;              // UAVs per block

__host__ __device__ inline int keys_ld(int K) { return (K + kColC - 1) / kColC * kColC; }

__device__ __forceinline__ double readlane_f64(double v, int l)
{
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)b, l);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(b >> 32), l);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// kMat: the source is a matrix (src.cands; the generator path is compiled out), kKeys: write the
// index's keys (matrix sources only).
template <bool kMat, bool kKeys>
__global__ __launch_bounds__(kColThreads) void column_pass_kernel(uint64_t* ts, CandSrc src, int N,
                                                                  int K, PenArgs pa, double penalty,
                                                                  double* __restrict__ vp,
                                                                  float* __restrict__ keysT,
                                                                  int* __restrict__ kbad)
{
    ts_begin(ts);   // profiling only (the chain's first launch: k_common.h)
    __shared__ double sb[3][kColB];             // candidate 0's values (keys)
    __shared__ double su[5][kColB];             // prev x, y, z / tan, r_max, cons3 threshold
    __shared__ float kt[kColB][kColC + 1];      // one variable block's keys: [UAV][candidate]
    __shared__ int kfl[3][kColB];
    const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
    const int k0 = blockIdx.x * kColC;
    const int k = k0 + w;
    const int kc = min(k, K - 1);
    const int ldk = keys_ld(K);
    const bool obj = vp != nullptr;
    double acc = 0.0;
    bool bad = false;
    for (int ib = 0; ib < N; ib += kColB) {
        const int nb = min(kColB, N - ib);
        // this lane's values: UAV ib + lane + 64 j, variables x, y, r (all loads in flight)
        double v[3][kColJ];
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
            for (int j = 0; j < kColJ; ++j) {
                const int i = ib + min(lane + kWave * j, nb - 1);
                v[a][j] = kMat ? src.cands[(int64_t)kc * src.ldc + a * N + i] : src.get(kc, a * N + i, N);
            }
        // what every candidate shares, staged once per workgroup
        for (int q = tid; q < nb; q += kColThreads) {
            const int i = ib + q;
            if (kKeys) {
#pragma unroll
                for (int a = 0; a < 3; ++a) sb[a][q] = src.cands[a * N + i];
#pragma unroll
                for (int a = 0; a < 3; ++a) kfl[a][q] = 0;
            }
            if (obj) {
                su[0][q] = pa.prev ? pa.prev[i] : 0.0;
                su[1][q] = pa.prev ? pa.prev[N + i] : 0.0;
                su[2][q] = pa.prev ? pa.prev[2 * N + i] / pa.tan_half_fov : 0.0;   // z1
                su[3][q] = pa.rmax ? pa.rmax[i] : 0.0;
                su[4][q] = pen_threshold(pa, i);
            }
        }
        __syncthreads();
        if (obj) {
            // the terms of this lane's UAVs (pen_term's operations in the same order), then the
            // chain over the block in UAV order: term of UAV ib + 64 j + l is lane l's t[j]
            double t[kColJ];
#pragma unroll
            for (int j = 0; j < kColJ; ++j) {
                const int q = min(lane + kWave * j, nb - 1);
                const double R2 = v[2][j];
                double tt = pa.rmax ? __builtin_fabs(R2 - su[3][q]) : 0.0;
                if (pa.prev) {
                    const double z2 = R2 / pa.tan_half_fov;
                    const double ddx = su[0][q] - v[0][j], ddy = su[1][q] - v[1][j], ddz = su[2][q] - z2;
                    const double sq = ddx * ddx + ddy * ddy + ddz * ddz;
                    if (sq > su[4][q]) tt = -1.0;
                }
                t[j] = tt;
                bad |= __ballot(lane + kWave * j < nb && tt < 0.0) != 0;
            }
#pragma unroll
            for (int j = 0; j < kColJ; ++j) {
                if (kWave * j >= nb) break;   // uniform
                const int n = min(kWave, nb - kWave * j);
                if (n == kWave) {
#pragma unroll
                    for (int l = 0; l < kWave; ++l) acc += readlane_f64(t[j], l);
                } else {
                    for (int l = 0; l < n; ++l) acc += readlane_f64(t[j], l);
                }
            }
        }
        if (kKeys) {
            // per variable block: the keys through LDS, then 64-B row segments
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                bool ok = true;
#pragma unroll
                for (int j = 0; j < kColJ; ++j) {
                    const int q = lane + kWave * j;
                    if (q >= nb) break;
                    const double b = sb[a][q];
                    const float f = (float)(v[a][j] - b);
                    const bool e = __builtin_bit_cast(uint64_t, b + (double)f) == __builtin_bit_cast(uint64_t, v[a][j]);
                    if (!e && k < K) atomicOr(&kfl[a][q], 1);
                    kt[q][w] = f;
                }
                __syncthreads();
                for (int q4 = tid; q4 < nb * (kColC / 4); q4 += kColThreads) {
                    const int q = q4 / (kColC / 4), part = q4 % (kColC / 4);
                    const float* s4 = &kt[q][4 * part];
                    *reinterpret_cast<float4*>(keysT + ((int64_t)a * N + ib + q) * ldk + k0 + 4 * part) =
                        make_float4(s4[0], s4[1], s4[2], s4[3]);
                }
                __syncthreads();
                (void)ok;
            }
            for (int q = tid; q < 3 * nb; q += kColThreads) {
                const int a = q / nb, qq = q - a * nb;
                kbad[(int64_t)blockIdx.x * 3 * N + a * N + ib + qq] = kfl[a][qq];
            }
        }
        __syncthreads();   // LDS reuse by the next block
    }
    if (obj && lane == 0 && k < K) vp[k] = bad ? __builtin_inf() : acc * penalty;
    ts_end(ts);
}

// cands: see CandSrc. Writes disks[k*N + i] (the streaming scan's records).
__global__ void disk_prep_kernel(CandSrc src, int N, int K, DiskRec* __restrict__ disks)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)N * K) return;
    const int k = (int)(t / N), i = (int)(t % N);
    disks[t] = make_disk(src.get(k, i, N), src.get(k, N + i, N), src.get(k, 2 * N + i, N));
}

}  // namespace mac
