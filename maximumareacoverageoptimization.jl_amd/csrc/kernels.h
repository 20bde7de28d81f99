// kernels.h — gfx950 (CDNA4, wave64) device code of libmaxcover.
//
// Hot path (one MADS poll = K candidates x full coverage scan, src/TDM_STATIC_opt.jl:82-100 via
// src/AreaCoverageCalculation.jl:63-78):
//   disk_prep_kernel     per (candidate, disk): {cx, cy, T(r), r} with T the exact threshold
//   coverage_tiled_kernel disk-major walk over the tile-binned point list; one workgroup (or G)
//                         per candidate; a point is counted by the lowest-index disk covering it
//   coverage_scan_kernel  streaming brute force: every point against every disk (scalar-cache
//                         disk operands, branch-free), KB candidates per pass
//   finalize_kernel       fixed-order partial sum -> area; objective penalty; cons3 mask
//   argmin_kernel         lexicographic (objective, index) minimum
// Set-up path (once per MPC step): bbox, tile keys, gather, offsets, covered flags.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "predicate.h"

#pragma clang fp contract(off)

namespace mac {

constexpr int kWave = 64;
constexpr int kBlock = 256;        // 4 waves
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr int kNbrCap = 6;         // lower-index overlapping disks kept per disk in LDS

struct Grid {
    double gx0, gy0;     // origin (bbox min of the finite points)
    double invS;         // 1 / tile pitch (same pitch on both axes)
    double S;
    int nTx, nTy;
};

struct DiskRec {         // 32 B, one per (candidate, disk)
    double cx, cy, T, r;
};

// ------------------------------------------------------------------ wave / block helpers

__device__ __forceinline__ double wave_sum_f64(double v)
{
    // fixed butterfly: deterministic
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, kWave);
    return v;
}

__device__ __forceinline__ int wave_incl_scan_i32(int v, int lane)
{
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
        const int t = __shfl_up(v, off, kWave);
        if (lane >= off) v += t;
    }
    return v;
}

// Block sum in fixed order (wave butterfly, then waves 0..3 in order). Result valid in thread 0.
__device__ __forceinline__ double block_sum_f64(double v, double* red /* kWavesPerBlock */)
{
    const int lane = threadIdx.x & (kWave - 1);
    const int wid = threadIdx.x / kWave;
    v = wave_sum_f64(v);
    if (lane == 0) red[wid] = v;
    __syncthreads();
    double s = 0.0;
    if (threadIdx.x == 0) {
#pragma unroll
        for (int i = 0; i < kWavesPerBlock; ++i) s += red[i];
    }
    return s;
}

// ------------------------------------------------------------------ per-batch disk prep

// cands: 3N x K column-major (candidate k at cands + k*ldc). Writes disks[k*N + i].
__global__ void disk_prep_kernel(const double* __restrict__ cands, int N, int ldc, int K,
                                 DiskRec* __restrict__ disks)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)N * K) return;
    const int k = (int)(t / N), i = (int)(t % N);
    const double* c = cands + (int64_t)k * ldc;
    DiskRec d;
    d.cx = c[i];
    d.cy = c[N + i];
    d.r = c[2 * N + i];
    d.T = cover_threshold(d.r);
    disks[t] = d;
}

// ------------------------------------------------------------------ streaming scan

// Every point against every disk of KB candidates. Disk operands are wave-uniform loads
// (scalar cache); each lane holds PPT points in registers. Branch-free inner loop: the
// first-hit `break` of the reference changes which disk is credited, never the sum.
template <int KB, int PPT>
__global__ __launch_bounds__(kBlock) void coverage_scan_kernel(
    const double2* __restrict__ xy, const double* __restrict__ w, int64_t M,
    const DiskRec* __restrict__ disks, int N, int K, int64_t chunk, int nblk,
    double* __restrict__ partial /* K x nblk */)
{
    __shared__ double red[kWavesPerBlock];
    const int blk = blockIdx.x;
    const int k0 = blockIdx.y * KB;
    const int64_t begin = (int64_t)blk * chunk;
    const int64_t end = begin + chunk < M ? begin + chunk : M;

    double acc[KB];
#pragma unroll
    for (int q = 0; q < KB; ++q) acc[q] = 0.0;

    for (int64_t base = begin; base < end; base += (int64_t)kBlock * PPT) {
        double px[PPT], py[PPT], pw[PPT];
#pragma unroll
        for (int u = 0; u < PPT; ++u) {
            const int64_t p = base + (int64_t)u * kBlock + threadIdx.x;
            if (p < end) {
                const double2 v = xy[p];
                px[u] = v.x;
                py[u] = v.y;
                pw[u] = w[p];
            } else {
                px[u] = __builtin_nan("");  // NaN: never covered
                py[u] = 0.0;
                pw[u] = 0.0;
            }
        }
#pragma unroll
        for (int q = 0; q < KB; ++q) {
            const int k = k0 + q;
            if (k >= K) break;
            const DiskRec* dk = disks + (int64_t)k * N;
            bool cov[PPT];
#pragma unroll
            for (int u = 0; u < PPT; ++u) cov[u] = false;
            for (int c = 0; c < N; ++c) {
                const double cx = dk[c].cx, cy = dk[c].cy, T = dk[c].T;
#pragma unroll
                for (int u = 0; u < PPT; ++u) cov[u] |= sqdist(px[u], py[u], cx, cy) <= T;
            }
#pragma unroll
            for (int u = 0; u < PPT; ++u)
                if (cov[u]) acc[q] += pw[u];
        }
    }
#pragma unroll
    for (int q = 0; q < KB; ++q) {
        const int k = k0 + q;
        const double s = block_sum_f64(acc[q], red);
        if (threadIdx.x == 0 && k < K) partial[(int64_t)k * nblk + blk] = s;
        __syncthreads();
    }
}

// ------------------------------------------------------------------ tiled (culled) walk

// LDS layout for the tiled kernel, N disks (dynamic shared memory, 16-B aligned carve):
//   double cx[N], cy[N], T[N]; int4 span[N]; uint16 ncnt[N]; uint16 nbr[N][kNbrCap];
//   per wave: int rowStart[64], rowPre[64]
__host__ __device__ inline size_t tiled_lds_bytes(int N)
{
    size_t b = (size_t)N * 3 * sizeof(double);
    b += (size_t)N * 4 * sizeof(int);
    b += (size_t)N * sizeof(uint16_t) * (1 + kNbrCap);
    b = (b + 15) & ~(size_t)15;
    b += (size_t)kWavesPerBlock * 2 * kWave * sizeof(int);
    return b;
}

// One workgroup per (candidate k, slice gi of G). Each wave walks whole disks: for disk c it
// reads the tile-row runs of c's bounding box from the CSR offsets (tile rows are contiguous
// in the sorted list), tests every point in them, and credits a covered point only when no
// lower-index disk also covers it (exactly-once union count; lower-index overlap candidates
// come from a conservative disk-disk intersection list built in LDS).
__global__ __launch_bounds__(kBlock) void coverage_tiled_kernel(
    const double2* __restrict__ xy, const double* __restrict__ w,
    const int32_t* __restrict__ off, Grid g,
    const DiskRec* __restrict__ disks, int N, int K, int G,
    double* __restrict__ partial /* K x G */)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    double* sx = (double*)lds;
    double* sy = sx + N;
    double* sT = sy + N;
    int4* span = (int4*)(sT + N);
    uint16_t* ncnt = (uint16_t*)(span + N);
    uint16_t* nbr = ncnt + N;
    size_t wofs = (size_t)N * 3 * sizeof(double) + (size_t)N * 4 * sizeof(int) +
                  (size_t)N * sizeof(uint16_t) * (1 + kNbrCap);
    wofs = (wofs + 15) & ~(size_t)15;
    const int lane = threadIdx.x & (kWave - 1);
    const int wid = threadIdx.x / kWave;
    int* rowStart = (int*)(lds + wofs) + wid * 2 * kWave;
    int* rowPre = rowStart + kWave;
    __shared__ double red[kWavesPerBlock];

    const int k = blockIdx.x / G;
    const int gi = blockIdx.x % G;
    const DiskRec* dk = disks + (int64_t)k * N;

    // 1. disks -> LDS, spans
    for (int c = threadIdx.x; c < N; c += kBlock) {
        const DiskRec d = dk[c];
        sx[c] = d.cx;
        sy[c] = d.cy;
        sT[c] = d.T;
        int x0, x1, y0, y1;
        const bool okx = d.T >= 0.0 && tile_span(d.cx, d.r, g.gx0, g.invS, g.nTx, x0, x1);
        const bool oky = okx && tile_span(d.cy, d.r, g.gy0, g.invS, g.nTy, y0, y1);
        span[c] = oky ? make_int4(x0, x1, y0, y1) : make_int4(1, 0, 1, 0);
    }
    __syncthreads();

    // 2. lower-index overlap lists for this slice's disks (disk c belongs to slice c % G)
    for (int c = gi + G * threadIdx.x; c < N; c += G * kBlock) {
        int cnt = 0;
        if (span[c].x <= span[c].y) {
            const double cx = sx[c], cy = sy[c], r = dk[c].r;
            for (int c2 = 0; c2 < c; ++c2) {
                if (span[c2].x > span[c2].y) continue;  // covers nothing
                if (disks_may_overlap(cx, cy, r, sx[c2], sy[c2], dk[c2].r)) {
                    if (cnt < kNbrCap) nbr[c * kNbrCap + cnt] = (uint16_t)c2;
                    ++cnt;
                }
            }
        }
        ncnt[c] = (uint16_t)(cnt > kNbrCap ? 0xffff : cnt);
    }
    __syncthreads();

    // 3. walk: wave `wid` of slice gi takes disks c = gi + G*(wid + kWavesPerBlock*j)
    double acc = 0.0;
    const int stride = G * kWavesPerBlock;
    for (int c = gi + G * wid; c < N; c += stride) {
        const int4 sp = span[c];
        if (sp.x > sp.y) continue;
        const double cx = sx[c], cy = sy[c], T = sT[c];
        const int nc = ncnt[c];
        for (int rb = sp.z; rb <= sp.w; rb += kWave) {
            const int nr = (sp.w - rb + 1) < kWave ? (sp.w - rb + 1) : kWave;
            int s = 0, len = 0;
            if (lane < nr) {
                const int64_t rowbase = (int64_t)(rb + lane) * g.nTx;
                s = off[rowbase + sp.x];
                len = off[rowbase + sp.y + 1] - s;
            }
            const int incl = wave_incl_scan_i32(len, lane);
            const int total = __shfl(incl, kWave - 1, kWave);
            rowStart[lane] = s;
            rowPre[lane] = incl - len;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            for (int i = lane; i < total; i += kWave) {
                int lo = 0, hi = nr - 1;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (rowPre[mid] <= i) lo = mid; else hi = mid - 1;
                }
                const int j = rowStart[lo] + (i - rowPre[lo]);
                const double2 p = xy[j];
                if (sqdist(p.x, p.y, cx, cy) <= T) {
                    bool owned = true;
                    if (nc != 0xffff) {
                        for (int q = 0; q < nc; ++q) {
                            const int c2 = nbr[c * kNbrCap + q];
                            if (sqdist(p.x, p.y, sx[c2], sy[c2]) <= sT[c2]) { owned = false; break; }
                        }
                    } else {
                        for (int c2 = 0; c2 < c; ++c2) {
                            if (sqdist(p.x, p.y, sx[c2], sy[c2]) <= sT[c2]) { owned = false; break; }
                        }
                    }
                    if (owned) acc += w[j];
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
    const double s = block_sum_f64(acc, red);
    if (threadIdx.x == 0) partial[(int64_t)k * G + gi] = s;
}

// ------------------------------------------------------------------ finalize / argmin

// area_k = sum_g partial[k][g] (fixed order). obj_k = -area_k + penalty * violation_k with
// violation_k = sum_i |x[2N+i] - rmax[i]| sequentially (src/TDM_STATIC_opt.jl:89-97).
// cons3 (src/TDM_Constraints.jl:54-75) when prev != null: infeasible -> obj = +inf and
// feasible flag 0. The test sqrt(s) > d_lim is evaluated exactly as !(s <= T(nextup(d))).
__global__ void finalize_kernel(const double* __restrict__ partial, int G, int K,
                                const double* __restrict__ cands, int N, int ldc,
                                const double* __restrict__ rmax, double penalty,
                                const double* __restrict__ prev, const double* __restrict__ dlimT,
                                double tan_half_fov, double* __restrict__ area_out,
                                double* __restrict__ obj_out)
{
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= K) return;
    double area = 0.0;
    for (int g = 0; g < G; ++g) area += partial[(int64_t)k * G + g];
    if (area_out) area_out[k] = area;
    if (!obj_out) return;
    const double* x = cands + (int64_t)k * ldc;
    bool feasible = true;
    if (prev) {
        for (int i = 0; i < N; ++i) {
            const double x1 = prev[i], y1 = prev[N + i], z1 = prev[2 * N + i] / tan_half_fov;
            const double x2 = x[i], y2 = x[N + i], z2 = x[2 * N + i] / tan_half_fov;
            const double ddx = x1 - x2, ddy = y1 - y2, ddz = z1 - z2;
            const double s = ddx * ddx + ddy * ddy + ddz * ddz;
            // dlimT[i] = threshold for "sqrt(s) <= d": +inf sentinel means never infeasible
            if (s > dlimT[i]) { feasible = false; break; }
        }
    }
    double violation = 0.0;
    if (rmax)
        for (int i = 0; i < N; ++i) violation += __builtin_fabs(x[i + 2 * N] - rmax[i]);
    const double obj = -area + violation * penalty;
    obj_out[k] = feasible ? obj : __builtin_inf();
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

// ------------------------------------------------------------------ set-up kernels

// Per-block min/max of finite x and y: out[blk] = {xmin, xmax, ymin, ymax}.
__global__ __launch_bounds__(kBlock) void bbox_kernel(const double* __restrict__ x,
                                                      const double* __restrict__ y, int64_t M,
                                                      double4* __restrict__ out)
{
    double xmn = __builtin_inf(), xmx = -__builtin_inf();
    double ymn = __builtin_inf(), ymx = -__builtin_inf();
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < M;
         i += (int64_t)gridDim.x * kBlock) {
        const double a = x[i], b = y[i];
        if (__builtin_isfinite(a)) { xmn = a < xmn ? a : xmn; xmx = a > xmx ? a : xmx; }
        if (__builtin_isfinite(b)) { ymn = b < ymn ? b : ymn; ymx = b > ymx ? b : ymx; }
    }
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
