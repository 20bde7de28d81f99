// kernels.h — gfx950 (CDNA4, wave64) device code of libmaxcover.
//
// Hot path: one MADS poll = K candidates x full coverage of the fire-point list
// (src/TDM_STATIC_opt.jl:82-100 via src/AreaCoverageCalculation.jl:63-78), as a short chain:
//   disk_prep*_kernel     per (candidate, disk): {cx, cy, T(r), r}, T the exact threshold
//   region_kernel         per disk i: union of its tile spans over the K candidates + costs
//   decide_kernel         picks the poll walk or the per-candidate walk on the device
//   coverage_poll_kernel  workgroup = (disk i, 256 candidates): the entries of disk i's region
//                         staged in LDS once, one candidate per lane, broadcast LDS reads
//   coverage_tiled_kernel workgroup = candidate: each wave walks whole disks over the CSR rows
//   coverage_scan_kernel  streaming brute force (every entry x every disk), the fallback
//   finalize_kernel       fixed-order sum of per-slice partials -> area; penalty; cons3 mask
//   argmin_kernel         lexicographic (objective, index) minimum
// An entry is credited to the LOWEST-index disk covering it (exactly-once union count), so the
// area is the reference's first-hit-break sum (:67-78) over the same multiset of entries.
// Partials are laid out [slice][candidate] and summed in slice order: bit-reproducible.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "predicate.h"

#pragma clang fp contract(off)

namespace mac {

constexpr int kWave = 64;
constexpr int kBlock = 256;        // 4 waves
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr int kNbrCap = 6;         // tiled walk: lower-index overlapping disks kept per disk
constexpr int kPollCH = 1024;      // poll walk: entries staged in LDS per chunk
constexpr int kPollRB = 64;        // poll walk: region rows per batch
constexpr int kPollNbr = 64;       // poll walk: lower-index overlapping regions kept

constexpr int kModePoll = 1;
constexpr int kModeTiled = 2;

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
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, kWave);  // fixed butterfly
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

__device__ __forceinline__ DiskRec make_disk(double cx, double cy, double r)
{
    DiskRec d;
    d.cx = cx;
    d.cy = cy;
    d.r = r;
    d.T = cover_threshold(r);
    return d;
}

__device__ __forceinline__ bool disk_span(const DiskRec& d, const Grid& g, int4& sp)
{
    int x0, x1, y0, y1;
    if (!(d.T >= 0.0)) return false;
    if (!tile_span(d.cx, d.r, g.gx0, g.invS, g.nTx, x0, x1)) return false;
    if (!tile_span(d.cy, d.r, g.gy0, g.invS, g.nTy, y0, y1)) return false;
    sp = make_int4(x0, x1, y0, y1);
    return true;
}

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
    if (threadIdx.x == 0) *mode = forced ? forced : (A <= ratio * B ? kModePoll : kModeTiled);
}

// ------------------------------------------------------------------ streaming scan

// Every entry against every disk of KB candidates (disks[k*N + c], wave-uniform loads through
// the scalar cache); each lane holds PPT entries in registers. Branch-free inner loop: the
// reference's first-hit `break` changes which disk is credited, never the sum.
// partial[blk*K + k]: this block's share of candidate k.
template <int KB, int PPT>
__global__ __launch_bounds__(kBlock) void coverage_scan_kernel(
    const double2* __restrict__ xy, const double* __restrict__ w, int64_t M,
    const DiskRec* __restrict__ disks, int N, int K, int64_t chunk,
    double* __restrict__ partial)
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
        if (threadIdx.x == 0 && k < K) partial[(int64_t)blk * K + k] = s;
        __syncthreads();
    }
}

// ------------------------------------------------------------------ per-candidate tiled walk

// LDS layout, N disks (dynamic shared memory, 16-B aligned carve):
//   double cx[N], cy[N], T[N], r[N]; int4 span[N]; uint16 ncnt[N]; uint16 nbr[N][kNbrCap];
//   per wave: int rowStart[64], rowPre[64]
__host__ __device__ inline size_t tiled_lds_head(int N)
{
    size_t b = (size_t)N * 4 * sizeof(double);
    b += (size_t)N * 4 * sizeof(int);
    b += (size_t)N * sizeof(uint16_t) * (1 + kNbrCap);
    return (b + 15) & ~(size_t)15;
}
__host__ __device__ inline size_t tiled_lds_bytes(int N)
{
    return tiled_lds_head(N) + (size_t)kWavesPerBlock * 2 * kWave * sizeof(int);
}

// Workgroup = (candidate k, slice gi of G). Each wave walks whole disks: for disk c it reads
// the tile-row runs of c's span from the CSR offsets (a row of tiles is contiguous in the
// sorted list), tests every entry in them, and credits a covered entry only when no lower-index
// disk also covers it (candidates for that come from a conservative disk-disk intersection
// list built in LDS). disksT[c*K + k]; partial[gi*K + k]. Runs only when *mode == kModeTiled
// (or mode == null).
__global__ __launch_bounds__(kBlock) void coverage_tiled_kernel(
    const double2* __restrict__ xy, const double* __restrict__ w,
    const int32_t* __restrict__ off, Grid g,
    const DiskRec* __restrict__ disksT, int N, int K, int G, const int* __restrict__ mode,
    double* __restrict__ partial)
{
    if (mode && *mode != kModeTiled) return;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    double* sx = (double*)lds;
    double* sy = sx + N;
    double* sT = sy + N;
    double* sR = sT + N;
    int4* span = (int4*)(sR + N);
    uint16_t* ncnt = (uint16_t*)(span + N);
    uint16_t* nbr = ncnt + N;
    const int lane = threadIdx.x & (kWave - 1);
    const int wid = threadIdx.x / kWave;
    int* rowStart = (int*)(lds + tiled_lds_head(N)) + wid * 2 * kWave;
    int* rowPre = rowStart + kWave;
    __shared__ double red[kWavesPerBlock];

    const int k = blockIdx.x / G;
    const int gi = blockIdx.x % G;

    // 1. disks -> LDS, spans
    for (int c = threadIdx.x; c < N; c += kBlock) {
        const DiskRec d = disksT[(int64_t)c * K + k];
        sx[c] = d.cx;
        sy[c] = d.cy;
        sT[c] = d.T;
        sR[c] = d.r;
        int4 sp;
        span[c] = disk_span(d, g, sp) ? sp : make_int4(1, 0, 1, 0);
    }
    __syncthreads();

    // 2. lower-index overlap lists for this slice's disks (disk c belongs to slice c % G)
    for (int c = gi + G * threadIdx.x; c < N; c += G * kBlock) {
        int cnt = 0;
        if (span[c].x <= span[c].y) {
            const double cx = sx[c], cy = sy[c], r = sR[c];
            for (int c2 = 0; c2 < c; ++c2) {
                if (span[c2].x > span[c2].y) continue;  // covers nothing
                if (disks_may_overlap(cx, cy, r, sx[c2], sy[c2], sR[c2])) {
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
    if (threadIdx.x == 0) partial[(int64_t)gi * K + k] = s;
}

// ------------------------------------------------------------------ poll walk

// Workgroup = (disk i, candidates k = 256*blockIdx.y + lane). The entries of disk i's region
// (union of its spans over the whole poll) are staged in LDS in chunks; every lane then tests
// its own candidate's disk i against each staged entry (one broadcast LDS read per entry per
// wave) and credits it when no lower-index disk j of the SAME candidate covers it (j ranges
// over the disks whose regions overlap region i). partialT[i*K + k]. Runs when *mode == poll.
__global__ __launch_bounds__(kBlock) void coverage_poll_kernel(
    const double2* __restrict__ xy, const double* __restrict__ w,
    const int32_t* __restrict__ off, Grid g, const DiskRec* __restrict__ disksT,
    const int4* __restrict__ region, int N, int K, const int* __restrict__ mode,
    double* __restrict__ partialT)
{
    if (mode && *mode != kModePoll) return;
    __shared__ double2 sxy[kPollCH];
    __shared__ double sw[kPollCH];
    __shared__ int rs[kPollRB], rpre[kPollRB + 1];
    __shared__ uint16_t nbr[kPollNbr];
    __shared__ int ncnt;

    const int i = blockIdx.x;
    const int tid = threadIdx.x;
    const int k = blockIdx.y * kBlock + tid;
    const bool valid = k < K;
    const int4 R = region[i];
    if (R.x > R.y) {  // disk i covers nothing in any candidate
        if (valid) partialT[(int64_t)i * K + k] = 0.0;
        return;
    }
    DiskRec d;
    if (valid) d = disksT[(int64_t)i * K + k];
    else d = DiskRec{0.0, 0.0, -1.0, 0.0};

    // lower-index disks whose regions overlap region i (order is irrelevant: boolean OR)
    if (tid == 0) ncnt = 0;
    __syncthreads();
    for (int j = tid; j < i; j += kBlock) {
        const int4 Q = region[j];
        if (Q.x <= Q.y && Q.x <= R.y && R.x <= Q.y && Q.z <= R.w && R.z <= Q.w) {
            const int p = atomicAdd(&ncnt, 1);
            if (p < kPollNbr) nbr[p] = (uint16_t)j;
        }
    }
    __syncthreads();
    const int nc = ncnt;

    double acc = 0.0;
    for (int rb = R.z; rb <= R.w; rb += kPollRB) {
        const int nr = min(kPollRB, R.w - rb + 1);
        if (tid < nr) {
            const int64_t rowbase = (int64_t)(rb + tid) * g.nTx;
            const int s = off[rowbase + R.x];
            rs[tid] = s;
            rpre[tid + 1] = off[rowbase + R.y + 1] - s;
        }
        __syncthreads();
        if (tid == 0) {
            rpre[0] = 0;
            for (int r = 0; r < nr; ++r) rpre[r + 1] += rpre[r];
        }
        __syncthreads();
        const int total = rpre[nr];
        for (int base = 0; base < total; base += kPollCH) {
            const int n = min(kPollCH, total - base);
            for (int q = tid; q < n; q += kBlock) {
                const int f = base + q;
                int lo = 0, hi = nr - 1;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (rpre[mid] <= f) lo = mid; else hi = mid - 1;
                }
                const int j = rs[lo] + (f - rpre[lo]);
                sxy[q] = xy[j];
                sw[q] = w[j];
            }
            __syncthreads();
            if (d.T >= 0.0) {
                for (int q = 0; q < n; ++q) {
                    const double2 p = sxy[q];
                    if (sqdist(p.x, p.y, d.cx, d.cy) <= d.T) {
                        bool owned = true;
                        if (nc <= kPollNbr) {
                            for (int u = 0; u < nc; ++u) {
                                const DiskRec e = disksT[(int64_t)nbr[u] * K + k];
                                if (sqdist(p.x, p.y, e.cx, e.cy) <= e.T) { owned = false; break; }
                            }
                        } else {
                            for (int j = 0; j < i; ++j) {
                                const int4 Q = region[j];
                                if (!(Q.x <= Q.y && Q.x <= R.y && R.x <= Q.y && Q.z <= R.w &&
                                      R.z <= Q.w))
                                    continue;
                                const DiskRec e = disksT[(int64_t)j * K + k];
                                if (sqdist(p.x, p.y, e.cx, e.cy) <= e.T) { owned = false; break; }
                            }
                        }
                        if (owned) acc += sw[q];
                    }
                }
            }
            __syncthreads();
        }
    }
    if (valid) partialT[(int64_t)i * K + k] = acc;
}

// ------------------------------------------------------------------ finalize / argmin

// area_k = sum over slices g of partial[g*K + k] (fixed order); the slice count is n_poll when
// *mode == poll, else n_other. obj_k = -area_k + penalty * violation_k with violation_k =
// sum_i |x[2N+i] - rmax[i]| sequentially (src/TDM_STATIC_opt.jl:89-97). cons3
// (src/TDM_Constraints.jl:54-75) when prev != null: infeasible -> obj = +inf; the test
// sqrt(s) > d_lim is evaluated exactly as s > dlimT (predicate.h dlim_threshold).
__global__ void finalize_kernel(const double* __restrict__ partial, const int* __restrict__ mode,
                                int n_poll, int n_other, int K,
                                const double* __restrict__ cands, int N, int ldc,
                                const double* __restrict__ rmax, double penalty,
                                const double* __restrict__ prev, const double* __restrict__ dlimT,
                                double tan_half_fov, double* __restrict__ area_out,
                                double* __restrict__ obj_out)
{
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= K) return;
    const int G = (mode && *mode == kModePoll) ? n_poll : n_other;
    double area = 0.0;
    for (int g = 0; g < G; ++g) area += partial[(int64_t)g * K + k];
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
