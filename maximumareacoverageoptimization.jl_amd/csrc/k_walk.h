// k_walk.h — the three coverage walks (streaming scan, per-candidate tiled walk, poll walk).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "predicate.h"
#include "k_common.h"
#include "k_index.h"
#include "k_poll_shared.h"

#pragma clang fp contract(off)

namespace mac {

// ------------------------------------------------------------------ streaming scan

// Every entry against every disk of KB candidates (disks[k*N + c], wave-uniform loads through
// the scalar cache); each lane holds PPT entries in registers. Branch-free inner loop: the
// reference's first-hit `break` changes which disk is credited, never the sum.
// partial[blk*K + k]: this block's share of candidate k.
template <int KB, int PPT>
__device__ __forceinline__ void coverage_scan_body(
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
//   double cx[N], cy[N], T[N], r[N]; int4 span[N]; int ncnt[N]; uint16 nbr[N][kNbrCap];
//   per wave: int rowStart[64], rowPre[64]
__host__ __device__ inline size_t tiled_lds_head(int N)
{
    size_t b = (size_t)N * 4 * sizeof(double);
    b += (size_t)N * 4 * sizeof(int);
    b += (size_t)N * sizeof(int);
    b += (size_t)N * sizeof(uint16_t) * kNbrCap;
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
// list built in LDS). Disk c of candidate k through the disk index (k_index.h);
// partial[gi*K + k]. Runs only when *mode == kModeTiled
// (or mode == null). Workgroups loop over units (grid-stride).
// Poll chain (nbrP != null): the lower-index candidates of disk c are the poll-level neighbour
// list walk_setup built once per poll (k_poll_shared.h neighbors_block: disks whose regions — the
// unions of their spans over the poll — overlap c's; a superset of any candidate's overlaps), so a
// unit tests sum over its disks of |list| pairs instead of every lower-index disk; an overflowed
// poll-level list (more than kPollNbr) falls back to every lower-index disk.
__device__ __forceinline__ void coverage_tiled_body(
    const double2* __restrict__ xy, const double* __restrict__ w,
    const int32_t* __restrict__ off, Grid g,
    const DiskRec* __restrict__ urec, const int* __restrict__ umap, int N, int K, int G,
    const int* __restrict__ mode, double* __restrict__ partial,
    const uint16_t* __restrict__ nbrP = nullptr, const int* __restrict__ ncountP = nullptr)
{
    if (mode && *mode != kModeTiled) return;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    double* sx = (double*)lds;
    double* sy = sx + N;
    double* sT = sy + N;
    double* sR = sT + N;
    int4* span = (int4*)(sR + N);
    int* ncnt = (int*)(span + N);
    uint16_t* nbr = (uint16_t*)(ncnt + N);
    const int lane = threadIdx.x & (kWave - 1);
    const int wid = threadIdx.x / kWave;
    int* rowStart = (int*)(lds + tiled_lds_head(N)) + wid * 2 * kWave;
    int* rowPre = rowStart + kWave;
    __shared__ double red[kWavesPerBlock];

    // grid-stride over the K*G (candidate, slice) units: the grid is capped so that the
    // launch stays cheap when the device-side choice is the poll walk
    for (int64_t unit = blockIdx.x; unit < (int64_t)K * G; unit += gridDim.x) {
    const int k = (int)(unit / G);
    const int gi = (int)(unit % G);
    __syncthreads();  // LDS reuse across units

    // 1. disks -> LDS, spans
    for (int c = threadIdx.x; c < N; c += kBlock) {
        const DiskRec d = rec_of(urec, umap, c, K, k);
        sx[c] = d.cx;
        sy[c] = d.cy;
        sT[c] = d.T;
        sR[c] = d.r;
        int4 sp;
        span[c] = disk_span(d, g, sp) ? sp : make_int4(1, 0, 1, 0);
        ncnt[c] = 0;
    }
    __syncthreads();

    // 2. lower-index overlap lists for this slice's disks (disk c belongs to slice c % G): the
    // pairs (c, c2 < c) spread over the whole workgroup (c2 = tid, tid + kBlock, ...), appended
    // with LDS atomics — the list order is irrelevant, ownership below is an OR over it
    for (int c = gi; c < N; c += G) {
        if (span[c].x > span[c].y) continue;   // uniform
        const double cx = sx[c], cy = sy[c], r = sR[c];
        auto test = [&](int c2) {
            if (span[c2].x > span[c2].y) return;  // covers nothing
            if (disks_may_overlap(cx, cy, r, sx[c2], sy[c2], sR[c2])) {
                const int q = atomicAdd(&ncnt[c], 1);
                if (q < kNbrCap) nbr[c * kNbrCap + q] = (uint16_t)c2;
            }
        };
        const int pc = nbrP ? ncountP[c] : kPollNbr + 1;   // (uniform)
        if (pc <= kPollNbr) {
            for (int q = threadIdx.x; q < pc; q += kBlock) test(nbrP[c * kPollNbr + q]);
        } else {
            for (int c2 = threadIdx.x; c2 < c; c2 += kBlock) test(c2);
        }
    }
    __syncthreads();

    // 3. walk: wave `wid` of slice gi takes disks c = gi + G*(wid + kWavesPerBlock*j)
    double acc = 0.0;
    const int stride = G * kWavesPerBlock;
    for (int c = gi + G * wid; c < N; c += stride) {
        const int4 sp = span[c];
        if (sp.x > sp.y) continue;
        const double cx = sx[c], cy = sy[c], T = sT[c];
        const int nc = ncnt[c] > kNbrCap ? 0xffff : ncnt[c];   // overflow: below
        const int pcl = nbrP ? ncountP[c] : kPollNbr + 1;
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
                    } else if (pcl <= kPollNbr) {   // overflowed: the poll-level list
                        for (int q = 0; q < pcl; ++q) {
                            const int c2 = nbrP[c * kPollNbr + q];
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
}

// timed entry points (ts: in-kernel launch timing, k_common.h)
template <int KB, int PPT>
__global__ __launch_bounds__(kBlock) void coverage_scan_kernel(
    uint64_t* ts, const double2* __restrict__ xy, const double* __restrict__ w, int64_t M,
    const DiskRec* __restrict__ disks, int N, int K, int64_t chunk, double* __restrict__ partial)
{
    ts_begin(ts);
    coverage_scan_body<KB, PPT>(xy, w, M, disks, N, K, chunk, partial);
    ts_end(ts);
}

__global__ __launch_bounds__(kBlock) void coverage_tiled_kernel(
    uint64_t* ts, const double2* __restrict__ xy, const double* __restrict__ w,
    const int32_t* __restrict__ off, Grid g, const DiskRec* __restrict__ urec,
    const int* __restrict__ umap, int N, int K, int G, const int* __restrict__ mode,
    double* __restrict__ partial)
{
    ts_begin(ts);
    coverage_tiled_body(xy, w, off, g, urec, umap, N, K, G, mode, partial);
    ts_end(ts);
}

// The poll chain's per-candidate walk (launched after walk_setup when the lane's recent polls
// chose it, or it is forced; maxcover.hip enqueue_eval): every block makes the walk choice with
// the poll-level neighbour counts known (k_poll_shared.h walk_choice), block 0 stores it in
// mode[0] (the poll kernel, the bit-word kernel and finalize read it) and in the lane's mapped
// hint word; when the per-candidate walk wins, the blocks grid-stride over its (candidate,
// slice) units with the poll-level lists. A stopped pipelined MADS loop (mode[0] == 0 from
// walk_setup) returns at once.
__global__ __launch_bounds__(kBlock) void coverage_tiled_poll_kernel(
    uint64_t* ts, const double2* __restrict__ xy, const double* __restrict__ w,
    const int32_t* __restrict__ off, Grid g, const DiskRec* __restrict__ urec,
    const int* __restrict__ umap, int N, int K, int G, int* __restrict__ mode,
    double* __restrict__ partial, const uint16_t* __restrict__ nbr, const int* __restrict__ ncount,
    const double2* __restrict__ cost, double ratio, int forced, int* __restrict__ hint)
{
    ts_begin(ts);
    const int m0 = *mode;
    if (m0 == 0) {   // (uniform) the pipelined MADS loop has stopped
        ts_end(ts);
        return;
    }
    const int m = walk_choice(N, K, cost, ncount, ratio, forced);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        mode[0] = m;
        if (hint) *(volatile int*)hint = m;
    }
    if (m == kModeTiled) coverage_tiled_body(xy, w, off, g, urec, umap, N, K, G, nullptr, partial, nbr, ncount);
    ts_end(ts);
}

// The poll chain's set-up after the index: block i < N builds disk i's neighbour list (k_poll_shared.h
// neighbors_block) for the poll kernel, the bit-word kernel, finalize and the per-candidate walk;
// block 0 sets mode[0] to the poll walk (coverage_tiled_poll_kernel, when launched, makes the choice
// after it), or to 0 when the pipelined MADS loop has stopped.
// With orj (the union pass, k_or.h, will run on this poll): block i also builds disk i's UPPER
// neighbour boxes and lists the union pass's jobs for the shared entries region i owns.
struct OrSetup {
    int4* nboxU;
    int* ncountU;
    int2* jobs;        // kOrBuckets lists of cap jobs (k_or.h or_list_jobs)
    int cap;
    const int32_t* off;
    Grid g;
    const int* ucount; // positions per disk (the index)
};

__global__ __launch_bounds__(kBlock) void walk_setup_kernel(
    uint64_t* ts, int N, const int4* __restrict__ region, uint16_t* __restrict__ nbr,
    int4* __restrict__ nboxT, int* __restrict__ ncount, int* __restrict__ dlist,
    int* __restrict__ dcount, int* __restrict__ mode, int* __restrict__ qual,
    const MadsState* __restrict__ halt, OrSetup orj)
{
    ts_begin(ts);
    // the neighbour lists' regions, loaded beside the halt word (one round trip)
    const int i = blockIdx.x;
    const int4 none = make_int4(0x7fffffff, -1, 0x7fffffff, -1);
    const int4 R = i < N ? region[i] : none;
    int4 Q[kNbrPre];
#pragma unroll
    for (int q = 0; q < kNbrPre; ++q) {
        const int j = threadIdx.x + q * kBlock;
        Q[q] = j < i && i < N ? region[j] : none;
    }
    // a stopped pipelined MADS loop, or a poll its prep rejected whole (k_prep.h MadsState): no
    // walk; the poll kernel, the shared-entry passes and the finalize's argmin see mode 0 / the
    // state and return
    if (halt && (halt->ell < 0 || halt->skip)) {
        if (blockIdx.x == 0 && threadIdx.x == 0) mode[0] = 0;
        ts_end(ts);
        return;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) mode[0] = kModePoll;
    if (i < N && !orj.jobs) {
        neighbors_block(i, N, R, Q, region, nbr, nboxT, ncount, dlist, dcount, qual);
    } else if (i < N) {
        __shared__ int4 lbox[kPollNbr], ubox[kPollNbr];
        __shared__ int cnt2[2];
        neighbors_block(i, N, R, Q, region, nbr, nboxT, ncount, dlist, dcount, qual, orj.nboxU,
                        orj.ncountU, lbox, ubox, cnt2);
        __syncthreads();
        or_list_jobs(i, R, lbox, cnt2[0], ubox, cnt2[1], orj.off, orj.g, orj.jobs, orj.cap, dcount,
                     orj.ucount[i]);
    }
    ts_end(ts);
}


}  // namespace mac
