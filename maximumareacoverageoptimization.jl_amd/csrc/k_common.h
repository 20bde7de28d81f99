// k_common.h — constants, records and wave/block helpers shared by libmaxcover's kernels.
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
constexpr int kPollCH = 512;       // poll walk: entries staged in LDS per chunk
constexpr int kPollRB = 64;        // poll walk: region rows per batch
constexpr int kPollNbr = 64;       // poll walk: lower-index overlapping regions kept
constexpr int kPollSlots = 8;      // poll walk: candidate positions per lane (every wave)
constexpr int kPollPairs = kPollSlots / 2;
constexpr int kPollThreads = 256;  // poll walk: workgroup size (4 waves share one staging)
constexpr int kPollWaves = kPollThreads / kWave;
constexpr int kPollKPB = kWave * kPollSlots;  // poll walk: positions per slice
constexpr int kSharedWG = 256;     // poll walk: shared-entry workgroups (grid-stride over jobs)
constexpr int kBitsTab = 2048;     // bit-word kernel: positions per table group (k_bits.h)
constexpr int kBitsMinDisks = 16;  // bit-word kernel: used above this many disks with neighbours
// poll walk counters (dcount[]): [0] disks with neighbours the bit-word kernel can take (dlist
// from the front), [1] poll-kernel jobs taken, [2] the other disks with neighbours (dlist from the
// back), [3] bit-word / union-pass jobs taken, [4..7] union-pass jobs listed per weight bucket,
// heaviest first (k_or.h), [8] disks with lower neighbours whose upper list overflowed (the union
// pass stands down); cleared by the index kernel (the lane's mode buffer holds [walk, dcount])
constexpr int kOrBuckets = 4;
constexpr int kDcBits = 0, kDcPollJobs = 1, kDcOther = 2, kDcBitsJobs = 3, kDcOrJobs = 4,
              kDcOrBad = kDcOrJobs + kOrBuckets;
constexpr int kDcCount = kDcOrBad + 1;

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
template <int W = kWavesPerBlock>
__device__ __forceinline__ double block_sum_f64(double v, double* red /* W */)
{
    const int lane = threadIdx.x & (kWave - 1);
    const int wid = threadIdx.x / kWave;
    v = wave_sum_f64(v);
    if (lane == 0) red[wid] = v;
    __syncthreads();
    double s = 0.0;
    if (threadIdx.x == 0) {
#pragma unroll
        for (int i = 0; i < W; ++i) s += red[i];
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


__device__ __forceinline__ bool box_overlap(const int4& a, const int4& b)
{
    return a.x <= a.y && a.x <= b.y && b.x <= a.y && a.z <= b.w && b.z <= a.w;
}

__device__ __forceinline__ bool box_has(const int4& b, int tx, int ty)
{
    return b.x <= tx && tx <= b.y && b.z <= ty && ty <= b.w;
}

// tile span of disk (x, y, r): the same decision as disk_span(make_disk(x, y, r)) without the
// threshold (T(r) >= 0 exactly when r > 0)
__device__ __forceinline__ bool span_of(double x, double y, double r, const Grid& g, int4& sp)
{
    int x0, x1, y0, y1;
    if (!(r > 0.0)) return false;
    if (!tile_span(x, r, g.gx0, g.invS, g.nTx, x0, x1)) return false;
    if (!tile_span(y, r, g.gy0, g.invS, g.nTy, y0, y1)) return false;
    sp = make_int4(x0, x1, y0, y1);
    return true;
}

// ------------------------------------------------------------------ in-kernel launch timing
// Profiling only (ts == null otherwise): workgroup b writes ts[2b] = its start and ts[2b+1] = the
// end of its last wave, in s_memrealtime ticks (the constant 100 MHz clock, 10 ns). The host takes
// max(end) - min(start) over the launch's workgroups. Unlike HIP events this puts no extra packet
// or dependency into the stream, so the timed region runs as it does unprofiled; per workgroup
// it costs two plain stores, one barrier at entry and one LDS atomic per wave.
constexpr double kRealtimeHz = 100.0e6;

__device__ __forceinline__ uint64_t* ts_slot(uint64_t* ts)
{
    return ts + 2 * ((uint64_t)blockIdx.y * gridDim.x + blockIdx.x);
}

__device__ __forceinline__ int& ts_waves_done()
{
    __shared__ int done;
    return done;
}

__device__ __forceinline__ void ts_begin(uint64_t* ts)
{
    if (!ts) return;   // uniform
    if (threadIdx.x == 0) {
        ts_slot(ts)[0] = __builtin_amdgcn_s_memrealtime();
        ts_waves_done() = 0;
    }
    __syncthreads();
}

__device__ __forceinline__ void ts_end(uint64_t* ts)
{
    if (ts && (threadIdx.x & (kWave - 1)) == 0) {
        const int nw = (int)((blockDim.x + kWave - 1) / kWave);
        if (atomicAdd(&ts_waves_done(), 1) == nw - 1)   // the workgroup's last wave
            ts_slot(ts)[1] = __builtin_amdgcn_s_memrealtime();
    }
}

}  // namespace mac
