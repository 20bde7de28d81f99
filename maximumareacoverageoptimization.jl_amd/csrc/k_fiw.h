// k_fiw.h — the fused poll chain: prep_kernel -> fiw_kernel -> fin2_kernel (three launches).
//
// The five-launch chain (prep, disk index, walk set-up, poll walk, finalize) hands each disk's
// index outputs (records, map, lane constants) to the walk through HBM and needs the set-up launch
// between them only to find, for every disk, the lower-index disks whose regions overlap its own
// (exactly-once ownership, k_poll.h "Ownership"). Those regions are unions of spans over all K
// candidates, known only once every disk's index has run. Here each disk's region is instead a
// SUPERSET box computed from candidate 0's disk and one poll-wide displacement bound
// D = (max |x - x0|, max |y - y0|, max r - r0, max r0 - r) over the live candidates (the prep
// launch's per-workgroup maxima, k_prep.h): every workgroup can compute every disk's box from the
// matrix's first column, so one workgroup per disk i runs, in one launch:
//   * the index: the K packed keys of disk i (one coalesced row, k_prep.h) deduplicated into its
//     distinct disks ("positions"): a direct-mapped table over the box of key offsets D allows
//     (ell <= 3 polls), else an LDS hash; a row with an escaped key takes one position per candidate;
//   * its lower neighbours: the disks j < i whose boxes overlap box i;
//   * the poll walk over box i's entries that no lower box holds (k_poll.h's staging, exact fp32
//     filter and hot loop), one credit per position;
//   * the shared entries (box i's entries inside a lower box): handed to fin2_kernel (their
//     coordinates and the neighbour ids), or, past kFwShCap entries or kFwNbr neighbours, decided
//     here per candidate in fp64;
//   * one row per disk of per-candidate credits (uint32 counts when every entry weighs the same,
//     else fp64 credits).
// fin2_kernel sums the N rows per candidate (no map gather), adds the shared entries' credit (an
// entry counts for disk i of candidate k when disk i covers it and no listed lower neighbour disk
// of candidate k does, every disk read from its key word: the same exact doubles; the decisions of
// all handed-off disks split over every finalize block), applies the penalty and takes the argmin
// (k_final.h finalize_argmin). Every entry is credited to the lowest-index disk covering it, so the
// area is the reference's first-hit sum (src/AreaCoverageCalculation.jl:67-78).
// The boxes only decide which entries the walk stages and which the shared decisions take: a box
// larger than the exact region costs work, never a result. DESIGN.md §4.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "predicate.h"
#include "k_common.h"
#include "k_prep.h"
#include "k_index.h"
#include "k_lane.h"
#include "k_poll.h"
#include "k_poll_shared.h"
#include "k_final.h"

#pragma clang fp contract(off)

namespace mac {

constexpr int kFwThreads = 256;                  // 4 waves; two workgroups per CU (LDS), so the walk's
                                                 // registers fit without spills (2 waves per SIMD)
constexpr int kFwWaves = kFwThreads / kWave;
constexpr int kFwPer = 12;                       // candidates per thread: k = 12 t + j (16-B loads)
constexpr int kFwMaxK = kFwThreads * kFwPer;     // 3072 (+ 1: thread 0 also takes k = 3072)
constexpr int kFwHash = 4096;                    // hash slots (load <= 3/4)
constexpr int kFwIdBits = 12;
constexpr int kFwDirect = 6144;                  // direct-mapped slots (the dead slot included)
constexpr int kFwKPB = kWave * kPollSlots;       // positions per walk slice (8 per lane)
constexpr int kFwCH = 512;                       // entries staged per chunk
constexpr int kFwR = kFwCH / kFwThreads;         // ... per thread
constexpr int kFwShE = 64;                       // shared entries per decision word (in place)
constexpr int kFwNbr = kPollNbr;                 // lower neighbours kept (more: every lower disk)
constexpr int kFwShCap = 1024;                   // shared entries a disk hands to fin2_kernel

// Hint words (device ints, zero between polls: fin2_kernel's last block copies them to the lane's
// mapped host memory and clears them): [0] the most shared entries x neighbours of one disk,
// [1] disks that took one position per candidate (an escaped key), [2] disks with lower
// neighbours, [3] disks whose shared entries were decided in place (overflow)
constexpr int kFwHints = 4;

// The shared entries a disk hands to fin2_kernel: a disk with at most kFwHand lower neighbours and
// kFwShCap shared entries appends one 16-B record {disk, neighbours | entries << 8, neighbour ids
// 0 | 1 << 16, 2 | 3 << 16} to a compact list (any order: fin2 sorts it by disk; the count is
// zeroed by the next poll's prep launch), else decides them in place
constexpr int kFwHand = 4;
constexpr int kF2ListCap = 1024;   // listed disks fin2_kernel takes (the rest decide in place)
struct FwShared {
    int* count;       // listed disks
    int4* list;       // [N] their records
    double2* xy;      // [N][kFwShCap] the entries' coordinates, in a fixed order
    double* w;        // [N][kFwShCap] and weights
};

struct FwArgs {
    CandSrc src;               // keysP / ldk: the prep launch's packed keys (one row per disk)
    int N, K;
    Grid g;
    const uint8_t* dead;       // per candidate: 1 = failed cons3, left out (null: none); >= ldk bytes
    const double4* pd;         // prep: per workgroup {max |x-x0|, max |y-y0|, max r-r0, max r0-r}
    int npd;
    const double2* xy;         // tile-sorted entries
    const double* w;
    const int32_t* off;        // CSR over tiles
    int counts;                // every entry weighs the same: uint32 counts, else fp64 credits
    unsigned* crow;            // [N][ldk] counts per candidate (counts)
    double* frow;              // [N][ldk] credits per candidate (weighted)
    int ldk;
    int* hint;                 // kFwHints device ints
    FwShared sh;
};

// Tile range [lo, hi] holding the span (predicate.h tile_span) of every disk (c, r) with
// a <= c - r, c + r <= b and |c| + r <= m: partial_range's steps (k_prep.h) with a margin 100x
// wider, which dominates every rounding by which a, b and m — computed from a base disk and the
// displacement bound — can differ from the values tile_span rounds per disk.
__device__ __forceinline__ bool sup_range(double a, double b, double m, double g0, double invS, int n,
                                          int& lo, int& hi)
{
    const double ulo = (a - g0) * invS;
    const double uhi = (b - g0) * invS;
    const double err = (m + __builtin_fabs(g0)) * invS * 1e-12 + 1e-9;
    const double flo = __builtin_floor(ulo - err);
    const double fhi = __builtin_floor(uhi + err);
    if (!(flo == flo) || !(fhi == fhi)) { lo = 0; hi = n - 1; return true; }
    if (fhi < 0.0 || flo > (double)(n - 1)) return false;
    lo = flo < 0.0 ? 0 : (int)flo;
    hi = fhi > (double)(n - 1) ? n - 1 : (int)fhi;
    return true;
}

// The superset box of disk (x0, y0, r0) (candidate 0's) under the displacement bound (dx, dy, dr):
// it holds the tile span of every live candidate's disk of that UAV. False: empty (no live disk
// covers anything); NaN anywhere: the whole grid.
__device__ __forceinline__ bool sup_box(double x0, double y0, double r0, double dx, double dy, double dr,
                                        const Grid& g, int4& B)
{
    const double R = r0 + dr;
    if (!(R > 0.0) && R == R) return false;
    int a0, a1, b0, b1;
    if (!sup_range(x0 - dx - R, x0 + dx + R, __builtin_fabs(x0) + dx + R, g.gx0, g.invS, g.nTx, a0, a1))
        return false;
    if (!sup_range(y0 - dy - R, y0 + dy + R, __builtin_fabs(y0) + dy + R, g.gy0, g.invS, g.nTy, b0, b1))
        return false;
    B = make_int4(a0, a1, b0, b1);
    return true;
}

__device__ __forceinline__ DiskRec inert_disk() { return DiskRec{0.0, 0.0, -1.0, 0.0}; }

// Disk i of candidate k from a packed key word (k_prep.h): base + offsets, the exact doubles.
__device__ __forceinline__ DiskRec word_disk(uint32_t w, double bx, double by, double br)
{
    if (w == kDeadWord) return inert_disk();
    float fx, fy, fr;
    key_unpack(w, fx, fy, fr);
    return make_disk(bx + (double)fx, by + (double)fy, br + (double)fr);
}

__device__ __forceinline__ double src_val(const CandSrc& s, int k, int v, int N)
{
    return s.cands ? s.cands[(int64_t)k * s.ldc + v] : s.get(k, v, N);
}

// Disk jj of candidate k from its key word, or the candidate's own values when the key escaped
__device__ __forceinline__ DiskRec key_disk(const CandSrc& s, uint32_t key, int jj, int k, int N, double bx,
                                            double by, double br)
{
    if (key != kKeyEsc) return word_disk(key, bx, by, br);
    return make_disk(src_val(s, k, jj, N), src_val(s, k, N + jj, N), src_val(s, k, 2 * N + jj, N));
}

#ifdef MAC_DIAG
__device__ uint64_t g_diag_fiw[16 * 65536];  // diagnostic build only: per-disk phase stamps
#define MAC_FW_STAMP(q) if (threadIdx.x == 0 && i < 65536) g_diag_fiw[16 * i + (q)] = __builtin_amdgcn_s_memrealtime()
__device__ uint64_t g_diag_f2[8 * 4096];      // per fin2 block
#define MAC_F2_STAMP(q)                                                                      \
    if (threadIdx.x == 0 && blockIdx.x < 4096) {                                             \
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                          \
        g_diag_f2[8 * blockIdx.x + (q)] = __builtin_amdgcn_s_memrealtime();                  \
    }
#else
#define MAC_FW_STAMP(q)
#define MAC_F2_STAMP(q)
#endif

// per-position / per-candidate credit: exact integer counts (every entry weighs the same) or fp64
template <bool C> struct FwAcc { typedef double T; };
template <> struct FwAcc<true> { typedef unsigned T; };

// kCounts == (a.counts != 0): the equal-weight build keeps its credits in 32-bit integers (half the
// registers of the walk's accumulators and of the shared credits)
template <bool kCounts>
__global__ __launch_bounds__(kFwThreads) __attribute__((amdgpu_waves_per_eu(2))) void fiw_kernel(
    uint64_t* ts, FwArgs a)
{
    typedef typename FwAcc<kCounts>::T Acc;
    ts_begin(ts);
    CandSrc src = a.src;
    const int N = a.N, K = a.K;
    const Grid g = a.g;
    // workgroup b on disk (b % 8) * ceil(N/8) + b / 8: consecutive disks share an XCD
    const int per_xcd = (N + 7) / 8;
    const int i = (int)(blockIdx.x % 8) * per_xcd + (int)(blockIdx.x / 8);
    if (i >= N || !src.resolve()) {   // uniform
        ts_end(ts);
        return;
    }
    MAC_FW_STAMP(0);
    // LDS, by phase (index | walk and shared entries):
    //   X: hash: key word per candidate        | key word per position (poskey)
    //   Y: dedup table (direct or hash)        | credit per position (u32 counts or f64)
    //   Z: per candidate: slot | failed << 15  | per candidate: position | failed << 15
    //   wbuf: hash: a candidate of each position (owner_of)
    //   wbuf: -                                | walk: slice lane constants + staging;
    //                                            in-place shared decisions: coverage words
    __shared__ uint32_t xbuf[kFwMaxK + 1];
    __shared__ double tabbuf[kFwMaxK + 1];
    __shared__ uint16_t zbuf[kFwMaxK + 1];
    constexpr int kSl4 = kFwKPB * 16, kSlx = kFwKPB * 4, kS32 = (kFwCH + 4) * 16, kSix = kFwCH * 4,
                  kSw = kFwCH * 8;
    constexpr int kWB = kSl4 + kSlx + kS32 + kSix + kSw;
    __shared__ __attribute__((aligned(16))) unsigned char wbuf[kWB];
    static_assert(sizeof(uint64_t) * (kFwMaxK + 1) <= kWB, "coverage words fit the walk buffer");
    static_assert(sizeof(int) * (kFwDirect + 1) <= sizeof(double) * (kFwMaxK + 1), "direct table fits");
    __shared__ double2 shp[kFwShE];
    __shared__ double shw[kFwShE];
    __shared__ int shidx[kFwCH];
    __shared__ int rs[kPollRB], rpre[kPollRB + 1];
    __shared__ int nb_id[kFwNbr];
    __shared__ int4 nb_box[kFwNbr];
    __shared__ double nb_b[kFwNbr][3];
    __shared__ double dred[kFwWaves][4];
    __shared__ double sbase[7];   // candidate 0's disk i, the displacement bound
    __shared__ uint8_t scov[kFwKPB]; // per slice slot: its position's disk covers (finite, r > 0)
    __shared__ unsigned ninner;      // entries every position covers (the annulus, counts only)
    __shared__ int ucnt, ncnt, lslot;
    __shared__ int wkeep[kFwR][kFwWaves];
    __shared__ int wshr[kFwR][kFwWaves];   // per round and wave: shared entries handed off
    __shared__ int wsum[kFwWaves];
    uint32_t* const kx = xbuf;
    uint32_t* const poskey = xbuf;
    int* const table = reinterpret_cast<int*>(tabbuf);
    unsigned* const pcnt = reinterpret_cast<unsigned*>(tabbuf);
    double* const pcred = tabbuf;
    uint16_t* const owner_of = reinterpret_cast<uint16_t*>(wbuf);   // (hash numbering only)
    uint16_t* const cinfo = zbuf;
    float4* const sl4 = reinterpret_cast<float4*>(wbuf);
    float* const slx = reinterpret_cast<float*>(wbuf + kSl4);
    float4* const s32 = reinterpret_cast<float4*>(wbuf + kSl4 + kSlx);
    int* const six = reinterpret_cast<int*>(wbuf + kSl4 + kSlx + kS32);
    double* const sw = reinterpret_cast<double*>(wbuf + kSl4 + kSlx + kS32 + kSix);
    uint64_t* const Wd = reinterpret_cast<uint64_t*>(wbuf);

    const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
    constexpr int P = kFwPer + 1;
    auto kof = [&](int j) { return j < kFwPer ? tid * kFwPer + j : (tid == 0 ? kFwMaxK : K); };

    // ---- one round trip: this disk's key row and failure bytes (16-B and 4-B vector loads),
    // candidate 0's disk i, the displacement partials, the lower disks' bases (first two batches)
    int4 RG = make_int4(0, -1, 0, -1);
    bool ident;
    int rf0 = 0, rf1 = 0;   // the first row batch's runs (thread tid: row RG.z + tid), kept in flight
    double2 ppr[kFwR];      // the walk's first chunk of entries, loaded ahead (pjg: list index, -1 none)
    double pwr[kFwR];
    int pjg[kFwR];
    {
        const uint32_t* krow = src.keysP + (int64_t)i * src.ldk;
        uint32_t pq[P];
        bool dj[P];
#pragma unroll
        for (int c = 0; c < kFwPer / 4; ++c) {
            const int b0 = tid * kFwPer + 4 * c;   // (b0 % 4 == 0 and ldk % 32 == 0: b0 < ldk => b0 + 4 <= ldk)
            const uint4 q4 = b0 < src.ldk ? *reinterpret_cast<const uint4*>(krow + b0) : make_uint4(0, 0, 0, 0);
            const uint32_t d4 = a.dead && b0 < src.ldk ? *reinterpret_cast<const uint32_t*>(a.dead + b0) : 0u;
            pq[4 * c] = q4.x;
            pq[4 * c + 1] = q4.y;
            pq[4 * c + 2] = q4.z;
            pq[4 * c + 3] = q4.w;
#pragma unroll
            for (int e = 0; e < 4; ++e) dj[4 * c + e] = ((d4 >> (8 * e)) & 0xFFu) != 0 && b0 + e < K;
        }
        pq[kFwPer] = tid == 0 && K > kFwMaxK ? krow[kFwMaxK] : 0u;
        dj[kFwPer] = tid == 0 && K > kFwMaxK && a.dead && a.dead[kFwMaxK] != 0;
        const double bx = src_val(src, 0, i, N), by = src_val(src, 0, N + i, N),
                     br = src_val(src, 0, 2 * N + i, N);
        double dmx = -__builtin_inf(), dmy = -__builtin_inf(), dmr = -__builtin_inf(), dml = -__builtin_inf();
        for (int q = tid; q < a.npd; q += kFwThreads) {
            const double4 d4 = a.pd[q];
            dmx = fmax(dmx, d4.x);
            dmy = fmax(dmy, d4.y);
            dmr = fmax(dmr, d4.z);
            dml = fmax(dml, d4.w);
        }
        double jb[2][3];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int j = tid + q * kFwThreads;
            const int jc = min(j, N - 1);
            jb[q][0] = j < i ? src_val(src, 0, jc, N) : 0.0;
            jb[q][1] = j < i ? src_val(src, 0, N + jc, N) : 0.0;
            jb[q][2] = j < i ? src_val(src, 0, 2 * N + jc, N) : 0.0;
        }
        if (tid == 0) {
            ucnt = 0;
            ncnt = 0;
            ninner = 0u;
        }
        // the key words (failed: the dead word) and failure bits into LDS, this thread's own
        // candidates (no barrier needed to read them back): no per-candidate registers stay live
        // through the index (the walk needs every register it can get)
        bool esc = false;
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const int k = kof(j);
            esc |= k < K && !dj[j] && pq[j] == kKeyEsc;
            if (k < K) {
                kx[k] = dj[j] ? kDeadWord : pq[j];
                zbuf[k] = dj[j] ? (uint16_t)0x8000 : (uint16_t)0;
            }
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            dmx = fmax(dmx, __shfl_xor(dmx, o, kWave));
            dmy = fmax(dmy, __shfl_xor(dmy, o, kWave));
            dmr = fmax(dmr, __shfl_xor(dmr, o, kWave));
            dml = fmax(dml, __shfl_xor(dml, o, kWave));
        }
        if (lane == 0) {
            dred[wid][0] = dmx;
            dred[wid][1] = dmy;
            dred[wid][2] = dmr;
            dred[wid][3] = dml;
        }
        // one position per candidate when a key escaped (a disk off the packed grid)
        ident = __syncthreads_or(esc);
        MAC_FW_STAMP(1);
#pragma unroll
        for (int q = 0; q < kFwWaves; ++q) {
            dmx = fmax(dmx, dred[q][0]);
            dmy = fmax(dmy, dred[q][1]);
            dmr = fmax(dmr, dred[q][2]);
            dml = fmax(dml, dred[q][3]);
        }
        if (tid == 0) {
            sbase[0] = bx;
            sbase[1] = by;
            sbase[2] = br;
            sbase[3] = dmx;
            sbase[4] = dmy;
            sbase[5] = dmr;
            sbase[6] = dml;
        }
        const bool rany = sup_box(bx, by, br, dmx, dmy, dmr, g, RG);
        if (!rany) RG = make_int4(0, -1, 0, -1);
        // the first row batch's runs, in flight through the deduplication
        const int nrows = rany ? RG.w - RG.z + 1 : 0;
        if (tid < min(nrows, kPollRB)) {
            const int64_t rb = (int64_t)(RG.z + tid) * g.nTx;
            rf0 = a.off[rb + RG.x];
            rf1 = a.off[rb + RG.y + 1];
        }
        // ---- lower neighbours: disks j < i whose boxes overlap box i
        if (rany) {
            auto test = [&](int j, double x0, double y0, double r0) {
                int4 B;
                if (sup_box(x0, y0, r0, dmx, dmy, dmr, g, B) && box_overlap(B, RG)) {
                    const int p = atomicAdd(&ncnt, 1);
                    if (p < kFwNbr) {
                        nb_id[p] = j;
                        nb_box[p] = B;
                        nb_b[p][0] = x0;
                        nb_b[p][1] = y0;
                        nb_b[p][2] = r0;
                    }
                }
            };
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int j = tid + q * kFwThreads;
                if (j < i) test(j, jb[q][0], jb[q][1], jb[q][2]);
            }
            for (int j = tid + 2 * kFwThreads; j < i; j += kFwThreads)
                test(j, src_val(src, 0, j, N), src_val(src, 0, N + j, N), src_val(src, 0, 2 * N + j, N));
        }
        MAC_FW_STAMP(12);
        // ---- positions. Direct-mapped when the live candidates' key offsets fit a small box
        // (every live key packs to (dx, dy, dr) with |dx| <= Dx, |dy| <= Dy, -Dl <= dr <= Dr: the
        // displacement bound): one slot per offset triple, plain stores, positions numbered in slot
        // order; a candidate whose disk has r <= 0 (covers nothing) goes to the dead slot. Else an
        // LDS hash over the key words (linear probing).
        const bool dfits = !ident && dmx >= 0.0 && dmx <= 1023.0 && dmy >= 0.0 && dmy <= 1023.0 &&
                           dmr >= -511.0 && dmr <= 511.0 && dml >= -511.0 && dml <= 511.0;
        const int Dx = dfits ? (int)dmx : 0, Dy = dfits ? (int)dmy : 0;
        const int Dr = dfits ? (int)dmr : 0, Dl = dfits ? (int)dml : 0;
        const int nyd = 2 * Dy + 1, nrd = Dr + Dl + 1;
        const int nslot = dfits && nrd >= 1 ? (2 * Dx + 1) * nyd * nrd : 0;
        bool direct = dfits && nrd >= 1 && (double)Dx == dmx && (double)Dy == dmy && (double)Dr == dmr &&
                      (double)Dl == dml && nslot + 1 <= kFwDirect;
        if (direct) {
            for (int q = tid; q <= nslot; q += kFwThreads) table[q] = 0;
        }
        lds_barrier();   // (the table is cleared; the row runs' loads stay in flight)
        MAC_FW_STAMP(15);
        bool miss = false;
        if (direct) {   // per candidate its slot (zbuf, beside the failure bit); branch-free
#pragma unroll
            for (int j = 0; j < P; ++j) {
                const int k = kof(j);
                const uint32_t w = pq[j];
                const int dx = (int)(w << 21) >> 21, dy = (int)(w << 10) >> 21, dr = (int)w >> 22;
                // (r <= 0 covers nothing: the dead slot, as a failed candidate)
                const bool live = k < K && !dj[j] && br + (double)dr > 0.0;
                const bool inr = dx >= -Dx && dx <= Dx && dy >= -Dy && dy <= Dy && dr >= -Dl && dr <= Dr;
                miss |= live && !inr;
                const int sl = live && inr ? ((dx + Dx) * nyd + (dy + Dy)) * nrd + (dr + Dl) : nslot;
                if (k < K) {
                    table[sl] = 1;
                    zbuf[k] = (uint16_t)((dj[j] ? 0x8000 : 0) | sl);
                }
            }
        }
        MAC_FW_STAMP(13);
        {   // any miss: the hash (an LDS word, not __syncthreads_or: that would wait for the row runs)
            const uint64_t mb = __ballot(miss);
            if (lane == 0) wsum[wid] = mb != 0;
            lds_barrier();
            bool any = false;
#pragma unroll
            for (int q = 0; q < kFwWaves; ++q) any |= wsum[q] != 0;
            direct = direct && !any;
            lds_barrier();   // (wsum is reused below)
        }
        MAC_FW_STAMP(14);
        if (direct) {
            // number the occupied slots in slot order: each thread a run of consecutive slots
            const int per = (nslot + 1 + kFwThreads - 1) / kFwThreads;
            const int s0 = min(tid * per, nslot + 1), s1 = min(s0 + per, nslot + 1);
            int c = 0;
            for (int s = s0; s < s1; ++s) c += table[s];
            const int incl = wave_incl_scan_i32(c, lane);
            if (lane == kWave - 1) wsum[wid] = incl;
            lds_barrier();
            int id = incl - c;
            for (int q = 0; q < wid; ++q) id += wsum[q];
            for (int s = s0; s < s1; ++s) {
                if (table[s]) {
                    uint32_t wk = kDeadWord;
                    if (s < nslot) {
                        const int dr = s % nrd - Dl, t2 = s / nrd;
                        const int dy = t2 % nyd - Dy, dx = t2 / nyd - Dx;
                        wk = key_pack(dx, dy, dr);
                    }
                    poskey[id] = wk;
                    table[s] = id++;
                }
            }
            if (tid == kFwThreads - 1) ucnt = id;
        } else if (!ident) {
            for (int q = tid; q < kFwHash; q += kFwThreads) table[q] = -1;
            lds_barrier();
            constexpr uint32_t mask = kFwHash - 1;
#pragma unroll
            for (int j = 0; j < P; ++j) {
                const int k = kof(j);
                if (k >= K) continue;
                const uint32_t key = kx[k];
                uint32_t s = word_hash(key) & mask;
                for (;;) {
                    int cur = table[s];
                    if (cur < 0) {
                        cur = atomicCAS(&table[s], -1, k);
                        if (cur < 0) break;
                    }
                    if (kx[cur] == key) break;
                    s = (s + 1) & mask;
                }
                zbuf[k] = (uint16_t)((zbuf[k] & 0x8000) | s);   // (the slot, beside the failure bit)
            }
            lds_barrier();
            for (int q = tid; q < kFwHash; q += kFwThreads) {
                const int owner = table[q];
                if (owner >= 0) {
                    const int u = atomicAdd(&ucnt, 1);
                    owner_of[u] = (uint16_t)owner;
                    table[q] = (owner << kFwIdBits) | u;
                }
            }
        }
        lds_barrier();
        MAC_FW_STAMP(2);
        // the walk's first row batch (its runs have arrived by now) and the first chunk's entry
        // loads, left in flight through the positions and the slice's lane constants
        if (rany && tid < kWave) {
            const int nr = min(kPollRB, RG.w - RG.z + 1);
            const int len = tid < nr ? rf1 - rf0 : 0;
            const int incl = wave_incl_scan_i32(len, tid);
            if (tid < nr) {
                rs[tid] = rf0;
                rpre[tid + 1] = incl;
            }
            if (tid == 0) rpre[0] = 0;
        }
        lds_barrier();
        if (rany) {
            const int nr = min(kPollRB, RG.w - RG.z + 1);
            const int nraw = min(kFwCH, rpre[nr]);
#pragma unroll
            for (int r = 0; r < kFwR; ++r) {
                const int qd = tid + r * kFwThreads;
                pjg[r] = -1;
                if (qd < nraw) {
                    int lo = 0, hi = nr - 1;
                    while (lo < hi) {
                        const int mid = (lo + hi + 1) >> 1;
                        if (rpre[mid] <= qd) lo = mid; else hi = mid - 1;
                    }
                    pjg[r] = rs[lo] + (qd - rpre[lo]);
                    ppr[r] = a.xy[pjg[r]];
                    pwr[r] = a.w[pjg[r]];
                }
            }
        }
        // per candidate its position; hash: per position its key word (through registers: the
        // buffers change roles at the barrier)
        const int U0 = ident ? K : ucnt;
        constexpr int PU = (kFwMaxK + 1 + kFwThreads - 1) / kFwThreads;
        uint32_t pkr[PU];
        const bool hashed = !direct && !ident;
#pragma unroll
        for (int q = 0; q < PU; ++q) {
            const int u = tid + q * kFwThreads;
            pkr[q] = hashed && u < U0 ? kx[owner_of[u]] : 0u;
        }
        // per candidate its position (this thread's own zbuf words: slot -> position), read
        // before the barrier: the table's words become the position credits after it
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const int k = kof(j);
            if (k >= K) continue;
            const uint16_t zb = zbuf[k];
            const int sl = zb & 0x7FFF;
            const int u = ident ? k : direct ? table[sl] : table[sl] & ((1 << kFwIdBits) - 1);
            cinfo[k] = (uint16_t)(u | (zb & 0x8000));
        }
        lds_barrier();
        if (hashed) {
#pragma unroll
            for (int q = 0; q < PU; ++q)
                if (tid + q * kFwThreads < U0) poskey[tid + q * kFwThreads] = pkr[q];
        }
        for (int u = tid; u < U0; u += kFwThreads) {
            if (kCounts) pcnt[u] = 0u;
            else pcred[u] = 0.0;
        }
        lds_barrier();
    }
    MAC_FW_STAMP(3);
    const int U = ident ? K : ucnt;
    const int nc = ncnt;
    const bool rany = RG.x <= RG.y;
    // position u's disk: its key word (or, one position per candidate, the candidate's own disk)
    auto pos_disk = [&](int u) -> DiskRec {
        if (ident) {
            if (cinfo[u] & 0x8000) return inert_disk();
            return make_disk(src_val(src, u, i, N), src_val(src, u, N + i, N), src_val(src, u, 2 * N + i, N));
        }
        return word_disk(poskey[u], sbase[0], sbase[1], sbase[2]);
    };

    // The walk's lane constants need T(r) only to within the fp32 filter's spare error budget
    // (k_poll.h: the filter's error is below 38.1 eps M^2 S, the band half-width X' is 64 eps M^2 S,
    // eps = 2^-24): fl(r * r) differs from T(r) by a few ulp of r^2 (2^-51 M^2), far inside it, and
    // every entry in the band is re-decided with the exact T (pos_disk). So the lane constants take
    // the disk from its key word and r * r, without the 128-bit threshold (cover_threshold).
    auto walk_disk = [&](int u) -> DiskRec {
        DiskRec d;
        if (ident) {
            if (cinfo[u] & 0x8000) return inert_disk();
            d.cx = src_val(src, u, i, N);
            d.cy = src_val(src, u, N + i, N);
            d.r = src_val(src, u, 2 * N + i, N);
        } else {
            const uint32_t w = poskey[u];
            if (w == kDeadWord) return inert_disk();
            float fx, fy, fr;
            key_unpack(w, fx, fy, fr);
            d.cx = sbase[0] + (double)fx;
            d.cy = sbase[1] + (double)fy;
            d.r = sbase[2] + (double)fr;
        }
        d.T = d.r > 0.0 ? d.r * d.r : -1.0;
        return d;
    };
    // The annulus (equal weights): every position's disk (c, r) lies within the displacement
    // bound of candidate 0's, |cx - x0| <= Dx, |cy - y0| <= Dy, r >= r0 - Dl, r <= r0 + Dr, so an
    // entry at distance d from (x0, y0) is covered by all of them when d + hypot(Dx, Dy) < r0 - Dl
    // and by none when d - hypot(Dx, Dy) > r0 + Dr; margins of 1e-9 (relative) dominate every
    // rounding of d, the bound and the reference's sqrt(d^2) < r. Those entries skip the tests:
    // the first are counted once and credited to every covering position, the second dropped.
    double rin2 = -1.0, rout2 = __builtin_inf();
    if (kCounts && rany) {
        const double bx0 = sbase[2], ex = sbase[3], ey = sbase[4], er = sbase[5], el = sbase[6];
        const double e = __builtin_sqrt(ex * ex + ey * ey) * (1.0 + 1e-9);
        const double rin = (bx0 - el) - e - 1e-9 * (__builtin_fabs(bx0) + __builtin_fabs(el) + e + 1.0);
        if (rin > 0.0 && rin < 1e150) rin2 = rin * rin * (1.0 - 1e-9);
        const double rout = (bx0 + er) + e + 1e-9 * (__builtin_fabs(bx0) + __builtin_fabs(er) + e + 1.0);
        if (rout > 0.0 && rout < 1e150) rout2 = rout * rout * (1.0 + 1e-9);
    }

    // the shared entries (box i's entries inside a lower box) are handed to fin2_kernel from the
    // walk's own compaction (slice 0), in its fixed order, when the list can take the disk
    const bool hand_ok = nc > 0 && nc <= kFwHand;
    int nsh_walk = 0;
    // ---- the walk of box i over the entries no lower box holds (k_poll.h)
    if (rany) {
        const double ox = g.gx0 + 0.5 * (double)(RG.x + RG.y + 1) * g.S;
        const double oy = g.gy0 + 0.5 * (double)(RG.z + RG.w + 1) * g.S;
        const double Umax = 0.5 * (double)max(RG.y - RG.x + 1, RG.w - RG.z + 1) * g.S + 2.0 * g.S;
        for (int kb = 0; kb < U; kb += kFwKPB) {
            const int ke = min(U, kb + kFwKPB);
            for (int t = tid; t < kFwKPB; t += kFwThreads) {   // the slice's lane constants
                const int u = kb + t;
                PollLane L = inert_lane();
                bool cov = false;
                if (u < ke) {
                    const DiskRec d = walk_disk(u);
                    // (a finite disk with r > 0 whose span misses the grid covers no entry: its
                    // lane decides every staged entry "not covered", exactly as an inert lane)
                    cov = d.T >= 0.0 && __builtin_isfinite(d.cx) && __builtin_isfinite(d.cy);
                    if (cov) L = poll_lane(d, ox, oy, Umax);
                }
                sl4[t] = make_float4(L.sa, L.sb, L.stm, L.ns);
                slx[t] = L.xp;
                scov[t] = cov ? 1 : 0;
            }
            __syncthreads();
            if (kb == 0) MAC_FW_STAMP(8);
            f32x2 sa[kPollPairs], sb[kPollPairs], st[kPollPairs], ns[kPollPairs];
            float xp[kPollSlots];
            Acc acc[kPollSlots];
            uint32_t live = 0, covm = 0;
#pragma unroll
            for (int u = 0; u < kPollSlots; ++u) {
                const int p = u * kWave + lane;
                const float4 c = sl4[p];
                xp[u] = kb + p < ke ? slx[p] : -1.0f;
                if (kb + p < ke) live |= 1u << u;
                if (kb + p < ke && scov[p]) covm |= 1u << u;
                acc[u] = 0;
                const int j = u >> 1;
                if (u & 1) {
                    sa[j].y = c.x; sb[j].y = c.y; st[j].y = c.z; ns[j].y = c.w;
                } else {
                    sa[j].x = c.x; sb[j].x = c.y; st[j].x = c.z; ns[j].x = c.w;
                }
            }
            const int np = (ke - kb + 2 * kWave - 1) / (2 * kWave);
            for (int rb = RG.z; rb <= RG.w; rb += kPollRB) {
                const int nr = min(kPollRB, RG.w - rb + 1);
                const bool first_rb = kb == 0 && rb == RG.z;   // (its runs are scanned already)
                if (!first_rb) {
                    int rs0 = 0, rs1 = 0;
                    if (rb == RG.z) {
                        if (tid < nr) {
                            rs0 = rf0;
                            rs1 = rf1;
                        }
                    } else if (tid < nr) {   // later row batches (boxes over 64 rows): their runs now
                        const int64_t rowb = (int64_t)(rb + tid) * g.nTx;
                        rs0 = a.off[rowb + RG.x];
                        rs1 = a.off[rowb + RG.y + 1];
                    }
                    __syncthreads();   // (the previous batch's rows are read)
                    if (tid < kWave) {
                        const int len = tid < nr ? rs1 - rs0 : 0;
                        const int incl = wave_incl_scan_i32(len, tid);
                        if (tid < nr) {
                            rs[tid] = rs0;
                            rpre[tid + 1] = incl;
                        }
                        if (tid == 0) rpre[0] = 0;
                    }
                    __syncthreads();
                }
                const int total = rpre[nr];
                for (int base = 0; base < total; base += kFwCH) {
                    // the chunk's entries disk i may own (no lower box holds them, finite),
                    // compacted in a fixed order (round, wave, lane)
                    const int nraw = min(kFwCH, total - base);
                    const bool pre = first_rb && base == 0;   // loaded ahead (ppr, pwr, pjg)
                    double2 pr[kFwR];
                    double wr[kFwR];
                    int jg[kFwR];
                    uint64_t bal[kFwR], hbal[kFwR];
#pragma unroll
                    for (int r = 0; r < kFwR; ++r) {
                        const int qd = tid + r * kFwThreads;
                        bool keep = false, inner = false, hs = false;
                        pr[r] = make_double2(0.0, 0.0);
                        wr[r] = 0.0;
                        jg[r] = 0;
                        if (qd < nraw) {
                            const int f = base + qd;
                            int lo = 0, hi = nr - 1;
                            while (lo < hi) {
                                const int mid = (lo + hi + 1) >> 1;
                                if (rpre[mid] <= f) lo = mid; else hi = mid - 1;
                            }
                            if (pre) {
                                jg[r] = pjg[r];
                                pr[r] = ppr[r];
                                wr[r] = pwr[r];
                            } else {
                                jg[r] = rs[lo] + (f - rpre[lo]);
                                pr[r] = a.xy[jg[r]];
                                wr[r] = a.w[jg[r]];
                            }
                            const bool shared = nc > 0 &&
                                entry_shared(nc, nb_box, tile_of(pr[r].x, g.gx0, g.invS, g.nTx), rb + lo);
                            const bool fin = __builtin_isfinite(pr[r].x) && __builtin_isfinite(pr[r].y);
                            keep = !shared && fin;
                            hs = shared && fin;
                            if (keep) {   // the annulus: inside every disk / outside all
                                const double ux = pr[r].x - sbase[0], uy = pr[r].y - sbase[1];
                                const double d0 = ux * ux + uy * uy;
                                if (d0 <= rin2) {
                                    keep = false;
                                    inner = true;
                                } else if (d0 >= rout2) {
                                    keep = false;
                                }
                            }
                        }
                        const uint64_t ib = __ballot(inner);
                        if (kb == 0 && lane == 0 && ib) atomicAdd(&ninner, (unsigned)__popcll(ib));
                        bal[r] = __ballot(keep);
                        if (lane == 0) wkeep[r][wid] = __popcll(bal[r]);
                        hbal[r] = __ballot(hs && kb == 0 && hand_ok);
                        if (lane == 0) wshr[r][wid] = __popcll(hbal[r]);
                    }
                    __syncthreads();
                    if (kb == 0 && hand_ok) {   // (uniform) hand-off copies, in the fixed order
#pragma unroll
                        for (int r = 0; r < kFwR; ++r) {
                            int hd = nsh_walk + __popcll(hbal[r] & ((1ull << lane) - 1));
#pragma unroll
                            for (int w2 = 0; w2 < kFwWaves; ++w2) {
                                if (w2 < wid) hd += wshr[r][w2];
                                nsh_walk += wshr[r][w2];
                            }
                            if (((hbal[r] >> lane) & 1) && hd < kFwShCap) {
                                a.sh.xy[(int64_t)i * kFwShCap + hd] = pr[r];
                                a.sh.w[(int64_t)i * kFwShCap + hd] = wr[r];
                            }
                        }
                    }
                    int n = 0;
#pragma unroll
                    for (int r = 0; r < kFwR; ++r) {
                        int dst = n + __popcll(bal[r] & ((1ull << lane) - 1));
#pragma unroll
                        for (int w2 = 0; w2 < kFwWaves; ++w2) {
                            if (w2 < wid) dst += wkeep[r][w2];
                            n += wkeep[r][w2];
                        }
                        if ((bal[r] >> lane) & 1) {
                            six[dst] = jg[r];
                            sw[dst] = wr[r];
                            const float fu = (float)(pr[r].x - ox), fv = (float)(pr[r].y - oy);
                            s32[dst] = __builtin_isfinite(fu) && __builtin_isfinite(fv)
                                           ? make_float4(__builtin_fmaf(fu, fu, fv * fv), fu, fv, 0.0f)
                                           : make_float4(__builtin_inff(), 0.0f, 0.0f, 0.0f);
                        }
                    }
                    if (tid < ((4 - (n & 3)) & 3)) s32[n + tid] = make_float4(__builtin_inff(), 0.0f, 0.0f, 0.0f);
                    __syncthreads();
                    bool uniform = true;   // (equal weights: always)
                    if constexpr (!kCounts) {
                        const uint64_t w0b = __builtin_bit_cast(uint64_t, sw[0]);
                        bool mixed = false;
                        for (int e = tid; e < n; e += kFwThreads) mixed |= __builtin_bit_cast(uint64_t, sw[e]) != w0b;
                        uniform = !__syncthreads_or(mixed);
                    }
                    if (kb == 0 && rb == RG.z && base == 0) MAC_FW_STAMP(9);
                    const int ng = (n + 3) >> 2;
                    float bmin[kPollSlots];
#pragma unroll
                    for (int u = 0; u < kPollSlots; ++u) bmin[u] = __builtin_inff();
                    if (uniform) {
                        f32x2 h[kPollPairs];
                        switch (np) {
                        case 1: poll_hot<1, kFwWaves>(s32, ng, wid, sa, sb, st, ns, h, bmin); break;
                        case 2: poll_hot<2, kFwWaves>(s32, ng, wid, sa, sb, st, ns, h, bmin); break;
                        case 3: poll_hot<3, kFwWaves>(s32, ng, wid, sa, sb, st, ns, h, bmin); break;
                        default: poll_hot<4, kFwWaves>(s32, ng, wid, sa, sb, st, ns, h, bmin); break;
                        }
                        const double wu = kCounts ? 1.0 : sw[0];
#pragma unroll
                        for (int u = 0; u < kPollSlots; ++u) {
                            const float hc = (u & 1) ? h[u >> 1].y : h[u >> 1].x;
                            if ((live & (1u << u)) && !(bmin[u] <= xp[u])) {
                                if constexpr (kCounts) acc[u] += (unsigned)hc;
                                else acc[u] += (double)hc * wu;
                            }
                        }
                    } else {
                        for (int q4 = wid; q4 < ng; q4 += kFwWaves) {
                            for (int e = 0; e < 4; ++e) {
                                const int qe = 4 * q4 + e;
                                const float4 en = s32[qe];
                                const double wq = qe < n ? sw[qe] : 0.0;
#pragma unroll
                                for (int u = 0; u < kPollSlots; ++u) {
                                    const int j = u >> 1;
                                    const float d = (u & 1)
                                        ? __builtin_fmaf(en.x, ns[j].y, __builtin_fmaf(en.z, sb[j].y, __builtin_fmaf(en.y, sa[j].y, st[j].y)))
                                        : __builtin_fmaf(en.x, ns[j].x, __builtin_fmaf(en.z, sb[j].x, __builtin_fmaf(en.y, sa[j].x, st[j].x)));
                                    if ((live & (1u << u)) && d > 0.0f) acc[u] += (Acc)wq;
                                    bmin[u] = __builtin_fminf(bmin[u], __builtin_fabsf(d));
                                }
                            }
                        }
                    }
                    // band: a slot with an entry within X' of the threshold re-decides this wave's
                    // entries of the chunk in fp64 (the position's disk from its key; the slot's
                    // constants from the slice arrays). The weighted loop above added the slot's
                    // fp32 decisions already: they are replaced.
                    if (kb == 0 && rb == RG.z && base == 0) MAC_FW_STAMP(10);
                    uint32_t bandm = 0;
#pragma unroll
                    for (int u = 0; u < kPollSlots; ++u)
                        if ((live & (1u << u)) && bmin[u] <= xp[u]) bandm |= 1u << u;
                    while (bandm) {
                        const int ub = __builtin_ctz(bandm);
                        bandm &= bandm - 1;
                        const int p = ub * kWave + lane;
                        const float4 c = sl4[p];
                        const float xpb = slx[p];
                        const DiskRec d = pos_disk(kb + p);
                        double cv = 0.0, fv = 0.0;   // the exact credit, the fp32 credit it replaces
                        for (int q4 = wid; q4 < ng; q4 += kFwWaves)
                            for (int e = 4 * q4; e < min(4 * q4 + 4, n); ++e) {
                                const float4 en = s32[e];
                                const float dp = __builtin_fmaf(en.x, c.w, __builtin_fmaf(en.z, c.y, __builtin_fmaf(en.y, c.x, c.z)));
                                bool cov;
                                if (__builtin_fabsf(dp) <= xpb) {
                                    const double2 q = a.xy[six[e]];
                                    cov = sqdist(q.x, q.y, d.cx, d.cy) <= d.T;
                                } else {
                                    cov = dp > 0.0f;
                                }
                                const double we = kCounts ? 1.0 : sw[e];
                                if (cov) cv += we;
                                if (dp > 0.0f) fv += we;
                            }
#pragma unroll
                        for (int u = 0; u < kPollSlots; ++u)
                            if (u == ub) acc[u] += (Acc)(uniform ? cv : cv - fv);
                    }
                    __syncthreads();   // the staging is read
                    if (kb == 0 && rb == RG.z && base == 0) MAC_FW_STAMP(11);
                }
            }
            // the slice's credit per position, the waves' shares added in wave order (wave 0
            // adds the annulus' inner entries to every covering position)
            if constexpr (kCounts) {
                const unsigned nin = wid == 0 ? ninner : 0u;
#pragma unroll
                for (int u = 0; u < kPollSlots; ++u)
                    if (live & (1u << u))
                        atomicAdd(&pcnt[kb + u * kWave + lane], (unsigned)acc[u] + ((covm >> u) & 1u ? nin : 0u));
            } else {
                for (int w2 = 0; w2 < kFwWaves; ++w2) {
                    if (w2 == wid) {
#pragma unroll
                        for (int u = 0; u < kPollSlots; ++u)
                            if (live & (1u << u)) pcred[kb + u * kWave + lane] += acc[u];
                    }
                    __syncthreads();
                }
            }
            __syncthreads();   // (the slice arrays are rewritten by the next slice)
        }
    }
    MAC_FW_STAMP(4);

    // ---- the shared entries (box i's entries inside a lower box): enumerated in a fixed order and
    // handed to fin2_kernel, or — past kFwShCap entries or kFwNbr neighbours — decided here
    Acc sh[P];
#pragma unroll
    for (int j = 0; j < P; ++j) sh[j] = 0;
    int swork = 0;
    bool handed = false;
    if (rany && hand_ok && nsh_walk <= kFwShCap) {   // (uniform) a place on the list, else in place
        if (tid == 0) lslot = atomicAdd(a.sh.count, 1);
        __syncthreads();
        if (lslot < kF2ListCap) {
            handed = true;
            swork = nsh_walk;
        }
    }
    if (rany && nc > 0 && !handed) {
        const int nclist = min(nc, kFwNbr);
        // decided in place: the entries enumerated again, in windows, per candidate in fp64
        {
            for (int rb = RG.z; rb <= RG.w; rb += kPollRB) {
                const int nr = min(kPollRB, RG.w - rb + 1);
                int rs0 = 0, rs1 = 0;
                if (tid < nr) {
                    const int64_t rowb = (int64_t)(rb + tid) * g.nTx;
                    rs0 = a.off[rowb + RG.x];
                    rs1 = a.off[rowb + RG.y + 1];
                }
                __syncthreads();
                if (tid < kWave) {
                    const int len = tid < nr ? rs1 - rs0 : 0;
                    const int incl = wave_incl_scan_i32(len, tid);
                    if (tid < nr) {
                        rs[tid] = rs0;
                        rpre[tid + 1] = incl;
                    }
                    if (tid == 0) rpre[0] = 0;
                }
                __syncthreads();
                const int total = rpre[nr];
                for (int base = 0; base < total; base += kFwCH) {
                    // the window's shared entries, compacted in a fixed order (their list indices)
                    const int nraw = min(kFwCH, total - base);
                    int jglob[kFwR];
                    uint64_t bal[kFwR];
#pragma unroll
                    for (int r = 0; r < kFwR; ++r) {
                        const int qd = tid + r * kFwThreads;
                        bool shared = false;
                        jglob[r] = 0;
                        if (qd < nraw) {
                            const int f = base + qd;
                            int lo = 0, hi = nr - 1;
                            while (lo < hi) {
                                const int mid = (lo + hi + 1) >> 1;
                                if (rpre[mid] <= f) lo = mid; else hi = mid - 1;
                            }
                            jglob[r] = rs[lo] + (f - rpre[lo]);
                            const double2 p = a.xy[jglob[r]];
                            shared = __builtin_isfinite(p.x) && __builtin_isfinite(p.y) &&
                                     entry_shared(nc, nb_box, tile_of(p.x, g.gx0, g.invS, g.nTx), rb + lo);
                        }
                        bal[r] = __ballot(shared);
                        if (lane == 0) wkeep[r][wid] = __popcll(bal[r]);
                    }
                    __syncthreads();
                    int nsh = 0;
#pragma unroll
                    for (int r = 0; r < kFwR; ++r) {
                        int dst = nsh + __popcll(bal[r] & ((1ull << lane) - 1));
#pragma unroll
                        for (int w2 = 0; w2 < kFwWaves; ++w2) {
                            if (w2 < wid) dst += wkeep[r][w2];
                            nsh += wkeep[r][w2];
                        }
                        if ((bal[r] >> lane) & 1) shidx[dst] = jglob[r];
                    }
                    __syncthreads();
                    swork += nsh;
                    for (int e0 = 0; e0 < nsh; e0 += kFwShE) {
                        const int ne = min(kFwShE, nsh - e0);
                        if (tid < ne) {
                            shp[tid] = a.xy[shidx[e0 + tid]];
                            shw[tid] = a.w[shidx[e0 + tid]];
                        }
                        __syncthreads();
                        // per position: the word of the chunk's entries its disk covers (exact)
                        for (int u = tid; u < U; u += kFwThreads) {
                            const DiskRec d = pos_disk(u);
                            uint64_t m = 0;
                            for (int e = 0; e < ne; ++e)
                                if (sqdist(shp[e].x, shp[e].y, d.cx, d.cy) <= d.T) m |= 1ull << e;
                            Wd[u] = m;
                        }
                        __syncthreads();
                        // per candidate: disk i's word, minus the entries a lower neighbour's disk
                        // of the same candidate covers
                        uint64_t Mj[P];
#pragma unroll
                        for (int j = 0; j < P; ++j) {
                            const int k = kof(j);
                            const uint16_t ci = k < K ? cinfo[k] : (uint16_t)0x8000;
                            Mj[j] = (ci & 0x8000) ? 0ull : Wd[ci & 0x7FFF];
                        }
                        auto strip = [&](int jj, double x0, double y0, double r0) {
                            uint32_t key[P];
#pragma unroll
                            for (int j = 0; j < P; ++j)
                                key[j] = Mj[j] ? src.keysP[(int64_t)jj * src.ldk + kof(j)] : 0u;
#pragma unroll
                            for (int j = 0; j < P; ++j) {
                                if (!Mj[j]) continue;
                                const DiskRec d = key_disk(src, key[j], jj, kof(j), N, x0, y0, r0);
                                for (uint64_t b = Mj[j]; b;) {
                                    const int e = __builtin_ctzll(b);
                                    b &= b - 1;
                                    if (sqdist(shp[e].x, shp[e].y, d.cx, d.cy) <= d.T) Mj[j] &= ~(1ull << e);
                                }
                            }
                        };
                        if (nc <= kFwNbr) {
                            for (int m = 0; m < nclist; ++m) strip(nb_id[m], nb_b[m][0], nb_b[m][1], nb_b[m][2]);
                        } else {   // overflowed list: every lower disk whose box overlaps box i
                            for (int jj = 0; jj < i; ++jj) {
                                const double x0 = src_val(src, 0, jj, N), y0 = src_val(src, 0, N + jj, N),
                                             r0 = src_val(src, 0, 2 * N + jj, N);
                                int4 B;
                                if (sup_box(x0, y0, r0, sbase[3], sbase[4], sbase[5], g, B) && box_overlap(B, RG))
                                    strip(jj, x0, y0, r0);
                            }
                        }
#pragma unroll
                        for (int j = 0; j < P; ++j) {
                            if constexpr (kCounts) {
                                sh[j] += (unsigned)__popcll(Mj[j]);
                            } else {
                                for (uint64_t b = Mj[j]; b;) {
                                    const int e = __builtin_ctzll(b);
                                    b &= b - 1;
                                    sh[j] += shw[e];
                                }
                            }
                        }
                        __syncthreads();   // the chunk and the words are reused
                    }
                }
            }
        }
    }
    if (tid == 0 && handed) {
        int id[kFwHand];
#pragma unroll
        for (int m = 0; m < kFwHand; ++m) id[m] = m < nc ? nb_id[m] : 0;
        a.sh.list[lslot] = make_int4(i, nc | (swork << 8), (int)((unsigned)id[0] | ((unsigned)id[1] << 16)),
                                     (int)((unsigned)id[2] | ((unsigned)id[3] << 16)));
    }
    MAC_FW_STAMP(5);
    // ---- the row: per candidate its position's credit (plus the shared credit decided in place)
    const int64_t orow = (int64_t)i * a.ldk;
#pragma unroll
    for (int c = 0; c < kFwPer / 4; ++c) {
        const int b0 = tid * kFwPer + 4 * c;
        if (b0 >= K) break;
        if constexpr (kCounts) {
            unsigned v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int k = b0 + e;
                const uint16_t ci = k < K ? cinfo[k] : (uint16_t)0x8000;
                v[e] = (ci & 0x8000) || !rany ? 0u : pcnt[ci & 0x7FFF] + (unsigned)sh[4 * c + e];
            }
            *reinterpret_cast<uint4*>(a.crow + orow + b0) = make_uint4(v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int k = b0 + e;
                if (k >= K) break;
                const uint16_t ci = cinfo[k];
                a.frow[orow + k] = (ci & 0x8000) || !rany ? 0.0 : pcred[ci & 0x7FFF] + sh[4 * c + e];
            }
        }
    }
    if (tid == 0 && K > kFwMaxK) {
        const uint16_t ci = cinfo[kFwMaxK];
        const bool dead = (ci & 0x8000) || !rany;
        if constexpr (kCounts) a.crow[orow + kFwMaxK] = dead ? 0u : pcnt[ci & 0x7FFF] + (unsigned)sh[kFwPer];
        else a.frow[orow + kFwMaxK] = dead ? 0.0 : pcred[ci & 0x7FFF] + sh[kFwPer];
    }
    if (tid == 0 && a.hint) {
        if (nc > 0) {
            atomicMax(&a.hint[0], swork * max(nc, 1));
            atomicAdd(&a.hint[2], 1);
            if (!handed) atomicAdd(&a.hint[3], 1);
        }
        if (ident) atomicAdd(&a.hint[1], 1);
    }
#ifdef MAC_DIAG
    if (tid == 0 && i < 65536)
        g_diag_fiw[16 * i + 7] = ((uint64_t)U << 32) | ((uint64_t)min(nc, 0xFFFF) << 16) |
                                (uint64_t)min((RG.y - RG.x + 1) * (RG.w - RG.z + 1), 0xFFFF);
#endif
    MAC_FW_STAMP(6);
    ts_end(ts);
}

// ------------------------------------------------------------------ finalize of the fused chain
// Block = C candidates x (1024 / C) row groups: thread (c, g) sums rows g, g + G, ... of candidate
// kb + c, all of its rows in flight at once (u32 counts: exact in any order; f64 credits: this
// fixed order), then the G group sums in group order. Then the shared entries the disks handed off
// (FwShared's list, sorted by disk), in batches of whole disks (at most kF2Slots disk records): per
// slot and candidate the disk from its key word (exact doubles), per (entry, candidate) the
// decision — disk i covers it, none of its listed lower neighbours does — with each disk's entries
// split over the row groups (its records held in registers) and added in that group's fixed order.
// obj_k = -area_k + vp_k; the argmin by the last-arriving block (k_final.h finalize_argmin), which
// also copies the fused kernel's hint words to the lane's mapped host memory (maxcover.hip
// enqueue_eval reads them before the next poll).
constexpr int kF2Threads = 1024;
constexpr int kF2C = 16;
constexpr int kF2G = kF2Threads / kF2C;
constexpr int kF2Slots = 64;      // disk records per batch (handed-off disks, their <= kFwHand neighbours)
constexpr int kF2Ent = 2048;      // shared entries staged at once
constexpr int kF2List = kF2ListCap;   // listed disks taken (a disk past it decided in place)
constexpr int kF2Pre = 64;        // list records loaded with the rows

struct F2Shared {
    CandSrc src;                  // keys (keysP / ldk) and candidate 0's column (the bases)
    const int* count;             // FwShared's list
    const int4* list;
    const double2* xy;
    const double* w;
    const uint8_t* dead;
};

template <bool kCounts>
__global__ __launch_bounds__(kF2Threads) void fin2_kernel(
    const unsigned* __restrict__ crow, const double* __restrict__ frow, int ldk, int N, int K,
    double w0, const double* __restrict__ vp, double* __restrict__ area_out, double* __restrict__ obj_out,
    FinBest fb, F2Shared sd, uint64_t* ts)
{
    ts_begin(ts);
    MAC_F2_STAMP(0);
    constexpr int C = kF2C, G = kF2G;
    const int t = threadIdx.x, c = t % C, gq = t / C;
    const int per = (int)(gridDim.x / 8);
    const int cb = per > 0 && gridDim.x % 8 == 0 ? (int)(blockIdx.x % 8) * per + (int)(blockIdx.x / 8)
                                                 : (int)blockIdx.x;
    const int k = cb * C + c;
    const int kc = min(k, K - 1);
    CandSrc src = sd.src;
    const bool run = src.resolve();   // (a stopped pipelined MADS loop: nothing to add)
    __shared__ double fred[G][C];
    __shared__ uint64_t ired[G][C];
    // one round trip: the list's count and first kF2Pre records, the candidate's penalty and
    // failure byte, and its rows (kF2R per thread in flight at once; more in later batches)
    constexpr int kF2R = 16;
    const int lc = min(*sd.count, min(kF2List, N));
    const int4 lr0 = t < kF2Pre ? sd.list[min(t, N - 1)] : make_int4(0, 0, 0, 0);
    const double vpk = (vp && gq == 0 && k < K) ? vp[k] : 0.0;
    const bool cdead = !(k < K) || !run || (sd.dead && sd.dead[kc]);
    uint64_t s = 0;
    double sf = 0.0;
    if (k < K) {
        for (int r = gq; r < N; r += kF2R * G) {
            if constexpr (kCounts) {
                unsigned v[kF2R];
#pragma unroll
                for (int b = 0; b < kF2R; ++b) {
                    const int rr = r + b * G;
                    v[b] = rr < N ? crow[(int64_t)rr * ldk + k] : 0u;
                }
#pragma unroll
                for (int b = 0; b < kF2R; ++b) s += v[b];
            } else {
                double v[kF2R];
#pragma unroll
                for (int b = 0; b < kF2R; ++b) {
                    const int rr = r + b * G;
                    v[b] = rr < N ? frow[(int64_t)rr * ldk + k] : 0.0;
                }
                double bs = 0.0;
#pragma unroll
                for (int b = 0; b < kF2R; ++b) bs += v[b];
                sf += bs;
            }
        }
    }
    MAC_F2_STAMP(1);
    // ---- the handed-off shared entries (lc: uniform)
    if (lc > 0 && run) {
        __shared__ int4 lraw[kF2List];
        __shared__ int flist[kF2List], fnc[kF2List], fsh[kF2List];
        __shared__ int fids[kF2List][kFwHand];
        __shared__ int bslot[kF2List + 1], bent[kF2List + 1];   // per listed disk: first slot, entry
        __shared__ double srec[kF2Slots][3][C];                  // per slot and candidate: x, y, T
        __shared__ double2 sxy[kF2Ent];
        __shared__ double swt[kF2Ent];
        __shared__ int nbat;
        for (int q = t; q < lc; q += kF2Threads) lraw[q] = q < kF2Pre ? lr0 : sd.list[q];
        __syncthreads();
        // sorted by disk: each record's rank among the listed disks (distinct ids)
        for (int q = t; q < lc; q += kF2Threads) {
            const int4 r = lraw[q];
            int rk = 0;
            for (int o = 0; o < lc; ++o) rk += lraw[o].x < r.x;
            flist[rk] = r.x;
            fnc[rk] = r.y & 0xFF;
            fsh[rk] = r.y >> 8;
            fids[rk][0] = r.z & 0xFFFF;
            fids[rk][1] = (int)((unsigned)r.z >> 16);
            fids[rk][2] = r.w & 0xFFFF;
            fids[rk][3] = (int)((unsigned)r.w >> 16);
        }
        __syncthreads();
        if (t == 0) {   // slots and entries per listed disk
            int sl = 0, en = 0;
            for (int q = 0; q < lc; ++q) {
                bslot[q] = sl;
                bent[q] = en;
                sl += 1 + fnc[q];
                en += fsh[q];
            }
            bslot[lc] = sl;
            bent[lc] = en;
        }
        __syncthreads();
        MAC_F2_STAMP(2);
        for (int q0 = 0; q0 < lc;) {
            // the batch: listed disks [q0, q1) whose records fit kF2Slots (one disk always fits)
            if (t == 0) {
                int q1 = q0 + 1;
                while (q1 < lc && bslot[q1 + 1] - bslot[q0] <= kF2Slots) ++q1;
                nbat = q1;
            }
            __syncthreads();
            const int q1 = nbat;
            const int sl0 = bslot[q0], ns = bslot[q1] - sl0;
            const int e0all = bent[q0], e1all = bent[q1];
            // the first chunk's entries, loaded before the records' keys (one round trip for both)
            constexpr int kEPT = kF2Ent / kF2Threads;
            double2 exy[kEPT];
            double ew[kEPT];
            {
                const int ne = min(kF2Ent, e1all - e0all);
#pragma unroll
                for (int r = 0; r < kEPT; ++r) {
                    const int e = t + r * kF2Threads;
                    exy[r] = make_double2(0.0, 0.0);
                    ew[r] = 0.0;
                    if (e < ne) {
                        const int eg = e0all + e;   // the listed disk holding it
                        int lo = q0, hi = q1 - 1;
                        while (lo < hi) {
                            const int mid = (lo + hi + 1) >> 1;
                            if (bent[mid] <= eg) lo = mid; else hi = mid - 1;
                        }
                        const int64_t se = (int64_t)flist[lo] * kFwShCap + (eg - bent[lo]);
                        exy[r] = sd.xy[se];
                        if constexpr (!kCounts) ew[r] = sd.w[se];
                    }
                }
            }
            // per slot and candidate: the disk (its key word, candidate 0's disk)
            for (int q = t; q < ns * C; q += kF2Threads) {
                const int sl = q / C, cc = q % C;
                int lo = q0, hi = q1 - 1;   // the listed disk holding slot sl0 + sl
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (bslot[mid] - sl0 <= sl) lo = mid; else hi = mid - 1;
                }
                const int m = sl - (bslot[lo] - sl0);
                const int jj = m == 0 ? flist[lo] : fids[lo][m - 1];
                const int kk = min(cb * C + cc, K - 1);
                const uint32_t key = src.keysP[(int64_t)jj * src.ldk + kk];
                const DiskRec d = key_disk(src, key, jj, kk, N, src_val(src, 0, jj, N),
                                           src_val(src, 0, N + jj, N), src_val(src, 0, 2 * N + jj, N));
                srec[sl][0][cc] = d.cx;
                srec[sl][1][cc] = d.cy;
                srec[sl][2][cc] = d.T;
            }
            for (int e0 = e0all; e0 < e1all; e0 += kF2Ent) {
                const int ne = min(kF2Ent, e1all - e0);
                if (e0 == e0all) {
#pragma unroll
                    for (int r = 0; r < kEPT; ++r) {
                        const int e = t + r * kF2Threads;
                        if (e < ne) {
                            sxy[e] = exy[r];
                            swt[e] = ew[r];
                        }
                    }
                } else {
                    for (int e = t; e < ne; e += kF2Threads) {
                        const int eg = e0 + e;
                        int lo = q0, hi = q1 - 1;
                        while (lo < hi) {
                            const int mid = (lo + hi + 1) >> 1;
                            if (bent[mid] <= eg) lo = mid; else hi = mid - 1;
                        }
                        const int64_t se = (int64_t)flist[lo] * kFwShCap + (eg - bent[lo]);
                        sxy[e] = sd.xy[se];
                        swt[e] = kCounts ? 0.0 : sd.w[se];
                    }
                }
                __syncthreads();
                MAC_F2_STAMP(3);
                // per listed disk: its records and its neighbours' in registers, then its entries
                // of this chunk, split over the row groups (group gq: entries gq, gq + G, ...)
                if (!cdead) {
                    for (int lq = q0; lq < q1; ++lq) {
                        const int ea = max(bent[lq], e0) - e0, eb = min(bent[lq + 1], e0 + ne) - e0;
                        if (ea >= eb) continue;
                        const int b = bslot[lq] - sl0, ncq = fnc[lq];
                        const double cx = srec[b][0][c], cy = srec[b][1][c], T = srec[b][2][c];
                        double nx[kFwHand], ny[kFwHand], nT[kFwHand];
#pragma unroll
                        for (int m = 0; m < kFwHand; ++m) {
                            const bool in = m < ncq;
                            nx[m] = in ? srec[b + 1 + m][0][c] : 0.0;
                            ny[m] = in ? srec[b + 1 + m][1][c] : 0.0;
                            nT[m] = in ? srec[b + 1 + m][2][c] : -1.0;   // (never covers)
                        }
                        // four entries per step, their LDS reads issued together
                        constexpr int kU = 4;
                        for (int e = ea + gq; e < eb; e += kU * G) {
                            double2 pp[kU];
#pragma unroll
                            for (int u = 0; u < kU; ++u)
                                pp[u] = e + u * G < eb ? sxy[e + u * G] : make_double2(0.0, 0.0);
#pragma unroll
                            for (int u = 0; u < kU; ++u) {
                                if (!(e + u * G < eb)) break;
                                const double2 p = pp[u];
                                if (!(sqdist(p.x, p.y, cx, cy) <= T)) continue;
                                bool stolen = false;
#pragma unroll
                                for (int m = 0; m < kFwHand; ++m)   // (ncq: uniform; usually 1)
                                    if (m < ncq && !stolen) stolen = sqdist(p.x, p.y, nx[m], ny[m]) <= nT[m];
                                if (!stolen) {
                                    if constexpr (kCounts) s += 1;
                                    else sf += swt[e + u * G];
                                }
                            }
                        }
                    }
                }
                __syncthreads();
            }
            q0 = q1;
        }
    }
    MAC_F2_STAMP(4);
    double o = __builtin_inf();
    if constexpr (kCounts) {
        ired[gq][c] = s;
        __syncthreads();
        if (gq == 0 && k < K) {
            uint64_t n = 0;
#pragma unroll
            for (int q = 0; q < G; ++q) n += ired[q][c];
            const double area = (double)n * w0;
            if (area_out) area_out[k] = area;
            if (vp) o = -area + vpk;
            if (obj_out) obj_out[k] = o;
        }
    } else {
        fred[gq][c] = sf;
        __syncthreads();
        if (gq == 0 && k < K) {
            double area = 0.0;
#pragma unroll
            for (int q = 0; q < G; ++q) area += fred[q][c];
            if (area_out) area_out[k] = area;
            if (vp) o = -area + vpk;
            if (obj_out) obj_out[k] = o;
        }
    }
    MAC_F2_STAMP(5);
    if (fb.best && t < kWave) {
        [[maybe_unused]] const bool last = finalize_argmin<C>(fb, o, k, k < K);   // (+ the hint words)
#ifdef MAC_DIAG
        if (t == 0 && blockIdx.x < 4096) g_diag_f2[8 * blockIdx.x + 7] = last;
#endif
    }
    MAC_F2_STAMP(6);
    ts_end(ts);
}

}  // namespace mac
