// k_fused.h — one MADS poll over an equal-weight point list in TWO launches (every reference
// input: w = dx*dy on every entry, src/CellFunctions.jl:53, src/AreaCoverageCalculation.jl:16).
//
// Reference: the poll of src/TDM_STATIC_opt.jl:162 — every trial point x evaluated by
// AreaMaxObjective (:82-100) = -calculateArea(x, points) (src/AreaCoverageCalculation.jl:63-78)
// + 1e5 * sum_i |x[2N+i] - r_max[i]|, behind the extreme barrier cons3
// (src/TDM_Constraints.jl:54-75), then the best trial point kept.
//
// launch 1, fused_prep_kernel (grid: penalty chains, then key tiles)
//   * chain workgroups (16 candidates): the sequential penalty sum and the cons3 mark of every
//     candidate, straight from the candidate source -> vp[k] (k_final.h's relay, terms computed
//     in place: nothing per (disk, candidate) is materialised);
//   * key tiles (32 disks x 64 candidates, coalesced 256-B rows of the column-major matrix): per
//     (disk i, candidate k) the exact int16 offsets of (x, y, r) from candidate 0's disk i
//     (keys, 6 B), an "inexact" flag per (disk, tile), the disk's tile span -> per-disk region by
//     generation-tagged 64-bit atomic min / max (no clearing pass), span areas; tiles of disk
//     tile 0 zero the count row cnt[k];
//   * the workgroup that arrives last (self-resetting atomicInc counter) reads the regions and
//     builds every disk's lower-index neighbour list (all pairs, regions tiled through LDS) and
//     the list of disks with neighbours.
// launch 2, fused_walk_kernel (grid: N walk workgroups, then shared-entry workgroups)
//   * walk workgroup = disk i: its candidates' keys hashed in LDS (64-bit packed keys, one CAS
//     per probe) -> the distinct disks ("positions", ~300 of 3073 in a config-4 poll); the
//     region's entries staged once as fp32 (k_poll.h's exact filter); every wave tests every
//     position against a quarter of the entries; the position counts are added to each
//     candidate's count by one integer atomic per candidate (exact in any order);
//   * shared-entry jobs (disk with lower-index neighbours x candidate slice; the shared
//     workgroups, then every walk workgroup once its disk is done): exact fp64 ownership of the
//     entries a lower-index disk can also cover, disks read from the source, integer atomics;
//   * the workgroup that arrives last: area_k = count_k * w, obj_k = -area_k + vp_k, the
//     lexicographic argmin, the 16-byte result mirrored to pinned host memory.
// No per-(disk, candidate) intermediate other than the 6-B keys goes through HBM, no launch
// between the index and the walk, no finalize / argmin launch.
//
// Cross-workgroup hand-offs inside a launch (MI355X_MICROARCH.md "Workgroup dispatch ... and
// inter-workgroup visibility"): producers publish only through device-scope atomics (region
// words, counts) or sc1 stores (span areas, regions), every storing wave drains its vmcnt
// before its workgroup's one arrival atomic, and the last arriver reads through atomics / sc1
// loads. Everything else crosses the launch boundary.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "predicate.h"
#include "k_common.h"
#include "k_prep.h"
#include "k_index.h"
#include "k_lane.h"
#include "k_poll_shared.h"
#include "k_poll.h"
#include "k_final.h"

#pragma clang fp contract(off)

namespace mac {

constexpr int kFD = 32;            // key tile: disks
constexpr int kFC = 64;            // key tile: candidates
constexpr int kFSlots = 4096;      // walk: LDS hash table (uint64 packed keys)
constexpr int kFMaxU = 3072;       // walk: distinct disks hashed at most (load <= 3/4)
constexpr int kFMaxK = 8192;       // walk: candidates whose table slot is kept in LDS (uint16)
constexpr int kFRegTile = 1024;    // prep (last workgroup): regions per LDS tile
constexpr int kFChainCands = 64;   // chain: candidates per workgroup (4 threads each)
constexpr int kFChainU = 4;        // chain: rounds of 16 disks per batch of loads
constexpr int kFChainThr = 256;    // chain: cons3 thresholds per LDS chunk

enum { kCtlDone1 = 0, kCtlDone2 = 1, kCtlDcount = 2, kCtlJobs = 3, kCtlWords = 8 };

struct FusedArgs {
    CandSrc src;
    int N, K, Kp;                  // Kp: key row pitch (multiple of kFC)
    int ndt, nct;                  // key tiles: ceil(N / kFD) x ceil(K / kFC)
    int n_chain, n_shared;
    Grid g;
    // objective: rmax == null -> areas only (no chains)
    const double* rmax;
    const double* prev;            // cons3 around prev (null: no cons3), raw d_lim per UAV
    const double* dlim;
    double tan_half_fov, penalty, w0;
    // lane scratch
    int16_t* keys;                 // [3][N][Kp]
    uint8_t* kbad;                 // [N][nct]
    int4* part;                    // [ndt][nct][kFD] partial regions (sc1)
    unsigned* dtctr;               // [ndt] per disk tile arrival counters (self-resetting)
    double* vp;                    // [K]
    unsigned* cnt;                 // [K]
    int4* region;                  // [N] (sc1)
    uint16_t* nbr;                 // [N][kPollNbr]
    int4* nboxT;                   // [N][kPollNbr]
    int* ncount;                   // [N]
    int* dlist;                    // [N]
    int* ctl;                      // [kCtlWords]
    // point list (tile order)
    const double2* xy;
    const int32_t* off;
    // outputs
    double* area_out;
    double* obj_out;
    double* best;
    double* mirror;
    uint64_t seq;
    int64_t idx_base;
};

__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// int4 through two 8-B agent-scope (sc1) accesses: the cross-workgroup hand-offs of launch 1
__device__ __forceinline__ void st_sc1(int4* p, const int4& v)
{
    unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
    __hip_atomic_store(q, (unsigned long long)(uint32_t)v.x | ((unsigned long long)(uint32_t)v.y << 32),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(q + 1, (unsigned long long)(uint32_t)v.z | ((unsigned long long)(uint32_t)v.w << 32),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int4 ld_sc1(const int4* p)
{
    const unsigned long long* q = reinterpret_cast<const unsigned long long*>(p);
    const unsigned long long a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return make_int4((int)(uint32_t)a, (int)(uint32_t)(a >> 32), (int)(uint32_t)b, (int)(uint32_t)(b >> 32));
}

__device__ __forceinline__ int4 empty_box() { return make_int4(0x7fffffff, -1, 0x7fffffff, -1); }
__device__ __forceinline__ void box_join(int4& R, const int4& P)
{
    R.x = min(R.x, P.x);
    R.y = max(R.y, P.y);
    R.z = min(R.z, P.z);
    R.w = max(R.w, P.w);
}

// exact int16 offset of v from b: b + (double)key reproduces v bit for bit, else ok = false
__device__ __forceinline__ int key16(double v, double b, bool& ok)
{
    const double d = v - b;
    const bool in = d >= -32767.0 && d <= 32767.0;    // NaN: false
    const int q = in ? (int)d : 0;
    ok &= in && (double)q == d &&
          __builtin_bit_cast(uint64_t, b + (double)q) == __builtin_bit_cast(uint64_t, v);
    return q;
}

__device__ __forceinline__ unsigned long long pack_key(int kx, int ky, int kr)
{
    return (unsigned long long)(uint16_t)kx | ((unsigned long long)(uint16_t)ky << 16) |
           ((unsigned long long)(uint16_t)kr << 32) | (1ull << 48);
}

__device__ __forceinline__ uint32_t hash_key(unsigned long long key)
{
    uint64_t z = key * 0x9E3779B97F4A7C15ull;
    z ^= z >> 29;
    z *= 0xBF58476D1CE4E5B9ull;
    return (uint32_t)(z >> 32);
}

// ================================================================== launch 1

// Penalty chains of candidates [k0, k0 + 64): violation_k = sum_{i=0..N-1} |R_i - r_max_i|
// accumulated IN ORDER from 0.0 (src/TDM_STATIC_opt.jl:89-93), +inf when cons3 rejects a UAV's
// move (pen_term, k_prep.h). Thread t: candidate k0 + t/4, quarter t%4. A round covers 16
// disks: the quarter loads disks [4q, 4q + 4) of the round from its candidate's contiguous
// column (one 128-B line per candidate and section, shared by its four lanes), and the running
// sum is relayed through the four lanes in quarter order by shuffles: the additions stay in
// disk order without a barrier. kFChainU rounds of loads are in flight at once.
__device__ __forceinline__ void fused_chain_block(const FusedArgs& a, int k0, unsigned char* lds)
{
    double* thr = (double*)lds;   // [kFChainThr] cons3 thresholds of the chunk
    const int t = threadIdx.x, lane = t & (kWave - 1), c = t >> 2, qq = t & 3;
    const int k = k0 + c, N = a.N;
    const bool kv = k < a.K;
    double carry = 0.0;
    bool bad = false;
    for (int c0 = 0; c0 < N; c0 += kFChainThr) {
        const int c1 = min(N, c0 + kFChainThr);
        __syncthreads();
        if (a.prev)
            for (int q = t; q < kFChainThr; q += kBlock) thr[q] = c0 + q < N ? dlim_threshold(a.dlim[c0 + q]) : 0.0;
        __syncthreads();
        for (int base = c0; base < c1; base += 16 * kFChainU) {
            double R[kFChainU][4], X[kFChainU][4], Y[kFChainU][4];
#pragma unroll
            for (int u = 0; u < kFChainU; ++u)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int ii = base + 16 * u + 4 * qq + e;
                    const bool v = kv && ii < c1;
                    R[u][e] = v ? a.src.get(k, 2 * N + ii, N) : 0.0;
                    X[u][e] = (v && a.prev) ? a.src.get(k, ii, N) : 0.0;
                    Y[u][e] = (v && a.prev) ? a.src.get(k, N + ii, N) : 0.0;
                }
#pragma unroll
            for (int u = 0; u < kFChainU; ++u) {
                double term[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int ii = base + 16 * u + 4 * qq + e;
                    term[e] = 0.0;   // pad: + 0.0, exact
                    if (kv && ii < c1) {
                        term[e] = __builtin_fabs(R[u][e] - a.rmax[ii]);
                        if (a.prev) {
                            const double x1 = a.prev[ii], y1 = a.prev[N + ii];
                            const double z1 = a.prev[2 * N + ii] / a.tan_half_fov;
                            const double z2 = R[u][e] / a.tan_half_fov;
                            const double ddx = x1 - X[u][e], ddy = y1 - Y[u][e], ddz = z1 - z2;
                            if (ddx * ddx + ddy * ddy + ddz * ddz > thr[ii - c0]) bad = true;
                        }
                    }
                }
#pragma unroll
                for (int step = 0; step < 4; ++step) {
                    if (qq == step) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) carry += term[e];
                    }
                    carry = __shfl(carry, (lane & ~3) | step, kWave);
                }
            }
        }
    }
    // a cons3 failure anywhere in the candidate's four quarters bars it
    const bool anybad = __shfl_xor((int)bad, 1, kWave) | __shfl_xor((int)bad, 2, kWave) |
                        __shfl_xor((int)bad, 3, kWave) | (int)bad;
    if (qq == 0 && kv) a.vp[k] = anybad ? __builtin_inf() : carry * a.penalty;
}

// Key tile (disk tile dt, candidate tile ct): keys, exactness flags, the tile's partial regions.
// Returns true on the workgroup that arrives last among its disk tile's nct tiles.
__device__ __forceinline__ bool fused_key_tile(const FusedArgs& a, int tile, unsigned char* lds)
{
    typedef int16_t KRow[kFC + 4];
    KRow* ks = (KRow*)lds;                                             // [3 * kFD] rows
    int4* rr = (int4*)(lds + 3 * kFD * sizeof(KRow));                  // [8][kFD]
    int* okv = (int*)(rr + 8 * kFD);                                   // [8][kFD]
    int* flag = okv + 8 * kFD;
    const int dt = tile % a.ndt, ct = tile / a.ndt;
    const int t = threadIdx.x, l = t & (kFD - 1), q = t / kFD;         // 32 disks x 8
    const int N = a.N, K = a.K;
    const int i = dt * kFD + l;
    const bool di = i < N;
    double bx = 0.0, by = 0.0, br = 0.0;
    double x[8], y[8], r[8];
    if (di) {
        bx = a.src.get(0, i, N);
        by = a.src.get(0, N + i, N);
        br = a.src.get(0, 2 * N + i, N);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {   // every load in flight at once
        const int k = ct * kFC + q + 8 * j;
        const bool v = di && k < K;
        x[j] = v ? a.src.get(k, i, N) : bx;
        y[j] = v ? a.src.get(k, N + i, N) : by;
        r[j] = v ? a.src.get(k, 2 * N + i, N) : br;
    }
    bool ok = true;
    int4 R = empty_box();
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int kk = q + 8 * j, k = ct * kFC + kk;
        int kx = 0, ky = 0, kr = 0;
        if (di && k < K) {
            kx = key16(x[j], bx, ok);
            ky = key16(y[j], by, ok);
            kr = key16(r[j], br, ok);
            int4 sp;
            if (span_of(x[j], y[j], r[j], a.g, sp)) box_join(R, sp);
        }
        ks[l][kk] = (int16_t)kx;
        ks[kFD + l][kk] = (int16_t)ky;
        ks[2 * kFD + l][kk] = (int16_t)kr;
    }
    rr[q * kFD + l] = R;
    okv[q * kFD + l] = ok ? 1 : 0;
    __syncthreads();
    if (t < kFD) {
        int4 Q = empty_box();
        int okall = 1;
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            box_join(Q, rr[g * kFD + t]);
            okall &= okv[g * kFD + t];
        }
        if (di) a.kbad[(int64_t)i * a.nct + ct] = okall ? 0 : 1;
        st_sc1(&a.part[((int64_t)dt * a.nct + ct) * kFD + t], Q);
    }
    // key rows: 3 x 32 rows of 64 int16 (128 B each), 8-B stores (Kp is a multiple of kFC)
#pragma unroll
    for (int r0 = 0; r0 < 3 * kFD; r0 += kBlock / 16) {
        const int row = r0 + t / 16, c4 = (t % 16) * 4;
        const int aa = row / kFD, ii = dt * kFD + (row % kFD);
        if (ii < N) {
            const int16_t* src = &ks[row][c4];
            uint2 v;
            v.x = (uint32_t)(uint16_t)src[0] | ((uint32_t)(uint16_t)src[1] << 16);
            v.y = (uint32_t)(uint16_t)src[2] | ((uint32_t)(uint16_t)src[3] << 16);
            *(uint2*)&a.keys[((int64_t)aa * N + ii) * a.Kp + ct * kFC + c4] = v;
        }
    }
    if (dt == 0 && t < kFC && ct * kFC + t < K) a.cnt[ct * kFC + t] = 0u;
    if (tile == 0 && t == 0) a.ctl[kCtlJobs] = 0;
    vm_drain();          // this wave's stores are complete ...
    __syncthreads();     // ... and every other wave's
    if (t == 0) *flag = atomicInc(&a.dtctr[dt], a.nct - 1) == (unsigned)(a.nct - 1);
    __syncthreads();
    return *flag != 0;
}

// The last tile of disk tile dt: the regions of its 32 disks from the nct partials.
__device__ __forceinline__ void fused_dt_regions(const FusedArgs& a, int dt, unsigned char* lds)
{
    int4* rr = (int4*)lds;   // [8][kFD]
    const int t = threadIdx.x, l = t & (kFD - 1), g = t / kFD;
    int4 R = empty_box();
    for (int c = g; c < a.nct; c += 8) box_join(R, ld_sc1(&a.part[((int64_t)dt * a.nct + c) * kFD + l]));
    rr[g * kFD + l] = R;
    __syncthreads();
    const int i = dt * kFD + t;
    if (t < kFD && i < a.N) {
        int4 Q = empty_box();
#pragma unroll
        for (int q = 0; q < 8; ++q) box_join(Q, rr[q * kFD + t]);
        if (Q.x > Q.y || Q.z > Q.w) Q = empty_box();
        st_sc1(&a.region[i], Q);
    }
    vm_drain();
    __syncthreads();
}

// The last disk tile's last tile: every disk's lower-index neighbour list (all pairs, the
// regions through LDS in tiles of kFRegTile) and the list of disks with neighbours.
__device__ __forceinline__ void fused_prep_last(const FusedArgs& a, unsigned char* lds)
{
    int4* sreg = (int4*)lds;                         // [kFRegTile]
    int* sd = (int*)(sreg + kFRegTile);
    const int t = threadIdx.x, N = a.N;
    if (t == 0) *sd = 0;
    // snake order over rounds of 256 disks: every thread walks about the same number of pairs
    for (int m = 0; m * kBlock < N; ++m) {
        const int i = m * kBlock + ((m & 1) ? kBlock - 1 - t : t);
        const int4 Ri = i < N ? ld_sc1(&a.region[i]) : empty_box();
        int cnt = 0;
        const int jend = min(N, (m + 1) * kBlock);
        for (int jb = 0; jb < jend; jb += kFRegTile) {
            __syncthreads();
            constexpr int PT = kFRegTile / kBlock;
            int4 v[PT];
#pragma unroll
            for (int q = 0; q < PT; ++q) {   // every load in flight at once
                const int j = jb + t + q * kBlock;
                v[q] = j < jend ? ld_sc1(&a.region[j]) : empty_box();
            }
#pragma unroll
            for (int q = 0; q < PT; ++q) sreg[t + q * kBlock] = v[q];
            __syncthreads();
            if (i < N && Ri.x <= Ri.y) {
                const int je = min(i, jb + kFRegTile);
                for (int j = jb; j < je; ++j) {
                    const int4 Q = sreg[j - jb];
                    if (box_overlap(Q, Ri)) {
                        if (cnt < kPollNbr) {
                            a.nbr[i * kPollNbr + cnt] = (uint16_t)j;
                            a.nboxT[i * kPollNbr + cnt] = Q;
                        }
                        ++cnt;
                    }
                }
            }
        }
        if (i < N) {
            a.ncount[i] = cnt;
            if (cnt > 0) a.dlist[atomicAdd(sd, 1)] = i;
        }
    }
    __syncthreads();
    if (t == 0) a.ctl[kCtlDcount] = *sd;
}

constexpr int kPrepLds = 3 * kFD * (kFC + 4) * 2 + 8 * kFD * 16 + 8 * kFD * 4 + 64;
static_assert(kPrepLds >= kFRegTile * 16 + 16, "the last workgroup's region tile fits");
static_assert(kPrepLds >= kFChainThr * 8, "the chain's thresholds fit");

// Grid: n_chain chain workgroups, then ndt * nct key tiles.
__global__ __launch_bounds__(kBlock) void fused_prep_kernel(uint64_t* ts, FusedArgs a)
{
    ts_begin(ts);
    __shared__ __attribute__((aligned(16))) unsigned char lds[kPrepLds];
    __shared__ int last;
    const int b = blockIdx.x;
    if (b < a.n_chain) {
        fused_chain_block(a, b * kFChainCands, lds);
    } else {
        const int tile = b - a.n_chain;
        if (fused_key_tile(a, tile, lds)) {   // the last of its disk tile
            fused_dt_regions(a, tile % a.ndt, lds);
            if (threadIdx.x == 0)
                last = atomicInc((unsigned*)&a.ctl[kCtlDone1], a.ndt - 1) == (unsigned)(a.ndt - 1);
            __syncthreads();
            if (last) fused_prep_last(a, lds);
        }
    }
    ts_end(ts);
}

// ================================================================== launch 2

// disk i of candidate k from the source
__device__ __forceinline__ DiskRec src_disk(const CandSrc& s, int N, int i, int k)
{
    return make_disk(s.get(k, i, N), s.get(k, N + i, N), s.get(k, 2 * N + i, N));
}

// Shared-entry job (k_poll_shared.h poll_shared_job) with the disks read from the source and
// integer counts added to cnt[k].
__device__ __forceinline__ void fused_shared_job(const FusedArgs& a, int i, int kb, int C,
                                                 unsigned char* lds)
{
    double2* sp = (double2*)lds;                             // [kPollThreads]
    int* rs = (int*)(sp + kPollThreads);                     // [kPollRB]
    int* rpre = rs + kPollRB;                                // [kPollRB + 1]
    int4* nbox = (int4*)(rpre + kPollRB + 4);                // [kPollNbr]
    uint16_t* nbr = (uint16_t*)(nbox + kPollNbr);            // [kPollNbr]
    int* wcount = (int*)(nbr + kPollNbr);                    // [kPollWaves]
    unsigned* gsum = (unsigned*)(wcount + kPollWaves);       // [kPollThreads]
    int* run_s = (int*)(gsum + kPollThreads);                // [kPollThreads]
    int* run_pre = run_s + kPollThreads;                     // [kPollThreads + 1]
    int* nruns = run_pre + kPollThreads + 1;

    const int N = a.N, K = a.K;
    const Grid& g = a.g;
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
    const int G = kPollThreads / C;
    const int c = tid % C, eg = tid / C;
    const int k = kb + c;
    const bool valid = k < K;
    const int nc = a.ncount[i];
    const int ncl = min(nc, kPollNbr);
    const int4 R = a.region[i];
    const int nrows = R.w - R.z + 1;
    __syncthreads();  // LDS reuse across jobs
    if (tid < ncl) {
        nbr[tid] = a.nbr[i * kPollNbr + tid];
        nbox[tid] = a.nboxT[i * kPollNbr + tid];
    }
    DiskRec d = DiskRec{0.0, 0.0, -1.0, 0.0};
    DiskRec e[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) e[m] = DiskRec{0.0, 0.0, -1.0, 0.0};
    if (valid) {
        d = src_disk(a.src, N, i, k);
#pragma unroll
        for (int m = 0; m < 4; ++m)
            if (m < ncl) e[m] = src_disk(a.src, N, a.nbr[i * kPollNbr + m], k);
    }
    unsigned acc = 0;
    __syncthreads();

    // the exact decision of this round's staged entries sp[0, ns) for this thread's candidate:
    // its entries s = eg + G*j (j < 256 / G) as a 256-bit mask of those disk i covers, then each
    // lower-index neighbour strips the entries it covers — a neighbour disk is read once per
    // round, not once per entry
    auto decide = [&](int ns) {
        if (!(valid && d.T >= 0.0) || ns <= eg) return;
        const int nj = (ns - eg + G - 1) / G;
        uint64_t m0 = 0, m1 = 0, m2 = 0, m3 = 0;
        for (int j = 0; j < nj; ++j) {
            const double2 q = sp[eg + G * j];
            if (sqdist(q.x, q.y, d.cx, d.cy) <= d.T) {
                const uint64_t bit = 1ull << (j & 63);
                const int w = j >> 6;
                m0 |= w == 0 ? bit : 0ull;
                m1 |= w == 1 ? bit : 0ull;
                m2 |= w == 2 ? bit : 0ull;
                m3 |= w == 3 ? bit : 0ull;
            }
        }
        auto strip_word = [&](uint64_t& mw, int w, const DiskRec& x) {
            uint64_t m = mw;
            while (m) {
                const int b = __builtin_ctzll(m);
                m &= m - 1;
                const double2 q = sp[eg + G * (64 * w + b)];
                if (sqdist(q.x, q.y, x.cx, x.cy) <= x.T) mw &= ~(1ull << b);
            }
        };
        auto strip = [&](const DiskRec& x) {
            strip_word(m0, 0, x);
            strip_word(m1, 1, x);
            strip_word(m2, 2, x);
            strip_word(m3, 3, x);
        };
#pragma unroll
        for (int m = 0; m < 4; ++m)
            if (m < ncl && (m0 | m1 | m2 | m3)) strip(e[m]);
        if (nc > 4 && (m0 | m1 | m2 | m3)) {
            if (nc <= kPollNbr) {
                for (int m = 4; m < nc && (m0 | m1 | m2 | m3); ++m) strip(src_disk(a.src, N, nbr[m], k));
            } else {  // overflowed list: every lower-index overlapping region
                for (int j = 0; j < i && (m0 | m1 | m2 | m3); ++j)
                    if (box_overlap(a.region[j], R)) strip(src_disk(a.src, N, j, k));
            }
        }
        acc += (unsigned)(__popcll(m0) + __popcll(m1) + __popcll(m2) + __popcll(m3));
    };

    // shared tiles of each row: runs of a 64-bit tile mask (the union of the neighbour boxes);
    // regions wider or higher than 64 tiles take the row-by-row path below
    const int tw = R.y - R.x + 1;
    bool fast = tw <= kWave && nrows <= kWave;
    if (fast) {
        if (tid < kWave) {
            uint64_t mask = 0;
            const int r = R.z + tid;
            if (tid < nrows) {
                const uint64_t all = tw == 64 ? ~0ull : ((1ull << tw) - 1);
                if (nc > kPollNbr) {
                    mask = all;
                } else {
                    for (int m = 0; m < ncl; ++m) {
                        const int4 Q = nbox[m];
                        if (r < Q.z || r > Q.w) continue;
                        const int lo = max(R.x, Q.x) - R.x, hi = min(R.y, Q.y) - R.x;
                        if (lo <= hi) mask |= (hi - lo == 63 ? ~0ull : ((1ull << (hi - lo + 1)) - 1)) << lo;
                    }
                }
            }
            const uint64_t starts = mask & ~(mask << 1);
            const int cnt = __popcll(starts);
            const int incl = wave_incl_scan_i32(cnt, tid);
            const int tot = __shfl(incl, kWave - 1, kWave);
            if (tid == 0) *nruns = tot;
            if (tot <= kPollThreads) {
                int qq = incl - cnt;
                uint64_t m2 = mask;
                const int64_t rowbase = (int64_t)r * g.nTx + R.x;
                while (m2) {
                    const int lo = __builtin_ctzll(m2);
                    const uint64_t from = m2 >> lo;
                    const int len = ~from ? __builtin_ctzll(~from) : 64 - lo;
                    const int s0 = a.off[rowbase + lo];
                    run_s[qq] = s0;
                    run_pre[qq + 1] = a.off[rowbase + lo + len] - s0;
                    ++qq;
                    m2 &= len + lo >= 64 ? 0ull : (~0ull << (lo + len));
                }
            }
        }
        __syncthreads();
        const int nrun = *nruns;
        fast = nrun <= kPollThreads;
        if (fast) {
            const int len = tid < nrun ? run_pre[tid + 1] : 0;
            const int incl = wave_incl_scan_i32(len, lane);
            if (lane == kWave - 1) wcount[wid] = incl;
            __syncthreads();
            int pre = incl - len, total = 0;
            for (int qq = 0; qq < kPollWaves; ++qq) {
                if (qq < wid) pre += wcount[qq];
                total += wcount[qq];
            }
            __syncthreads();
            if (tid < nrun) run_pre[tid] = pre;
            if (tid == 0) run_pre[nrun] = total;
            __syncthreads();
            for (int base = 0; base < total; base += kPollThreads) {
                const int n = min(kPollThreads, total - base);
                if (tid < n) {
                    const int f = base + tid;
                    int lo = 0, hi = nrun - 1;
                    while (lo < hi) {
                        const int mid = (lo + hi + 1) >> 1;
                        if (run_pre[mid] <= f) lo = mid; else hi = mid - 1;
                    }
                    sp[tid] = a.xy[run_s[lo] + (f - run_pre[lo])];
                }
                __syncthreads();
                decide(n);
                __syncthreads();
            }
        }
    }
    for (int rb = R.z; !fast && rb <= R.w; rb += kPollRB) {
        const int nr = min(kPollRB, R.w - rb + 1);
        if (tid < nr) {
            const int64_t rowbase = (int64_t)(rb + tid) * g.nTx;
            const int s0 = a.off[rowbase + R.x];
            rs[tid] = s0;
            rpre[tid + 1] = a.off[rowbase + R.y + 1] - s0;
        }
        __syncthreads();
        if (tid < kWave) {
            const int v = wave_incl_scan_i32(tid < nr ? rpre[tid + 1] : 0, tid);
            if (tid < nr) rpre[tid + 1] = v;
            if (tid == 0) rpre[0] = 0;
        }
        __syncthreads();
        const int total = rpre[nr];
        for (int base = 0; base < total; base += kPollThreads) {
            const int f = base + tid;
            bool shared = false;
            double2 p = make_double2(0.0, 0.0);
            if (f < total) {
                int lo = 0, hi = nr - 1;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (rpre[mid] <= f) lo = mid; else hi = mid - 1;
                }
                p = a.xy[rs[lo] + (f - rpre[lo])];
                shared = entry_shared(nc, nbox, tile_of(p.x, g.gx0, g.invS, g.nTx), rb + lo);
            }
            const uint64_t bal = __ballot(shared);
            if (lane == 0) wcount[wid] = __popcll(bal);
            __syncthreads();
            int pos = __popcll(bal & ((1ull << lane) - 1)), ns = 0;
            for (int qq = 0; qq < kPollWaves; ++qq) {
                if (qq < wid) pos += wcount[qq];
                ns += wcount[qq];
            }
            if (shared) sp[pos] = p;
            __syncthreads();
            decide(ns);
            __syncthreads();
        }
    }
    gsum[eg * C + c] = acc;
    __syncthreads();
    if (eg == 0 && valid) {
        unsigned s = 0;
        for (int qq = 0; qq < G; ++qq) s += gsum[qq * C + c];
        if (s) atomicAdd(&a.cnt[k], s);
    }
}

// Walk of disk i (poll walk, k_poll.h, with the disk index built in LDS).
constexpr int kFStage = (kPollCH + 4) * 16 + kPollCH * 16;                 // s32 + s64
constexpr int kFWalkLds = kFSlots * 8 + kFMaxK * 2 + kFMaxU * 2 + kFStage +
                          (kPollRB + kPollRB + 4) * 4 + kPollNbr * 16 + 64;
static_assert(kPollWaves * kPollKPB * 4 + kPollKPB * 4 <= kFStage, "counts alias the staging");

#ifdef MAC_DIAG
#define MAC_FW_STAMP(q) if (threadIdx.x == 0 && i < 65536) g_diag_walk[8 * i + (q)] = __builtin_amdgcn_s_memrealtime()
#else
#define MAC_FW_STAMP(q)
#endif

__device__ __forceinline__ void fused_walk_disk(const FusedArgs& a, int i, unsigned char* lds)
{
    MAC_FW_STAMP(0);
    unsigned long long* table = (unsigned long long*)lds;                 // [kFSlots]
    uint16_t* cslot = (uint16_t*)(table + kFSlots);                       // [kFMaxK]
    uint16_t* pslot = cslot + kFMaxK;                                     // [kFMaxU]
    unsigned char* stage = (unsigned char*)(pslot + kFMaxU);
    float4* const s32 = (float4*)stage;                                   // [kPollCH + 4]
    double2* const s64 = (double2*)(stage + (kPollCH + 4) * 16);          // [kPollCH]
    unsigned (*const red)[kPollKPB] = (unsigned (*)[kPollKPB])stage;      // [4][512] (alias)
    unsigned* const pcnt = (unsigned*)(stage + kPollWaves * kPollKPB * 4); // [512] (alias)
    int* rs = (int*)(stage + kFStage);                                    // [kPollRB]
    int* rpre = rs + kPollRB;                                             // [kPollRB + 4]
    int4* nbox = (int4*)(rpre + kPollRB + 4);                             // [kPollNbr]
    int* misc = (int*)(nbox + kPollNbr);                                  // [0] distinct, [1] overflow, [2] scan

    const int N = a.N, K = a.K;
    const Grid& g = a.g;
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;

    // ---- prologue: one memory round trip for what disk i needs
    const int4 R = a.region[i];
    const int nc = a.ncount[i];
    const int4 nb = tid < kPollNbr ? a.nboxT[i * kPollNbr + tid] : make_int4(0, 0, 0, 0);
    bool bad = false;
    for (int q = tid; q < a.nct; q += kPollThreads) bad |= a.kbad[(int64_t)i * a.nct + q] != 0;
    const double bx = a.src.get(0, i, N), by = a.src.get(0, N + i, N), br = a.src.get(0, 2 * N + i, N);
    const bool hash_ok = K <= kFMaxK;
    // this thread's candidates: k = 4 * (tid + kPollThreads * j) + e
    constexpr int kKC = kFMaxK / (4 * kPollThreads);   // chunks of 4 candidates per thread
    uint2 qx[kKC], qy[kKC], qr[kKC];
    if (hash_ok) {
        const int16_t* kxr = a.keys + (int64_t)i * a.Kp;
        const int16_t* kyr = kxr + (int64_t)N * a.Kp;
        const int16_t* krr = kyr + (int64_t)N * a.Kp;
#pragma unroll
        for (int j = 0; j < kKC; ++j) {
            const int k4 = 4 * (tid + kPollThreads * j);
            if (k4 < K) {
                qx[j] = *(const uint2*)&kxr[k4];
                qy[j] = *(const uint2*)&kyr[k4];
                qr[j] = *(const uint2*)&krr[k4];
            }
        }
    }
    for (int q = tid; q < kFSlots; q += kPollThreads) table[q] = 0ull;
    if (tid < 3) misc[tid] = 0;
    if (tid < min(nc, kPollNbr)) nbox[tid] = nb;
    const bool hashed0 = hash_ok && !__syncthreads_or(bad);

    // ---- the distinct disks: insert, then ids in slot order
    if (hashed0) {
        constexpr uint32_t mask = kFSlots - 1;
#pragma unroll
        for (int j = 0; j < kKC; ++j) {
            const int k4 = 4 * (tid + kPollThreads * j);
            if (k4 >= K) continue;
            const uint32_t wx[2] = {qx[j].x, qx[j].y}, wy[2] = {qy[j].x, qy[j].y},
                           wr[2] = {qr[j].x, qr[j].y};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int k = k4 + e;
                if (k >= K) break;
                const int sh = (e & 1) * 16;
                const int kx = (int16_t)(wx[e >> 1] >> sh), ky = (int16_t)(wy[e >> 1] >> sh),
                          kr = (int16_t)(wr[e >> 1] >> sh);
                const unsigned long long key = pack_key(kx, ky, kr);
                uint32_t s = hash_key(key) & mask;
                bool placed = false;
                for (int pr = 0; pr < kFSlots; ++pr) {
                    const unsigned long long old = atomicCAS(&table[s], 0ull, key);
                    if (old == 0ull) {
                        atomicAdd(&misc[0], 1);
                        placed = true;
                        break;
                    }
                    if (old == key) {
                        placed = true;
                        break;
                    }
                    s = (s + 1) & mask;
                }
                if (!placed) misc[1] = 1;
                cslot[k] = (uint16_t)s;
            }
        }
    }
    __syncthreads();
    MAC_FW_STAMP(1);
    const bool hashed = hashed0 && misc[0] <= kFMaxU && misc[1] == 0;
    int U = K;
    if (hashed) {
        // ids in slot order: thread t owns slots [16t, 16t + 16)
        constexpr int per = kFSlots / kPollThreads;
        int occ = 0;
#pragma unroll
        for (int q = 0; q < per; ++q) occ += table[tid * per + q] != 0ull;
        const int incl = wave_incl_scan_i32(occ, lane);
        int* wsum = misc + 4;   // (misc has 16 words)
        if (lane == kWave - 1) wsum[wid] = incl;
        __syncthreads();
        int id = incl - occ;
        for (int w = 0; w < wid; ++w) id += wsum[w];
#pragma unroll
        for (int q = 0; q < per; ++q) {
            const int s = tid * per + q;
            const unsigned long long v = table[s];
            if (v != 0ull) {
                table[s] = v | ((unsigned long long)id << 52);
                pslot[id] = (uint16_t)s;
                ++id;
            }
        }
        U = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        __syncthreads();
    }
    MAC_FW_STAMP(2);
    // position p -> its disk (hashed: candidate 0's disk + the exact key; identity: candidate p)
    auto pos_disk = [&](int p) {
        if (hashed) {
            const unsigned long long key = table[pslot[p]];
            const int kx = (int16_t)(key & 0xffff), ky = (int16_t)((key >> 16) & 0xffff),
                      kr = (int16_t)((key >> 32) & 0xffff);
            return make_disk(bx + (double)kx, by + (double)ky, br + (double)kr);
        }
        return src_disk(a.src, N, i, p);
    };
    // candidate k -> its position
    auto pos_of = [&](int k) { return hashed ? (int)(table[cslot[k]] >> 52) : k; };

    if (R.x > R.y) return;   // disk i covers nothing in any candidate (uniform)

    // region rows: run start and entries before it, batches of kPollRB rows
    const double ox = g.gx0 + 0.5 * (double)(R.x + R.y + 1) * g.S;
    const double oy = g.gy0 + 0.5 * (double)(R.z + R.w + 1) * g.S;
    const double Umax = 0.5 * (double)max(R.y - R.x + 1, R.w - R.z + 1) * g.S + 2.0 * g.S;

    f32x2 sa[kPollPairs], sb[kPollPairs], st[kPollPairs], ns[kPollPairs];
    float xp[kPollSlots];
    for (int kb = 0; kb < U; kb += kPollKPB) {
        const int ke = min(U, kb + kPollKPB);
        uint32_t live = 0;
        double acc[kPollSlots];
#pragma unroll
        for (int u = 0; u < kPollSlots; ++u) {
            acc[u] = 0.0;
            const int p = kb + u * kWave + lane;
            PollLane L = inert_lane();
            if (p < ke) {
                live |= 1u << u;
                const DiskRec d = pos_disk(p);
                int4 sp;
                if (disk_span(d, g, sp)) L = poll_lane(d, ox, oy, Umax);
            }
            xp[u] = L.xp;
            const int j = u >> 1;
            if (u & 1) {
                sa[j].y = L.sa; sb[j].y = L.sb; st[j].y = L.stm; ns[j].y = L.ns;
            } else {
                sa[j].x = L.sa; sb[j].x = L.sb; st[j].x = L.stm; ns[j].x = L.ns;
            }
        }
        if (kb == 0) MAC_FW_STAMP(3);
        const int np = (ke - kb + 2 * kWave - 1) / (2 * kWave);
        auto dprime = [&](const float4& e, int u) {
            const int j = u >> 1;
            const float a_ = (u & 1) ? sa[j].y : sa[j].x, b_ = (u & 1) ? sb[j].y : sb[j].x;
            const float t_ = (u & 1) ? st[j].y : st[j].x, n_ = (u & 1) ? ns[j].y : ns[j].x;
            return __builtin_fmaf(e.x, n_, __builtin_fmaf(e.z, b_, __builtin_fmaf(e.y, a_, t_)));
        };
        for (int rb = R.z; rb <= R.w; rb += kPollRB) {
            const int nr = min(kPollRB, R.w - rb + 1);
            __syncthreads();
            if (tid < nr) {
                const int64_t rowbase = (int64_t)(rb + tid) * g.nTx;
                const int s0 = a.off[rowbase + R.x];
                rs[tid] = s0;
                rpre[tid + 1] = a.off[rowbase + R.y + 1] - s0;
            }
            __syncthreads();
            if (tid < kWave) {
                const int v = wave_incl_scan_i32(tid < nr ? rpre[tid + 1] : 0, tid);
                if (tid < nr) rpre[tid + 1] = v;
                if (tid == 0) rpre[0] = 0;
            }
            __syncthreads();
            const int total = rpre[nr];
            for (int base = 0; base < total; base += kPollCH) {
                const int n = min(kPollCH, total - base);
                for (int q = tid; q < n; q += kPollThreads) {
                    const int f = base + q;
                    int lo = 0, hi = nr - 1;
                    while (lo < hi) {
                        const int mid = (lo + hi + 1) >> 1;
                        if (rpre[mid] <= f) lo = mid; else hi = mid - 1;
                    }
                    const double2 p = a.xy[rs[lo] + (f - rpre[lo])];
                    s64[q] = p;
                    const bool shared =
                        nc > 0 && entry_shared(nc, nbox, tile_of(p.x, g.gx0, g.invS, g.nTx), rb + lo);
                    const float fu = (float)(p.x - ox), fv = (float)(p.y - oy);
                    s32[q] = !shared && __builtin_isfinite(fu) && __builtin_isfinite(fv)
                                 ? make_float4(__builtin_fmaf(fu, fu, fv * fv), fu, fv, 0.0f)
                                 : make_float4(__builtin_inff(), 0.0f, 0.0f, 0.0f);
                }
                if (tid < ((4 - (n & 3)) & 3)) s32[n + tid] = make_float4(__builtin_inff(), 0.0f, 0.0f, 0.0f);
                __syncthreads();
                const int ng = (n + 3) >> 2;
                float bmin[kPollSlots];
#pragma unroll
                for (int u = 0; u < kPollSlots; ++u) bmin[u] = __builtin_inff();
                auto band = [&](int u) {
                    const DiskRec d = pos_disk(kb + u * kWave + lane);
                    double c = 0.0;
                    for (int q4 = wid; q4 < ng; q4 += kPollWaves)
                        for (int q = 4 * q4; q < min(4 * q4 + 4, n); ++q) {
                            const float4 e = s32[q];
                            const float dp = dprime(e, u);
                            bool cov;
                            if (__builtin_fabsf(dp) <= xp[u]) {
                                const double2 p = s64[q];
                                if (e.x == __builtin_inff() && nc > 0 &&
                                    entry_shared(nc, nbox, tile_of(p.x, g.gx0, g.invS, g.nTx),
                                                 tile_of(p.y, g.gy0, g.invS, g.nTy)))
                                    continue;
                                cov = sqdist(p.x, p.y, d.cx, d.cy) <= d.T;
                            } else {
                                cov = dp > 0.0f;
                            }
                            if (cov) c += 1.0;
                        }
                    return c;
                };
                f32x2 h[kPollPairs];
                switch (np) {
                case 1: poll_hot<1>(s32, ng, wid, sa, sb, st, ns, h, bmin); break;
                case 2: poll_hot<2>(s32, ng, wid, sa, sb, st, ns, h, bmin); break;
                case 3: poll_hot<3>(s32, ng, wid, sa, sb, st, ns, h, bmin); break;
                default: poll_hot<4>(s32, ng, wid, sa, sb, st, ns, h, bmin); break;
                }
#pragma unroll
                for (int u = 0; u < kPollSlots; ++u) {
                    if (!(live & (1u << u))) continue;
                    const float hc = (u & 1) ? h[u >> 1].y : h[u >> 1].x;
                    acc[u] += bmin[u] <= xp[u] ? band(u) : (double)hc;
                }
                __syncthreads();
            }
        }
        if (kb == 0) MAC_FW_STAMP(4);
        // the slice's count per position: the four waves' shares (integers: any order)
#pragma unroll
        for (int u = 0; u < kPollSlots; ++u) red[wid][u * kWave + lane] = (unsigned)acc[u];
        __syncthreads();
        for (int p = tid; p < ke - kb; p += kPollThreads)
            pcnt[p] = red[0][p] + red[1][p] + red[2][p] + red[3][p];
        __syncthreads();
        // every candidate whose disk i sits at one of this slice's positions: one atomic add
        for (int k = tid; k < K; k += kPollThreads) {
            const int u = pos_of(k) - kb;
            if (u >= 0 && u < ke - kb) {
                const unsigned v = pcnt[u];
                if (v) atomicAdd(&a.cnt[k], v);
            }
        }
        if (kb == 0) MAC_FW_STAMP(5);
    }
}

// The last arriver of launch 2: areas, objectives, argmin (k_final.h argmin_kernel's order).
__device__ __forceinline__ void fused_final(const FusedArgs& a, unsigned char* lds)
{
    double* sv = (double*)lds;
    int* si = (int*)(sv + kPollWaves);
    const int K = a.K;
    double bv = __builtin_inf();
    int bi = -1;
    constexpr int B = 4;
    for (int k0 = threadIdx.x; k0 < K; k0 += B * kPollThreads) {
        unsigned n[B];
#pragma unroll
        for (int b = 0; b < B; ++b) {
            const int k = k0 + b * kPollThreads;
            n[b] = k < K ? __hip_atomic_fetch_add(&a.cnt[k], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                         : 0u;
        }
#pragma unroll
        for (int b = 0; b < B; ++b) {
            const int k = k0 + b * kPollThreads;
            if (k >= K) break;
            // the reference's sum of n equal weights, exact when every partial sum is;
            // nothing covered: 0.0 (also for a NaN / infinite / signed-zero weight)
            const double area = (n[b] == 0u || a.w0 == 0.0) ? 0.0 : (double)n[b] * a.w0;
            if (a.area_out) a.area_out[k] = area;
            if (a.rmax) {
                const double o = -area + a.vp[k];
                if (a.obj_out) a.obj_out[k] = o;
                if (o < bv) {   // ascending k per thread: first minimum kept
                    bv = o;
                    bi = k;
                }
            }
        }
    }
    if (!a.best) return;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1)
        argmin_take(bv, bi, __shfl_xor(bv, off, kWave), __shfl_xor(bi, off, kWave));
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    if (lane == 0) {
        sv[wid] = bv;
        si[wid] = bi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int q = 1; q < kPollWaves; ++q) argmin_take(sv[0], si[0], sv[q], si[q]);
        const int i = si[0];
        a.best[0] = i >= 0 ? sv[0] : __builtin_inf();
        const int64_t gidx = i >= 0 ? a.idx_base + i : (int64_t)-1;
        a.best[1] = __builtin_bit_cast(double, gidx);
        if (a.mirror) {
            a.mirror[0] = a.best[0];
            a.mirror[1] = a.best[1];
            __threadfence_system();
            __hip_atomic_store(reinterpret_cast<uint64_t*>(a.mirror + 2), a.seq, __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

__global__ __launch_bounds__(kPollThreads) void fused_walk_kernel(uint64_t* ts, FusedArgs a)
{
    ts_begin(ts);
    __shared__ __attribute__((aligned(16))) unsigned char lds[kFWalkLds];
    __shared__ int sjob, last;
    const int bx = blockIdx.x, N = a.N;
    if (bx < N) {
        // consecutive disks on one XCD (blocks b, b + 8, ... share one): block b is the
        // (b / 8)-th block of XCD slot b % 8, which owns a contiguous run of disks
        const int x = bx % 8, r = bx / 8, fl = N / 8, rem = N % 8;
        const int i = x < rem ? x * (fl + 1) + r : rem * (fl + 1) + (x - rem) * fl + r;
        fused_walk_disk(a, i, lds);
#ifdef MAC_DIAG
        vm_drain();
        __syncthreads();
        if (threadIdx.x == 0 && i < 65536) g_diag_walk[8 * i + 6] = __builtin_amdgcn_s_memrealtime();
#endif
    }
    // shared-entry jobs: [0, n_shared) one each to the shared workgroups, the rest from the
    // counter (walk workgroups join once their disk is done)
    const int dcount = a.ctl[kCtlDcount];
    if (dcount > 0) {
        const int C = dcount * ((a.K + kShC - 1) / kShC) > 2 * (int)gridDim.x ? kShCWide : kShC;
        const int nsub = (a.K + C - 1) / C;
        const int total = dcount * nsub;
        int job = bx >= N ? bx - N : -1;
        for (;;) {
            if (job < 0) {
                __syncthreads();
                if (threadIdx.x == 0) sjob = a.n_shared + atomicAdd(&a.ctl[kCtlJobs], 1);
                __syncthreads();
                job = sjob;
            }
            if (job >= total) break;   // uniform
            fused_shared_job(a, a.dlist[job / nsub], (job % nsub) * C, C, lds);
            job = -1;
        }
    }
    vm_drain();
    __syncthreads();
    if (threadIdx.x == 0)
        last = atomicInc((unsigned*)&a.ctl[kCtlDone2], gridDim.x - 1) == gridDim.x - 1;
    __syncthreads();
    if (last) fused_final(a, lds);
    ts_end(ts);
}

}  // namespace mac
