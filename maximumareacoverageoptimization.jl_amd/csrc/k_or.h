// k_or.h — shared entries by per-entry union (equal weights): the shared-entry pass of crowded
// polls (config 5's clustered disks over the fire, config 4 "clustered").
//
// Ownership recap (k_poll.h): the walk of disk d credits every entry of region d that lies in no
// LOWER neighbour's box; an entry e that lies in several region boxes ("shared") has its disk set
// D_e = {d : tile(e) in box d}, and the walk of j0 = min D_e credits it when disk j0 of the
// candidate covers it (no lower box holds e, so it is not shared for j0). The reference counts
// e once when ANY disk covers it (src/AreaCoverageCalculation.jl:67-78, first hit + break), so
// the missing part of e's count is
//     [OR_{d in D_e} cov_d(e, k)] AND NOT cov_{j0}(e, k).
// This pass adds exactly that, once per shared entry: e belongs to the job list of i = max D_e
// (the entries of region i in some lower box and in no UPPER box, so D_e is {i} plus lower
// neighbours of i, the lists walk_setup builds), split in blocks of 64 entries (walk_setup lists
// the jobs). Per job:
//   1. stage the 64 entries; per disk slot m ({i} + lower neighbours) the 64-bit mask live[m] of
//      entries inside its box, and lmask[m] of entries whose j0 is that disk;
//   2. per disk with live entries, per distinct position u of that disk (k_index.h), the 64-bit
//      word T[u] of the entries it covers — the walk's exact fp32 filter (k_poll.h header), band
//      entries re-decided in fp64 — then per candidate k: Y |= T[u_d(k)], Z |= T[u_d(k)] & lmask;
//   3. per candidate: popcount(Y & ~Z) added (integer atomics: exact in any order) to spart row i
//      (kept as popcount(Y) - sum of popcount(T & lmask): the lmask sets are disjoint).
// Tests: sum over shared entries of sum over d in D_e of U_d (distinct positions), against the
// bit-word kernel's per-owner (U_i + sum over ALL neighbours of U_j) x |S_i|: the owner form tests
// each shared entry once per owner and against every neighbour's positions (3.4e9 tests on the
// slowest config-5 poll, 6e8 here).
// Used when every disk with neighbours fits the lists (at most kPollNbr lower and upper
// neighbours, regions at most 64 x 64 tiles) and the list is not weighted; otherwise the poll
// kernel's fp64 jobs take every disk (k_poll.h shared_route).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "predicate.h"
#include "k_common.h"
#include "k_lane.h"

#pragma clang fp contract(off)

namespace mac {

#ifdef MAC_DIAG
// diagnostic build only: per workgroup, ticks (s_memrealtime, 10 ns) spent in each phase and counts
__device__ uint64_t g_diag_or[1024 * 16];
#define MAC_OR_T(q) do { if (threadIdx.x == 0) { const uint64_t t_ = __builtin_amdgcn_s_memrealtime(); dg[q] += t_ - dt; dt = t_; } } while (0)
#define MAC_OR_N(q, v) do { if (threadIdx.x == 0) dg[q] += (v); } while (0)
#else
#define MAC_OR_T(q)
#define MAC_OR_N(q, v)
#endif

constexpr int kOrThreads = 512;                 // 8 waves
constexpr int kOrPT = 7;                        // candidates per thread per candidate chunk (K = 3073: one)
constexpr int kOrKC = kOrPT * kOrThreads;       // 3584 candidates per chunk
constexpr int kOrE = 64;                        // entries per job
constexpr int kOrTab = 4096;                    // positions per table chunk (32 KB of words)
constexpr int kOrRuns = 64 * 32;                // tile runs of a region (64 rows x 32 runs)

// Which shared-entry pass a poll takes (device side, uniform; the host's hint bits_on: 0 none,
// 1 above kBitsMinDisks disks with neighbours, 2 always): 0 the poll kernel's fp64 jobs for
// every disk with neighbours; 1 the bit-word kernel (k_bits.h, weighted lists) for the disks it
// qualifies + fp64 jobs for the others; 2 this union pass for every disk (equal weights).
__device__ __forceinline__ int shared_route(const int* __restrict__ dcount, int bits_on, int counts,
                                            int K)
{
    const int nA = dcount[kDcBits], nB = dcount[kDcOther];
    if (!bits_on || nA + nB <= (bits_on == 2 ? 0 : kBitsMinDisks)) return 0;
    if (!counts) return 1;
    (void)K;
    return nB == 0 && dcount[kDcOrBad] == 0 ? 2 : 0;
}

// One wave's 64 32-bit words global -> LDS with no register (global_load_lds_dword): lane l
// reads g_lane (its own address) into l_wave + 4 l; l_wave is wave-uniform. Drained by the next
// __syncthreads (hipcc waits vmcnt(0) there).
__device__ __forceinline__ void glds_u32(const void* g_lane, void* l_wave)
{
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g_lane,
                                     (__attribute__((address_space(3))) void*)l_wave, 4, 0, 0);
}

// Row r's tiles of region R (at most 64 x 64 tiles) that lie in some lower box and in no upper
// box, as a mask of tile columns relative to R.x.
__device__ __forceinline__ uint64_t or_row_mask(const int4& R, int r, const int4* lbox, int nl,
                                                const int4* ubox, int nu)
{
    if (r < R.z || r > R.w) return 0;
    auto span = [&](const int4& Q) -> uint64_t {
        if (r < Q.z || r > Q.w) return 0;
        const int a = max(R.x, Q.x) - R.x, b = min(R.y, Q.y) - R.x;
        if (a > b) return 0;
        return (b - a == 63 ? ~0ull : ((1ull << (b - a + 1)) - 1)) << a;
    };
    uint64_t lo = 0, up = 0;
    for (int m = 0; m < nl; ++m) lo |= span(lbox[m]);
    for (int m = 0; m < nu; ++m) up |= span(ubox[m]);
    const int tw = R.y - R.x + 1;
    uint64_t mask = lo & ~up;
    if (tw < 64) mask &= (1ull << tw) - 1;
    return mask;
}

// Entries of row r's masked runs (wave 0: lane = row). The first four runs' offsets are loaded
// together (a row of a MADS poll's region has one to three), further runs one by one.
__device__ __forceinline__ int or_row_count(const int32_t* __restrict__ off, const Grid& g,
                                            const int4& R, int r, uint64_t mask)
{
    const int64_t rowbase = (int64_t)r * g.nTx + R.x;
    int lo[4], hi[4];
    uint64_t m2 = mask;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        lo[q] = hi[q] = 0;
        if (m2) {
            const int a = __builtin_ctzll(m2);
            const uint64_t from = m2 >> a;
            const int len = ~from ? __builtin_ctzll(~from) : 64 - a;
            lo[q] = a;
            hi[q] = a + len;
            m2 &= len + a >= 64 ? 0ull : (~0ull << (a + len));
        }
    }
    int v[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        v[2 * q] = hi[q] > lo[q] ? off[rowbase + lo[q]] : 0;
        v[2 * q + 1] = hi[q] > lo[q] ? off[rowbase + hi[q]] : 0;
    }
    int n = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) n += v[2 * q + 1] - v[2 * q];
    while (m2) {
        const int a = __builtin_ctzll(m2);
        const uint64_t from = m2 >> a;
        const int len = ~from ? __builtin_ctzll(~from) : 64 - a;
        n += off[rowbase + a + len] - off[rowbase + a];
        m2 &= len + a >= 64 ? 0ull : (~0ull << (a + len));
    }
    return n;
}

// A job's weight bucket (0 heaviest): its tables test about U_i * (1 + nl) positions (disk i's
// positions and its lower neighbours'), so jobs are handed out heaviest first and the launch's
// tail is made of light jobs (longest-processing-time order).
__device__ __forceinline__ int or_bucket(int U, int nl)
{
    const int w = U * (1 + min(nl, 8));
    return w >= 8192 ? 0 : w >= 4096 ? 1 : w >= 2048 ? 2 : 3;
}

// walk_setup's part (block i, after neighbors_block with the lists in LDS): the number of entries
// of region i that this pass owns (lower box, no upper box) and one job per 64 of them, appended
// ({i, block}) to its weight bucket's list (jobs + bucket * cap) from the counter
// dcount[kDcOrJobs + bucket]. A list past `cap` (cannot happen: the owned sets are disjoint,
// cap >= M / 64 + N) makes the pass stand down (kDcOrBad).
__device__ __forceinline__ void or_list_jobs(int i, const int4& R, const int4* lbox, int nl,
                                             const int4* ubox, int nu, const int32_t* __restrict__ off,
                                             const Grid& g, int2* __restrict__ jobs, int cap,
                                             int* __restrict__ dcount, int U)
{
    __shared__ int s_base, s_nblk;
    const int tid = threadIdx.x;
    if (nl == 0 || nl > kPollNbr || nu > kPollNbr || R.y - R.x + 1 > 64 || R.w - R.z + 1 > 64)
        return;   // (uniform) nothing owned, or the pass stands down for this poll
    if (tid < kWave) {
        const int r = R.z + tid;
        const uint64_t mask = or_row_mask(R, r, lbox, nl, ubox, nu);
        int n = or_row_count(off, g, R, r, mask);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) n += __shfl_xor(n, o, kWave);
        if (tid == 0) {
            const int nblk = (n + kOrE - 1) / kOrE;
            const int bk = or_bucket(U, nl);
            s_nblk = nblk;
            s_base = nblk ? atomicAdd(dcount + kDcOrJobs + bk, nblk) : 0;
            if (nblk && s_base + nblk > cap) atomicAdd(dcount + kDcOrBad, 1);
            s_base += bk * cap;
        }
    }
    __syncthreads();
    const int base = s_base, nblk = s_nblk;
    for (int b = tid; b < nblk; b += kBlock)
        if (base % cap + b < cap) jobs[base + b] = make_int2(i, b);
}

struct OrArgs {
    const double2* xy;
    const int32_t* off;
    Grid g;
    const DiskRec* urec;
    const int* umap;
    const int* ucount;
    const int4* region;
    const uint16_t* nbrT;
    const int4* nboxT;
    const int* ncount;
    const int4* nboxU;
    const int* ncountU;
    const float4* lane4;
    const float* lanexp;
    const int2* jobs;
    int* dcount;
    const int* mode;
    unsigned* spart;   // uint32 count rows [N][K] (the poll kernel zeroed the rows of disks with neighbours)
    int N, K, bits_on;
    int cap;           // jobs per bucket list (jobs + bucket * cap)
};

// (cur << 1) | sign bit of v (v_alignbit_b32 {cur, v} >> 31)
__device__ __forceinline__ uint32_t or_shift_sign(uint32_t cur, float v)
{
    uint32_t r;
    asm("v_alignbit_b32 %0, %1, %2, 31" : "=v"(r) : "v"(cur), "v"(v));
    return r;
}

__global__ __launch_bounds__(kOrThreads) __attribute__((amdgpu_waves_per_eu(4))) void shared_or_kernel(uint64_t* ts, OrArgs a)
{
    __shared__ int sid[kPollNbr + 1], sU[kPollNbr + 1];
    __shared__ int4 sbox[kPollNbr + 1], subox[kPollNbr];
    __shared__ int wrun[kWave];
    __shared__ double2 s64[kOrE];
    __shared__ int2 stile[kOrE];
    __shared__ int js[kOrE];
    __shared__ uint64_t live[kPollNbr + 1], lmask[kPollNbr + 1];
    __shared__ int rel[kPollNbr + 1];
    __shared__ __attribute__((aligned(16))) float4 ent[kOrE / 2];   // {U0, U1, V0, V1} per entry pair
    __shared__ f32x2 entq[kOrE / 2];                                 // {Q0, Q1}
    __shared__ __attribute__((aligned(16))) uint2 tab[kOrTab];   // the tables (the set-up's runs alias them)
    static_assert((3 * kOrRuns + 1) * sizeof(int) <= sizeof(uint2) * kOrTab, "runs fit the tables");
    int* const run_s = reinterpret_cast<int*>(tab);
    int* const run_pre = run_s + kOrRuns;
    int* const run_row = run_pre + kOrRuns + 1;
    __shared__ int um32[2][kOrKC];   // a disk's position of every candidate of the chunk (two buffers)
    __shared__ int s_nrel, s_total, s_next[2];

    ts_begin(ts);
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
    constexpr int kWaves = kOrThreads / kWave;
    if ((a.mode && *a.mode != kModePoll) || shared_route(a.dcount, a.bits_on, 1, a.K) != 2) {   // uniform
        ts_end(ts);
        return;
    }
    int nb[kOrBuckets], njobs = 0;   // the buckets' job counts, heaviest bucket first
#pragma unroll
    for (int b = 0; b < kOrBuckets; ++b) {
        nb[b] = a.dcount[kDcOrJobs + b];
        njobs += nb[b];
    }
    const int K = a.K;
#ifdef MAC_DIAG
    uint64_t dg[16] = {};
    uint64_t dt = __builtin_amdgcn_s_memrealtime();
    const uint64_t dt0 = dt;
#endif
    const Grid g = a.g;
    // the candidates' positions of slot m's disk (chunk kc0) straight into LDS buffer bb (no
    // registers); the barrier after the next staging drains them
    auto issue_pos = [&](int m, int bb, int kc0) {
        const int64_t row = (int64_t)sid[m] * K;
#pragma unroll
        for (int c = 0; c < kOrPT; ++c) {
            const int kw = kc0 + c * kOrThreads + wid * kWave;   // the wave's first candidate
            if (kw < K) glds_u32(a.umap + row + min(kw + lane, K - 1), &um32[bb][c * kOrThreads + wid * kWave]);
        }
    };
    int it = 0;
    for (int job = blockIdx.x; job < njobs; ++it) {
        int q = job, bk = 0;
#pragma unroll
        for (int b = 0; b < kOrBuckets - 1; ++b)
            if (bk == b && q >= nb[b]) {
                q -= nb[b];
                bk = b + 1;
            }
        // the next job's counter add, in flight during this job (two slots: a wave still reading
        // this job's slot never sees the next job's write)
        if (tid == 0) s_next[it & 1] = (int)gridDim.x + atomicAdd(a.dcount + kDcBitsJobs, 1);
        const int2 jb = a.jobs[(int64_t)bk * a.cap + q];
        const int i = jb.x, blk = jb.y;
        // disk i's lists (slot 0: disk i itself, slots 1..nc: its lower neighbours)
        const int nc = a.ncount[i], ncU = a.ncountU[i];
        if (tid < nc) {
            sid[1 + tid] = a.nbrT[i * kPollNbr + tid];
            sbox[1 + tid] = a.nboxT[i * kPollNbr + tid];
        }
        if (tid < ncU) subox[tid] = a.nboxU[i * kPollNbr + tid];
        if (tid == 0) {
            sid[0] = i;
            sbox[0] = a.region[i];
        }
        __syncthreads();
        const int4 R = sbox[0];
        // the owned runs of region i (wave 0: lane = row), and the disks' position counts
        if (tid < kWave) {
            const int r = R.z + lane;
            const uint64_t mask = or_row_mask(R, r, sbox + 1, nc, subox, ncU);
            const int64_t rowbase = (int64_t)r * g.nTx + R.x;
            const int cnt = __popcll(mask & ~(mask << 1));   // runs of the row
            const int qi = wave_incl_scan_i32(cnt, lane);
            // the row's runs: first entry and length (every off load in flight), then the
            // lengths turned into the exclusive prefix over the region's runs
            int qq = qi - cnt, len_row = 0;
            for (uint64_t m2 = mask; m2;) {
                const int a0 = __builtin_ctzll(m2);
                const uint64_t from = m2 >> a0;
                const int len = ~from ? __builtin_ctzll(~from) : 64 - a0;
                const int s0 = a.off[rowbase + a0];
                const int n0 = a.off[rowbase + a0 + len] - s0;
                run_s[qq] = s0;
                run_pre[qq] = n0;
                run_row[qq] = r;
                len_row += n0;
                ++qq;
                m2 &= len + a0 >= 64 ? 0ull : (~0ull << (a0 + len));
            }
            const int ei = wave_incl_scan_i32(len_row, lane);
            int pre = ei - len_row;
            for (int z = qi - cnt; z < qi; ++z) {
                const int n0 = run_pre[z];
                run_pre[z] = pre;
                pre += n0;
            }
            if (lane == kWave - 1) {
                wrun[0] = qi;
                run_pre[qi] = ei;
                s_total = ei;
            }
        } else if (tid - kWave <= nc) {
            sU[tid - kWave] = a.ucount[sid[tid - kWave]];
        }
        __syncthreads();
        const int nrun = wrun[0], total = s_total;
        // the job's 64 entries: exact coordinates, tiles (x from the coordinate as the walk does,
        // y = the run's row); past the owned list: NaN, tile -1 (in no box)
        if (tid < kOrE) {
            const int f = blk * kOrE + tid;
            double2 p = make_double2(__builtin_nan(""), __builtin_nan(""));
            int2 tl = make_int2(-1, -1);
            if (f < total) {
                int lo = 0, hi = nrun - 1;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (run_pre[mid] <= f) lo = mid; else hi = mid - 1;
                }
                p = a.xy[run_s[lo] + (f - run_pre[lo])];
                tl = make_int2(tile_of(p.x, g.gx0, g.invS, g.nTx), run_row[lo]);
            }
            s64[tid] = p;
            stile[tid] = tl;
            // j0: the lowest disk whose box holds the entry (slot index; -1: none)
            int best = -1, bid = 0x7fffffff;
            for (int m = 0; m <= nc; ++m)
                if (tl.x >= 0 && box_has(sbox[m], tl.x, tl.y) && sid[m] < bid) {
                    bid = sid[m];
                    best = m;
                }
            js[tid] = best;
        }
        __syncthreads();
        // per disk slot: live entries (inside its box) and the entries it is j0 of
        for (int m = wid; m <= nc; m += kWaves) {
            const int2 tl = stile[lane];
            const uint64_t lv = __ballot(tl.x >= 0 && box_has(sbox[m], tl.x, tl.y));
            const uint64_t lm = __ballot(js[lane] == m);
            if (lane == 0) {
                live[m] = lv;
                lmask[m] = lm;
            }
        }
        __syncthreads();
        if (tid < kWave) {   // the disks with live entries, in slot order
            int n = 0;
            for (int m0 = 0; m0 <= nc; m0 += kWave) {
                const int m = m0 + lane;
                const bool has = m <= nc && live[m] != 0;
                const uint64_t bal = __ballot(has);
                if (has) rel[n + __popcll(bal & ((1ull << lane) - 1))] = m;
                n += __popcll(bal);
            }
            if (lane == 0) s_nrel = n;
        }
        __syncthreads();
        const int nrel = s_nrel;
        MAC_OR_T(0);
        MAC_OR_N(8, 1);
        MAC_OR_N(9, nrel);

        for (int kc0 = 0; kc0 < K; kc0 += kOrKC) {
            // per candidate: Y = the union word; zc = the j0 part's count (the lmask sets of the
            // disks are disjoint, so popcount(OR of (T & lmask)) is the sum of their popcounts)
            uint64_t Y[kOrPT];
            uint32_t zc[kOrPT];
#pragma unroll
            for (int c = 0; c < kOrPT; ++c) {
                Y[c] = 0;
                zc[c] = 0;
            }
            if (nrel > 0) issue_pos(rel[0], 0, kc0);
            for (int r = 0; r < nrel; ++r) {
                const int m = rel[r], bb = r & 1;
                const int d = sid[m], U = sU[m];
                const int64_t row = (int64_t)d * K;
                const uint64_t lv = live[m], lm = lmask[m];
                // the entries relative to region d's centre, as the walk stages them; entries
                // outside box d, past the list or non-finite are inert (Q = +inf: d' = -inf)
                if (tid < kOrE) {
                    const int4 Rd = sbox[m];
                    const double ox = g.gx0 + 0.5 * (double)(Rd.x + Rd.y + 1) * g.S;
                    const double oy = g.gy0 + 0.5 * (double)(Rd.z + Rd.w + 1) * g.S;
                    const double2 p = s64[tid];
                    const float fu = (float)(p.x - ox), fv = (float)(p.y - oy);
                    const bool f = ((lv >> tid) & 1) && __builtin_isfinite(fu) && __builtin_isfinite(fv);
                    float* const eu = reinterpret_cast<float*>(&ent[tid >> 1]);
                    eu[tid & 1] = f ? fu : 0.0f;
                    eu[2 + (tid & 1)] = f ? fv : 0.0f;
                    reinterpret_cast<float*>(&entq[tid >> 1])[tid & 1] =
                        f ? __builtin_fmaf(fu, fu, fv * fv) : __builtin_inff();
                }
                __syncthreads();   // (this disk's positions have landed too)
                // the next disk's positions into the other buffer, in flight during this disk
                if (r + 1 < nrel) issue_pos(rel[r + 1], bb ^ 1, kc0);
                MAC_OR_T(1);
                MAC_OR_N(10, U);
                MAC_OR_N(11, __popcll(lv));
                // work items (position, 32-entry half with live entries): both halves of a
                // position are separate items, so the waves stay balanced and an item's lane
                // constants load one item ahead of its tests
                const bool w0 = (uint32_t)lv != 0, w1 = (uint32_t)(lv >> 32) != 0;
                const int nh = (w0 ? 1 : 0) + (w1 ? 1 : 0), h1 = w0 ? 0 : 1;   // uniform
                uint32_t* const tab32 = reinterpret_cast<uint32_t*>(tab);
                for (int u0 = 0; u0 < U; u0 += kOrTab) {
                    const int u1 = min(U, u0 + kOrTab);
                    const int nit = (u1 - u0) * nh;
                    int q = tid;
                    float4 c4n = make_float4(0.0f, 0.0f, -1.0f, -1.0f);
                    float xpn = -1.0f;
                    if (q < nit) {
                        const int p = u0 + (nh == 2 ? q >> 1 : q);
                        c4n = a.lane4[row + p];
                        xpn = a.lanexp[row + p];
                    }
                    for (; q < nit; q += kOrThreads) {
                        const int p = u0 + (nh == 2 ? q >> 1 : q);
                        const int hv = nh == 2 ? (q & 1) : h1;   // the half: entries 32 hv ..
                        const float4 c4 = c4n;
                        const float xp = xpn;
                        const int qn = q + kOrThreads;
                        if (qn < nit) {   // the next item's constants, in flight during the tests
                            const int pn = u0 + (nh == 2 ? qn >> 1 : qn);
                            c4n = a.lane4[row + pn];
                            xpn = a.lanexp[row + pn];
                        }
                        const f32x2 sa = {c4.x, c4.x}, sb = {c4.y, c4.y}, st = {c4.z, c4.z},
                                    ns = {c4.w, c4.w}, xp2 = {xp, xp};
                        uint32_t cw = 0u;
                        float bmin = __builtin_inff();
                        const float4* const eh = ent + 16 * hv;
                        const f32x2* const qh = entq + 16 * hv;
                        const uint32_t lvh = (uint32_t)(lv >> (32 * hv));   // the half's live entries
                        // groups of 8 entries; a group with no live entry (uniform) only shifts
                        // its 8 zero bits in (entries in tile order: live ones come in runs)
                        for (int g8 = 0; g8 < 4; ++g8) {
                            if (((lvh >> (8 * g8)) & 0xffu) == 0u) {
                                cw <<= 8;
                                continue;
                            }
#pragma unroll 2
                            for (int j = 4 * g8; j < 4 * g8 + 4; ++j) {
                                const float4 uv = eh[j];
                                const f32x2 qq = qh[j];
                                const f32x2 U2 = {uv.x, uv.y}, V2 = {uv.z, uv.w};
                                const f32x2 dd = __builtin_elementwise_fma(
                                    qq, ns, __builtin_elementwise_fma(V2, sb, __builtin_elementwise_fma(U2, sa, st)));
                                // covered iff d' > X' iff X' - d' < 0: its sign bit shifted in
                                const f32x2 sd2 = xp2 - dd;
                                cw = or_shift_sign(cw, sd2.x);
                                cw = or_shift_sign(cw, sd2.y);
                                bmin = __builtin_fminf(bmin, __builtin_fminf(__builtin_fabsf(dd.x),
                                                                             __builtin_fabsf(dd.y)));
                            }
                        }
                        uint32_t t = __builtin_bitreverse32(cw);
                        // X' < 2 for every normal position: no |d'| <= 2 means no band entry; a
                        // band (or forced) position re-decides its half's entries, band ones in fp64
                        if (bmin <= 2.0f || !(xp < 2.0f)) {
                            const DiskRec rr = a.urec[row + p];
                            t = 0u;
                            for (int e = 0; e < 32; ++e) {
                                const float4 uv = eh[e >> 1];
                                const float qv = qh[e >> 1][e & 1];
                                const float U1 = (e & 1) ? uv.y : uv.x, V1 = (e & 1) ? uv.w : uv.z;
                                const float dp = __builtin_fmaf(qv, c4.w, __builtin_fmaf(V1, c4.y, __builtin_fmaf(U1, c4.x, c4.z)));
                                bool cov = dp > xp;
                                if (__builtin_fabsf(dp) <= xp) {
                                    const double2 qd = s64[32 * hv + e];
                                    cov = qv != __builtin_inff() && sqdist(qd.x, qd.y, rr.cx, rr.cy) <= rr.T;
                                }
                                if (cov) t |= 1u << e;
                            }
                        }
                        if (nh == 2)
                            tab32[2 * (p - u0) + hv] = t;
                        else
                            tab[p - u0] = hv ? make_uint2(0u, t) : make_uint2(t, 0u);
                    }
                    __syncthreads();
                    MAC_OR_T(2);
                    // combine: the union word and the j0 word of every candidate
#pragma unroll
                    for (int c = 0; c < kOrPT; ++c) {
                        const int k = kc0 + tid + c * kOrThreads;
                        const int u = k < K ? um32[bb][c * kOrThreads + tid] : -1;
                        if (u >= u0 && u < u1) {
                            const uint2 t2 = tab[u - u0];
                            const uint64_t t = (uint64_t)t2.x | ((uint64_t)t2.y << 32);
                            Y[c] |= t;
                            zc[c] += (uint32_t)__popcll(t & lm);
                        }
                    }
                    __syncthreads();   // the next chunk / disk overwrites the tables and entries
                    MAC_OR_T(3);
                }
            }
#pragma unroll
            for (int c = 0; c < kOrPT; ++c) {
                const int k = kc0 + tid + c * kOrThreads;
                const int n = __popcll(Y[c]) - (int)zc[c];   // popcount(Y & ~Z): Z is in Y
                if (k < K && n) atomicAdd(a.spart + (int64_t)i * K + k, (unsigned)n);
            }
        }
        // the next job (its counter add went out at the start of this one)
        __syncthreads();
        job = s_next[it & 1];
        MAC_OR_T(4);
    }
#ifdef MAC_DIAG
    if (tid == 0 && blockIdx.x < 1024) {
        dg[12] = __builtin_amdgcn_s_memrealtime() - dt0;
        for (int q = 0; q < 16; ++q) g_diag_or[16 * blockIdx.x + q] = dg[q];
    }
#endif
    ts_end(ts);
}

}  // namespace mac
