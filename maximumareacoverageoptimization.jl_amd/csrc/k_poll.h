// k_poll.h — the poll walk: one workgroup per (disk i, slice of the poll's candidates).
//
// Across one poll, disk i of candidate k sits at x_inc + delta*d_k: a few metres around the
// incumbent. region[i] (k_prep.h) is the union of disk i's tile spans over all K candidates.
// The workgroup stages the entries of region[i] in LDS once (chunks of kPollCH) and each lane
// tests kPollKPL of its candidates' disk i against every staged entry: one broadcast LDS read
// per entry per wave feeds kPollKPL tests, there is no cross-lane reduction, and entries come
// from HBM once per (disk, slice) instead of once per (candidate, disk). An entry is credited to
// disk i of candidate k only when no lower-index disk j of candidate k covers it (exactly-once
// union counting), so the area is the reference's first-hit sum
// (src/AreaCoverageCalculation.jl:67-78) over the same multiset of entries.
//
// Ownership. Only disks j < i whose regions overlap region i can also cover an entry of region
// i, and only inside their region box. Entries whose tile lies in such a box ("shared") are
// left out here and decided exactly by the shared-entry workgroups (k_poll_shared.h); every
// other entry of region i can only be credited to disk i.
//
// Exact fp32 filter. With o the region centre, x = px - ox, y = py - oy, cu = cx - ox,
// cv = cy - oy (fp64; errors relative to these small offsets): the reference decision
// a64 <= T (sqrt(a64) < r, predicate.h) is, up to fp64 noise, sign(T - A) with
// T - A = (T - C) - (x^2 + y^2) + 2x*cu + 2y*cv, C = cu^2 + cv^2.
// Entries are staged once as fp32 (U, V, Q = U^2 + V^2); each lane keeps, per candidate, a
// power of two S and fp32 Sa = S*2cu, Sb = S*2cv, STm = S*fl32(T - C), and computes
//     d' = fma(Q, -S, fma(V, Sb, fma(U, Sa, STm)))      ( = S*(T - A) + error )
// With M = max(Umax, |cu|, |cv|, r) and eps = 2^-24 the error is below 38.1 eps M^2 * S
// (staging of U, V, Q: 14.1, the fp32 constants: 6, the three fmas: 18), so with
// X = RU32(2^-18 M^2) (= 64 eps M^2) and S = 2^k such that X' = S*X is in [1, 2):
//     d' >  X'   =>  a64 <  T   covered         (then clamp(d') = 1 exactly)
//     d' < -X'   =>  a64 >  T   not covered     (clamp(d') = 0)
//     |d'| <= X' (the band)     => the lane re-decides the whole chunk, band entries in fp64.
// The hot loop is therefore, per 2 entries x 2 candidates, six packed fmas, two packed clamps
// (v_pk_add_f32 ... clamp), two packed adds and two v_min3 (the band detector): three VALU ops
// per test. On the reference lattices the band is empty (|a - T| >= 1/2 >> X).
// Non-finite and shared entries are staged with Q = +inf, U = V = 0: d' = -inf, never counted,
// never in the band. A lane whose M is outside [2^-60, 2^60] is "forced": S = 1, X' = +inf, every
// entry goes to the exact pass.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "predicate.h"
#include "k_common.h"
#include "k_poll_shared.h"
#include "k_bits.h"
#include "k_final.h"
#include "k_index.h"
#include "k_lane.h"

#pragma clang fp contract(off)

namespace mac {

#ifdef MAC_DIAG
constexpr uint64_t kDiagMax = 1 << 16;
__device__ uint64_t g_diag[4 * kDiagMax];
#endif

#ifdef MAC_DIAG
// diagnostic build only: per-workgroup (start, end, role << 56 | info, XCC) stamps indexed by the
// linear block id; nothing else reads them
__device__ __forceinline__ void diag_stamp(uint64_t t0, uint64_t role, uint64_t info)
{
    if (threadIdx.x != 0) return;
    const uint64_t b = (uint64_t)blockIdx.y * gridDim.x + blockIdx.x;
    if (b >= kDiagMax) return;
    g_diag[4 * b + 0] = t0;
    g_diag[4 * b + 1] = __builtin_amdgcn_s_memrealtime();
    g_diag[4 * b + 2] = (role << 56) | (info & 0xffffffffffffffull);
    g_diag[4 * b + 3] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));
}
#define MAC_DIAG_STAMP(t0, role, info) diag_stamp(t0, role, info)
__device__ uint64_t g_diag_walk[8 * 65536];   // walk role, grid row 0: per-disk phase stamps
#define MAC_WALK_STAMP(q) if (threadIdx.x == 0 && blockIdx.y == 0 && i < 65536) g_diag_walk[8 * i + (q)] = __builtin_amdgcn_s_memrealtime()
#else
#define MAC_DIAG_STAMP(t0, role, info)
#define MAC_WALK_STAMP(q)
#endif

// Hot loop of the poll walk over this wave's groups of 4 staged entries (q4 = w, w + 4, ...):
// NP candidate pairs per entry pair, per 2 entries x 2 candidates six packed fmas, two packed
// clamps (count), two packed adds and two v_min3 (band detector). h[j]: covered counts of pair j.
// NW: the waves splitting the groups (wave w takes groups w, w + NW, ...).
template <int NP, int NW = kPollWaves>
__device__ __forceinline__ void poll_hot(const float4* __restrict__ s32, int ng, int w,
                                         const f32x2 (&sa)[kPollPairs], const f32x2 (&sb)[kPollPairs],
                                         const f32x2 (&st)[kPollPairs], const f32x2 (&ns)[kPollPairs],
                                         f32x2 (&h)[kPollPairs], float (&bmin)[kPollSlots])
{
    const f32x2 zero2 = {0.0f, 0.0f};
#pragma unroll
    for (int j = 0; j < kPollPairs; ++j) h[j] = zero2;
#define MAC_POLL_PAIR(E0, E1, J)                                                                \
    {                                                                                         \
        const f32x2 d0 = fma2(E0.x, ns[J], fma2(E0.z, sb[J], fma2(E0.y, sa[J], st[J])));       \
        const f32x2 d1 = fma2(E1.x, ns[J], fma2(E1.z, sb[J], fma2(E1.y, sa[J], st[J])));       \
        h[J] += clamp01x2(d0, zero2);                                                         \
        h[J] += clamp01x2(d1, zero2);                                                         \
        bmin[2 * J] = __builtin_fminf(__builtin_fminf(bmin[2 * J], __builtin_fabsf(d0.x)),     \
                                      __builtin_fabsf(d1.x));                                  \
        bmin[2 * J + 1] = __builtin_fminf(__builtin_fminf(bmin[2 * J + 1], __builtin_fabsf(d0.y)), \
                                          __builtin_fabsf(d1.y));                              \
    }
    for (int q4 = w; q4 < ng; q4 += NW) {
        const float4 e0 = s32[4 * q4], e1 = s32[4 * q4 + 1], e2 = s32[4 * q4 + 2], e3 = s32[4 * q4 + 3];
#pragma unroll
        for (int j = 0; j < NP; ++j) {
            MAC_POLL_PAIR(e0, e1, j)
            MAC_POLL_PAIR(e2, e3, j)
        }
    }
#undef MAC_POLL_PAIR
}

// Grid (N + n_shared); roles by x, in dispatch order: x < N, when
// *mode == kModePoll (or mode == null): one workgroup per disk i, over slices of kPollKPB
// positions of disk i's distinct disks (urec / ucount, k_index.h): partial[i*K + p] = weight of
// the non-shared entries credited to position p (finalize gathers it for every candidate through
// the map). Within a slice every wave holds all positions (8 per lane) and the waves split the
// staged entries: per entry group the LDS reads feed up to 4 candidate pairs, so the loop is
// VALU-dense even when a disk has only a few hundred positions. Then n_shared workgroups
// deciding the shared entries into spart, grid-striding over the jobs (disk with neighbours x
// kShC-candidate slice, k_poll_shared.h).
__device__ __forceinline__ void coverage_poll_body(
    const double2* __restrict__ xy, const double* __restrict__ w,
    const int32_t* __restrict__ off, Grid g, const DiskRec* __restrict__ urec,
    const int* __restrict__ umap, const int* __restrict__ ucount,
    const int4* __restrict__ region, const uint16_t* __restrict__ nbrT,
    const int4* __restrict__ nboxT, const float4* __restrict__ lane4,
    const float* __restrict__ lanexp, const int2* __restrict__ rows,
    const int* __restrict__ ncount, const int* __restrict__ dlist, const int* __restrict__ dcount,
    int* __restrict__ jobctr, int N, int K, const int* __restrict__ mode, double* __restrict__ partial,
    double* __restrict__ spart, int n_shared, int counts, int bits_on, int* __restrict__ dc_out,
    const int* __restrict__ qual, const double2* __restrict__ cost, double ratio)
{
    static_assert(kPollSlots == 2 * kPollPairs, "the hot loop pairs candidate slots");
#ifdef MAC_DIAG
    const uint64_t diag_t0 = __builtin_amdgcn_s_memrealtime();
#endif
    const int bx = blockIdx.x, by = blockIdx.y;
    // the walk the device chose: loaded first, checked once each role's first loads are out
    const int mv = mode ? *mode : kModePoll;
    // launch hints for the next poll (mapped host memory, maxcover.hip): the disks with
    // neighbours (the bit-word kernel) and the most distinct positions of a disk (walk rows)
    if (bx == 0 && by == 0 && dc_out && mv == kModePoll) {
        int um = 0;
        for (int d = threadIdx.x; d < N; d += kPollThreads) um = max(um, ucount[d]);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) um = max(um, __shfl_xor(um, o, kWave));
        __shared__ int sum_[kPollWaves];
        if ((threadIdx.x & (kWave - 1)) == 0) sum_[threadIdx.x / kWave] = um;
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int q = 1; q < kPollWaves; ++q) um = max(um, sum_[q]);
            *(volatile int*)dc_out = dcount[kDcBits] + dcount[kDcOther];
            *((volatile int*)dc_out + 2) = sum_[0] > um ? sum_[0] : um;
        }
    }
    // walk workgroups first: 8 * ceil(N/8) of them, workgroup b on disk (b % 8) * ceil(N/8) + b / 8
    // (the disk index's map, k_index.h: a disk's index outputs are in its XCD's L2); then the
    // shared-entry workgroups. Grid rows past the first: further walk workgroups of the same
    // disks (position slices by, by + gridDim.y, ...); every other role runs in row 0 only
    const int per_xcd = (N + 7) / 8, nwalk = 8 * per_xcd;
    if (by > 0 && bx >= nwalk) return;

    // The shared-entry jobs (disk with neighbours x kShC-candidate slice, k_poll_shared.h) are
    // taken from a counter (the index kernel cleared it) by the shared workgroups and by every
    // walk workgroup once its disk is done: few jobs (separated disks) finish at once, many (a
    // crowded poll) spread over the whole grid.
    // Jobs [0, n_shared) go to the shared workgroups one each, without the counter; the rest are
    // taken as n_shared + counter.
    auto shared_jobs = [&](int first) {
        __shared__ int sjob;
        // fp64 jobs of 64 candidates while the jobs fill the chip, 256 when the disks with
        // neighbours alone would (fewer re-stagings of each region). With more than
        // kBitsMinDisks disks with neighbours the bit-word kernel (k_bits.h, launched next) takes
        // every disk it qualifies for; the jobs of those disks return at once here.
        const int nA = dcount[kDcBits], nB = dcount[kDcOther];
        // (k_or.h shared_route) 0: every disk with neighbours here; 1: the bit-word kernel takes
        // the qualifying disks (the rest here); 2: the union pass takes every disk
        const int route = lane4 != nullptr ? shared_route(dcount, bits_on, counts, K) : 0;
        const int nlist = route == 1 ? nB : route == 2 ? 0 : nA + nB;   // list position q: dlist[N-1-q], then dlist[q-nB]
        const int C = nlist * ((K + kShC - 1) / kShC) > 2 * (int)gridDim.x ? kShCWide : kShC;
        const int nsub = (K + C - 1) / C;
        const int total = nlist * nsub;
        int job = first;
        for (;;) {
            if (job < 0) {
                if (threadIdx.x == 0) sjob = n_shared + atomicAdd(jobctr, 1);
                __syncthreads();
                job = sjob;
                __syncthreads();
            }
            if (job >= total) break;   // uniform
            const int ql = job / nsub;
            const int di = ql < nB ? dlist[N - 1 - ql] : dlist[ql - nB];
                poll_shared_job(xy, w, off, g, urec, umap, region, nbrT, nboxT, rows, ncount,
                                di, K, (job % nsub) * C, C, spart, counts);
            job = -1;
        }
    };
    if (bx >= nwalk) {  // then: the shared entries
        if (mv != kModePoll) return;
        if (bx == nwalk && cost && dc_out) {
            // launch hint for the next poll: the walk AUTO would choose now that the neighbour
            // lists exist (k_poll_shared.h walk_choice); the host launches the per-candidate walk's
            // kernel after a poll that would have chosen it (maxcover.hip enqueue_eval)
            const int m = walk_choice(N, K, cost, ncount, ratio, 0);
            if (threadIdx.x == 0) *((volatile int*)dc_out + 4) = m;
        }
        shared_jobs(bx - nwalk);
        MAC_DIAG_STAMP(diag_t0, 2, (uint64_t)(dcount[kDcBits] + dcount[kDcOther]));
        return;
    }
    do {  // the walk of disk bx (break: nothing more to credit)
#ifdef MAC_DIAG
    int diag_entries = 0;
#endif
    // s32: (Q, U, V, 0) per staged entry, (+inf, 0, 0) for shared / non-finite / pad; s64: exact
    // coordinates (band decisions); red: per-wave credit of each position, used only between
    // slices, over the staging area
    constexpr int kStageBytes = (kPollCH + 4) * (int)sizeof(float4) + kPollCH * (int)sizeof(double2);
    constexpr int kRedBytes = kPollWaves * kPollKPB * (int)sizeof(double);
    static_assert(kRedBytes <= kStageBytes, "red aliases the staging arrays");
    __shared__ __attribute__((aligned(16))) unsigned char stage[kStageBytes];
    float4* const s32 = (float4*)stage;
    double2* const s64 = (double2*)(stage + (kPollCH + 4) * sizeof(float4));
    double (*const red)[kPollKPB] = (double (*)[kPollKPB])stage;
    __shared__ double sw[kPollCH];
    __shared__ int rs[kPollRB], rpre[kPollRB + 1];
    __shared__ int4 nbox[kPollNbr];

    const int i = (bx % 8) * per_xcd + bx / 8;
    if (i >= N) break;   // uniform: a padding workgroup (takes shared jobs below)
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
    const int64_t row = (int64_t)i * K;
    // One memory round trip for everything indexed by disk i, loaded speculatively (bounds are
    // checked once it has arrived): the position count, region, neighbour count and boxes, the
    // region's row descriptors and the first slice's lane constants (k_index.h).
    const int U = ucount[i];
    const int4 R = region[i];
    const int nc = ncount[i];
    const int2 rinfo = tid <= kRowInfo ? rows[(int64_t)i * (kRowInfo + 1) + tid] : make_int2(0, 0);
    const int4 nb = tid < kPollNbr ? nboxT[i * kPollNbr + tid] : make_int4(0, 0, 0, 0);
    // every wave holds every position of a slice: p = kb + 64 s + lane (slot s); the waves split
    // the staged entries instead (groups of 4, wave w takes groups w, w + 4, ...). Per slot: the
    // lane constants as pair vectors (slots 2j, 2j+1) and X'.
    f32x2 sa[kPollPairs], sb[kPollPairs], st[kPollPairs], ns[kPollPairs];
    float xp[kPollSlots];
    auto load_lanes = [&](int kb) {   // speculative: any p < K is allocated
#pragma unroll
        for (int u = 0; u < kPollSlots; ++u) {
            const int p = kb + u * kWave + lane;
            const float4 c = p < K ? lane4[row + p] : make_float4(0.0f, 0.0f, -1.0f, -1.0f);
            xp[u] = p < K ? lanexp[row + p] : -1.0f;
            const int j = u >> 1;
            if (u & 1) {
                sa[j].y = c.x;
                sb[j].y = c.y;
                st[j].y = c.z;
                ns[j].y = c.w;
            } else {
                sa[j].x = c.x;
                sb[j].x = c.y;
                st[j].x = c.z;
                ns[j].x = c.w;
            }
        }
    };
    const int kb0 = by * kPollKPB;   // this workgroup's first position slice
    if (by > 0 && kb0 >= U) break;     // uniform: no slice of this disk for this row
    load_lanes(kb0);
    if (mv != kModePoll) return;       // (after the first loads: the check costs no round trip)
    // the union pass (launched next, k_or.h) adds its counts into spart row i of every disk
    // with neighbours (finalize reads those rows)
    if (by == 0 && counts && nc > 0 && shared_route(dcount, bits_on, counts, K) == 2)
        for (int k = tid; k < K; k += kPollThreads) reinterpret_cast<unsigned*>(spart)[row + k] = 0u;
    if (R.x > R.y) {  // disk i covers nothing in any candidate (uniform across the block)
        if (by > 0)
            ;   // row 0 writes the zeros
        else if (counts)
            for (int p = tid; p < U; p += kPollThreads) reinterpret_cast<unsigned*>(partial)[row + p] = 0u;
        else
            for (int p = tid; p < U; p += kPollThreads) partial[row + p] = 0.0;
        break;
    }
    if (tid < min(nc, kPollNbr)) nbox[tid] = nb;
    // regions of at most kRowInfo rows (every MADS poll) take their row runs from the index
    const int nrows = R.w - R.z + 1;
    const bool fastrows = nrows <= kRowInfo;
    if (fastrows && tid <= nrows) {
        rs[tid] = rinfo.x;
        rpre[tid] = rinfo.y;
    }
    __syncthreads();

    // region centre: the origin of the staged offsets and of the index's lane constants
    const double ox = g.gx0 + 0.5 * (double)(R.x + R.y + 1) * g.S;
    const double oy = g.gy0 + 0.5 * (double)(R.z + R.w + 1) * g.S;

    // slices of kPollKPB positions (one for any MADS poll: a few hundred distinct disks)
    for (int kb = kb0; kb < U; kb += (int)gridDim.y * kPollKPB) {
        const int ke = min(U, kb + kPollKPB);
        MAC_WALK_STAMP(0);
        if (kb > kb0) load_lanes(kb);
        uint32_t live = 0;
        double acc[kPollSlots];
#pragma unroll
        for (int u = 0; u < kPollSlots; ++u) {
            acc[u] = 0.0;
            if (kb + u * kWave + lane < ke) live |= 1u << u;
            else xp[u] = -1.0f;   // past the slice's last position: never band (its lane
                                  // constants may be another disk's or stale: never credited)
        }
        // candidate pairs with a position (block-uniform)
        const int np = (ke - kb + 2 * kWave - 1) / (2 * kWave);
        // d' of slot u for a staged entry (the hot loop's arithmetic, one candidate)
        auto dprime = [&](const float4& e, int u) {
            const int j = u >> 1;
            const float a_ = (u & 1) ? sa[j].y : sa[j].x, b_ = (u & 1) ? sb[j].y : sb[j].x;
            const float t_ = (u & 1) ? st[j].y : st[j].x, n_ = (u & 1) ? ns[j].y : ns[j].x;
            return __builtin_fmaf(e.x, n_, __builtin_fmaf(e.z, b_, __builtin_fmaf(e.y, a_, t_)));
        };
        MAC_WALK_STAMP(1);

        for (int rb = R.z; rb <= R.w; rb += kPollRB) {
            const int nr = min(kPollRB, R.w - rb + 1);
            if (!fastrows) {  // row runs of this batch from the CSR offsets
                if (tid < nr) {
                    const int64_t rowbase = (int64_t)(rb + tid) * g.nTx;
                    const int s0 = off[rowbase + R.x];
                    rs[tid] = s0;
                    rpre[tid + 1] = off[rowbase + R.y + 1] - s0;
                }
                __syncthreads();
                if (tid < kWave) {  // inclusive scan of the row lengths (nr <= 64: one wave)
                    const int v = wave_incl_scan_i32(tid < nr ? rpre[tid + 1] : 0, tid);
                    if (tid < nr) rpre[tid + 1] = v;
                    if (tid == 0) rpre[0] = 0;
                }
                __syncthreads();
            }
            const int total = rpre[nr];
#ifdef MAC_DIAG
            diag_entries += total;
            if (rb == R.z) MAC_WALK_STAMP(2);
#endif
            for (int base = 0; base < total; base += kPollCH) {
                const int nraw = min(kPollCH, total - base);
                // the chunk's entries disk i may own: shared ones (the shared-entry pass decides
                // them) and non-finite ones (never covered) are left out, the rest compacted in a
                // fixed order (round, wave, lane) so the walk only tests what it can credit
                constexpr int kR = kPollCH / kPollThreads;
                __shared__ int wkeep[kR][kPollWaves];
                double2 pr[kR];
                double wr[kR];
                uint64_t bal[kR];
#pragma unroll
                for (int r = 0; r < kR; ++r) {
                    const int q = tid + r * kPollThreads;
                    bool keep = false;
                    pr[r] = make_double2(0.0, 0.0);
                    wr[r] = 0.0;
                    if (q < nraw) {
                        const int f = base + q;
                        int lo = 0, hi = nr - 1;
                        while (lo < hi) {
                            const int mid = (lo + hi + 1) >> 1;
                            if (rpre[mid] <= f) lo = mid; else hi = mid - 1;
                        }
                        const int j = rs[lo] + (f - rpre[lo]);
                        pr[r] = xy[j];
                        wr[r] = w[j];
                        const bool shared =
                            nc > 0 && entry_shared(nc, nbox, tile_of(pr[r].x, g.gx0, g.invS, g.nTx), rb + lo);
                        // (an entry whose fp32 offset overflows stays: inert for the filter, a
                        // forced lane decides it in fp64)
                        keep = !shared && __builtin_isfinite(pr[r].x) && __builtin_isfinite(pr[r].y);
                    }
                    bal[r] = __ballot(keep);
                    if (lane == 0) wkeep[r][wid] = __popcll(bal[r]);
                }
                __syncthreads();
                int n = 0;
#pragma unroll
                for (int r = 0; r < kR; ++r) {
                    int dst = n + __popcll(bal[r] & ((1ull << lane) - 1));
                    for (int q = 0; q < kPollWaves; ++q) {
                        if (q < wid) dst += wkeep[r][q];
                        n += wkeep[r][q];
                    }
                    if ((bal[r] >> lane) & 1) {
                        s64[dst] = pr[r];
                        sw[dst] = wr[r];
                        const float fu = (float)(pr[r].x - ox), fv = (float)(pr[r].y - oy);
                        s32[dst] = __builtin_isfinite(fu) && __builtin_isfinite(fv)
                                       ? make_float4(__builtin_fmaf(fu, fu, fv * fv), fu, fv, 0.0f)
                                       : make_float4(__builtin_inff(), 0.0f, 0.0f, 0.0f);
                    }
                }
                // pad to a multiple of 4 entries with inert ones (d' = -inf: never counted, never band)
                if (tid < ((4 - (n & 3)) & 3)) s32[n + tid] = make_float4(__builtin_inff(), 0.0f, 0.0f, 0.0f);
                __syncthreads();
                // weights identical across the chunk?
                const uint64_t w0 = __builtin_bit_cast(uint64_t, sw[0]);
                bool mixed = false;
                for (int q = tid; q < n; q += kPollThreads)
                    mixed |= __builtin_bit_cast(uint64_t, sw[q]) != w0;
                const bool uniform = !__syncthreads_or(mixed);
#ifdef MAC_DIAG
                if (rb == R.z && base == 0) MAC_WALK_STAMP(3);
#endif
                const int ng = (n + 3) >> 2;   // groups of 4 entries; this wave: wid, wid + 4, ...
                float bmin[kPollSlots];
#pragma unroll
                for (int u = 0; u < kPollSlots; ++u) bmin[u] = __builtin_inff();
                // band: the lane re-decides this wave's entries of the chunk for slot u; entries
                // with |d'| <= X' in fp64. Shared entries (q = +inf, d' = -inf) are skipped: the
                // shared kernel owns them; for a forced lane (X' = +inf) they are told apart from
                // non-finite ones here.
                auto band = [&](int u) {
                    const DiskRec d = urec[row + kb + u * kWave + lane];
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
                            if (cov) c += counts ? 1.0 : sw[q];
                        }
                    return c;
                };
                if (uniform) {
                    f32x2 h[kPollPairs];
                    switch (np) {   // hot loop: 3 VALU ops per test, np pairs per entry pair
                    case 1: poll_hot<1>(s32, ng, wid, sa, sb, st, ns, h, bmin); break;
                    case 2: poll_hot<2>(s32, ng, wid, sa, sb, st, ns, h, bmin); break;
                    case 3: poll_hot<3>(s32, ng, wid, sa, sb, st, ns, h, bmin); break;
                    default: poll_hot<4>(s32, ng, wid, sa, sb, st, ns, h, bmin); break;
                    }
                    // counts < 2^24: exact in fp32 when no entry is in the band
                    const double wu = sw[0];
#pragma unroll
                    for (int u = 0; u < kPollSlots; ++u) {
                        if (!(live & (1u << u))) continue;
                        const float hc = (u & 1) ? h[u >> 1].y : h[u >> 1].x;
                        acc[u] += bmin[u] <= xp[u] ? band(u) : (counts ? (double)hc : (double)hc * wu);
                    }
                } else {
                    // weighted loop: covered entries add their own weight (clamp(d') is 0 or 1
                    // off the band; a band chunk is recomputed)
                    double cw[kPollSlots];
#pragma unroll
                    for (int u = 0; u < kPollSlots; ++u) cw[u] = 0.0;
                    for (int q4 = wid; q4 < ng; q4 += kPollWaves) {
                        for (int e = 0; e < 4; ++e) {
                            const int q = 4 * q4 + e;
                            const float4 en = s32[q];
                            const double wq = q < n ? sw[q] : 0.0;
#pragma unroll
                            for (int u = 0; u < kPollSlots; ++u) {
                                if ((u >> 1) >= np) continue;
                                const float d = dprime(en, u);
                                cw[u] += d > 0.0f ? wq : 0.0;
                                bmin[u] = __builtin_fminf(bmin[u], __builtin_fabsf(d));
                            }
                        }
                    }
#pragma unroll
                    for (int u = 0; u < kPollSlots; ++u) {
                        if (!(live & (1u << u))) continue;
                        acc[u] += bmin[u] <= xp[u] ? band(u) : cw[u];
                    }
                }
#ifdef MAC_DIAG
                if (rb == R.z && base == 0) MAC_WALK_STAMP(4);
#endif
                __syncthreads();
            }
        }
        // the slice's credit per position: the four waves' shares, added in wave order
#pragma unroll
        for (int u = 0; u < kPollSlots; ++u) red[wid][u * kWave + lane] = acc[u];
        __syncthreads();
        // per position: its credit (equal weights: the covered-entry count, a uint32; finalize
        // reads candidate k's through the map)
        for (int p = tid; p < ke - kb; p += kPollThreads) {
            double a = 0.0;
#pragma unroll
            for (int q = 0; q < kPollWaves; ++q) a += red[q][p];
            if (counts) reinterpret_cast<unsigned*>(partial)[row + kb + p] = (unsigned)a;
            else partial[row + kb + p] = a;
        }
        __syncthreads();
        MAC_WALK_STAMP(5);
    }
    MAC_DIAG_STAMP(diag_t0, 3, ((uint64_t)nc << 40) | ((uint64_t)U << 20) | (uint64_t)diag_entries);
    } while (0);
    if (mv == kModePoll) shared_jobs(-1);
}

// timed entry point (ts: in-kernel launch timing, k_common.h)
__global__ __launch_bounds__(kPollThreads) __attribute__((amdgpu_waves_per_eu(3))) void coverage_poll_kernel(
    uint64_t* ts, const double2* __restrict__ xy, const double* __restrict__ w,
    const int32_t* __restrict__ off, Grid g, const DiskRec* __restrict__ urec,
    const int* __restrict__ umap, const int* __restrict__ ucount,
    const int4* __restrict__ region, const uint16_t* __restrict__ nbrT,
    const int4* __restrict__ nboxT, const float4* __restrict__ lane4,
    const float* __restrict__ lanexp, const int2* __restrict__ rows,
    const int* __restrict__ ncount, const int* __restrict__ dlist, const int* __restrict__ dcount,
    int* __restrict__ jobctr, int N, int K, const int* __restrict__ mode, double* __restrict__ partial,
    double* __restrict__ spart, int n_shared, int counts, int bits_on, int* __restrict__ dc_out,
    const int* __restrict__ qual, const double2* __restrict__ cost, double ratio)
{
    ts_begin(ts);
    coverage_poll_body(xy, w, off, g, urec, umap, ucount, region, nbrT, nboxT, lane4, lanexp, rows,
                       ncount, dlist, dcount, jobctr, N, K, mode, partial, spart, n_shared, counts,
                       bits_on, dc_out, qual, cost, ratio);
    ts_end(ts);
}

}  // namespace mac
