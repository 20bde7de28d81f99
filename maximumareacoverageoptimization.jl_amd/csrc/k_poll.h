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
#include "k_final.h"
#include "k_index.h"

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

__device__ __forceinline__ float next_down_f32(float f)
{
    if (f != f || f == -__builtin_inff()) return f;
    if (f == 0.0f) return -__builtin_bit_cast(float, 1u);
    uint32_t b = __builtin_bit_cast(uint32_t, f);
    b = f > 0.0f ? b - 1 : b + 1;
    return __builtin_bit_cast(float, b);
}

__device__ __forceinline__ float next_up_f32(float f)
{
    if (f != f || f == __builtin_inff()) return f;
    if (f == 0.0f) return __builtin_bit_cast(float, 1u);
    uint32_t b = __builtin_bit_cast(uint32_t, f);
    b = f > 0.0f ? b + 1 : b - 1;
    return __builtin_bit_cast(float, b);
}

// largest float <= v (NaN -> -inf: the fast "covered" test then never fires)
__device__ __forceinline__ float f32_down(double v)
{
    if (!(v == v)) return -__builtin_inff();
    float f = (float)v;
    if ((double)f > v) f = next_down_f32(f);
    return f;
}

// smallest float >= v (NaN -> +inf: everything not surely covered goes to the exact pass)
__device__ __forceinline__ float f32_up(double v)
{
    if (!(v == v)) return __builtin_inff();
    float f = (float)v;
    if ((double)f < v) f = next_up_f32(f);
    return f;
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

// clamp to [0, 1] of both halves in one packed op (d' > X' >= 1 -> 1, d' < 0 -> 0)
__device__ __forceinline__ f32x2 clamp01x2(f32x2 x, f32x2 zero)
{
    f32x2 r;
    asm("v_pk_add_f32 %0, %1, %2 clamp" : "=v"(r) : "v"(x), "v"(zero));
    return r;
}

__device__ __forceinline__ f32x2 fma2(float a, f32x2 b, f32x2 c)
{
    return __builtin_elementwise_fma((f32x2)a, b, c);
}

// Per-candidate constants of the scaled fp32 filter (see the header comment).
struct PollLane {
    float sa, sb, stm, ns, xp;   // S*2cu, S*2cv, S*fl32(T - C), -S, X'
};

__device__ __forceinline__ PollLane poll_lane(const DiskRec& d, double ox, double oy, double U)
{
    PollLane L;
    const double cu = d.cx - ox, cv = d.cy - oy;
    const double M = __builtin_fmax(__builtin_fmax(U, d.r),
                                    __builtin_fmax(__builtin_fabs(cu), __builtin_fabs(cv)));
    if (!(M <= 0x1p60 && M >= 0x1p-60)) {  // forced: everything to the exact pass
        L.sa = L.sb = L.stm = 0.0f;
        L.ns = -1.0f;
        L.xp = __builtin_inff();
        return L;
    }
    const float X = f32_up(M * M * 0x1p-18 + 0x1p-120);
    const int ex = (int)((__builtin_bit_cast(uint32_t, X) >> 23) & 0xff) - 127;  // X normal
    const double S = __builtin_ldexp(1.0, -ex);   // S*X in [1, 2)
    const double C = cu * cu + cv * cv;
    L.sa = (float)(2.0 * cu * S);
    L.sb = (float)(2.0 * cv * S);
    L.stm = (float)((d.T - C) * S);
    L.ns = (float)(-S);
    L.xp = (float)((double)X * S);
    return L;
}

__device__ __forceinline__ float poll_dprime(const float4& e, const PollLane& L)
{
    return __builtin_fmaf(e.x, L.ns, __builtin_fmaf(e.z, L.sb, __builtin_fmaf(e.y, L.sa, L.stm)));
}

// Grid (n_chain + n_shared + N, slices); roles by x, in dispatch order (the first ones overlap
// the walk): x < n_chain: objective-penalty chains of candidates [16c, 16c + 16),
// c = y * n_chain + x, into vp (k_final.h), whatever the walk; then, when *mode == kModePoll (or mode == null),
// n_shared x slices workgroups deciding the shared entries into spart, grid-striding over the
// jobs (disk with neighbours x kShC-candidate slice, k_poll_shared.h), and one
// workgroup per (disk i,
// slice g): positions [g*kPollKPB, min(U_i, (g+1)*kPollKPB)) of disk i's distinct disks
// (urec / ucount, k_index.h), thread t pass u ->
// p = kb + 256u + t; partial[i*K + p] = weight of the non-shared entries credited to that disk
// (finalize gathers it for every candidate through the map).
__device__ __forceinline__ void coverage_poll_body(
    const double2* __restrict__ xy, const double* __restrict__ w,
    const int32_t* __restrict__ off, Grid g, const DiskRec* __restrict__ urec,
    const int* __restrict__ umap, const int* __restrict__ ucount,
    const int4* __restrict__ region, const uint16_t* __restrict__ nbrT,
    const int* __restrict__ ncount, const int* __restrict__ dlist, const int* __restrict__ dcount,
    int N, int K, const int* __restrict__ mode, double* __restrict__ partial,
    double* __restrict__ spart, int n_chain, const double* __restrict__ pen, double penalty,
    double* __restrict__ vp, int n_shared)
{
    static_assert(kPollKPL == 4, "the hot loop pairs candidates (0,1) and (2,3)");
#ifdef MAC_DIAG
    const uint64_t diag_t0 = __builtin_amdgcn_s_memrealtime();
#endif
    if ((int)blockIdx.x < n_chain) {  // first: the objective-penalty chains (any walk)
        static_assert(kPollThreads == kBlock, "penalty_chain_block needs kBlock threads");
        const int k0 = (blockIdx.y * n_chain + blockIdx.x) * kChainC;
        if (k0 < K) penalty_chain_block(pen, K, N, k0, penalty, vp);
        MAC_DIAG_STAMP(diag_t0, 1, 0);
        return;
    }
    const int bx = blockIdx.x - n_chain;
    if (mode && *mode != kModePoll) return;
    if (bx < n_shared) {  // then: the shared entries (k_poll_shared.h), over every row
        const int nd = *dcount;
        const int nsub = (K + kShC - 1) / kShC;
        for (int job = blockIdx.y * n_shared + bx; job < nd * nsub; job += n_shared * gridDim.y)
                poll_shared_job(xy, w, off, g, urec, umap, region, nbrT, ncount,
                                dlist[job / nsub], K, (job % nsub) * kShC, spart);
        MAC_DIAG_STAMP(diag_t0, 2, (uint64_t)nd);
        return;
    }
#ifdef MAC_DIAG
    int diag_entries = 0;
#endif
    __shared__ float4 s32[kPollCH + 4];  // (Q, U, V, 0); (+inf, 0, 0) for shared / non-finite / pad
    __shared__ double2 s64[kPollCH];   // exact coordinates (band decisions)
    __shared__ double sw[kPollCH];
    __shared__ int rs[kPollRB], rpre[kPollRB + 1];
    __shared__ int4 nbox[kPollNbr];

    const int i = bx - n_shared;
    const int tid = threadIdx.x;
    // positions p = distinct disks of disk i (k_dedup.h; all K candidates without dedup)
    const int U = ucount[i];
    const int kb = blockIdx.y * kPollKPB;
    if (kb >= U) return;  // uniform: this slice has no position
    MAC_WALK_STAMP(0);
    const int ke = min(U, kb + kPollKPB);
    const int4 R = region[i];
    const int nc = ncount[i];
    const int64_t row = (int64_t)i * K;

    // lane-major positions p = kb + 256u + t: a disk's few hundred distinct disks spread over
    // all four waves first (latency hiding beats packing them into fewer waves)
    int kk[kPollKPL];
#pragma unroll
    for (int u = 0; u < kPollKPL; ++u) {
        const int p = kb + u * kPollThreads + tid;
        kk[u] = p < ke ? p : -1;
    }
    if (R.x > R.y) {  // disk i covers nothing in any candidate (uniform across the block)
#pragma unroll
        for (int u = 0; u < kPollKPL; ++u)
            if (kk[u] >= 0) partial[row + kk[u]] = 0.0;
        return;
    }
    if (tid < min(nc, kPollNbr)) nbox[tid] = region[nbrT[i * kPollNbr + tid]];

    // region centre and the bound Umax on every staged offset (entries of tile t satisfy
    // t <= (p - g0)/S < t + 1 up to rounding; two tiles of slack absorb it)
    const double ox = g.gx0 + 0.5 * (double)(R.x + R.y + 1) * g.S;
    const double oy = g.gy0 + 0.5 * (double)(R.z + R.w + 1) * g.S;
    const double Umax = 0.5 * (double)max(R.y - R.x + 1, R.w - R.z + 1) * g.S + 2.0 * g.S;

    PollLane pl[kPollKPL];
    bool live[kPollKPL];
    double acc[kPollKPL];
#pragma unroll
    for (int u = 0; u < kPollKPL; ++u) {
        acc[u] = 0.0;
        live[u] = false;
        pl[u] = PollLane{0.0f, 0.0f, -1.0f, -1.0f, 0.5f};  // d' < -X' for every entry: inert
        if (kk[u] < 0) continue;
        const DiskRec d = urec[row + kk[u]];
        int4 sp;
        if (!disk_span(d, g, sp)) continue;
        live[u] = true;
        pl[u] = poll_lane(d, ox, oy, Umax);
    }
    // wave-uniform: which candidate pairs have any live lane in this wave
    const bool pair0 = __any(live[0] || live[1]);
    const bool pair1 = __any(live[2] || live[3]);
    const f32x2 zero2 = {0.0f, 0.0f};
    const f32x2 sa01 = {pl[0].sa, pl[1].sa}, sb01 = {pl[0].sb, pl[1].sb};
    const f32x2 st01 = {pl[0].stm, pl[1].stm}, ns01 = {pl[0].ns, pl[1].ns};
    const f32x2 sa23 = {pl[2].sa, pl[3].sa}, sb23 = {pl[2].sb, pl[3].sb};
    const f32x2 st23 = {pl[2].stm, pl[3].stm}, ns23 = {pl[2].ns, pl[3].ns};

    MAC_WALK_STAMP(1);
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
#ifdef MAC_DIAG
        diag_entries += total;
        if (rb == R.z) MAC_WALK_STAMP(2);
#endif
        for (int base = 0; base < total; base += kPollCH) {
            const int n = min(kPollCH, total - base);
            bool mixed = false;
            double wfirst = 0.0;
            for (int q = tid; q < n; q += kPollThreads) {
                const int f = base + q;
                int lo = 0, hi = nr - 1;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (rpre[mid] <= f) lo = mid; else hi = mid - 1;
                }
                const int j = rs[lo] + (f - rpre[lo]);
                const double2 p = xy[j];
                const double wj = w[j];
                s64[q] = p;
                sw[q] = wj;
                const bool shared =
                    nc > 0 && entry_shared(nc, nbox, tile_of(p.x, g.gx0, g.invS, g.nTx), rb + lo);
                const float fu = (float)(p.x - ox), fv = (float)(p.y - oy);
                s32[q] = !shared && __builtin_isfinite(fu) && __builtin_isfinite(fv)
                             ? make_float4(__builtin_fmaf(fu, fu, fv * fv), fu, fv, 0.0f)
                             : make_float4(__builtin_inff(), 0.0f, 0.0f, 0.0f);
                if (q == tid) wfirst = wj;
                mixed |= __builtin_bit_cast(uint64_t, wj) != __builtin_bit_cast(uint64_t, wfirst);
            }
            // pad to a multiple of 4 entries with inert ones (d' = -inf: never counted, never band)
            if (tid < ((4 - (n & 3)) & 3)) s32[n + tid] = make_float4(__builtin_inff(), 0.0f, 0.0f, 0.0f);
            __syncthreads();
            // weights identical across the chunk? (compare with entry 0 after staging)
            const uint64_t w0 = __builtin_bit_cast(uint64_t, sw[0]);
            mixed |= (tid < n) && __builtin_bit_cast(uint64_t, sw[tid]) != w0;
            const bool uniform = !__syncthreads_or(mixed);
#ifdef MAC_DIAG
            if (rb == R.z && base == 0) MAC_WALK_STAMP(3);
#endif

            if (pair0 || pair1) {
                float bmin[kPollKPL];
#pragma unroll
                for (int u = 0; u < kPollKPL; ++u) bmin[u] = __builtin_inff();
                double cw[kPollKPL];   // this chunk's credited weight per candidate
                if (uniform) {
                    // hot loop: 2 entries x 2 candidates per step, 3 VALU ops per test
                    f32x2 h01 = zero2, h23 = zero2;
                    // entries staged as (Q, U, V, 0); bmin updates chained so they form v_min3
#define MAC_POLL_PAIR(E0, E1, SA, SB, ST, NS, H, B0, B1)                                       \
    {                                                                                         \
        const f32x2 d0 = fma2(E0.x, NS, fma2(E0.z, SB, fma2(E0.y, SA, ST)));                   \
        const f32x2 d1 = fma2(E1.x, NS, fma2(E1.z, SB, fma2(E1.y, SA, ST)));                   \
        H += clamp01x2(d0, zero2);                                                            \
        H += clamp01x2(d1, zero2);                                                            \
        B0 = __builtin_fminf(__builtin_fminf(B0, __builtin_fabsf(d0.x)), __builtin_fabsf(d1.x)); \
        B1 = __builtin_fminf(__builtin_fminf(B1, __builtin_fabsf(d0.y)), __builtin_fabsf(d1.y)); \
    }
                    if (pair1) {
                        for (int q = 0; q < n; q += 4) {
                            const float4 e0 = s32[q], e1 = s32[q + 1], e2 = s32[q + 2], e3 = s32[q + 3];
                            MAC_POLL_PAIR(e0, e1, sa01, sb01, st01, ns01, h01, bmin[0], bmin[1])
                            MAC_POLL_PAIR(e0, e1, sa23, sb23, st23, ns23, h23, bmin[2], bmin[3])
                            MAC_POLL_PAIR(e2, e3, sa01, sb01, st01, ns01, h01, bmin[0], bmin[1])
                            MAC_POLL_PAIR(e2, e3, sa23, sb23, st23, ns23, h23, bmin[2], bmin[3])
                        }
                    } else {
                        for (int q = 0; q < n; q += 4) {
                            const float4 e0 = s32[q], e1 = s32[q + 1], e2 = s32[q + 2], e3 = s32[q + 3];
                            MAC_POLL_PAIR(e0, e1, sa01, sb01, st01, ns01, h01, bmin[0], bmin[1])
                            MAC_POLL_PAIR(e2, e3, sa01, sb01, st01, ns01, h01, bmin[0], bmin[1])
                        }
                    }
#undef MAC_POLL_PAIR
                    // counts < 2^24: exact in fp32 when no entry is in the band
                    const double wu = sw[0];
                    cw[0] = (double)h01.x * wu;
                    cw[1] = (double)h01.y * wu;
                    cw[2] = (double)h23.x * wu;
                    cw[3] = (double)h23.y * wu;
                } else {
                    // weighted loop: covered entries add their own weight (clamp(d') is 0 or 1
                    // off the band; a band chunk is recomputed below)
#pragma unroll
                    for (int u = 0; u < kPollKPL; ++u) cw[u] = 0.0;
                    for (int q = 0; q < n; ++q) {
                        const float4 e = s32[q];
                        const double wq = sw[q];
#pragma unroll
                        for (int u = 0; u < kPollKPL; ++u) {
                            const float d = poll_dprime(e, pl[u]);
                            cw[u] += d > 0.0f ? wq : 0.0;
                            bmin[u] = __builtin_fminf(bmin[u], __builtin_fabsf(d));
                        }
                    }
                }
                // band: the lane re-decides this chunk; entries with |d'| <= X' in fp64.
                // Shared entries (q = +inf, d' = -inf) are skipped: the shared kernel owns them;
                // for a forced lane (X' = +inf) they are told apart from non-finite ones here.
#pragma unroll
                for (int u = 0; u < kPollKPL; ++u) {
                    if (live[u] && bmin[u] <= pl[u].xp) {
                        const DiskRec d = urec[row + kk[u]];
                        double c = 0.0;
                        for (int q = 0; q < n; ++q) {
                            const float4 e = s32[q];
                            const float dp = poll_dprime(e, pl[u]);
                            bool cov;
                            if (__builtin_fabsf(dp) <= pl[u].xp) {
                                const double2 p = s64[q];
                                if (e.x == __builtin_inff() && nc > 0 &&
                                    entry_shared(nc, nbox, tile_of(p.x, g.gx0, g.invS, g.nTx),
                                                 tile_of(p.y, g.gy0, g.invS, g.nTy)))
                                    continue;
                                cov = sqdist(p.x, p.y, d.cx, d.cy) <= d.T;
                            } else {
                                cov = dp > 0.0f;
                            }
                            if (cov) c += sw[q];
                        }
                        cw[u] = c;
                    }
                    if (live[u]) acc[u] += cw[u];
                }
            }
#ifdef MAC_DIAG
            if (rb == R.z && base == 0) MAC_WALK_STAMP(4);
#endif
            __syncthreads();
        }
    }
#pragma unroll
    for (int u = 0; u < kPollKPL; ++u)
        if (kk[u] >= 0) partial[row + kk[u]] = acc[u];
    MAC_WALK_STAMP(5);
    MAC_DIAG_STAMP(diag_t0, 3, ((uint64_t)nc << 40) | ((uint64_t)(ke - kb) << 20) | (uint64_t)diag_entries);
}

// timed entry point (ts: in-kernel launch timing, k_common.h)
__global__ __launch_bounds__(kPollThreads) __attribute__((amdgpu_waves_per_eu(4))) void coverage_poll_kernel(
    uint64_t* ts, const double2* __restrict__ xy, const double* __restrict__ w,
    const int32_t* __restrict__ off, Grid g, const DiskRec* __restrict__ urec,
    const int* __restrict__ umap, const int* __restrict__ ucount,
    const int4* __restrict__ region, const uint16_t* __restrict__ nbrT,
    const int* __restrict__ ncount, const int* __restrict__ dlist, const int* __restrict__ dcount,
    int N, int K, const int* __restrict__ mode, double* __restrict__ partial,
    double* __restrict__ spart, int n_chain, const double* __restrict__ pen, double penalty,
    double* __restrict__ vp, int n_shared)
{
    ts_begin(ts);
    coverage_poll_body(xy, w, off, g, urec, umap, ucount, region, nbrT, ncount, dlist, dcount, N, K,
                       mode, partial, spart, n_chain, pen, penalty, vp, n_shared);
    ts_end(ts);
}

}  // namespace mac
