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
// left out here and decided exactly by coverage_poll_shared_kernel (k_poll_shared.h); every
// other entry of region i can only be credited to disk i.
//
// Exact fp32 filter. With o the region origin, u = px - ox, v = py - oy, cu = cx - ox,
// cv = cy - oy: a = (u-cu)^2 + (v-cv)^2 = q - 2u*cu - 2v*cv + C, q = u^2 + v^2, C = cu^2 + cv^2.
// Entries are staged as fp32 (u~, v~, q~); each test is t = fma(v~, -2cv~, fma(u~, -2cu~, q~))
// compared with fp32 thresholds around T - C. With eps = 2^-24, |u|,|v| <= U (every staged
// entry) and D = U + max(|cu|, |cv|): |t - (a - C)| <= 28.2 eps D^2 (q: 10 eps D^2, the two
// products 8.04 eps D^2, the three roundings 10 eps D^2), while the fp64 reference value a64 and
// the fp64 C differ from the real ones by < 2^-50 D^2. So with delta = 2^-18 D^2 (= 64 eps D^2):
//     t <= RD32(T - C - delta)   =>  a64 <= T    covered, the reference decision
//     t >  RU32(T - C + delta)   =>  a64 >  T    not covered
//     otherwise (the band)       =>  decided in fp64 from the staged exact coordinates.
// On the reference lattices the band is empty (a = n + 1/2 never lies within delta of T).
// Non-finite entries (never covered) and shared entries are staged with q = +inf, so t = +inf
// is never NaN and never under a threshold; a lane with D > 2^60 sends every entry to the exact
// pass.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "predicate.h"
#include "k_common.h"
#include "k_poll_shared.h"

#pragma clang fp contract(off)

namespace mac {

#ifdef MAC_DIAG
constexpr uint64_t kDiagMax = 1 << 16;
__device__ uint64_t g_diag[4 * kDiagMax];
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

// c + [t > T] computed as c + sign(T - t): t is never NaN, T never -0, and distinct floats never
// subtract to zero, so the sign bit of T - t is exactly [t > T] (no compare, no VCC hazard).
__device__ __forceinline__ uint32_t count_above(uint32_t c, float T, float t)
{
    return c + (__builtin_bit_cast(uint32_t, T - t) >> 31);
}

// Slice g: candidates [g*kPollKPB, min(K, (g+1)*kPollKPB)); lane t, pass u -> k = kb + u*256 + t.
// partial[i*K + k] = weight of the non-shared entries credited to disk i of candidate k.
// Runs when mode == null or *mode == kModePoll.
__global__ __launch_bounds__(kBlock) void coverage_poll_kernel(
    const double2* __restrict__ xy, const double* __restrict__ w,
    const int32_t* __restrict__ off, Grid g, const DiskRec* __restrict__ disksT,
    const int4* __restrict__ region, const uint16_t* __restrict__ nbrT,
    const int* __restrict__ ncount, int N, int K, const int* __restrict__ mode,
    double* __restrict__ partial)
{
    if (mode && *mode != kModePoll) return;
#ifdef MAC_DIAG
    const uint64_t diag_t0 = __builtin_amdgcn_s_memrealtime();
    int diag_entries = 0;
#endif
    __shared__ float4 s32[kPollCH];    // (u~, v~, q~, 0); q~ = +inf for shared / non-finite
    __shared__ double2 s64[kPollCH];   // exact coordinates (band decisions)
    __shared__ double sw[kPollCH];
    __shared__ int rs[kPollRB], rpre[kPollRB + 1];
    __shared__ int4 nbox[kPollNbr];

    const int i = blockIdx.x;
    const int tid = threadIdx.x;
    const int kb = blockIdx.y * kPollKPB;
    const int ke = min(K, kb + kPollKPB);
    const int4 R = region[i];
    const int nc = ncount[i];

    int kk[kPollKPL];
#pragma unroll
    for (int u = 0; u < kPollKPL; ++u) {
        const int k = kb + u * kBlock + tid;
        kk[u] = k < ke ? k : -1;
    }
    if (R.x > R.y) {  // disk i covers nothing in any candidate (uniform across the block)
#pragma unroll
        for (int u = 0; u < kPollKPL; ++u)
            if (kk[u] >= 0) partial[(int64_t)i * K + kk[u]] = 0.0;
        return;
    }
    if (tid < min(nc, kPollNbr)) nbox[tid] = region[nbrT[i * kPollNbr + tid]];

    // region origin and the bound U on every staged offset (entries of tile t satisfy
    // t <= (p - g0)/S < t + 1 up to rounding; two tiles of slack absorb it)
    const double ox = g.gx0 + (double)R.x * g.S;
    const double oy = g.gy0 + (double)R.z * g.S;
    const double U = (double)max(R.y - R.x, R.w - R.z) * g.S + 2.0 * g.S;

    float m2cx[kPollKPL], m2cy[kPollKPL], Tlo[kPollKPL], Thi[kPollKPL];
    bool live[kPollKPL];
    double acc[kPollKPL];
#pragma unroll
    for (int u = 0; u < kPollKPL; ++u) {
        acc[u] = 0.0;
        live[u] = false;
        m2cx[u] = m2cy[u] = 0.0f;
        Tlo[u] = Thi[u] = -__builtin_inff();
        if (kk[u] < 0) continue;
        const DiskRec d = disksT[(int64_t)i * K + kk[u]];
        int4 sp;
        if (!disk_span(d, g, sp)) continue;
        live[u] = true;
        const double cu = d.cx - ox, cv = d.cy - oy;
        const double D = U + __builtin_fmax(__builtin_fabs(cu), __builtin_fabs(cv));
        if (!(D <= 0x1p60)) {  // keep fp32 far from overflow: exact pass for everything
            Tlo[u] = -__builtin_inff();
            Thi[u] = __builtin_inff();
            continue;
        }
        const double C = cu * cu + cv * cv;
        const double delta = D * D * 0x1p-18 + 0x1p-120;
        m2cx[u] = (float)(-2.0 * cu);
        m2cy[u] = (float)(-2.0 * cv);
        Tlo[u] = f32_down(d.T - C - delta);
        Thi[u] = f32_up(d.T - C + delta);
    }
    bool any_live = false;
#pragma unroll
    for (int u = 0; u < kPollKPL; ++u) any_live |= live[u];
    const bool wave_live = __any(any_live);

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
#endif
        for (int base = 0; base < total; base += kPollCH) {
            const int n = min(kPollCH, total - base);
            bool mixed = false;
            double wfirst = 0.0;
            for (int q = tid; q < n; q += kBlock) {
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
                             ? make_float4(fu, fv, __builtin_fmaf(fu, fu, fv * fv), 0.0f)
                             : make_float4(0.0f, 0.0f, __builtin_inff(), 0.0f);
                if (q == tid) wfirst = wj;
                mixed |= __builtin_bit_cast(uint64_t, wj) != __builtin_bit_cast(uint64_t, wfirst);
            }
            __syncthreads();
            // weights identical across the chunk? (compare with entry 0 after staging)
            const uint64_t w0 = __builtin_bit_cast(uint64_t, sw[0]);
            mixed |= (tid < n) && __builtin_bit_cast(uint64_t, sw[tid]) != w0;
            const bool uniform = !__syncthreads_or(mixed);

            if (wave_live) {
                bool band[kPollKPL];
                uint32_t nlo[kPollKPL], nhi[kPollKPL];
#pragma unroll
                for (int u = 0; u < kPollKPL; ++u) nlo[u] = nhi[u] = 0;
                if (uniform) {
                    // hot loop: per staged entry, kPollKPL tests of 2 FMAs + 2 sign-bit counts
#pragma unroll 4
                    for (int q = 0; q < n; ++q) {
                        const float4 e = s32[q];
#pragma unroll
                        for (int u = 0; u < kPollKPL; ++u) {
                            const float t = __builtin_fmaf(e.y, m2cy[u], __builtin_fmaf(e.x, m2cx[u], e.z));
                            nlo[u] = count_above(nlo[u], Tlo[u], t);
                            nhi[u] = count_above(nhi[u], Thi[u], t);
                        }
                    }
#pragma unroll
                    for (int u = 0; u < kPollKPL; ++u) {
                        const int clo = n - (int)nlo[u];
                        if (clo) acc[u] += (double)clo * sw[0];
                    }
                } else {
                    // weighted loop: the surely covered entries add their own weight
#pragma unroll 2
                    for (int q = 0; q < n; ++q) {
                        const float4 e = s32[q];
                        const double wq = sw[q];
#pragma unroll
                        for (int u = 0; u < kPollKPL; ++u) {
                            const float t = __builtin_fmaf(e.y, m2cy[u], __builtin_fmaf(e.x, m2cx[u], e.z));
                            const uint32_t a = count_above(0u, Tlo[u], t);
                            acc[u] += a ? 0.0 : wq;
                            nlo[u] += a;
                            nhi[u] = count_above(nhi[u], Thi[u], t);
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < kPollKPL; ++u) band[u] = nhi[u] != nlo[u];
                // exact fp64 decisions for the band entries (rare; never on reference lattices).
                // Shared and non-finite entries have t = +inf: never in the band unless the lane
                // is fp32-disabled (Thi = +inf), and then the exact test rejects non-finite ones
                // while shared ones are skipped here (decided by the shared kernel).
#pragma unroll
                for (int u = 0; u < kPollKPL; ++u) {
                    if (!band[u]) continue;
                    const DiskRec d = disksT[(int64_t)i * K + kk[u]];
                    for (int q = 0; q < n; ++q) {
                        const float4 e = s32[q];
                        const float t = __builtin_fmaf(e.y, m2cy[u], __builtin_fmaf(e.x, m2cx[u], e.z));
                        if (!(t > Tlo[u] && t <= Thi[u])) continue;
                        const double2 p = s64[q];
                        if (e.z == __builtin_inff() && nc > 0 &&
                            entry_shared(nc, nbox, tile_of(p.x, g.gx0, g.invS, g.nTx),
                                         tile_of(p.y, g.gy0, g.invS, g.nTy)))
                            continue;
                        if (sqdist(p.x, p.y, d.cx, d.cy) <= d.T) acc[u] += sw[q];
                    }
                }
            }
            __syncthreads();
        }
    }
#pragma unroll
    for (int u = 0; u < kPollKPL; ++u)
        if (kk[u] >= 0) partial[(int64_t)i * K + kk[u]] = acc[u];
#ifdef MAC_DIAG
    if (tid == 0) {
        // diagnostic build only: per-workgroup stamps into a buffer nothing else reads
        const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
        const uint64_t b = (uint64_t)blockIdx.y * gridDim.x + blockIdx.x;
        if (b < kDiagMax) {
            g_diag[4 * b + 0] = diag_t0;
            g_diag[4 * b + 1] = t1;
            g_diag[4 * b + 2] = ((uint64_t)nc << 32) | (uint32_t)diag_entries;
            g_diag[4 * b + 3] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));
        }
    }
#endif
}

}  // namespace mac
