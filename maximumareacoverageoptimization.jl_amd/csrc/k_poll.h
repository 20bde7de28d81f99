// k_poll.h — the poll walk: one workgroup per (disk i, 256 candidates) over a whole MADS poll.
//
// Across one poll, disk i of candidate k sits at x_inc + delta*d_k: a few metres around the
// incumbent. region[i] (k_prep.h) is the union of disk i's tile spans over all K candidates.
// The workgroup stages the entries of region[i] in LDS once (chunks of kPollCH) and every lane
// tests ITS candidate's disk i against every staged entry: one broadcast LDS read per entry per
// wave, no cross-lane reduction, entries read from HBM once per disk instead of once per
// (candidate, disk). An entry is credited to disk i of candidate k only when no lower-index disk
// j of candidate k covers it (j over the disks whose regions overlap region i): exactly-once
// union counting, so the area is the reference's first-hit sum (src/AreaCoverageCalculation.jl:
// 67-78) over the same multiset of entries.
//
// Exact fp32 filter. Entries are staged as fp32 offsets from the region origin o, the lane's
// centre likewise. With eps = 2^-24, |u| <= U for every staged offset and D = U + |c - o| >= |dx|,
// |dy|: |dx32 - dx| <= 2.01 eps D, |a32 - a| <= 12.2 eps D^2 and |a64 - a| <= 6.1 * 2^-53 D^2,
// so with delta = 2^-20 D^2 (> 12.3 eps D^2):
//     a32 <= RD32(T - delta)          =>  a64 <= T   (covered, the reference decision)
//     a32 >  RU32(T + delta)          =>  a64 >  T   (not covered)
//     otherwise (the band)            =>  decided in fp64 from the staged exact coordinates.
// On the reference lattices the band is empty: a = n + 1/2 never lies within delta of T.
// NaN/inf coordinates fail both fp32 tests and every fp64 test, like the reference.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "predicate.h"
#include "k_common.h"

#pragma clang fp contract(off)

namespace mac {

constexpr int kPollCH2 = kPollCH / 2;  // staged fp32 pairs

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

__device__ __forceinline__ bool box_overlap(const int4& a, const int4& b)
{
    return a.x <= a.y && a.x <= b.y && b.x <= a.y && a.z <= b.w && b.z <= a.w;
}

// partialT[i*K + k] = weight of the entries credited to disk i of candidate k.
// Runs when mode == null or *mode == kModePoll.
__global__ __launch_bounds__(kBlock) void coverage_poll_kernel(
    const double2* __restrict__ xy, const double* __restrict__ w,
    const int32_t* __restrict__ off, Grid g, const DiskRec* __restrict__ disksT,
    const int4* __restrict__ region, int N, int K, const int* __restrict__ mode,
    double* __restrict__ partialT)
{
    if (mode && *mode != kModePoll) return;
    __shared__ float4 s32[kPollCH2];   // (rx, ry) of entries 2q, 2q+1
    __shared__ double2 s64[kPollCH];   // exact coordinates (band + ownership tests)
    __shared__ double sw[kPollCH];
    __shared__ int rs[kPollRB], rpre[kPollRB + 1];
    __shared__ uint16_t nbr[kPollNbr];
    __shared__ int ncnt;

    const int i = blockIdx.x;
    const int tid = threadIdx.x;
    const int k = blockIdx.y * kBlock + tid;
    const bool valid = k < K;
    const int4 R = region[i];
    if (R.x > R.y) {  // disk i covers nothing in any candidate (uniform across the block)
        if (valid) partialT[(int64_t)i * K + k] = 0.0;
        return;
    }
    DiskRec d = DiskRec{0.0, 0.0, -1.0, 0.0};
    if (valid) d = disksT[(int64_t)i * K + k];
    int4 sp;
    const bool live = valid && disk_span(d, g, sp);

    // region origin and the bound U on every staged offset |p - o| (entries of tile t satisfy
    // t <= (p - g0)/S < t + 1 up to rounding; two tiles of slack absorb it)
    const double ox = g.gx0 + (double)R.x * g.S;
    const double oy = g.gy0 + (double)R.z * g.S;
    const double U = (double)max(R.y - R.x, R.w - R.z) * g.S + 2.0 * g.S;
    float rcx = 0.0f, rcy = 0.0f, Tlo = -__builtin_inff(), Thi = -__builtin_inff();
    if (live) {
        const double ccx = d.cx - ox, ccy = d.cy - oy;
        const double D = U + __builtin_fmax(__builtin_fabs(ccx), __builtin_fabs(ccy));
        const double delta = D * D * 0x1p-20 + 0x1p-100;
        rcx = (float)ccx;
        rcy = (float)ccy;
        Tlo = f32_down(d.T - delta);
        Thi = f32_up(d.T + delta);
    }

    // lower-index disks whose regions overlap region i (order irrelevant: a boolean OR)
    if (tid == 0) ncnt = 0;
    __syncthreads();
    for (int j = tid; j < i; j += kBlock) {
        const int4 Q = region[j];
        if (box_overlap(Q, R)) {
            const int p = atomicAdd(&ncnt, 1);
            if (p < kPollNbr) nbr[p] = (uint16_t)j;
        }
    }
    __syncthreads();
    const int nc = ncnt;

    // is the entry at exact coordinates p covered by a lower-index disk of candidate k?
    auto stolen = [&](const double2 p) -> bool {
        if (nc <= kPollNbr) {
            for (int u = 0; u < nc; ++u) {
                const DiskRec e = disksT[(int64_t)nbr[u] * K + k];
                if (sqdist(p.x, p.y, e.cx, e.cy) <= e.T) return true;
            }
        } else {
            for (int j = 0; j < i; ++j) {
                if (!box_overlap(region[j], R)) continue;
                const DiskRec e = disksT[(int64_t)j * K + k];
                if (sqdist(p.x, p.y, e.cx, e.cy) <= e.T) return true;
            }
        }
        return false;
    };

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
            float* s32f = (float*)s32;
            for (int q = tid; q < n; q += kBlock) {
                const int f = base + q;
                int lo = 0, hi = nr - 1;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (rpre[mid] <= f) lo = mid; else hi = mid - 1;
                }
                const int j = rs[lo] + (f - rpre[lo]);
                const double2 p = xy[j];
                s64[q] = p;
                sw[q] = w[j];
                s32f[2 * q] = (float)(p.x - ox);
                s32f[2 * q + 1] = (float)(p.y - oy);
            }
            if (tid == 0 && (n & 1)) {  // pad the last pair: NaN is never covered, never in band
                s32f[2 * n] = __builtin_nanf("");
                s32f[2 * n + 1] = __builtin_nanf("");
            }
            __syncthreads();
            const uint64_t w0 = __builtin_bit_cast(uint64_t, sw[0]);
            bool mixed = false;
            for (int q = tid; q < n; q += kBlock) mixed |= __builtin_bit_cast(uint64_t, sw[q]) != w0;
            const bool uniform = !__syncthreads_or(mixed);

            if (live) {
                bool band = false;
                if (nc == 0 && uniform) {
                    // hot loop: two entries per iteration, count the surely covered ones
                    int cnt = 0;
                    const int n2 = (n + 1) >> 1;
                    for (int q2 = 0; q2 < n2; ++q2) {
                        const float4 v = s32[q2];
                        const float dx0 = v.x - rcx, dy0 = v.y - rcy;
                        const float dx1 = v.z - rcx, dy1 = v.w - rcy;
                        const float a0 = __builtin_fmaf(dx0, dx0, dy0 * dy0);
                        const float a1 = __builtin_fmaf(dx1, dx1, dy1 * dy1);
                        cnt += (a0 <= Tlo) + (a1 <= Tlo);
                        band |= (a0 > Tlo) & (a0 <= Thi);
                        band |= (a1 > Tlo) & (a1 <= Thi);
                    }
                    if (cnt) acc += (double)cnt * sw[0];
                } else {
                    const float2* s2 = (const float2*)s32;
                    for (int q = 0; q < n; ++q) {
                        const float2 v = s2[q];
                        const float dx = v.x - rcx, dy = v.y - rcy;
                        const float a = __builtin_fmaf(dx, dx, dy * dy);
                        if (a <= Tlo) {
                            if (nc == 0 || !stolen(s64[q])) acc += sw[q];
                        } else if (a <= Thi) {
                            band = true;
                        }
                    }
                }
                if (band) {  // exact fp64 decision for the band entries (rare)
                    const float2* s2 = (const float2*)s32;
                    for (int q = 0; q < n; ++q) {
                        const float2 v = s2[q];
                        const float dx = v.x - rcx, dy = v.y - rcy;
                        const float a = __builtin_fmaf(dx, dx, dy * dy);
                        if (!(a > Tlo && a <= Thi)) continue;
                        const double2 p = s64[q];
                        if (sqdist(p.x, p.y, d.cx, d.cy) <= d.T && (nc == 0 || !stolen(p)))
                            acc += sw[q];
                    }
                }
            }
            __syncthreads();
        }
    }
    if (valid) partialT[(int64_t)i * K + k] = acc;
}

}  // namespace mac
