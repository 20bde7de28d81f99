// predicate.h — the reference's coverage predicate made exact and cheap, shared by host and
// device code of libmaxcover.
//
// Reference predicate (src/AreaCoverageCalculation.jl:70, also src/CellFunctions.jl:90):
//     sqrt((px - cx)^2 + (py - cy)^2) < r          (Float64, ^2 = x*x, no FMA)
// Let a = fl(fl(dx*dx) + fl(dy*dy)) with dx = fl(px - cx), dy = fl(py - cy). With sqrt
// correctly rounded (IEEE, as Julia's sqrt is), fl(sqrt(a)) < r holds iff a <= T(r), where
// T(r) = RD(m^2) and m = (pred(r) + r) / 2 is the rounding boundary just below r:
//   fl(sqrt a) < r  <=>  fl(sqrt a) <= pred(r)  <=>  sqrt a < m  <=>  a < m^2  <=>  a <= RD(m^2).
// sqrt a == m is impossible: m needs one bit more than a double, so m^2 (an odd 107+-bit
// significand, or below the subnormal range) is never a double. T is computed once per disk
// with integer arithmetic, so every point test is two subtractions, two multiplications,
// one addition and one comparison — and bit-for-bit the reference's decision.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define MAC_HD __host__ __device__ __forceinline__
#else
#define MAC_HD static inline
#endif

#pragma clang fp contract(off)

namespace mac {

constexpr double kDblMax = 1.7976931348623157e308;

// Full 128-bit square of M (M < 2^56) as (hi, lo), portable 32-bit limb arithmetic.
MAC_HD void square_u64(uint64_t M, uint64_t& hi, uint64_t& lo)
{
    const uint64_t ml = M & 0xffffffffull, mh = M >> 32;  // mh < 2^24
    const uint64_t ll = ml * ml;
    const uint64_t mid = (ml * mh) << 1;                    // < 2^57
    const uint64_t mid_lo = mid << 32, mid_hi = mid >> 32;
    lo = ll + mid_lo;
    const uint64_t carry = lo < ll ? 1u : 0u;
    hi = mh * mh + mid_hi + carry;
}

MAC_HD int clz64(uint64_t v) { return v ? __builtin_clzll(v) : 64; }

// T(r): largest double T with (fl(sqrt(a)) < r) <=> (a <= T) for every double a >= 0.
// r <= 0 or NaN: nothing is ever covered -> -1 (a >= +0 or NaN never satisfies a <= -1).
// r = +inf: every finite a is covered -> DBL_MAX (a = inf is not: sqrt(inf) < inf is false).
MAC_HD double cover_threshold(double r)
{
    if (!(r > 0.0)) return -1.0;
    const uint64_t b = __builtin_bit_cast(uint64_t, r);
    const int e = (int)((b >> 52) & 0x7ff);
    const uint64_t f = b & ((1ull << 52) - 1);
    if (e == 0x7ff) return kDblMax;  // +inf (NaN excluded above)
    uint64_t M;
    int F;  // m = M * 2^F exactly, M odd
    if (e == 0) {  // subnormal r = f * 2^-1074: m = (2f - 1) * 2^-1075
        M = 2 * f - 1;
        F = -1075;
    } else {
        const uint64_t R = f | (1ull << 52);
        const int E = e - 1075;  // r = R * 2^E
        if (f == 0 && e > 1) {   // power of two: the gap below r is half the gap above
            M = 4 * R - 1;
            F = E - 2;
        } else {
            M = 2 * R - 1;
            F = E - 1;
        }
    }
    uint64_t hi, lo;
    square_u64(M, hi, lo);
    const int L = hi ? 128 - clz64(hi) : 64 - clz64(lo);  // bit length of M^2
    int s = L - 53;                                        // keep 53 significant bits ...
    const int s_sub = -1074 - 2 * F;                       // ... or stop at the 2^-1074 grid
    if (s_sub > s) s = s_sub;
    if (s < 0) s = 0;  // unreachable (m^2 is never a double); keeps the shift defined
    uint64_t Q;
    if (s >= 128) {
        Q = 0;
    } else if (s >= 64) {
        Q = hi >> (s - 64);
    } else if (s == 0) {
        Q = lo;
    } else {
        Q = (lo >> s) | (hi << (64 - s));
    }
    // Q < 2^53: exact as a double; the scaling is exact (result on the double grid).
    double T = (double)Q;
    int ex = s + 2 * F;
    // ldexp without libm: scale in steps that stay exact.
    while (ex > 0) {
        const int st = ex > 1000 ? 1000 : ex;
        T *= __builtin_bit_cast(double, (uint64_t)(1023 + st) << 52);
        ex -= st;
    }
    while (ex < 0) {
        // Scale down by at most 2^-1000 at a time; the final step lands on the grid exactly
        // because s was chosen so that the result is a multiple of 2^-1074.
        const int st = ex < -1000 ? 1000 : -ex;
        T *= __builtin_bit_cast(double, (uint64_t)(1023 - st) << 52);
        ex += st;
    }
    if (T > kDblMax) T = kDblMax;  // m^2 above the largest double: RD = DBL_MAX
    return T;
}

// The reference's squared distance, rounded exactly as Julia rounds it (no contraction).
MAC_HD double sqdist(double px, double py, double cx, double cy)
{
    const double dx = px - cx;
    const double dy = py - cy;
    return dx * dx + dy * dy;
}

// Tile index of a coordinate on a uniform grid (origin g0, inverse pitch invS, n tiles).
// NaN maps to 0; values are clamped into [0, n-1]. Monotone non-decreasing in v.
MAC_HD int tile_of(double v, double g0, double invS, int n)
{
    double u = (v - g0) * invS;
    if (!(u == u)) return 0;
    u = __builtin_floor(u);
    if (u < 0.0) return 0;
    if (u > (double)(n - 1)) return n - 1;
    return (int)u;
}

// Conservative span [lo, hi] of tiles that can hold a point covered by a disk (centre c,
// radius r) along one axis: any covered point has |p - c| < r(1 + 3*2^-53), and the margin
// below dominates every rounding of (v - g0) * invS for both the disk bound and the point.
// Returns false when no tile can hold a covered point.
MAC_HD bool tile_span(double c, double r, double g0, double invS, int n, int& lo, int& hi)
{
    if (!(c == c) || !(r > 0.0)) return false;         // NaN centre, r <= 0 or NaN: covers nothing
    if (__builtin_isinf(c)) return false;               // distance to every point is inf
    if (__builtin_isinf(r)) { lo = 0; hi = n - 1; return true; }
    const double ulo = ((c - r) - g0) * invS;
    const double uhi = ((c + r) - g0) * invS;
    const double err = (__builtin_fabs(c) + r + __builtin_fabs(g0)) * invS * 1e-14 + 1e-9;
    const double flo = __builtin_floor(ulo - err);
    const double fhi = __builtin_floor(uhi + err);
    if (!(flo == flo) || !(fhi == fhi)) { lo = 0; hi = n - 1; return true; }
    if (fhi < 0.0 || flo > (double)(n - 1)) return false;
    lo = flo < 0.0 ? 0 : (int)flo;
    hi = fhi > (double)(n - 1) ? n - 1 : (int)fhi;
    return true;
}

// Smallest double > d (d finite or -inf); +inf stays +inf.
MAC_HD double next_up(double d)
{
    if (d != d || d == __builtin_inf()) return d;
    if (d == 0.0) return __builtin_bit_cast(double, (uint64_t)1);  // +denorm_min (also for -0)
    uint64_t b = __builtin_bit_cast(uint64_t, d);
    b = d > 0.0 ? b + 1 : b - 1;
    return __builtin_bit_cast(double, b);
}

// cons3 (src/TDM_Constraints.jl:67) rejects when fl(sqrt(s)) > d. With T as above:
// fl(sqrt s) > d  <=>  !(fl(sqrt s) < next_up(d))  <=>  s > T(next_up(d))   (s not NaN;
// NaN s gives false on both sides). d = NaN or +inf never rejects -> +inf sentinel.
MAC_HD double dlim_threshold(double d)
{
    if (d != d || d == __builtin_inf()) return __builtin_inf();
    return cover_threshold(next_up(d));
}

// Can disks (c1, r1) and (c2, r2) share a covered point? Conservative (may say yes when no).
// A shared point p has |c1 - c2| <= |c1 - p| + |p - c2| < (r1 + r2)(1 + 3*2^-53).
MAC_HD bool disks_may_overlap(double x1, double y1, double r1, double x2, double y2, double r2)
{
    if (__builtin_isinf(r1) || __builtin_isinf(r2)) return true;
    const double dx = x1 - x2, dy = y1 - y2;
    const double d2 = dx * dx + dy * dy;
    const double rr = r1 + r2;
    return !(d2 > rr * rr * (1.0 + 1e-9) + 1e-300);
}

}  // namespace mac
