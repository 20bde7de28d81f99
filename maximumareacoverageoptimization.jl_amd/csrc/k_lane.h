// k_lane.h — per-candidate constants of the poll walk's scaled fp32 filter (k_poll.h header
// comment): computed once per distinct disk by the index kernel (k_index.h), read by the walk.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "k_common.h"

#pragma clang fp contract(off)

namespace mac {

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

// Inert lane: d' = -Q - 1 < 0 for every entry (never counted), X' = -1 (never in the band).
__device__ __forceinline__ PollLane inert_lane() { return PollLane{0.0f, 0.0f, -1.0f, -1.0f, -1.0f}; }

}  // namespace mac
