// k_prep.h — the prep launch (penalty chains, fp32 keys, per-disk range records) and the scan's disk records.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "predicate.h"
#include "k_common.h"

#pragma clang fp contract(off)

namespace mac {

// ------------------------------------------------------------------ per-batch disk prep

// Objective-penalty inputs (src/TDM_STATIC_opt.jl:89-97) and the cons3 constraint
// (src/TDM_Constraints.jl:54-75). rmax == null: no penalty term; prev == null: no cons3.
struct PenArgs {
    const double* rmax;
    const double* prev;
    const double* dlimT;   // per UAV: cons3 holds iff s <= dlimT[i] (predicate.h dlim_threshold)
    const double* dlim;    // ... or the raw d_lim[i], thresholded where it is read (dlimT == null)
    double tan_half_fov;
};

// UAV i's cons3 threshold: dlimT[i], or dlim_threshold(d_lim[i]) (evaluated once per disk by the
// callers that loop over candidates, so the device API needs no threshold launch of its own)
__device__ __forceinline__ double pen_threshold(const PenArgs& pa, int i)
{
    if (!pa.prev) return 0.0;
    return pa.dlimT ? pa.dlimT[i] : dlim_threshold(pa.dlim[i]);
}

// Term i of candidate (x_i, y_i, R_i): |R_i - rmax_i| (0 without rmax), or -1 when UAV i's move
// violates cons3 (sqrt(dx^2 + dy^2 + dz^2) > d_lim[i], z = R / tan(FOV/2), evaluated exactly as
// s > T3 = pen_threshold(pa, i)). A negative term marks the candidate infeasible; the finalize
// chain sums the others sequentially in i (bit-exact with the reference's loop).
__device__ __forceinline__ double pen_term(double x2, double y2, double R2, int i, int N,
                                           const PenArgs& pa, double T3)
{
    if (pa.prev) {
        const double x1 = pa.prev[i], y1 = pa.prev[N + i], z1 = pa.prev[2 * N + i] / pa.tan_half_fov;
        const double z2 = R2 / pa.tan_half_fov;
        const double ddx = x1 - x2, ddy = y1 - y2, ddz = z1 - z2;
        const double s = ddx * ddx + ddy * ddy + ddz * ddz;
        if (s > T3) return -1.0;
    }
    return pa.rmax ? __builtin_fabs(R2 - pa.rmax[i]) : 0.0;
}

// Whether UAV i's diagonal LTMADS steps reject every candidate that carries them: with the
// incumbent's value v of one of UAV i's variables (q = 0 x, 1 y, 2 r), both v + b and v - b (b =
// 2^ell; the generator's x +- entry with entry = +-b gives exactly these doubles) put that
// variable's own term of cons3's sum above T3. The sum dx^2 + dy^2 + dz^2 in floating point is at
// least each of its terms (adding non-negative terms is monotone under rounding), so the whole
// candidate fails cons3 then, whatever its other entries. Every variable is the diagonal of one
// column of B, so when this holds for all 3N variables no candidate of the poll passes cons3.
// pen_term's arithmetic (x1 - x2, z = R / tan(FOV/2), z1 - z2).
__host__ __device__ __forceinline__ bool diag_rejects(double v, double b, double p, int q,
                                                      double tan_half_fov, double T3)
{
    bool all = true;
#pragma unroll
    for (int sg = 0; sg < 2; ++sg) {
        const double c = sg == 0 ? v + b : v - b;
        double d;
        if (q < 2) {
            d = p - c;
        } else {
            const double z1 = p / tan_half_fov, z2 = c / tan_half_fov;
            d = z1 - z2;
        }
        const double sq = d * d;
        all = all && sq > T3;
    }
    return all;
}

// ------------------------------------------------------------------ candidate sources

// splitmix64 stream value number `idx` (1-based) after `state` (workloads.SplitMix64).
__host__ __device__ __forceinline__ uint64_t splitmix_at(uint64_t state, uint64_t idx)
{
    uint64_t z = state + idx * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__host__ __device__ __forceinline__ double splitmix_uniform_at(uint64_t state, uint64_t idx)
{
    return (double)(splitmix_at(state, idx) >> 11) * (1.0 / 9007199254740992.0);
}

// Entry (r, c) of the lower-triangular LTMADS matrix L drawn from the stream at `state`
// (workloads.ltmads_basis): diagonal sign(u_{r+1} < 0.5 ? -1 : 1) * 2^ell; strictly lower
// entries uniform integers in [-(2^ell - 1), 2^ell - 1] from stream values n + 1 + r(r-1)/2 + c
// (numpy's tril_indices order); zero above the diagonal.
__host__ __device__ __forceinline__ double ltmads_entry(uint64_t state, int64_t n, int64_t b,
                                                        int64_t r, int64_t c)
{
    if (r < c) return 0.0;
    if (r == c) return (splitmix_uniform_at(state, (uint64_t)r + 1) < 0.5 ? -1.0 : 1.0) * (double)b;
    const int64_t lo = -b + 1, span = 2 * b - 1;
    const double u = splitmix_uniform_at(state, (uint64_t)(n + 1 + r * (r - 1) / 2 + c));
    return (double)(lo + (int64_t)__builtin_floor(u * (double)span));
}

// The native MADS loop's state on the device when its polls are pipelined (maxcover.hip
// mads_run_pipelined): the finalize of poll t applies poll t's update (k_final.h mads_step) and
// poll t + 1's launches read the mesh index from here, so the host enqueues polls ahead of their
// outcomes. ell < 0 (the mesh precision limit) stops the loop: every later launch returns at once.
// A poll that cons3 rejects whole (skip = 1, written by the poll's prep launch: every variable's
// diagonal step ±2^ell alone violates its UAV's d_lim, k_prep.h poll_rejected) is a failure with
// no evaluation: the launches after the prep return at once and the finalize applies the failure
// update. feas counts the candidates that pass cons3 (the evaluations the reference makes).
struct MadsState {
    double f;      // objective at the incumbent
    int64_t it;    // polls applied
    int ell;       // mesh index of the next poll (step 2^ell)
    int skip;      // the current poll is rejected whole (set by its prep launch)
    unsigned long long feas;   // candidates evaluated (passing cons3)
    int64_t skipped;           // polls rejected whole
    int64_t succ;              // successful polls (the incumbent moved)
};

// Where candidate coordinates come from: a 3N x K column-major matrix (the batch APIs), or a
// complete LTMADS poll around an incumbent generated on the fly (the native MADS driver):
// candidate k < n is x + B[:, k], k >= n is x - B[:, k - n], B = L[rp][:, cp] (variable v of a
// candidate = x_i for v = i, y_i for v = N + i, r_i for v = 2N + i).
struct CandSrc {
    const double* cands;   // matrix source when non-null
    int ldc;
    const uint32_t* keysP; // packed integer keys, one row per disk (the prep launch), when non-null
    const float* keysT;    // ... and the fp32 keys of the escaped values, variable-major rows
    int ldk;               // row pitch of both (keys_ld(K))
    const double* xinc;    // generator: incumbent (3N), row / column permutations (n each)
    const int* rp;
    const int* cp;
    uint64_t state;
    int64_t b;             // 2^ell
    int k0;                // generator: candidate k of this source is candidate k0 + k of the poll
                           // (a rank's shard of it)
    const MadsState* mst;  // generator, pipelined MADS loop: b from the device state (else null)
    // the basis form (mac_poll_basis_f64: a caller-owned poll, DirectSearch's B = L[rp][:, cp] and
    // mesh size delta, src/TDM_STATIC_opt.jl:22-44): L's lower triangle packed by rows (int16,
    // entry (r, c <= r) at r(r+1)/2 + c) and B's entries delta * L instead of the stream's draws
    // (null: the stream). b is then a bound on |L| (the index's int16 table) and delta scales it.
    const int16_t* ltri;
    double delta;
    // (host only) the chain a generated poll takes under MAC_CHAIN_AUTO: 1 = the five-launch chain
    // (the host found the poll crowded: maxcover.hip host_crowded_disks), 0 = AUTO's history
    int route_five;
    // Called at the top of every launch that reads the source: b = 2^ell from the device state;
    // false once the loop has stopped, or (launches after the prep: any_poll false) when the
    // prep rejected the poll whole (the launch returns at once). Uniform per workgroup.
    __device__ __forceinline__ bool resolve(bool any_poll = false)
    {
        if (!mst) return true;
        const int e = mst->ell;
        if (e < 0 || (!any_poll && mst->skip)) return false;
        b = (int64_t)1 << e;
        return true;
    }
    // B's entry (r, c) of a generated poll (n = 3N): the stream's LTMADS draw, or delta * L[r][c]
    __device__ __forceinline__ double entry(int n, int r, int c) const
    {
        if (ltri) return r < c ? 0.0 : delta * (double)ltri[(int64_t)r * (r + 1) / 2 + c];
        return ltmads_entry(state, n, b, r, c);
    }
    __device__ __forceinline__ double get(int kl, int v, int N) const
    {
        if (cands) return cands[(int64_t)kl * ldc + v];
        const int n = 3 * N;
        const int k = kl + k0;
        const int kk = k < n ? k : k - n;
        const double d = entry(n, rp[v], cp[kk]);
        return k < n ? xinc[v] + d : xinc[v] - d;
    }
};

// ------------------------------------------------------------------ the prep launch
// The first launch of every evaluation: workgroup cw takes candidates [8cw, 8cw + 8), thread u
// UAV u of each block of kPrepU UAVs, and reads that UAV's (x, y, r) of its 8 candidates — 24
// coalesced loads, all in flight at once — from the 3N x K matrix as Julia hands it over (or the
// LTMADS generator). The matrix is read once per evaluation, here; from those values:
//   objective (vp != null): term_i = |R_i - rmax_i|, or -1 when UAV i's move fails cons3
//     (pen_term's arithmetic), into LDS; lane c of wave 0 folds candidate 8cw + c's terms IN
//     ORDER i = 0, 1, ..., N-1 from 0.0, as src/TDM_STATIC_opt.jl:88-92 does (bit-exact): one
//     lane per chain. vp[k] = violation * penalty, or +inf when a term is negative (the extreme
//     barrier of src/TDM_Constraints.jl:54-75);
//   poll walk (prec != null): one 16-B record per (workgroup, UAV), prec[cw*N + i] (a
//     coalesced store): {x range, y range, span-area estimate, key flag}. The range is a tile box
//     containing the tile span (predicate.h tile_span) of every one of the 8 disks,
//     from min(c - r), max(c + r) and max(|c| + r) per axis: tile_span's rounding steps are
//     monotone in those, so the box bounds each span from outside (a superset region only
//     makes the walk stage or share more entries, never changes a result), packed as two
//     16-bit tile numbers (range_pack); the estimate is the disks' span areas as (2r/S + 1)^2
//     (the walk choice's cost). The disk index reduces disk i's records (k_index.h);
//   keys (keysP != null; matrix or generator): the packed key of each disk (below), relative to
//     candidate 0's, into keysP[i*ldk + k] (8 consecutive words: two 16-B stores); an escaped
//     disk's three fp32 offsets fl32(v - v0) into keysT[v*ldk + k]; the record's key flag is 1
//     when one of those does not reproduce its double bit for bit (k_index.h "Keys": the disk
//     then takes the identity map).
#ifndef MAC_PREP_C
#define MAC_PREP_C 8
#endif
constexpr int kPrepC = MAC_PREP_C;   // candidates per workgroup (a multiple of 4)
constexpr int kPrepU = 512;      // UAVs per block = threads per workgroup

// keysP / keysT row pitch: rows start on 128-B boundaries (and hold every workgroup's kPrepC keys:
// a workgroup writes kPrepC keys from k0 = its index * kPrepC, so 32 must be a multiple of kPrepC
// or the last workgroup's keys would spill into the next row); the chain fold is one wave
static_assert(kPrepC % 4 == 0 && 32 % kPrepC == 0 && kPrepC <= 64,
              "MAC_PREP_C must divide 32 and be a multiple of 4");
__host__ __device__ inline int keys_ld(int K) { return (K + 31) & ~31; }

struct PrepArgs {
    CandSrc src;
    int N, K;
    PenArgs pa;
    double penalty;
    double* vp;                // per-candidate penalty (null: no objective)
    int pair;                  // generated complete polls (K = 2n, n % 4 == 0): workgroup cw takes
                               // x + B[:, k] and x - B[:, k] for k in [4cw, 4cw + 4) (one draw of
                               // each B entry for both: prep_cand)
    int nchain;                // workgroups
    int skip_failed;           // 1: the records leave out cons3 failures (no area is reported for them)
    int4* prec;                // [nchain][N] records (null: no poll walk)
    Grid g;
    uint32_t* keysP;           // packed keys (null: none), one row per disk, pitch ldk
    float* keysT;              // fp32 keys of escaped values, 3N rows of pitch ldk
    int ldk;
    // the fused chain (k_fiw.h; null: none): per workgroup the largest displacement of a disk from
    // candidate 0's over its live candidates {max |x - x0|, max |y - y0|, max r - r0, max r0 - r}
    // (keysP needed; a NaN difference counts as +inf),
    // and one byte per candidate: 1 when it fails cons3 and is left out (skip_failed, N <= kPrepU)
    double4* pd;
    uint8_t* dead8;
    // the pipelined MADS loop with cons3 (null: none): the state whose skip word this launch
    // writes (workgroup 0), the poll being rejected whole when every variable's diagonal step
    // fails (diag_rejects); then every workgroup returns before its records
    MadsState* mst_w;
    unsigned long long* feas;  // += the candidates that pass cons3 (null: not counted)
    int* lreset;               // the fused chain's hand-off list count, zeroed for this poll (null: none)
    int xbase;                 // (prep_x_kernel) workgroup cw also takes candidate xbase + cw when < K
};

// The fused chain's prep over a matrix source (prep_x_kernel): kPrepCX candidates per workgroup
// and floor(K / kPrepCX) workgroups, the remainder (fewer than the workgroups) one more each to
// the first. At config 4 (K = 3073) that is 512 workgroups, two on every CU; kPrepC = 8 gives 385,
// two on 129 CUs and one on the rest, and the doubled CUs set the launch's length.
constexpr int kPrepCX = 6;

// Packed keys. Disk i of candidate k is keyed by its offsets (dx, dy, dr) from candidate 0's
// disk. When all three are integers that reproduce the doubles exactly (v0 + (double)d == v bit
// for bit) with |dx|, |dy| <= 1023 and |dr| <= 511 — every MADS poll on the granular mesh up to
// step 2^9 — the key is one 32-bit word (11 + 11 + 10 bits, two's complement); else the word is
// the escape kKeyEsc (r field -512) and the value's three fp32 offsets go to the keysT rows
// (k_index.h "Keys"). Either encoding satisfies v == v0 + (double)key, so equal keys still mean
// equal disks; the index reads one word per candidate instead of three.
constexpr uint32_t kKeyEsc = 0x200u << 22;
__device__ __forceinline__ bool key_int(double v, double b, double lim, int& d)
{
    const double f = v - b;
    if (!(f >= -lim && f <= lim)) return false;   // (NaN: false)
    d = (int)f;
    return (double)d == f && __builtin_bit_cast(uint64_t, b + (double)d) == __builtin_bit_cast(uint64_t, v);
}
__device__ __forceinline__ uint32_t key_pack(int dx, int dy, int dr)
{
    return ((uint32_t)dx & 0x7FFu) | (((uint32_t)dy & 0x7FFu) << 11) | (((uint32_t)dr & 0x3FFu) << 22);
}
__device__ __forceinline__ void key_unpack(uint32_t p, float& x, float& y, float& r)
{
    x = (float)((int)(p << 21) >> 21);
    y = (float)((int)(p << 10) >> 21);
    r = (float)((int)p >> 22);
}

// the tile range [lo, hi] on one axis covering every span of disks with min(c - r) = a,
// max(c + r) = b, max(|c| + r) = m (tile_span's steps, each monotone); false: empty
__device__ __forceinline__ bool partial_range(double a, double b, double m, double g0, double invS,
                                              int n, int& lo, int& hi)
{
    const double ulo = (a - g0) * invS;
    const double uhi = (b - g0) * invS;
    const double err = (m + __builtin_fabs(g0)) * invS * 1e-14 + 1e-9;
    const double flo = __builtin_floor(ulo - err);
    const double fhi = __builtin_floor(uhi + err);
    if (!(flo == flo) || !(fhi == fhi)) { lo = 0; hi = n - 1; return true; }
    if (fhi < 0.0 || flo > (double)(n - 1)) return false;
    lo = flo < 0.0 ? 0 : (int)flo;
    hi = fhi > (double)(n - 1) ? n - 1 : (int)fhi;
    return true;
}

// A tile range [lo, hi] of an axis of n tiles as two 16-bit numbers lo >> s, hi >> s, with s the
// least shift that fits n - 1 below 0xFFFF (0 for every grid of up to 65535 tiles a side);
// unpacking rounds outwards (a superset); the empty range packs as {0xFFFF, 0}, the identity of
// the (min, max) reduction.
__host__ __device__ inline int range_shift(int n)
{
    int s = 0;
    while (((n - 1) >> s) > 0xFFFE) ++s;
    return s;
}
__device__ __forceinline__ uint32_t range_pack(bool any, int lo, int hi, int s)
{
    return any ? (uint32_t)(lo >> s) | ((uint32_t)(hi >> s) << 16) : 0xFFFFu;
}
__device__ __forceinline__ void range_unpack(uint32_t lo16, uint32_t hi16, int s, int n, int& lo, int& hi)
{
    lo = (int)(lo16 << s);
    hi = min((int)(((hi16 + 1) << s) - 1), n - 1);
}

#ifdef MAC_DIAG
__device__ uint64_t g_diag_prep[64 * 16];   // diagnostic build only: workgroup phase stamps
#define MAC_PREP_STAMP_T(q, t) if (threadIdx.x == (t) && cw < 64 && (q) < 16) g_diag_prep[16 * cw + (q)] = __builtin_amdgcn_s_memrealtime()
#else
#define MAC_PREP_STAMP_T(q, t)
#endif
#define MAC_PREP_STAMP(q) MAC_PREP_STAMP_T(q, 0)

// A workgroup barrier for LDS only: global stores still in flight are not waited for
// (__syncthreads would drain them first)
__device__ __forceinline__ void lds_barrier()
{
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// the workgroup's LDS (one block for both source kinds: their instantiations would each
// declare their own)
template <int PC>   // (PC: candidate slots per workgroup)
struct PrepLds {
    double term[PC][kPrepU + 2];   // [candidate][UAV]; rows 16-B aligned (the fold reads pairs),
                                   // 4 banks apart (+2)
    int wbad[kPrepU / kWave][PC];  // per wave: a term of the candidate is negative
    uint32_t wbadm[kPrepU / kWave];   // ... wbad as a mask over the candidates
    int wrej[kPrepU / kWave];         // per wave: every UAV's diagonal steps fail (mst_w)
    double dred[kPrepU / kWave][4];   // per wave: its share of the displacement bound
};

template <bool kMat, int PC>
__device__ __forceinline__ void prep_block(const PrepArgs& a, int cw, unsigned char* lds)
{
    constexpr int NC = PC;   // candidate slots
    PrepLds<NC>& L = *reinterpret_cast<PrepLds<NC>*>(lds);
    auto& term = L.term;
    auto& wbad = L.wbad;
    auto& wbadm = L.wbadm;
    auto& wrej = L.wrej;
    auto& dred = L.dred;
    const int N = a.N, K = a.K;
    const int u = threadIdx.x, lane = u & (kWave - 1), wid = u / kWave;
    const int k0 = cw * PC;
    const int n3 = 3 * N;
    // candidate c of the workgroup: k0 + c, or (pairs) the plus / minus candidates of B's columns
    // [4cw, 4cw + 4): c < 4 -> 4cw + c, c >= 4 -> n + 4cw + c - 4
    auto cand = [&](int c) { return a.pair ? (c < 4 ? 4 * cw + c : n3 + 4 * cw + c - 4) : k0 + c; };
    const bool obj = a.vp != nullptr;
    const PenArgs& pa = a.pa;
    MAC_PREP_STAMP(0);
    double acc = 0.0;   // the chain (lane c of wave 0: candidate k0 + c)
    bool bad = false;   // ... and whether a term of it is negative (cons3)
    // Candidates that fail cons3 (the extreme barrier, src/TDM_Constraints.jl:54-75) are not
    // evaluated by the reference's DirectSearch poll, and their objective is +inf whatever they
    // cover. With one block of UAVs (N <= kPrepU) their failure is known before the records are
    // written, so the records leave them out (the regions, and with them the walks' work, shrink
    // to the feasible candidates; the index maps them to an inert position, k_index.h). Uniform.
    const bool excl = obj && pa.prev && (a.prec || a.pd) && a.skip_failed && N <= kPrepU;
    double dmx = -__builtin_inf(), dmy = -__builtin_inf(), dmr = -__builtin_inf();   // (pd)
    double dml = -__builtin_inf();   // (pd) max r0 - r
    uint32_t dead = 0u;   // (excl) bit c: candidate c fails cons3 (0 otherwise)
    for (int ib = 0; ib < N; ib += kPrepU) {
        const int nb = min(kPrepU, N - ib);
        const int i = ib + u;
        const bool iv = u < nb;
        const int ii = min(i, N - 1);
        double v[NC][3];
        if (!kMat && PC == 8 && a.pair) {
            // x +- B[v][col]: each draw once for the candidate pair (PC == 8: four columns)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int col = 4 * cw + c;
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    const int vv = q * N + ii;
                    const double d = a.src.entry(n3, a.src.rp[vv], a.src.cp[col]);
                    v[c][q] = a.src.xinc[vv] + d;
                    v[c + 4][q] = a.src.xinc[vv] - d;
                }
            }
        } else {
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const int k = min(cand(c), K - 1);
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    if constexpr (kMat) v[c][q] = a.src.cands[(int64_t)k * a.src.ldc + q * N + ii];
                    else v[c][q] = a.src.get(k, q * N + ii, N);
                }
            }
        }
        double base[3] = {0.0, 0.0, 0.0};   // candidate 0's values: the keys' base
        if (a.keysP) {
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                if constexpr (kMat) base[q] = a.src.cands[q * N + ii];
                else base[q] = a.src.get(0, q * N + ii, N);
            }
        }
        if (obj) {
            // pen_term (above), the same operations in the same order
            const double x1 = pa.prev ? pa.prev[ii] : 0.0, y1 = pa.prev ? pa.prev[N + ii] : 0.0;
            const double z1 = pa.prev ? pa.prev[2 * N + ii] / pa.tan_half_fov : 0.0;
            const double rm = pa.rmax ? pa.rmax[ii] : 0.0;
            const double T3 = pen_threshold(pa, ii);
            uint32_t wdead = 0u;   // this wave's part of the failures
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const double R2 = v[c][2];
                double t = pa.rmax ? __builtin_fabs(R2 - rm) : 0.0;
                if (pa.prev) {
                    const double z2 = R2 / pa.tan_half_fov;
                    const double ddx = x1 - v[c][0], ddy = y1 - v[c][1], ddz = z1 - z2;
                    const double sq = ddx * ddx + ddy * ddy + ddz * ddz;
                    if (sq > T3) t = -1.0;
                }
                term[c][u] = t;
                const uint64_t neg = __ballot(iv && t < 0.0);
                if (lane == 0) wbad[wid][c] = neg != 0;
                wdead |= (neg != 0 ? 1u : 0u) << c;
            }
            if (lane == 0) wbadm[wid] = wdead;
            if (a.mst_w) {   // (excl, one block of UAVs: uniform) the whole-poll rejection
                bool rej = true;
                if (iv) {
                    const double bb = (double)a.src.b;
                    rej = diag_rejects(a.src.xinc[ii], bb, x1, 0, pa.tan_half_fov, T3) &&
                          diag_rejects(a.src.xinc[N + ii], bb, y1, 1, pa.tan_half_fov, T3) &&
                          diag_rejects(a.src.xinc[2 * N + ii], bb, pa.prev[2 * N + ii], 2, pa.tan_half_fov, T3);
                }
                const uint64_t keep = __ballot(!rej);
                if (lane == 0) wrej[wid] = keep == 0;
            }
            MAC_PREP_STAMP(1 + 3 * (ib / kPrepU));
            lds_barrier();   // every wave's terms and failures
            if (excl) {   // (the records below leave the failures out)
                dead = 0u;
#pragma unroll
                for (int w = 0; w < kPrepU / kWave; ++w) dead |= wbadm[w];
                if (a.mst_w) {
                    bool rej = true;
#pragma unroll
                    for (int w = 0; w < kPrepU / kWave; ++w) rej = rej && wrej[w] != 0;
                    if (cw == 0 && u == 0) a.mst_w->skip = rej ? 1 : 0;
                    if (rej) return;   // (uniform) the later launches see skip and return
                }
            }
            if (u < NC) {
                // the chain, sequential in UAV order: lane c of wave 0 folds candidate slot c
                // while the other waves go on to the bound and the keys below (wave 0 does its own
                // share of them after the fold, which sets the launch's length)
#pragma unroll
                for (int w = 0; w < kPrepU / kWave; ++w) bad |= wbad[w][u] != 0;
                if (!bad) {   // (a cons3 failure's vp is +inf: no chain to fold)
                    // the chain's wave first at issue: the dependent adds are the launch's
                    // critical path, the other waves on its SIMD have slack
                    __builtin_amdgcn_s_setprio(3);
                    // batches of 2 kB terms (pair reads), the next batch's reads in flight while
                    // this batch's adds run: the dependent adds, not the LDS latency, set the pace
                    constexpr int kB = 3;   // (the most that fits 128 VGPRs beside v)
                    const double2* row2 = reinterpret_cast<const double2*>(&term[u][0]);
                    const int nfull = nb / (2 * kB);
                    // ping-pong buffers (no register moves between batches); the reads past the
                    // last batch re-read it (clamped) and are never added
                    auto batch = [&](double2 (&buf)[kB], int bt) {
                        const int at = (bt < nfull ? bt : nfull - 1) * kB;
#pragma unroll
                        for (int j = 0; j < kB; ++j) buf[j] = row2[at + j];
                    };
                    auto add = [&](const double2 (&buf)[kB]) {
#pragma unroll
                        for (int j = 0; j < kB; ++j) {
                            acc += buf[j].x;
                            acc += buf[j].y;
                        }
                    };
                    if (nfull > 0) {
                        double2 A[kB], B[kB];
                        batch(A, 0);
#pragma unroll 1
                        for (int bt = 0; bt < nfull; bt += 2) {
                            batch(B, bt + 1);
                            __builtin_amdgcn_sched_barrier(0);   // (the reads stay ahead of the adds)
                            add(A);
                            if (bt + 1 >= nfull) break;
                            batch(A, bt + 2);
                            __builtin_amdgcn_sched_barrier(0);
                            add(B);
                        }
                    }
                    for (int q = nfull * 2 * kB; q < nb; ++q) acc += term[u][q];
                    __builtin_amdgcn_s_setprio(0);
                }
            }
            MAC_PREP_STAMP(2 + 3 * (ib / kPrepU));
        }
        if (a.pd && a.keysP && iv) {
            // the fused chain's displacement bound (k_fiw.h sup_box): over this workgroup's live
            // candidates (the ones the records below would take), a NaN difference counts as +inf
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const double x = v[c][0], y = v[c][1], r = v[c][2];
                if (cand(c) < K && !((dead >> c) & 1u) && r > 0.0 && __builtin_isfinite(x) &&
                    __builtin_isfinite(y)) {
                    double ex = __builtin_fabs(x - base[0]), ey = __builtin_fabs(y - base[1]), er = r - base[2];
                    double el = base[2] - r;
                    if (!(ex <= kDblMax)) ex = __builtin_inf();
                    if (!(ey <= kDblMax)) ey = __builtin_inf();
                    if (!(er == er)) er = __builtin_inf();
                    if (!(el == el)) el = __builtin_inf();
                    dmx = fmax(dmx, ex);
                    dmy = fmax(dmy, ey);
                    dmr = fmax(dmr, er);
                    dml = fmax(dml, el);
                }
            }
        }
        if (a.pd && ib + kPrepU >= N) {   // (uniform) this wave's share of the bound, into LDS
            // (thread 0 combines the waves at the end)
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
        }
        if ((a.prec || a.keysP) && iv) {
            double xa = __builtin_inf(), xb = -__builtin_inf(), ya = __builtin_inf(), yb = -__builtin_inf();
            double xm = 0.0, ym = 0.0, est = 0.0;
            bool any = false;
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                if (!a.prec) break;   // (the fused chain: keys only, no region records)
                const double x = v[c][0], y = v[c][1], r = v[c][2];
                // span_of's cases: r <= 0 or NaN, or a non-finite centre, covers nothing
                if (cand(c) < K && !((dead >> c) & 1u) && r > 0.0 && __builtin_isfinite(x) &&
                    __builtin_isfinite(y)) {
                    any = true;
                    xa = fmin(xa, x - r);
                    xb = fmax(xb, x + r);
                    ya = fmin(ya, y - r);
                    yb = fmax(yb, y + r);
                    xm = fmax(xm, __builtin_fabs(x) + r);
                    ym = fmax(ym, __builtin_fabs(y) + r);
                    const double e = 2.0 * r * a.g.invS + 1.0;
                    est += e * e;
                }
            }
            bool kb = false;   // a key of this disk is inexact (k_index.h "Keys")
            if (a.keysP) {     // the keys: packed words (two 16-B stores), escapes in fp32
                uint32_t pk[NC];
#pragma unroll
                for (int c = 0; c < NC; ++c) {
                    int dx = 0, dy = 0, dr = 0;
                    const bool packs = key_int(v[c][0], base[0], 1023.0, dx) &&
                                       key_int(v[c][1], base[1], 1023.0, dy) &&
                                       key_int(v[c][2], base[2], 511.0, dr);
                    pk[c] = packs ? key_pack(dx, dy, dr) : kKeyEsc;
                    if (!packs) {
#pragma unroll
                        for (int q = 0; q < 3; ++q) {
                            const float f = (float)(v[c][q] - base[q]);
                            kb |= !((dead >> c) & 1u) && __builtin_bit_cast(uint64_t, base[q] + (double)f) != __builtin_bit_cast(uint64_t, v[c][q]);
                            a.keysT[(int64_t)(q * N + i) * a.ldk + cand(c)] = f;
                        }
                    }
                }
                uint32_t* const krow = a.keysP + (int64_t)i * a.ldk;
#pragma unroll
                for (int h = 0; h < PC / 4; ++h)   // candidates cand(4h) .. cand(4h) + 3
                    *reinterpret_cast<uint4*>(krow + cand(4 * h)) =
                        make_uint4(pk[4 * h], pk[4 * h + 1], pk[4 * h + 2], pk[4 * h + 3]);
            }
            if (a.prec) {
                int x0 = 0, x1 = -1, y0 = 0, y1 = -1;
                any = any && partial_range(xa, xb, xm, a.g.gx0, a.g.invS, a.g.nTx, x0, x1) &&
                      partial_range(ya, yb, ym, a.g.gy0, a.g.invS, a.g.nTy, y0, y1);
                a.prec[(int64_t)cw * N + i] =
                    make_int4((int)range_pack(any, x0, x1, range_shift(a.g.nTx)),
                              (int)range_pack(any, y0, y1, range_shift(a.g.nTy)),
                              __builtin_bit_cast(int, (float)est), kb ? 1 : 0);
            }
        }
        MAC_PREP_STAMP(3 + 3 * (ib / kPrepU));
        if (obj && ib + kPrepU < N) lds_barrier();   // the fold has read the terms
    }
    if (obj && u < NC && cand(u) < K) {
        a.vp[cand(u)] = bad ? __builtin_inf() : acc * a.penalty;
        if (a.dead8) a.dead8[cand(u)] = excl && bad ? 1 : 0;
    }
    if (obj && a.feas && wid == 0) {   // the evaluations: candidates that pass cons3
        const uint64_t ok = __ballot(u < NC && cand(u) < K && !bad);
        if (lane == 0 && ok) atomicAdd(a.feas, (unsigned long long)__popcll(ok));
    }
    if (a.pd) {   // the workgroup's displacement bound: the waves' shares in order
        lds_barrier();
        if (u == 0) {
            double4 m = make_double4(dred[0][0], dred[0][1], dred[0][2], dred[0][3]);
            for (int q = 1; q < kPrepU / kWave; ++q) {
                m.x = fmax(m.x, dred[q][0]);
                m.y = fmax(m.y, dred[q][1]);
                m.z = fmax(m.z, dred[q][2]);
                m.w = fmax(m.w, dred[q][3]);
            }
            a.pd[cw] = m;
        }
    }
}

// The fused chain's prep over a matrix source with one block of UAVs (N <= kPrepU; k_fiw.h):
// kPrepCX candidates per workgroup plus, for the first K - xbase workgroups, candidate xbase + cw
// (slot kPrepCX). Waves 0..7 hold a UAV per thread: loads, penalty terms and cons3 ballots, one
// barrier, then per candidate slot the packed key and the share of the displacement bound, while
// a ninth wave that holds no UAV folds the chains (lane c: slot c's, sequential in UAV order). The
// fold and the keys are exclusive branches, so the candidate values are dead on the folding
// wave's path (80 VGPRs: two workgroups, 18 waves, fit a CU). Results are prep_block's bit for bit
// (the same terms in the same order, the same keys and bound).
template <bool kGen>
__device__ __forceinline__ void prep_block_x(const PrepArgs& a, int cw, unsigned char* lds)
{
    // kGen: a generated complete poll (K = 2n, n = 3N): workgroup cw takes the columns 3cw .. 3cw + 2
    // of B, slots 0-2 their plus candidates (k = col), slots 3-5 their minus candidates (k = n + col),
    // each B entry drawn once for both; N workgroups
    constexpr int PC = kPrepCX, NC = kGen ? kPrepCX : kPrepCX + 1, NW = kPrepU / kWave;
    PrepLds<kPrepCX + 1>& L = *reinterpret_cast<PrepLds<kPrepCX + 1>*>(lds);
    auto& term = L.term;
    auto& wbad = L.wbad;
    auto& wbadm = L.wbadm;
    auto& wrej = L.wrej;
    auto& dred = L.dred;
    const int N = a.N, K = a.K;
    const int u = threadIdx.x, lane = u & (kWave - 1), wid = u / kWave;
    const bool fw = wid == NW;   // the folding wave
    const int k0 = cw * PC;
    const int n3 = 3 * N;
    auto cand = [&](int c) {   // (>= K: absent)
        if constexpr (kGen) return c < 3 ? 3 * cw + c : n3 + 3 * cw + c - 3;
        else return c < PC ? k0 + c : a.xbase + cw;
    };
    const bool obj = a.vp != nullptr;
    const PenArgs& pa = a.pa;
    const bool excl = obj && pa.prev && a.skip_failed;
    const bool iv = !fw && u < N;
    const int ii = min(u, N - 1);
    MAC_PREP_STAMP(0);
    double v[NC][3];
    double base[3] = {0.0, 0.0, 0.0};   // candidate 0's values: the keys' base
    if (!fw) {
        if constexpr (kGen) {
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                const int vv = q * N + ii;
                const int rv = a.src.rp[vv];
                const double xv = a.src.xinc[vv];
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    const double d = a.src.entry(n3, rv, a.src.cp[3 * cw + c]);
                    v[c][q] = xv + d;
                    v[c + 3][q] = xv - d;
                }
                base[q] = xv + a.src.entry(n3, rv, a.src.cp[0]);
            }
        } else {
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const int k = min(cand(c), K - 1);
#pragma unroll
                for (int q = 0; q < 3; ++q) v[c][q] = a.src.cands[(int64_t)k * a.src.ldc + q * N + ii];
            }
#pragma unroll
            for (int q = 0; q < 3; ++q) base[q] = a.src.cands[q * N + ii];
        }
        if (obj) {
            // pen_term (above), the same operations in the same order
            const double x1 = pa.prev ? pa.prev[ii] : 0.0, y1 = pa.prev ? pa.prev[N + ii] : 0.0;
            const double z1 = pa.prev ? pa.prev[2 * N + ii] / pa.tan_half_fov : 0.0;
            const double rm = pa.rmax ? pa.rmax[ii] : 0.0;
            const double T3 = pen_threshold(pa, ii);
            uint32_t wdead = 0u;
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const double R2 = v[c][2];
                double t = pa.rmax ? __builtin_fabs(R2 - rm) : 0.0;
                if (pa.prev) {
                    const double z2 = R2 / pa.tan_half_fov;
                    const double ddx = x1 - v[c][0], ddy = y1 - v[c][1], ddz = z1 - z2;
                    const double sq = ddx * ddx + ddy * ddy + ddz * ddz;
                    if (sq > T3) t = -1.0;
                }
                term[c][u] = t;
                const uint64_t neg = __ballot(iv && t < 0.0);
                if (lane == 0) wbad[wid][c] = neg != 0;
                wdead |= (neg != 0 ? 1u : 0u) << c;
            }
            if (lane == 0) wbadm[wid] = wdead;
            if (a.mst_w) {   // the whole-poll rejection (uniform)
                bool rej = true;
                if (iv) {
                    const double bb = (double)a.src.b;
                    rej = diag_rejects(a.src.xinc[ii], bb, x1, 0, pa.tan_half_fov, T3) &&
                          diag_rejects(a.src.xinc[N + ii], bb, y1, 1, pa.tan_half_fov, T3) &&
                          diag_rejects(a.src.xinc[2 * N + ii], bb, pa.prev[2 * N + ii], 2, pa.tan_half_fov, T3);
                }
                const uint64_t keep = __ballot(!rej);
                if (lane == 0) wrej[wid] = keep == 0;
            }
        }
    }
    MAC_PREP_STAMP(1);
    uint32_t dead = 0u;
    if (obj) {
        lds_barrier();   // every wave's terms and failures
        if (excl) {
#pragma unroll
            for (int w = 0; w < NW; ++w) dead |= wbadm[w];
            if (a.mst_w) {
                bool rej = true;
#pragma unroll
                for (int w = 0; w < NW; ++w) rej = rej && wrej[w] != 0;
                if (cw == 0 && u == 0) a.mst_w->skip = rej ? 1 : 0;
                if (rej) return;   // (uniform) the later launches see skip and return
            }
        }
    }
    MAC_PREP_STAMP(2);
    if (fw) {   // the chains
        bool bad = false;
        double acc = 0.0;
        if (obj && lane < NC) {
#pragma unroll
            for (int w = 0; w < NW; ++w) bad |= wbad[w][lane] != 0;
            if (!bad) {   // (a cons3 failure's vp is +inf: no chain to fold)
                // batches of 2 kB terms (pair reads), the next batch's reads in flight while this
                // batch's adds run; ping-pong buffers, the reads past the last batch re-read it
                // (clamped) and are never added
                constexpr int kB = 6;
                const double2* row2 = reinterpret_cast<const double2*>(&term[lane][0]);
                const int nfull = N / (2 * kB);
                __builtin_amdgcn_s_setprio(3);   // the launch's critical path: first at issue
                auto batch = [&](double2 (&buf)[kB], int bt) {
                    const int at = (bt < nfull ? bt : nfull - 1) * kB;
#pragma unroll
                    for (int j = 0; j < kB; ++j) buf[j] = row2[at + j];
                };
                auto add = [&](const double2 (&buf)[kB]) {
#pragma unroll
                    for (int j = 0; j < kB; ++j) {
                        acc += buf[j].x;
                        acc += buf[j].y;
                    }
                };
                if (nfull > 0) {
                    double2 A[kB], B[kB];
                    batch(A, 0);
#pragma unroll 1
                    for (int bt = 0; bt < nfull; bt += 2) {
                        batch(B, bt + 1);
                        __builtin_amdgcn_sched_barrier(0);   // (the reads stay ahead of the adds)
                        add(A);
                        if (bt + 1 >= nfull) break;
                        batch(A, bt + 2);
                        __builtin_amdgcn_sched_barrier(0);
                        add(B);
                    }
                }
                for (int q = nfull * 2 * kB; q < N; ++q) acc += term[lane][q];
                __builtin_amdgcn_s_setprio(0);
            }
            MAC_PREP_STAMP_T(3, kPrepU);
            if (cand(lane) < K) {
                a.vp[cand(lane)] = bad ? __builtin_inf() : acc * a.penalty;
                if (a.dead8) a.dead8[cand(lane)] = excl && bad ? 1 : 0;
            }
        }
        if (obj && a.feas) {   // the evaluations: candidates that pass cons3
            const uint64_t ok = __ballot(lane < NC && cand(lane) < K && !bad);
            if (lane == 0 && ok) atomicAdd(a.feas, (unsigned long long)__popcll(ok));
        }
    } else {
        // per candidate slot its key word (escapes: the fp32 offsets, k_index.h "Keys") and its
        // share of the displacement bound (k_fiw.h sup_box: live candidates only — r > 0, a finite
        // centre, not a cons3 failure; a NaN difference counts as +inf)
        double dmx = -__builtin_inf(), dmy = -__builtin_inf(), dmr = -__builtin_inf(), dml = -__builtin_inf();
        uint32_t pk[NC];
        bool kb = false;   // (records) a key of this disk is inexact (k_index.h "Keys")
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const double x = v[c][0], y = v[c][1], r = v[c][2];
            int dx = 0, dy = 0, dr = 0;
            const bool packs = key_int(x, base[0], 1023.0, dx) && key_int(y, base[1], 1023.0, dy) &&
                               key_int(r, base[2], 511.0, dr);
            pk[c] = packs ? key_pack(dx, dy, dr) : kKeyEsc;
            if (!packs && iv && cand(c) < K) {
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    const float f = (float)(v[c][q] - base[q]);
                    if constexpr (kGen)
                        kb |= !((dead >> c) & 1u) &&
                              __builtin_bit_cast(uint64_t, base[q] + (double)f) != __builtin_bit_cast(uint64_t, v[c][q]);
                    a.keysT[(int64_t)(q * N + u) * a.ldk + cand(c)] = f;
                }
            }
            if (a.pd && iv && cand(c) < K && !((dead >> c) & 1u) && r > 0.0 && __builtin_isfinite(x) &&
                __builtin_isfinite(y)) {
                double ex = __builtin_fabs(x - base[0]), ey = __builtin_fabs(y - base[1]), er = r - base[2];
                double el = base[2] - r;
                if (!(ex <= kDblMax)) ex = __builtin_inf();
                if (!(ey <= kDblMax)) ey = __builtin_inf();
                if (!(er == er)) er = __builtin_inf();
                if (!(el == el)) el = __builtin_inf();
                dmx = fmax(dmx, ex);
                dmy = fmax(dmy, ey);
                dmr = fmax(dmr, er);
                dml = fmax(dml, el);
            }
        }
        if (iv) {
            uint32_t* const krow = a.keysP + (int64_t)u * a.ldk;
            if constexpr (kGen) {   // two runs of three words (plus and minus candidates)
#pragma unroll
                for (int c = 0; c < NC; ++c) krow[cand(c)] = pk[c];
            } else {   // (k0 = PC * cw: even) 8-B stores, the extra word alone
                static_assert(PC % 2 == 0, "an even candidate count");
#pragma unroll
                for (int h = 0; h < PC / 2; ++h)
                    *reinterpret_cast<uint2*>(krow + k0 + 2 * h) = make_uint2(pk[2 * h], pk[2 * h + 1]);
                if (cand(PC) < K) krow[cand(PC)] = pk[PC];
            }
        }
        if (kGen && a.prec && iv) {
            // (generated polls only: a matrix source takes this kernel in the fused chain alone)
            // the five-launch chain's partial region record (prep_block's): a tile box holding the
            // spans of the live candidates' disks, the span-area estimate and the key flag
            double xa = __builtin_inf(), xb = -__builtin_inf(), ya = __builtin_inf(), yb = -__builtin_inf();
            double xm = 0.0, ym = 0.0, est = 0.0;
            bool any = false;
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const double x = v[c][0], y = v[c][1], r = v[c][2];
                if (cand(c) < K && !((dead >> c) & 1u) && r > 0.0 && __builtin_isfinite(x) &&
                    __builtin_isfinite(y)) {
                    any = true;
                    xa = fmin(xa, x - r);
                    xb = fmax(xb, x + r);
                    ya = fmin(ya, y - r);
                    yb = fmax(yb, y + r);
                    xm = fmax(xm, __builtin_fabs(x) + r);
                    ym = fmax(ym, __builtin_fabs(y) + r);
                    const double e = 2.0 * r * a.g.invS + 1.0;
                    est += e * e;
                }
            }
            int x0 = 0, x1 = -1, y0 = 0, y1 = -1;
            any = any && partial_range(xa, xb, xm, a.g.gx0, a.g.invS, a.g.nTx, x0, x1) &&
                  partial_range(ya, yb, ym, a.g.gy0, a.g.invS, a.g.nTy, y0, y1);
            a.prec[(int64_t)cw * N + u] =
                make_int4((int)range_pack(any, x0, x1, range_shift(a.g.nTx)),
                          (int)range_pack(any, y0, y1, range_shift(a.g.nTy)),
                          __builtin_bit_cast(int, (float)est), kb ? 1 : 0);
        }
        if (a.pd) {
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
        }
    }
    if (a.pd) {   // the workgroup's displacement bound: the waves' shares in order
        lds_barrier();
        if (u == 0) {
            double4 m = make_double4(dred[0][0], dred[0][1], dred[0][2], dred[0][3]);
            for (int q = 1; q < NW; ++q) {
                m.x = fmax(m.x, dred[q][0]);
                m.y = fmax(m.y, dred[q][1]);
                m.z = fmax(m.z, dred[q][2]);
                m.w = fmax(m.w, dred[q][3]);
            }
            a.pd[cw] = m;
        }
    }
}

template <int PC, bool kX = false, bool kGen = false>
__device__ __forceinline__ void prep_body(uint64_t* ts, PrepArgs& a)
{
    ts_begin(ts);   // profiling only (the chain's first launch: k_common.h)
    if (a.lreset && blockIdx.x == 0 && threadIdx.x == 0) *a.lreset = 0;   // (read by fin2 after fiw)
    if (!a.src.resolve(true)) {
        ts_end(ts);
        return;
    }
    // XCD-aware: workgroups b and b + 8 share an XCD (round-robin dispatch), so consecutive
    // candidate groups — which fill the same lines of keysP and of the records — go to one XCD
    const int per = (int)((gridDim.x + 7) / 8), b = (int)blockIdx.x;
    const int cw = (int)(gridDim.x % 8) == 0 ? (b % 8) * per + b / 8 : b;
    __shared__ __attribute__((aligned(16))) unsigned char lds[sizeof(PrepLds<kX ? PC + 1 : PC>)];
    if constexpr (kX) {   // (N <= kPrepU) a matrix, or a generated complete poll in column triples
        prep_block_x<kGen>(a, cw, lds);
    } else if (a.src.cands) {
        prep_block<true, PC>(a, cw, lds);
    } else {
        prep_block<false, PC>(a, cw, lds);
    }
    ts_end(ts);
}

// kPrepC candidates per workgroup, two workgroups per CU
__global__ __launch_bounds__(kPrepU) __attribute__((amdgpu_waves_per_eu(4))) void prep_kernel(uint64_t* ts, PrepArgs a)
{
    prep_body<kPrepC>(ts, a);
}

// the fused chain's prep over a matrix source: kPrepCX (+1) candidates per workgroup (xbase), a
// ninth wave folding the chains; two workgroups (18 waves) per CU. kGen: a generated complete poll
// in column triples, its own kernel: one code path per register allocation (80 VGPRs each; the
// matrix path spill-free, where one kernel holding both paths spilled 13 VGPRs: config 4's prep
// 20.7 -> 26.1 us). 6 waves per EU beat 5 for the generated path too (prep 17.9 vs 23.7 us with
// 82 VGPRs and no spill: the two it spills here are off the hot path)
template <bool kGen>
__global__ __launch_bounds__(kPrepU + kWave) __attribute__((amdgpu_waves_per_eu(6))) void prep_x_kernel(uint64_t* ts, PrepArgs a)
{
    prep_body<kPrepCX, true, kGen>(ts, a);
}

// cands: see CandSrc. Writes disks[k*N + i] (the streaming scan's records).
__global__ void disk_prep_kernel(CandSrc src, int N, int K, DiskRec* __restrict__ disks)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)N * K) return;
    const int k = (int)(t / N), i = (int)(t % N);
    disks[t] = make_disk(src.get(k, i, N), src.get(k, N + i, N), src.get(k, 2 * N + i, N));
}

}  // namespace mac
