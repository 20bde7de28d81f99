// k_index.h — per-poll disk index: one workgroup per UAV disk i, over all K candidates.
//
// Everything the tiled / poll walks need about disk i of candidate k depends only on that disk's
// own (cx, cy, r):
//   * its record {cx, cy, T(r), r};
//   * its tile span;
//   * in the poll walk, its credit over region i's non-shared entries (no other disk can cover
//     those, k_poll.h "Ownership").
// A MADS poll moves each UAV by small integer steps. LTMADS directions are columns of a
// lower-triangular basis with entries bounded by 2^ell, and about a quarter of them do not move a
// given UAV at all. So the K candidates hold far fewer DISTINCT disks per UAV: about 270 of 3073
// at ell = 2 in the config-4 polls.
//
// disk_index_kernel reads the K candidates' (x_i, y_i, r_i) once, straight from the candidate
// source (the matrix's fp32 keys, or the LTMADS generator). It numbers the distinct disks in an
// LDS hash table (exact keys, see "Keys" below) and writes per distinct disk u the record
// urec[i*K + u], plus, for every candidate, the map umap[i*K + k] = u, and the count ucount[i].
// Disk i's region (the union of its tile spans over the K candidates) and its walk costs
// (U_i * |region|, U_i its distinct positions, and the summed span areas) are reduced here from the prep launch's per-workgroup
// partials (k_prep.h), while the keys load; its row descriptors are in flight during the hashing.
// Consumers read disk i of candidate k as urec[i*K + umap[i*K + k]]: the result is bit-identical
// to per-candidate records (same inputs, same arithmetic), and every candidate is still
// evaluated. Polls larger than kIndexMaxK + 1 use the identity map (one position per candidate).
//
// Workgroup b handles disk (b % 8) * ceil(N/8) + b / 8: consecutive disks on one XCD.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "predicate.h"
#include "k_common.h"
#include "k_prep.h"
#include "k_lane.h"

#pragma clang fp contract(off)

namespace mac {

#ifdef MAC_DIAG
__device__ uint64_t g_diag_index[8 * 65536];  // diagnostic build only: per-disk phase stamps
#define MAC_IDX_STAMP(q) if (threadIdx.x == 0 && i < 65536) g_diag_index[8 * i + (q)] = __builtin_amdgcn_s_memrealtime()
#else
#define MAC_IDX_STAMP(q)
#endif
constexpr int kIdxThreads = 1024;            // 16 waves: the phases are latency-bound
constexpr int kIdxWaves = kIdxThreads / kWave;
// candidates per thread, held in registers: 3 up to K = 3073 (N <= 512: two workgroups per CU,
// ~60 KB LDS), 6 up to K = 6145 (N <= 1024: one per CU, ~118 KB LDS); larger polls use the
// identity map (one position per candidate: exact, only slower walks)
constexpr int kIdxPer = 3;
constexpr int kIdxPerWide = 6;
constexpr int kIndexMaxK = kIdxThreads * kIdxPer;          // 3072 (+ 1, below)
constexpr int kIndexMaxKWide = kIdxThreads * kIdxPerWide;  // 6144 (+ 1)
template <int P> struct IdxShape {
    static constexpr int MaxK = kIdxThreads * P;          // + 1: thread 0 takes k = MaxK
    static constexpr int Slots = P <= 3 ? 4096 : 8192;    // table load <= 3/4
    static constexpr int IdBits = P <= 3 ? 12 : 13;       // table word = owner << IdBits | id
};

__device__ __forceinline__ uint32_t key_hash(uint32_t a, uint32_t b, uint32_t c)
{
    uint64_t z = (uint64_t)a * 0x9E3779B97F4A7C15ull;
    z ^= (uint64_t)b + 0xBF58476D1CE4E5B9ull + (z << 6) + (z >> 2);
    z ^= (uint64_t)c + 0x94D049BB133111EBull + (z << 6) + (z >> 2);
    z = (z ^ (z >> 31)) * 0xD6E8FEB86659FD93ull;
    return (uint32_t)(z ^ (z >> 32));
}

constexpr int kRowInfo = 32;   // region rows described per disk (larger regions: walks read off)

struct IndexOut {
    DiskRec* urec;
    int* umap;
    int* ucount;
    int4* region;           // disk i's region (written)
    double2* cost;          // disk i's walk costs {U_i * |region|, summed span areas} (written)
    int* dcount;            // the poll walk's counters (k_common.h kDc*), cleared here
    const int4* prec;       // the prep launch's records [nchain][N] (k_prep.h)
    int nchain;
    // poll walk inputs (null: not needed): per position the scaled-filter constants (k_lane.h)
    // {S*2cu, S*2cv, S*(T - C), -S} and X' (-1: inert), relative to the region centre; per disk
    // kRowInfo + 1 row descriptors of its region {first entry of the row's run, entries before
    // it} (entry nr = {0, total}), written when the region has at most kRowInfo rows
    float4* lane4;
    float* lanexp;
    int2* rows;
    const int32_t* off;
    // the poll's penalties (k_prep.h; null: none): a candidate with vp = +inf failed cons3, is not
    // evaluated (its objective is +inf whatever it covers) and maps to one inert position
    const double* vp;
};

// Key of a candidate that failed cons3: a signalling-NaN pattern, which no fp32 key can hold
// (keys are small integers or fp32 conversions, and conversions produce quiet NaNs), so the
// failed candidates share one position; its record covers nothing (T = -1, r = 0) and its lane
// is inert.
constexpr uint32_t kDeadKey = 0x7FBADEADu;
// ... and in word mode (every key of the disk packed, k_prep.h): an escape pattern with a nonzero
// offset field, which the prep never writes (its escapes are exactly kKeyEsc)
constexpr uint32_t kDeadWord = kKeyEsc | 1u;

__device__ __forceinline__ uint32_t word_hash(uint32_t w)
{
    w *= 0x9E3779B1u;
    w ^= w >> 15;
    w *= 0x85EBCA77u;
    return w ^ (w >> 13);
}
__device__ __forceinline__ bool dead_cand(const double* vp, int k, int K)
{
    return vp && k < K && vp[k] == __builtin_inf();
}

// fp32 key of value v relative to the base b: exact when b + (double)key reproduces v bit for bit
__device__ __forceinline__ float key_of(double v, double b, bool& ok)
{
    const float f = (float)(v - b);
    ok &= __builtin_bit_cast(uint64_t, b + (double)f) == __builtin_bit_cast(uint64_t, v);
    return f;
}

// Keys. A candidate's disk (x, y, r) is keyed by three fp32 offsets from candidate 0's disk,
// kept only when they reproduce the doubles exactly (b + (double)key == value, bit for bit): then
// equal keys mean equal disks, so two candidates share a position only when their disks are
// identical. A MADS poll moves a UAV by mesh multiples, which always compress; a disk whose K
// values do not all compress gets the identity map (one position per candidate: still exact,
// only slower walks). Each thread holds its kIdxPer candidates' doubles in registers through
// every phase, and the LDS holds only the fp32 keys, the table and the owners (~60 KB), so two
// workgroups fit a CU and the whole index runs in one round at N = 512.
// kKeys: keys and exactness flags written by the prep launch (packed words src.keysP, fp32
// offsets of escaped values src.keysT, the records' flags; exact doubles from src.cands or the
// generator): a packed word (dx, dy, dr) is the fp32 key triple (dx, dy, dr), exact by
// construction; else keyed here from src.get (the generator's distinct directions drawn once per
// disk).
template <bool kKeys, int kPer>
__global__ __launch_bounds__(kIdxThreads) __attribute__((amdgpu_waves_per_eu(kPer <= 3 ? 8 : 4))) void disk_index_kernel(
    uint64_t* ts, CandSrc src0, int N, int K, Grid g, int dedup, IndexOut o)
{
    CandSrc src = src0;
    constexpr int kIdxPer = kPer;
    constexpr int kIndexMaxK = IdxShape<kPer>::MaxK;
    constexpr int kIndexSlots = IdxShape<kPer>::Slots;
    constexpr int kIdBits = IdxShape<kPer>::IdBits;
    ts_begin(ts);   // profiling only, when the index opens the chain (k_common.h)
    __shared__ float kx[kIndexMaxK + 1], ky[kIndexMaxK + 1], kr[kIndexMaxK + 1];
    __shared__ int table[kIndexSlots];       // owner candidate, then (owner << kIdBits | id)
    __shared__ uint16_t owner_of[kIndexMaxK + 1];
    __shared__ int ucnt;
    __shared__ int sred[4][kIdxWaves];
    __shared__ float fred[kIdxWaves];

    const int per_xcd = (N + 7) / 8;
    const int i = (int)(blockIdx.x % 8) * per_xcd + (int)(blockIdx.x / 8);
    if (i >= N || !src.resolve()) {   // uniform
        ts_end(ts);
        return;
    }
    MAC_IDX_STAMP(0);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        for (int q = 0; q < kDcCount; ++q) o.dcount[q] = 0;   // the poll walk's counters (k_common.h)
    }
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
    const int64_t row = (int64_t)i * K;
    // candidates of this thread: k = tid + j * kIdxThreads (j < kIdxPer), and thread 0 also
    // takes k = kIndexMaxK (a full MADS poll is 2n + 1 = kIndexMaxK + 1 candidates at most here)
    const bool fits = dedup && K > 0 && K <= kIndexMaxK + 1;

    // disk i's region, costs and key flag from the prep launch's records (k_prep.h): loaded
    // with the keys, reduced per wave into sred / fred (published by the keys phase's barrier),
    // then by every thread
    uint32_t ax = 0xFFFF, bx_ = 0, ay = 0xFFFF, by_ = 0;
    float ps = 0.0f;
    bool pbad = false;
    auto load_partials = [&]() {
        for (int q = tid; q < o.nchain; q += kIdxThreads) {
            const int4 r = o.prec[(int64_t)q * N + i];
            ax = min(ax, (uint32_t)r.x & 0xFFFFu);
            bx_ = max(bx_, (uint32_t)r.x >> 16);
            ay = min(ay, (uint32_t)r.y & 0xFFFFu);
            by_ = max(by_, (uint32_t)r.y >> 16);
            ps += __builtin_bit_cast(float, r.z);
            pbad |= r.w != 0;
        }
    };
    auto publish_partials = [&]() {
        int4 PR;
        range_unpack(ax, bx_, range_shift(g.nTx), g.nTx, PR.x, PR.y);
        range_unpack(ay, by_, range_shift(g.nTy), g.nTy, PR.z, PR.w);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            PR.x = min(PR.x, __shfl_xor(PR.x, off, kWave));
            PR.y = max(PR.y, __shfl_xor(PR.y, off, kWave));
            PR.z = min(PR.z, __shfl_xor(PR.z, off, kWave));
            PR.w = max(PR.w, __shfl_xor(PR.w, off, kWave));
            ps += __shfl_xor(ps, off, kWave);   // (the same butterfly in every lane: fixed order)
        }
        if (lane == 0) {
            sred[0][wid] = PR.x;
            sred[1][wid] = PR.y;
            sred[2][wid] = PR.z;
            sred[3][wid] = PR.w;
            fred[wid] = ps;
        }
    };
    auto get3 = [&](int k, double& x, double& y, double& r) {
        if (kKeys && src.cands) {  // the column-major matrix (strided: identity path and bases only)
            const double* c = src.cands + (int64_t)k * src.ldc;
            x = c[i];
            y = c[N + i];
            r = c[2 * N + i];
        } else {
            x = src.get(k, i, N);
            y = src.get(k, N + i, N);
            r = src.get(k, 2 * N + i, N);
        }
    };

    bool hashed = false;
    bool words = false;   // every key of the disk is a packed word: one-word keys (kx holds the bits)
    constexpr int P = kIdxPer + 1;
    int slot[P];
    double bx = 0.0, by = 0.0, br = 0.0;   // candidate 0's disk: the key base
    if (fits && kKeys) {
        // ---- keys: rows of the fp32 key matrix (coalesced) and the tiles' exactness flags
        get3(0, bx, by, br);
        const uint32_t* fp = src.keysP + (int64_t)i * src.ldk;
        uint32_t pq[P];
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const int k = min(j < kIdxPer ? tid + j * kIdxThreads : (tid == 0 ? kIndexMaxK : K), K - 1);
            pq[j] = fp[k];
        }
        load_partials();
        // packed words to fp32 offsets; an escaped value's offsets from the fp32 rows (k_prep.h)
        float qx[P], qy[P], qr[P];
#pragma unroll
        for (int j = 0; j < P; ++j) {
            key_unpack(pq[j], qx[j], qy[j], qr[j]);
            if (pq[j] == kKeyEsc) {
                const int k = min(j < kIdxPer ? tid + j * kIdxThreads : (tid == 0 ? kIndexMaxK : K), K - 1);
                const float* fx = src.keysT + (int64_t)i * src.ldk;
                qx[j] = fx[k];
                qy[j] = fx[(int64_t)N * src.ldk + k];
                qr[j] = fx[(int64_t)2 * N * src.ldk + k];
            }
        }
        bool dj[P], any_esc = false;
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const int k = j < kIdxPer ? tid + j * kIdxThreads : (tid == 0 ? kIndexMaxK : K);
            dj[j] = dead_cand(o.vp, k, K);
            if (dj[j]) qx[j] = qy[j] = qr[j] = __builtin_bit_cast(float, kDeadKey);
            any_esc |= k < K && !dj[j] && pq[j] == kKeyEsc;
        }
        const bool bad = pbad;   // a key of disk i is inexact (the records' flags)
        for (int q = tid; q < kIndexSlots; q += kIdxThreads) table[q] = -1;
        if (tid == 0) ucnt = 0;
        words = !__syncthreads_or(any_esc);
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const int k = j < kIdxPer ? tid + j * kIdxThreads : (tid == 0 ? kIndexMaxK : K);
            if (k < K) {
                if (words) {
                    kx[k] = __builtin_bit_cast(float, dj[j] ? kDeadWord : pq[j]);
                } else {
                    kx[k] = qx[j];
                    ky[k] = qy[j];
                    kr[k] = qr[j];
                }
            }
        }
        publish_partials();
        hashed = !__syncthreads_or(bad);                  // (the barrier also publishes the keys)
    } else if (fits) {
        double cx[P], cy[P], cr[P];
        // ---- keys: every load in flight at once, then the fp32 offsets (exactness voted)
        get3(0, bx, by, br);
        load_partials();
        const int n = 3 * N;
        if (!src.cands && 3 * n <= 2 * kIndexSlots && (src.ltri || src.b <= 16384)) {
            // the generator: candidates k and k + n are x + d and x - d of the same LTMADS entry
            // d = L[rp[v]][cp[k mod n]] (k_prep.h CandSrc), so disk i's 3 x n entries are drawn
            // once into the table's LDS (integers |d| <= b, as int16) and both signs built from
            // them: the same doubles as src.get, half the stream draws, spread over all threads.
            // The basis form's table holds L itself and d = (double)L * delta (src.entry's product)
            int16_t* const dtab = reinterpret_cast<int16_t*>(table);
            const int r3[3] = {src.rp[i], src.rp[N + i], src.rp[2 * N + i]};
            for (int t = tid; t < 3 * n; t += kIdxThreads) {
                const int a = t / n, kk = t - a * n;
                const int r = r3[a], c = src.cp[kk];
                dtab[t] = src.ltri ? (r < c ? (int16_t)0 : src.ltri[(int64_t)r * (r + 1) / 2 + c])
                                   : (int16_t)ltmads_entry(src.state, n, src.b, r, c);
            }
            __syncthreads();
            const double sc = src.ltri ? src.delta : 1.0;
            const double xi = src.xinc[i], yi = src.xinc[N + i], ri = src.xinc[2 * N + i];
#pragma unroll
            for (int j = 0; j < P; ++j) {
                const int kl = min(j < kIdxPer ? tid + j * kIdxThreads : (tid == 0 ? kIndexMaxK : K), K - 1);
                const int kg = kl + src.k0;
                const bool plus = kg < n;
                const int kk = plus ? kg : kg - n;
                const double dx = sc * (double)dtab[kk], dy = sc * (double)dtab[n + kk],
                             dr = sc * (double)dtab[2 * n + kk];
                cx[j] = plus ? xi + dx : xi - dx;
                cy[j] = plus ? yi + dy : yi - dy;
                cr[j] = plus ? ri + dr : ri - dr;
            }
            __syncthreads();   // the table is cleared next
        } else {
#pragma unroll
            for (int j = 0; j < P; ++j) {
                const int k = j < kIdxPer ? tid + j * kIdxThreads : (tid == 0 ? kIndexMaxK : K);
                get3(min(k, K - 1), cx[j], cy[j], cr[j]);
            }
        }
        for (int q = tid; q < kIndexSlots; q += kIdxThreads) table[q] = -1;
        if (tid == 0) ucnt = 0;
        bool ok = true;
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const int k = j < kIdxPer ? tid + j * kIdxThreads : (tid == 0 ? kIndexMaxK : K);
            if (dead_cand(o.vp, k, K)) {
                kx[k] = ky[k] = kr[k] = __builtin_bit_cast(float, kDeadKey);
            } else if (k < K) {
                kx[k] = key_of(cx[j], bx, ok);
                ky[k] = key_of(cy[j], by, ok);
                kr[k] = key_of(cr[j], br, ok);
            }
        }
        publish_partials();
        hashed = !__syncthreads_or(!ok);                  // (the barrier also publishes the keys)
    } else {
        load_partials();
        publish_partials();
        __syncthreads();
    }
    MAC_IDX_STAMP(1);
    // ---- region and costs (every thread reduces the waves' partials: no further barrier); the
    // region's row descriptors load now and are written after the map
    int4 Rg = make_int4(0x7fffffff, -1, 0x7fffffff, -1);
    float psum = 0.0f;
#pragma unroll
    for (int q = 0; q < kIdxWaves; ++q) {
        Rg.x = min(Rg.x, sred[0][q]);
        Rg.y = max(Rg.y, sred[1][q]);
        Rg.z = min(Rg.z, sred[2][q]);
        Rg.w = max(Rg.w, sred[3][q]);
        psum += fred[q];
    }
    if (Rg.x > Rg.y || Rg.z > Rg.w) Rg = make_int4(0x7fffffff, -1, 0x7fffffff, -1);
    const bool any = Rg.x <= Rg.y;
    // the walk costs: the poll walk tests region i against each DISTINCT position (written with
    // the count below), the per-candidate walk visits the summed spans (k_poll_shared.h walk_choice)
    const double rc = any ? (double)(Rg.y - Rg.x + 1) * (double)(Rg.w - Rg.z + 1) : 0.0;
    if (tid == 0) o.region[i] = Rg;
    const bool want_rows = o.rows && any && Rg.w - Rg.z + 1 <= kRowInfo && tid < kWave;
    const int nr = Rg.w - Rg.z + 1;
    int rs0 = 0, rs1 = 0;
    if (want_rows && tid < nr) {
        const int64_t rb = (int64_t)(Rg.z + tid) * g.nTx;
        rs0 = o.off[rb + Rg.x];
        rs1 = o.off[rb + Rg.y + 1];
    }
    if (!hashed) {  // identity: one position per candidate
        for (int k = tid; k < K; k += kIdxThreads) {
            double x, y, r;
            get3(k, x, y, r);
            o.urec[row + k] = make_disk(x, y, r);
            o.umap[row + k] = k;
        }
        if (tid == 0) {
            o.ucount[i] = K;
            o.cost[i] = make_double2(rc * (double)K, (double)psum);
        }
    } else {
        // ---- insert (exact fp32 keys; linear probing)
        constexpr uint32_t mask = kIndexSlots - 1;
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const int k = j < kIdxPer ? tid + j * kIdxThreads : (tid == 0 ? kIndexMaxK : K);
            slot[j] = 0;
            if (k >= K) continue;
            const uint32_t bx = __builtin_bit_cast(uint32_t, kx[k]);
            const uint32_t by = words ? 0u : __builtin_bit_cast(uint32_t, ky[k]);
            const uint32_t br = words ? 0u : __builtin_bit_cast(uint32_t, kr[k]);
            uint32_t s = (words ? word_hash(bx) : key_hash(bx, by, br)) & mask;
            for (;;) {
                int cur = table[s];
                if (cur < 0) {
                    cur = atomicCAS(&table[s], -1, k);
                    if (cur < 0) break;                      // claimed an empty slot
                }
                if (__builtin_bit_cast(uint32_t, kx[cur]) == bx &&
                    (words || (__builtin_bit_cast(uint32_t, ky[cur]) == by &&
                               __builtin_bit_cast(uint32_t, kr[cur]) == br)))
                    break;                                   // same disk: share the slot
                s = (s + 1) & mask;                          // another disk: probe on
            }
            slot[j] = (int)s;
        }
        __syncthreads();
        MAC_IDX_STAMP(2);
        // ---- ids for the occupied slots (any order: nothing computed depends on the numbering)
        for (int q = tid; q < kIndexSlots; q += kIdxThreads) {
            const int owner = table[q];
            if (owner >= 0) {
                const int u = atomicAdd(&ucnt, 1);
                owner_of[u] = (uint16_t)owner;
                table[q] = (owner << kIdBits) | u;
            }
        }
        __syncthreads();
        MAC_IDX_STAMP(3);
        // ---- per candidate: the map
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const int k = j < kIdxPer ? tid + j * kIdxThreads : (tid == 0 ? kIndexMaxK : K);
            if (k >= K) continue;
            o.umap[row + k] = table[slot[j]] & ((1 << kIdBits) - 1);
        }
        if (tid == 0) {
            o.ucount[i] = ucnt;
            o.cost[i] = make_double2(rc * (double)ucnt, (double)psum);
        }
    }
    MAC_IDX_STAMP(4);
    if (want_rows) {   // (wave-uniform)
        const int len = rs1 - rs0;
        const int incl = wave_incl_scan_i32(len, tid);
        if (tid <= nr) o.rows[(int64_t)i * (kRowInfo + 1) + tid] = make_int2(rs0, incl - len);
    }
    // ---- per position: the record (hashed: from the owner's exact key, base + offset; identity:
    // written above) and the poll walk's lane constants relative to the region centre (the same
    // origin and bound the walk stages its entries with, k_poll.h)
    const double ox = g.gx0 + 0.5 * (double)(Rg.x + Rg.y + 1) * g.S;
    const double oy = g.gy0 + 0.5 * (double)(Rg.z + Rg.w + 1) * g.S;
    const double Umax = 0.5 * (double)max(Rg.y - Rg.x + 1, Rg.w - Rg.z + 1) * g.S + 2.0 * g.S;
    const int U = hashed ? ucnt : K;
    if (hashed || o.lane4) {
        for (int u = tid; u < U; u += kIdxThreads) {
            DiskRec d;
            if (hashed) {
                const int k = owner_of[u];
                float fx = 0.0f, fy = 0.0f, fr = 0.0f;
                bool dead;
                if (words) {
                    const uint32_t wk = __builtin_bit_cast(uint32_t, kx[k]);
                    dead = wk == kDeadWord;
                    key_unpack(wk, fx, fy, fr);
                } else {
                    dead = __builtin_bit_cast(uint32_t, kr[k]) == kDeadKey;
                    fx = kx[k];
                    fy = ky[k];
                    fr = kr[k];
                }
                if (dead) {   // the failed candidates
                    d.cx = d.cy = d.r = 0.0;
                    d.T = -1.0;
                } else {
                    d = make_disk(bx + (double)fx, by + (double)fy, br + (double)fr);
                }
                o.urec[row + u] = d;
            } else {
                double x, y, r;
                get3(u, x, y, r);
                d = make_disk(x, y, r);
            }
            if (o.lane4) {
                PollLane L = inert_lane();
                int4 sp;
                if (any && disk_span(d, g, sp)) L = poll_lane(d, ox, oy, Umax);
                o.lane4[row + u] = make_float4(L.sa, L.sb, L.stm, L.ns);
                o.lanexp[row + u] = L.xp;
            }
        }
    }
    MAC_IDX_STAMP(5);
    ts_end(ts);
}

// Small batches (K < 64 under AUTO: the per-candidate walk, which shares nothing between
// candidates): the identity map built with one thread per (disk, candidate) instead of a
// workgroup per disk, and no key pass. urec[i*K + k], umap[i*K + k] = k.
__global__ __launch_bounds__(256) void disk_index_identity_kernel(CandSrc src, int N, int K,
                                                                  DiskRec* __restrict__ urec,
                                                                  int* __restrict__ umap)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)N * K) return;
    const int i = (int)(t / K), k = (int)(t % K);
    const double x = src.get(k, i, N), y = src.get(k, N + i, N), r = src.get(k, 2 * N + i, N);
    urec[t] = make_disk(x, y, r);
    umap[t] = k;
}

// disk i of candidate k through the index
__device__ __forceinline__ DiskRec rec_of(const DiskRec* __restrict__ urec,
                                          const int* __restrict__ umap, int i, int K, int k)
{
    const int64_t row = (int64_t)i * K;
    return urec[row + umap[row + k]];
}

}  // namespace mac
