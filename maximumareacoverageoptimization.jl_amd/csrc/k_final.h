// k_final.h — partial-sum reduction, objective (the prep launch's penalty, k_prep.h) and the
// poll argmin.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "predicate.h"
#include "k_common.h"
#include "k_prep.h"

#pragma clang fp contract(off)

namespace mac {

#ifndef MAC_FIN_C
#define MAC_FIN_C 16
#endif
constexpr int kFinC = MAC_FIN_C;   // candidates per finalize block (x 1024 / kFinC slice groups)
#ifndef MAC_FIN_MAXBLK
#define MAC_FIN_MAXBLK 256
#endif
constexpr int kFinMaxBlk = MAC_FIN_MAXBLK;   // finalize blocks whose minima the last block loads at once
constexpr int kFinThreads = 1024;

// Block = 16 candidates x 64 slice groups. area_k = sum over slices g of the slice's credit in a
// fixed order (thread (c, sg) sums g = sg, sg+64, ... in batches of 8, then the 64 groups in
// order): bit-reproducible. The slice count is n_poll when *mode == poll, else n_other.
// Poll walk (mode == poll, map and spart given): slice g is disk g; its credit for candidate k is
// partial[g*K + map[g*K + k]] (the distinct-disk position, k_index.h) plus, when disk g has
// lower-index neighbours (ncount[g] > 0), its shared-entry row spart[g*K + k] (rows of other
// disks are never written and never read). Per batch the map and ncount loads go first, then the
// gathers and shared rows they select: two memory round trips per batch.
// obj_k = -area_k + vp_k when obj_out != null. With `counts` (every entry weighs w0) and the poll
// walk chosen, the rows hold uint32 covered-entry counts (partial[i][u] per position, gathered
// through the map, and spart[i][k] per candidate of the disks with neighbours): area_k = (their
// integer sum) * w0.
// The poll argmin (fb.best != null) is taken here too, with no launch of its own: every block
// publishes the lexicographic minimum of its kFinC candidates and the block that arrives last
// reduces the published minima (finalize_argmin below).
struct FinBest {
    double* best;          // {objective, index bits} (null: no argmin)
    uint64_t* mirror;      // mapped host slot {obj bits, index, seq, check} (may be null)
    uint64_t seq;
    int64_t idx_base;
    unsigned long long* blk;   // [gridDim.x][2] per-block minima {obj bits, index}
    unsigned* arrive;          // arrival counter, zero between launches (the last block resets it)
    // the pipelined native MADS loop (k_prep.h MadsState): the last block also applies the poll's
    // update (mads_step); st == null: none
    MadsState* st;
    const double* x;           // the poll's incumbent (its generator's xinc), 3N
    double* x_next;            // the incumbent after the poll
    const int* rp;             // the poll's row / column permutations
    const int* cp;
    uint64_t state;            // the poll's stream state
    int n, ell_max;
    uint64_t done_seq;         // mirror seq word once the loop has stopped (the host's wait ends)
    // launch-hint words (device ints; null: none): the last block copies the first nhint to the
    // mapped host words hint_host (the lane's next enqueue reads them) and clears them
    int* hint;
    int* hint_host;
    int nhint;
    // a stepper's cumulative count of candidates that passed cons3 (k_prep.h PrepArgs.feas; null:
    // none): the last block also writes it to the mirror's word 4 (a 64-B slot), under the check
    const unsigned long long* feas;
};

// Check word of a mirrored result (host: mirror_check in maxcover.hip): the host accepts the slot
// only when seq is the one it waits for AND the check word matches the three words it read, so a
// slot read while its stores are still landing (no fence orders them: a system-scope release
// would write back the XCD's L2) is read again, never accepted torn.
__host__ __device__ __forceinline__ uint64_t mirror_check(uint64_t o, uint64_t i, uint64_t q, uint64_t f = 0)
{
    uint64_t z = o ^ (i * 0x9E3779B97F4A7C15ull) ^ (q * 0xC2B2AE3D27D4EB4Full) ^ (f * 0xD6E8FEB86659FD93ull) ^
                 0x5851F42D4C957F2Dull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// The pipelined MADS loop's update, by the wave that took the poll's argmin (every lane holds
// bo, gidx): mac_mads_update's arithmetic (maxcover.hip; src/TDM_STATIC_opt.jl's NOMAD poll
// acceptance: a strictly better objective moves the incumbent and coarsens the mesh, else the mesh
// is refined), with the same ltmads_entry values and per-variable adds, so the pipelined loop visits
// the stepper's incumbents bit for bit. ell, f: the state before the poll.
__device__ __forceinline__ void mads_step(const FinBest& fb, double bo, int64_t gidx, int ell, double f)
{
    const int lane = threadIdx.x & (kWave - 1);
    const int n = fb.n;
    const double* __restrict__ x = fb.x;
    double* __restrict__ xn = fb.x_next;
    const bool better = gidx >= 0 && bo < f;
    // batches of kB variables per lane: every load of a batch in flight at once, then the stores
    // (a load-then-store loop was one memory round trip per variable: ~10 us at n = 1536)
    constexpr int kB = 8;
    const int64_t b = (int64_t)1 << ell;
    const bool plus = gidx < n;
    const int c = better ? fb.cp[plus ? (int)gidx : (int)gidx - n] : 0;
    for (int v0 = lane; v0 < n; v0 += kB * kWave) {
        double xv[kB];
        int rv[kB];
#pragma unroll
        for (int j = 0; j < kB; ++j) {
            const int v = v0 + j * kWave;
            xv[j] = v < n ? x[v] : 0.0;
            rv[j] = better && v < n ? fb.rp[v] : 0;
        }
#pragma unroll
        for (int j = 0; j < kB; ++j) {
            const int v = v0 + j * kWave;
            if (v >= n) break;
            if (better) {
                const double d = ltmads_entry(fb.state, n, b, rv[j], c);
                xn[v] = plus ? xv[j] + d : xv[j] - d;
            } else {
                xn[v] = xv[j];
            }
        }
    }
    if (lane == 0) {
        const int e = better ? (ell + 1 < fb.ell_max ? ell + 1 : fb.ell_max) : ell - 1;
        fb.st->f = better ? bo : f;
        fb.st->ell = e;
        fb.st->it += 1;
        if (better) fb.st->succ += 1;
    }
}

__device__ __forceinline__ void argmin_take(double& v1, int& i1, double v2, int i2)
{
    if ((i2 >= 0) && (i1 < 0 || v2 < v1 || (v2 == v1 && i2 < i1))) {
        v1 = v2;
        i1 = i2;
    }
}

// Wave 0 of every finalize block, lanes 0..kFinC-1 holding (o, k) of the block's candidates
// (have: k < K). Cross-workgroup hand-off (MI355X_MICROARCH.md, inter-workgroup visibility, first
// row of the sc1 table): lane 0 alone stores its block's minimum with 8-B agent-scope (sc1) stores,
// waits for them (vmcnt(0)), then adds to ONE counter; the block whose add returns the last count
// loads every minimum with sc1 loads, in the same wave. The lexicographic (objective, index)
// minimum is order-independent (the sequential first-best order); NaN / +inf never selected.
// C: lanes holding the block's candidates (a power of two <= 64). Returns true in the last block.
template <int C = kFinC>
__device__ __forceinline__ bool finalize_argmin(const FinBest& fb, double o, int k, bool have)
{
    static_assert(C >= 1 && C <= kWave && (C & (C - 1)) == 0, "C: a power of two up to a wave");
    const int lane = threadIdx.x & (kWave - 1);
    double bv = __builtin_inf();
    int bi = -1;
    if (have && lane < C && o < bv) {
        bv = o;
        bi = k;
    }
#pragma unroll
    for (int off = C / 2; off >= 1; off >>= 1)
        argmin_take(bv, bi, __shfl_xor(bv, off, kWave), __shfl_xor(bi, off, kWave));
    unsigned old = 0;
    if (lane == 0) {
        __hip_atomic_store(fb.blk + 2 * blockIdx.x, __builtin_bit_cast(unsigned long long, bv),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(fb.blk + 2 * blockIdx.x + 1, (unsigned long long)(long long)bi,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        old = __hip_atomic_fetch_add(fb.arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    old = __shfl(old, 0, kWave);
    if (old != gridDim.x - 1) return false;   // wave-uniform: not the last block
    // the pipelined MADS loop's state, loaded beside the minima (a stopped loop: no result)
    const int ell = fb.st ? fb.st->ell : 0;
    const double fcur = fb.st ? fb.st->f : 0.0;
    const int rej = fb.st ? fb.st->skip : 0;   // the prep rejected the poll whole: a failure
    bv = __builtin_inf();
    bi = -1;
    // every block's minimum in flight at once (kFinMaxBlk / 64 per lane), then the reduction
    constexpr int kPer = kFinMaxBlk / kWave;
    unsigned long long v[kPer], ix[kPer];
#pragma unroll
    for (int r = 0; r < kPer; ++r) {
        const unsigned q = lane + r * kWave;
        v[r] = q < gridDim.x ? __hip_atomic_load(fb.blk + 2 * q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                             : __builtin_bit_cast(unsigned long long, __builtin_inf());
        ix[r] = q < gridDim.x ? __hip_atomic_load(fb.blk + 2 * q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                              : ~0ull;
    }
    // the hint words and the feasible count, in the same round trip
    const uint64_t fe = fb.feas ? __hip_atomic_load(fb.feas, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
    const bool hl = fb.hint && lane < fb.nhint;
    const int hv = hl ? __hip_atomic_load(fb.hint + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
#pragma unroll
    for (int r = 0; r < kPer; ++r)
        if ((long long)ix[r] >= 0) argmin_take(bv, bi, __builtin_bit_cast(double, v[r]), (int)(long long)ix[r]);
    for (unsigned q = lane + kFinMaxBlk; q < gridDim.x; q += kWave) {   // grids past kFinMaxBlk
        const unsigned long long vv = __hip_atomic_load(fb.blk + 2 * q, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long xx = __hip_atomic_load(fb.blk + 2 * q + 1, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
        argmin_take(bv, bi, __builtin_bit_cast(double, vv), (int)(long long)xx);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1)
        argmin_take(bv, bi, __shfl_xor(bv, off, kWave), __shfl_xor(bi, off, kWave));
    const bool none = bi < 0 || rej;
    const double bo = none ? __builtin_inf() : bv;
    const int64_t gidx = none ? (int64_t)-1 : fb.idx_base + bi;
    if (fb.st && ell < 0) {   // the loop stopped before this poll
        if (lane == 0) __hip_atomic_store(fb.arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return true;
    }
    if (fb.st) {
        mads_step(fb, bo, gidx, ell, fcur);
        if (rej && lane == 0) fb.st->skipped += 1;
    }
    if (lane == 0) {
        // d_best with agent-scope (sc1, write-through) stores: a host that has read the mirror may
        // hand d_best to device work on another stream (an RCCL all-gather, dist.DeviceGather)
        // while this launch retires, and a plain store would sit in this XCD's L2 only
        unsigned long long* const bw = reinterpret_cast<unsigned long long*>(fb.best);
        __hip_atomic_store(bw, __builtin_bit_cast(unsigned long long, bo), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(bw + 1, (unsigned long long)gidx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(fb.arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (fb.mirror) {
            // d_best's stores acknowledged first, then the slot: plain stores to the mapped
            // words, validated on the host by seq + check (no system-scope fence)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint64_t o = __builtin_bit_cast(uint64_t, bo);
            const uint64_t ix = (uint64_t)gidx;
            fb.mirror[0] = o;
            fb.mirror[1] = ix;
            fb.mirror[2] = fb.seq;
            if (fb.feas) fb.mirror[4] = fe;
            fb.mirror[3] = mirror_check(o, ix, fb.seq, fe);
            // a pipelined loop that has just stopped: polls after this one write no slot, so the
            // seq word jumps past every seq the host may wait for
            if (fb.st && !(gidx >= 0 && bo < fcur) && ell == 0) fb.mirror[2] = fb.done_seq;
        }
    }
    if (hl) {   // (read above; cleared for the next poll)
        if (fb.hint_host) ((volatile int*)fb.hint_host)[lane] = hv;
        __hip_atomic_store(fb.hint + lane, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return true;
}

__global__ __launch_bounds__(kFinThreads) void finalize_kernel(
    const double* __restrict__ partial, const int* __restrict__ mode, int n_poll, int n_other,
    int K, int N, const int* __restrict__ map, const double* __restrict__ spart,
    const int* __restrict__ ncount, int counts, double w0,
    const double* __restrict__ vp, double* __restrict__ area_out, double* __restrict__ obj_out,
    FinBest fb, uint64_t* ts)
{
    ts_begin(ts);   // profiling only: the chain's last launch (k_common.h)
    double o = __builtin_inf();   // lanes sg == 0: candidate k's objective (for the argmin)
    __shared__ double red[kFinThreads / kFinC][kFinC];
    const int t = threadIdx.x, c = t % kFinC, sg = t / kFinC;
    constexpr int SG = kFinThreads / kFinC;
    // XCD-aware: blocks b and b + 8 share an XCD (round-robin dispatch), so candidate block
    // (b % 8) * per + b / 8 puts neighbouring candidate blocks — the two halves of each 128-B
    // line of every count row — on one L2. The grid is 8 * per blocks; the ones past K only
    // take part in the argmin's arrival count.
    const int per = (int)(gridDim.x / 8);
    const int cb = per > 0 && gridDim.x % 8 == 0 ? (int)(blockIdx.x % 8) * per + (int)(blockIdx.x / 8)
                                                 : (int)blockIdx.x;
    const int k0 = cb * kFinC;
    const int k = k0 + c;
    // the walk the device chose, loaded first and checked once the first loads are out (the
    // poll walk's map and neighbour counts are read speculatively: both are valid memory for
    // either walk), so it costs no round trip of its own
    const int mv = mode ? *mode : 0;
    // the candidate's penalty, loaded with the first batch of rows (one round trip fewer); every
    // lane of the poll walk's counts path takes it: a candidate that failed cons3 (vp = +inf, no area
    // asked for) has objective +inf whatever it covers, so its count gathers — the second, dependent
    // round trip — are left out (config 5: most of a poll's candidates at l >= 2)
    const bool cnt_path = counts && spart && map;
    const double vpk = (vp && (sg == 0 || cnt_path) && k < K) ? vp[k] : 0.0;
    if (cnt_path) {  // equal weights: integer rows, exact in any order
        constexpr int B = 8;
        int pos0[B];
        bool sh0[B];
#pragma unroll
        for (int b = 0; b < B; ++b) {
            const int gb = sg + b * SG;
            const bool in = k < K && gb < n_poll;
            pos0[b] = in ? map[(int64_t)gb * K + k] : -1;
            sh0[b] = in && ncount[gb] > 0;
        }
        const bool skip = vp && !area_out && !(vpk < __builtin_inf());   // (+inf or NaN: no area needed)
        if (mv == kModePoll) {
            const unsigned* const crow = reinterpret_cast<const unsigned*>(partial);
            const unsigned* const srow = reinterpret_cast<const unsigned*>(spart);
            __shared__ uint64_t ired[kFinThreads / kFinC][kFinC];
            const int G = n_poll;
            uint64_t a = 0;
            if (k < K && !skip) {
                // per row: the count at candidate k's position (the poll walk writes one per
                // position, the map gives candidate k's), plus its shared-entry count when the
                // disk has neighbours
                for (int g = sg; g < G; g += B * SG) {
                    unsigned v[B], sv[B];
                    int pos[B];
                    bool sh[B];
#pragma unroll
                    for (int b = 0; b < B; ++b) {
                        const int gb = g + b * SG;
                        if (g == sg) {
                            pos[b] = pos0[b];
                            sh[b] = sh0[b];
                        } else {
                            pos[b] = gb < G ? map[(int64_t)gb * K + k] : -1;
                            sh[b] = gb < G && ncount[gb] > 0;
                        }
                    }
#pragma unroll
                    for (int b = 0; b < B; ++b) {
                        const int64_t rb = (int64_t)(g + b * SG) * K;
                        v[b] = pos[b] >= 0 ? crow[rb + pos[b]] : 0u;
                        sv[b] = sh[b] ? srow[rb + k] : 0u;
                    }
#pragma unroll
                    for (int b = 0; b < B; ++b) a += (uint64_t)v[b] + sv[b];
                }
            }
            ired[sg][c] = a;
            __syncthreads();
            if (sg == 0 && k < K) {
                uint64_t n = 0;
#pragma unroll
                for (int q = 0; q < SG; ++q) n += ired[q][c];
                const double area = (double)n * w0;
                if (area_out) area_out[k] = area;
                if (vp) o = -area + vpk;
                if (obj_out) obj_out[k] = o;
            }
            if (fb.best && t < kWave) finalize_argmin(fb, o, k, k < K);
            ts_end(ts);
            return;
        }
    }
    const bool poll = mv == kModePoll;
    const int G = poll ? n_poll : n_other;
    const bool rows = spart && poll;
    const int* mp = (map && poll) ? map : nullptr;
    constexpr int kFinB = 8;
    double acc = 0.0;
    if (k < K) {
        for (int g = sg; g < G; g += kFinB * SG) {
            int pos[kFinB];
            bool sh[kFinB];
#pragma unroll
            for (int b = 0; b < kFinB; ++b) {
                const int gb = g + b * SG;
                pos[b] = gb < G ? (mp ? mp[(int64_t)gb * K + k] : k) : -1;
                sh[b] = rows && gb < G && ncount[gb] > 0;
            }
            double v[kFinB], sv[kFinB];
#pragma unroll
            for (int b = 0; b < kFinB; ++b) {
                const int64_t rb = (int64_t)(g + b * SG) * K;
                v[b] = pos[b] >= 0 ? partial[rb + pos[b]] : 0.0;
                sv[b] = sh[b] ? spart[rb + k] : 0.0;
            }
            double bs = 0.0;
#pragma unroll
            for (int b = 0; b < kFinB; ++b) bs += v[b] + sv[b];
            acc += bs;
        }
    }
    red[sg][c] = acc;

    __syncthreads();
    if (sg == 0 && k < K) {
        double area = 0.0;
#pragma unroll
        for (int q = 0; q < SG; ++q) area += red[q][c];
        if (area_out) area_out[k] = area;
        if (vp) o = -area + vpk;
        if (obj_out) obj_out[k] = o;
    }
    if (fb.best && t < kWave) finalize_argmin(fb, o, k, k < K);
    ts_end(ts);
}

// The multi-GPU poll's exchange on the device (mac_best_reduce_dev): n 16-B records {objective,
// index as int64 bits} — the ranks' poll bests, all-gathered by RCCL into one buffer on this
// stream — reduced by one wave to their lexicographic minimum (dist.reduce_best's rule: a record
// with index < 0 or an objective that is not < +inf never wins, ties to the lowest index), written
// to best and to its mapped host slot exactly as finalize's last block writes a poll's result
// (d_best with agent-scope stores, acknowledged, then the slot words under seq + check), so the
// host reads the node's argmin with mac_best_fetch and no copy or stream synchronisation.
__global__ __launch_bounds__(kWave) void best_reduce_kernel(const unsigned long long* __restrict__ rec, int n,
                                                          unsigned long long* best, uint64_t* mirror,
                                                          uint64_t seq)
{
    const int lane = threadIdx.x;
    double bv = __builtin_inf();
    long long bi = -1;
    for (int q = lane; q < n; q += kWave) {
        const double o = __builtin_bit_cast(double, rec[2 * q]);
        const long long i = (long long)rec[2 * q + 1];
        if (i >= 0 && o < __builtin_inf() && (bi < 0 || o < bv || (o == bv && i < bi))) {
            bv = o;
            bi = i;
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const double o = __shfl_xor(bv, off, kWave);
        const long long i = __shfl_xor(bi, off, kWave);
        if (i >= 0 && (bi < 0 || o < bv || (o == bv && i < bi))) {
            bv = o;
            bi = i;
        }
    }
    if (lane == 0) {
        const uint64_t o = __builtin_bit_cast(uint64_t, bv);
        const uint64_t ix = (uint64_t)bi;
        __hip_atomic_store(best, (unsigned long long)o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(best + 1, (unsigned long long)ix, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (mirror) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            mirror[0] = o;
            mirror[1] = ix;
            mirror[2] = seq;
            mirror[3] = mirror_check(o, ix, seq);
        }
    }
}

}  // namespace mac
