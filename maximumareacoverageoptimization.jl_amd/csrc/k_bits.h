// k_bits.h — shared-entry ownership from per-position coverage bit-words (the poll kernel's
// shared role, k_poll.h).
//
// The shared entries S_i of disk i are the entries of region i that some lower-index disk j can
// also cover: their tile lies in region j's box (k_poll_shared.h). Entry e of S_i is credited to
// disk i of candidate k iff disk i at its position u_i(k) covers e and no neighbour j < i at its
// position u_j(k) does (src/AreaCoverageCalculation.jl:67-78: first hit in disk order). A MADS
// poll holds a few hundred distinct disks per UAV (k_index.h), so instead of testing every
// (candidate, shared entry, neighbour) triple in fp64 (poll_shared_job) this job
//   1. computes, for every distinct position u of every disk d in {i} + neighbours, the bit-word
//      B_d[u] of the shared entries it covers (64 entries per word, tested with the walk's exact
//      fp32 filter, k_poll.h header; band entries re-decided in fp64), into LDS;
//   2. per candidate k: W = B_i[u_i(k)] & ~B_j1[u_j1(k)] & ~B_j2[u_j2(k)] ..., and adds
//      popcount(W) (equal weights) or the weights of W's entries in list order.
// Tests drop from K x |S_i| x (1 + neighbours) fp64 to (U_i + sum U_j) x |S_i| fp32.
//
// Passes of kBitsWP words (two entries per lane, every wave holds the same entries); disks in
// groups whose positions fit the table (kBitsTab positions x kBitsWP words) and whose map values
// fit registers (kBitsGrp disks); candidates [kb, kb + kBitsK) in registers (kBitsPT per thread).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

#include "predicate.h"
#include "k_common.h"
#include "k_lane.h"
#include "k_poll_shared.h"

#pragma clang fp contract(off)

namespace mac {

#ifdef MAC_DIAG
// diagnostic build only: per workgroup, ticks (s_memrealtime, 10 ns) spent in each phase and counts
__device__ uint64_t g_diag_bits[256 * 16];
#define MAC_BITS_T(q) do { if (threadIdx.x == 0) { const uint64_t t_ = __builtin_amdgcn_s_memrealtime(); dg[q] += t_ - dt; dt = t_; } } while (0)
#define MAC_BITS_N(q) do { if (threadIdx.x == 0) dg[q] += 1; } while (0)
#else
#define MAC_BITS_T(q)
#define MAC_BITS_N(q)
#endif

constexpr int kBitsThreads = 1024;                  // 16 waves: one workgroup per CU
constexpr int kBitsWaves = kBitsThreads / kWave;
constexpr int kBitsPT = 4;                          // candidates per thread
constexpr int kBitsK = kBitsPT * kBitsThreads;      // candidates per job (4096)
constexpr int kBitsWP = 2;                          // 64-entry words per pass
constexpr int kBitsGrp = 4;                         // disks per table group
constexpr int kBitsD = kPollNbr + 1;
#ifndef MAC_BITS_SPLIT
#define MAC_BITS_SPLIT 2
#endif
constexpr int kBitsSplit = MAC_BITS_SPLIT;          // jobs per disk (equal weights)
constexpr int kBitsPL = 2;                          // positions per lane in the tables
constexpr int kBitsBlk = kBitsPL * kWave;           // positions per wave block
constexpr int kBitsE = 1024;                        // shared entries staged in LDS at a time
constexpr int kBitsUC = 16384;                      // map values cached per job (uint16)


// (cur << 1) | sign bit of v, one v_alignbit_b32 ({cur, v} >> 31). Written as asm: the compiler's
// funnel-shift folding was seen to drop the second half of a packed pair feeding this chain.
__device__ __forceinline__ uint32_t shift_in_sign(uint32_t cur, float v)
{
    uint32_t r;
    asm("v_alignbit_b32 %0, %1, %2, 31" : "=v"(r) : "v"(cur), "v"(v));
    return r;
}

__device__ __forceinline__ f32x2 fma2v(f32x2 a, float b, f32x2 c)
{
    return __builtin_elementwise_fma(a, (f32x2)b, c);
}

// Runs of shared tiles of region R (at most 64 tiles wide and 64 rows high, neighbors_block): per
// row, the union of the neighbour boxes as a 64-bit tile mask, whose runs of tiles are contiguous
// runs of entries (at most 32 per row). Wave 0 writes run_s / run_pre (exclusive prefix of the run
// lengths, run_pre[nrun] = total) and *nruns; returns the number of shared entries after a
// barrier (all threads call it; the result is block-uniform).
constexpr int kBitsRuns = 64 * 32;
__device__ __forceinline__ int shared_runs(const int32_t* __restrict__ off, const Grid& g,
                                           const int4& R, int ncl, const int4* nbox,
                                           int* run_s, int* run_pre, int* nruns)
{
    const int tid = threadIdx.x;
    const int tw = R.y - R.x + 1, nrows = R.w - R.z + 1;
    if (tid < kWave) {
        uint64_t mask = 0;
        const int r = R.z + tid;
        if (tid < nrows) {
            for (int m = 0; m < ncl; ++m) {
                const int4 Q = nbox[m];
                if (r < Q.z || r > Q.w) continue;
                const int a = max(R.x, Q.x) - R.x, b = min(R.y, Q.y) - R.x;
                if (a <= b)   // tiles a..b of the row
                    mask |= (b - a == 63 ? ~0ull : ((1ull << (b - a + 1)) - 1)) << a;
            }
            if (tw < 64) mask &= (1ull << tw) - 1;
        }
        const uint64_t starts = mask & ~(mask << 1);
        const int cnt = __popcll(starts);
        const int64_t rowbase = (int64_t)r * g.nTx + R.x;
        // this row's entries in its runs, then the rows' prefix
        int len_row = 0;
        for (uint64_t m2 = mask; m2;) {
            const int a = __builtin_ctzll(m2);
            const uint64_t from = m2 >> a;
            const int len = ~from ? __builtin_ctzll(~from) : 64 - a;   // tiles in the run
            len_row += off[rowbase + a + len] - off[rowbase + a];
            m2 &= len + a >= 64 ? 0ull : (~0ull << (a + len));
        }
        const int qi = wave_incl_scan_i32(cnt, tid);
        const int ei = wave_incl_scan_i32(len_row, tid);
        int q = qi - cnt, pre = ei - len_row;
        for (uint64_t m2 = mask; m2;) {
            const int a = __builtin_ctzll(m2);
            const uint64_t from = m2 >> a;
            const int len = ~from ? __builtin_ctzll(~from) : 64 - a;
            const int s0 = off[rowbase + a];
            run_s[q] = s0;
            run_pre[q] = pre;
            pre += off[rowbase + a + len] - s0;
            ++q;
            m2 &= len + a >= 64 ? 0ull : (~0ull << (a + len));
        }
        if (tid == kWave - 1) {
            *nruns = qi;
            run_pre[qi] = ei;
        }
    }
    __syncthreads();
    return run_pre[*nruns];
}

// sorted-list index of shared entry f (0 <= f < total) through the runs
__device__ __forceinline__ int run_entry(const int* run_s, const int* run_pre, int nrun, int f)
{
    int lo = 0, hi = nrun - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (run_pre[mid] <= f) lo = mid; else hi = mid - 1;
    }
    return run_s[lo] + (f - run_pre[lo]);
}

// Shared-entry pass by bit-words (the header): grid-strides over the jobs (disk N - 1 - j / nsub,
// candidates [kb, kb + kBitsK)), taking job blockIdx.x first, then jobs from
// a counter (cleared by the index kernel). Runs only when the poll walk was chosen and more than
// kBitsMinDisks disks have neighbours (fewer: the poll kernel's fp64 jobs take them all), over
// the disks neighbors_block flagged in qual (the others: the poll kernel's fp64 jobs). Writes
// spart[i*K + k]: uint32 counts (kCounts: every entry weighs the same) or fp64 weights.
template <bool kCounts>
__global__ __launch_bounds__(kBitsThreads) void shared_bits_kernel(
    uint64_t* ts, const double2* __restrict__ xy, const double* __restrict__ w, const int32_t* __restrict__ off,
    Grid g, const DiskRec* __restrict__ urec, const int* __restrict__ umap,
    const int* __restrict__ ucount, const int4* __restrict__ region,
    const uint16_t* __restrict__ nbrT, const float4* __restrict__ lane4,
    const float* __restrict__ lanexp, const int* __restrict__ ncount,
    const int* __restrict__ qual, int* __restrict__ dcount, const int* __restrict__ mode, int N,
    int K, double* __restrict__ spart, int min_disks)
{
    __shared__ int sd[kBitsD], sU[kBitsD];
    __shared__ int4 sbox[kBitsD];
    __shared__ double2 sorg[kBitsD];
    __shared__ int run_s[kBitsRuns], run_pre[kBitsRuns + 1];
    __shared__ int nruns, sjob;
    __shared__ __attribute__((aligned(16))) uint4 tab[kBitsTab];   // [position in group]: 2 words
    __shared__ double swa[kBitsE];       // the job's shared entries (kBitsE at a time): weights,
    __shared__ double2 s64a[kBitsE];     // exact coordinates (NaN past the list), tiles
    __shared__ int2 stilea[kBitsE];
    __shared__ uint16_t ucache[kBitsUC]; // map values of the job's disks, [m][k - kb] (when they fit)
    __shared__ float4 ent[kBitsGrp][kWave * kBitsWP / 2];   // {U0, U1, V0, V1} per entry pair
    __shared__ f32x2 entq[kBitsGrp][kWave * kBitsWP / 2];   // {Q0, Q1}
    __shared__ int slive[kBitsGrp], sg_toff[kBitsGrp], sg_bp[kBitsGrp + 1], sg_np, sg_next[2];
    __shared__ int sg_m[kBitsGrp], sg_lo[kBitsGrp], sg_hi[kBitsGrp];

    ts_begin(ts);   // profiling only (k_common.h)
    if ((mode && *mode != kModePoll) ||                            // uniform
        dcount[kDcBits] + dcount[kDcOther] <= min_disks) {         // the poll kernel's jobs
        ts_end(ts);
        return;
    }
    const int tid = threadIdx.x, lane = tid & (kWave - 1);
    const int wid = __builtin_amdgcn_readfirstlane(tid / kWave);   // wave-uniform (scalar loads)
#ifdef MAC_DIAG
    uint64_t dg[16] = {};
    uint64_t dt = __builtin_amdgcn_s_memrealtime();
    const uint64_t dt0 = dt;
#endif
    // jobs in descending disk order: higher-index disks have more lower-index neighbours, so the
    // heavy jobs go first; disks not listed for this kernel (qual[i] == 0) are skipped
    // equal weights: each disk's passes are split over kBitsSplit jobs whose counts add up in
    // spart with integer atomics (exact in any order; the poll kernel zeroed those rows);
    // weights: one job per disk and candidate chunk, stored (a fixed fp64 summation order)
    constexpr int kSplit = kCounts ? kBitsSplit : 1;
    const int nsub = (K + kBitsK - 1) / kBitsK;
    const int njobs = N * nsub * kSplit;
    constexpr int kPass = kWave * kBitsWP;
    typedef typename std::conditional<kCounts, uint32_t, double>::type Acc;

    for (int job = blockIdx.x;;) {
        if (job >= njobs) break;   // uniform
        const int i = N - 1 - job / (nsub * kSplit);
        const int kb = ((job / kSplit) % nsub) * kBitsK, split = job % kSplit;
        if (qual[i]) {
            const int nc = ncount[i], nd = 1 + nc;
            if (tid < nd) {
                const int d = tid == 0 ? i : (int)nbrT[i * kPollNbr + tid - 1];
                const int4 Rd = region[d];
                sd[tid] = d;
                sU[tid] = ucount[d];
                sbox[tid] = Rd;
                sorg[tid] = make_double2(g.gx0 + 0.5 * (double)(Rd.x + Rd.y + 1) * g.S,
                                         g.gy0 + 0.5 * (double)(Rd.z + Rd.w + 1) * g.S);
            }
            __syncthreads();
            const int total = shared_runs(off, g, sbox[0], nc, sbox + 1, run_s, run_pre, &nruns);
            MAC_BITS_T(0);
            MAC_BITS_N(8);
            const int nrun = nruns;
            const int kend = min(K, kb + kBitsK);
            const int kc = kend - kb;
            // the job's map values in LDS when they fit (positions < kBitsTab < 2^16)
            const bool cached = nd * kc <= kBitsUC;
            if (cached)
                for (int t = tid; t < nd * kc; t += kBitsThreads) {
                    const int m = t / kc, kk = t - m * kc;
                    ucache[t] = (uint16_t)umap[(int64_t)sd[m] * K + kb + kk];
                }

            // per candidate: the covered-entry count (kCounts) or the fp64 weight sum
            Acc acc[kBitsPT];
#pragma unroll
            for (int c = 0; c < kBitsPT; ++c) acc[c] = 0;
            // this job's passes: a contiguous share of the disk's
            const int npass = (total + kPass - 1) / kPass;
            const int pbeg = (split * npass / kSplit) * kPass, pend = min(total, ((split + 1) * npass / kSplit) * kPass);
            for (int pb = pbeg; pb < pend; pb += kPass) {
                __syncthreads();   // the previous pass's entries, weights and tables are done
                if ((pb - pbeg) % kBitsE == 0) {
                    // the next kBitsE shared entries: exact coordinates (NaN past the list),
                    // tiles, weights
                    for (int t = tid; t < kBitsE; t += kBitsThreads) {
                        const int e = pb + t;
                        double2 p = make_double2(__builtin_nan(""), __builtin_nan(""));
                        double ww = 0.0;
                        if (e < total) {
                            const int j = run_entry(run_s, run_pre, nrun, e);
                            p = xy[j];
                            if (!kCounts) ww = w[j];
                        }
                        s64a[t] = p;
                        stilea[t] = e < total ? make_int2(tile_of(p.x, g.gx0, g.invS, g.nTx),
                                                          tile_of(p.y, g.gy0, g.invS, g.nTy))
                                              : make_int2(-1, -1);
                        if (!kCounts) swa[t] = ww;
                    }
                }
                const double2* const s64 = s64a + (pb - pbeg) % kBitsE;
                const int2* const stile = stilea + (pb - pbeg) % kBitsE;
                const double* const sw = swa + (pb - pbeg) % kBitsE;
                uint64_t W0[kBitsPT], W1[kBitsPT];
#pragma unroll
                for (int c = 0; c < kBitsPT; ++c) W0[c] = W1[c] = 0;
                MAC_BITS_N(9);
                // groups of at most kBitsGrp pieces = (disk m, position range [lo, hi)) of at most
                // kBitsTab positions in all, in disk order then position order: disk i's pieces come
                // first (W |= its word: each candidate's position lies in exactly one piece), then
                // the neighbours' (W &= ~word)
                for (int gm = 0, gu = 0; gm < nd;) {
                    if (tid == 0) {
                        int m = gm, u = gu, used = 0, np = 0;
                        while (m < nd && np < kBitsGrp && used < kBitsTab) {
                            const int take = min(sU[m] - u, kBitsTab - used);
                            sg_m[np] = m;
                            sg_lo[np] = u;
                            sg_hi[np] = u + take;
                            sg_toff[np] = used;
                            used += take;
                            ++np;
                            u += take;
                            if (u == sU[m]) {
                                ++m;
                                u = 0;
                            }
                        }
                        sg_np = np;
                        sg_next[0] = m;
                        sg_next[1] = u;
                    }
                    if (tid < kBitsGrp) slive[tid] = 0;
                    __syncthreads();
                    MAC_BITS_T(1);
                    MAC_BITS_N(10);
                    const int np = sg_np;
                    // the pieces' entries relative to their disk's region centre, as the walk
                    // stages them (k_poll.h), in pairs {U0, U1, V0, V1}, {Q0, Q1}; entries outside
                    // region d's box, past the list or non-finite are inert: Q = +inf (d' = -inf)
                    for (int t = tid; t < kBitsGrp * kPass; t += kBitsThreads) {
                        const int q = t / kPass, e = t - q * kPass;
                        if (q >= np) continue;
                        const int m = sg_m[q];
                        const double2 p = s64[e];
                        const int2 tl = stile[e];
                        const int4 bx = sbox[m];
                        const bool in = tl.x >= 0 && (m == 0 || box_has(bx, tl.x, tl.y));
                        const double2 o = sorg[m];
                        const float fu = (float)(p.x - o.x), fv = (float)(p.y - o.y);
                        const bool f = in && __builtin_isfinite(fu) && __builtin_isfinite(fv);
                        float* const eu = reinterpret_cast<float*>(&ent[q][e >> 1]);
                        eu[(e & 1)] = f ? fu : 0.0f;
                        eu[2 + (e & 1)] = f ? fv : 0.0f;
                        reinterpret_cast<float*>(&entq[q][e >> 1])[e & 1] =
                            f ? __builtin_fmaf(fu, fu, fv * fv) : __builtin_inff();
                        if (in) atomicOr(&slive[q], 1 << (e >> 5));   // live 32-entry words
                    }
                    __syncthreads();
                    if (tid == 0) {   // kBitsPL * 64-position blocks of the live pieces, flattened
                        int nb = 0;
                        for (int q = 0; q < kBitsGrp; ++q) {
                            sg_bp[q] = nb;
                            if (q < np && slive[q]) nb += (sg_hi[q] - sg_lo[q] + kBitsBlk - 1) / kBitsBlk;
                        }
                        sg_bp[kBitsGrp] = nb;
                    }
                    __syncthreads();
                    MAC_BITS_T(2);
                    // tables: lane = kBitsPL positions of a disk, bits = their coverage of the entries
                    const int nbt = sg_bp[kBitsGrp];
#ifdef MAC_DIAG
                    if (tid == 0) dg[11] += nbt;
#endif
                    for (int b = wid; b < nbt; b += kBitsWaves) {
                        asm volatile("" ::: "memory");   // re-read the entries per block: not hoisted
                        int q = 0;
#pragma unroll
                        for (int z = 1; z < kBitsGrp; ++z) q += b >= sg_bp[z] ? 1 : 0;
                        const int m = sg_m[q], d = sd[m], U = sg_hi[q], lo = sg_lo[q];
                        const int64_t row = (int64_t)d * K;
                        const int p0 = lo + (b - sg_bp[q]) * kBitsBlk + lane;
                        float4 c[kBitsPL];
                        float xp[kBitsPL];
                        f32x2 sa[kBitsPL], sb[kBitsPL], st[kBitsPL], ns[kBitsPL], xp2[kBitsPL];
#pragma unroll
                        for (int h = 0; h < kBitsPL; ++h) {
                            const int pp = p0 + h * kWave;
                            c[h] = pp < U ? lane4[row + pp] : make_float4(0.0f, 0.0f, -1.0f, -1.0f);
                            xp[h] = pp < U ? lanexp[row + pp] : -1.0f;
                            sa[h] = f32x2{c[h].x, c[h].x};
                            sb[h] = f32x2{c[h].y, c[h].y};
                            st[h] = f32x2{c[h].z, c[h].z};
                            ns[h] = f32x2{c[h].w, c[h].w};
                            xp2[h] = f32x2{xp[h], xp[h]};
                        }
                        const float4* const eq = ent[q];
                        const f32x2* const eqq = entq[q];
                        const int wlive = slive[q];   // words holding an entry in the disk's box
                        float bmin[kBitsPL];
                        // per position the four words (32 entries each) side by side: independent
                        // chains (bit e % 32 of word e / 32 = entry e covered); every entry read
                        // from LDS serves kBitsPL positions
                        uint32_t cur[kBitsPL][4];
#pragma unroll
                        for (int h = 0; h < kBitsPL; ++h) {
                            bmin[h] = __builtin_inff();
#pragma unroll
                            for (int wv = 0; wv < 4; ++wv) cur[h][wv] = 0u;
                        }
#pragma unroll 1
                        for (int j = 0; j < 16; ++j) {
#pragma unroll
                            for (int wv = 0; wv < 4; ++wv) {
                                if (!((wlive >> wv) & 1)) continue;   // uniform: no entry of the
                                                                      // word can be covered (0 bits)
                                const float4 uv = eq[16 * wv + j];
                                const f32x2 qq = eqq[16 * wv + j];
                                const f32x2 U2 = {uv.x, uv.y}, V2 = {uv.z, uv.w};
#pragma unroll
                                for (int h = 0; h < kBitsPL; ++h) {
                                    const f32x2 dd = __builtin_elementwise_fma(
                                        qq, ns[h], __builtin_elementwise_fma(V2, sb[h], __builtin_elementwise_fma(U2, sa[h], st[h])));
                                    // covered iff d' > X' iff X' - d' < 0 (exact: d' is never NaN):
                                    // its sign bit, shifted in at the bottom (the word is
                                    // bit-reversed at the end, so entry e lands on bit e % 32)
                                    const f32x2 sd2 = xp2[h] - dd;
                                    cur[h][wv] = shift_in_sign(cur[h][wv], sd2.x);
                                    cur[h][wv] = shift_in_sign(cur[h][wv], sd2.y);
                                    bmin[h] = __builtin_fminf(bmin[h], __builtin_fminf(__builtin_fabsf(dd.x),
                                                                                       __builtin_fabsf(dd.y)));
                                }
                            }
                        }
#pragma unroll
                        for (int h = 0; h < kBitsPL; ++h) {
                            const int pp = p0 + h * kWave;
                            if (pp >= U) continue;
                            uint4 t4 = make_uint4(__builtin_bitreverse32(cur[h][0]), __builtin_bitreverse32(cur[h][1]),
                                                  __builtin_bitreverse32(cur[h][2]), __builtin_bitreverse32(cur[h][3]));
                            // X' < 2 for every normal position: no |d'| <= 2 means no band entry;
                            // a band (or forced) position re-decides its entries, band ones in fp64
                            if (bmin[h] <= 2.0f || !(xp[h] < 2.0f)) {
                                const DiskRec r = urec[row + pp];
                                uint32_t t[4] = {0u, 0u, 0u, 0u};
                                for (int e = 0; e < kPass; ++e) {
                                    const float4 uv = eq[e >> 1];
                                    const float qq = reinterpret_cast<const float*>(&eqq[e >> 1])[e & 1];
                                    const float U1 = (e & 1) ? uv.y : uv.x, V1 = (e & 1) ? uv.w : uv.z;
                                    const float dp = __builtin_fmaf(qq, c[h].w, __builtin_fmaf(V1, c[h].y, __builtin_fmaf(U1, c[h].x, c[h].z)));
                                    bool cov = dp > xp[h];
                                    if (__builtin_fabsf(dp) <= xp[h]) {
                                        const double2 p = s64[e];
                                        cov = qq != __builtin_inff() && sqdist(p.x, p.y, r.cx, r.cy) <= r.T;
                                    }
                                    if (cov) t[e >> 5] |= 1u << (e & 31);
                                }
                                t4 = make_uint4(t[0], t[1], t[2], t[3]);
                            }
                            tab[sg_toff[q] + pp - lo] = t4;
                        }
                    }
                    __syncthreads();
                    MAC_BITS_T(3);
                    // combine: W = B_i[u_i] & ~B_j[u_j] ... over the group's disks (the map
                    // values of this thread's candidates all in flight at once)
                    int um[kBitsPT][kBitsGrp];
#pragma unroll
                    for (int c = 0; c < kBitsPT; ++c) {
                        const int k = kb + tid + c * kBitsThreads;
#pragma unroll
                        for (int q = 0; q < kBitsGrp; ++q) {
                            const int m = sg_m[q];
                            um[c][q] = (k < kend && q < np && slive[q])
                                           ? (cached ? (int)ucache[m * kc + k - kb]
                                                     : umap[(int64_t)sd[m] * K + k])
                                           : -1;
                        }
                    }
#pragma unroll
                    for (int c = 0; c < kBitsPT; ++c) {
#pragma unroll
                        for (int q = 0; q < kBitsGrp; ++q) {
                            const int u = um[c][q] - sg_lo[q];
                            if (um[c][q] < 0 || u < 0 || um[c][q] >= sg_hi[q]) continue;
                            const uint4 t = tab[sg_toff[q] + u];
                            const uint64_t a0 = (uint64_t)t.x | ((uint64_t)t.y << 32);
                            const uint64_t a1 = (uint64_t)t.z | ((uint64_t)t.w << 32);
                            if (sg_m[q] == 0) {
                                W0[c] |= a0;
                                W1[c] |= a1;
                            } else {
                                W0[c] &= ~a0;
                                W1[c] &= ~a1;
                            }
                        }
                    }
                    __syncthreads();   // the next group overwrites the tables and its info
                    MAC_BITS_T(4);
                    gm = sg_next[0];
                    gu = sg_next[1];
                }
#pragma unroll
                for (int c = 0; c < kBitsPT; ++c) {
                    if constexpr (kCounts) {
                        acc[c] += (uint32_t)(__popcll(W0[c]) + __popcll(W1[c]));
                    } else {   // weights of the credited entries, in list order
                        uint64_t a = W0[c];
                        while (a) {
                            acc[c] += sw[__builtin_ctzll(a)];
                            a &= a - 1;
                        }
                        a = W1[c];
                        while (a) {
                            acc[c] += sw[kWave + __builtin_ctzll(a)];
                            a &= a - 1;
                        }
                    }
                }
            }
#pragma unroll
            for (int c = 0; c < kBitsPT; ++c) {
                const int k = kb + tid + c * kBitsThreads;
                if (k >= kend) continue;
                if constexpr (kCounts) {
                    if (acc[c]) atomicAdd(reinterpret_cast<unsigned*>(spart) + (int64_t)i * K + k, acc[c]);
                } else {
                    spart[(int64_t)i * K + k] = acc[c];
                }
            }
        }
        // the next job
        __syncthreads();
        MAC_BITS_T(5);
        if (tid == 0) sjob = (int)gridDim.x + atomicAdd(dcount + kDcBitsJobs, 1);
        __syncthreads();
        job = sjob;
    }
#ifdef MAC_DIAG
    if (tid == 0 && blockIdx.x < 256) {
        dg[12] = __builtin_amdgcn_s_memrealtime() - dt0;
        for (int q = 0; q < 16; ++q) g_diag_bits[16 * blockIdx.x + q] = dg[q];
    }
#endif
    ts_end(ts);
}

}  // namespace mac
