// k_poll_shared.h — ownership for the poll walk: per-disk neighbour lists (once per poll) and
// the exact pass over "shared" entries, the entries of region i that a lower-index disk j can
// also cover (their tile lies in region j's box, and boxes i, j overlap).
//
// The main poll kernel (k_poll.h) never credits a shared entry; this kernel adds, for every
// (disk i, candidate k), the weight of the shared entries that disk i of candidate k covers and
// no disk j < i of candidate k covers — in fp64, exactly the reference predicate — to
// partial[i*K + k]. Together: every entry is credited to the lowest-index disk covering it.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "predicate.h"
#include "k_common.h"
#include "k_index.h"
#include "k_or.h"

#pragma clang fp contract(off)

namespace mac {

// Disk i's lower-index neighbours: the disks j < i whose region boxes overlap region i's (at
// most kPollNbr kept in nbr[i*kPollNbr ...]; ncount[i] is the true count, > kPollNbr meaning
// "overflowed"), their region boxes in nboxT. Disks with neighbours are appended to dlist (order irrelevant: each is processed
// independently); *dcount must be zero on entry (the disk index clears it).
// A disk with neighbours goes to the bit-word kernel's list (front of dlist, k_bits.h) when its
// list did not overflow and its region is at most 64 x 64 tiles; otherwise to the back of dlist
// (the poll kernel's fp64 jobs).
// With nboxU (the shared-entry union pass, k_or.h): also the UPPER neighbours' boxes (j > i,
// nboxU / ncountU, at most kPollNbr kept), and the lists in LDS for the caller (lbox / ubox,
// counts in cnt2[0..1]); a disk with lower neighbours whose upper list overflows is counted in
// dcount[kDcOrBad] (the union pass then stands down for the poll).
// R: region i; Q[q]: region j = threadIdx.x + q * kBlock (j < i), loaded by the caller beside the
// walk choice's costs (one round trip); further j are loaded here.
constexpr int kNbrPre = 4;   // regions per thread loaded up front (i <= 1024)
__device__ __forceinline__ void neighbors_block(int i, int N, const int4& R, const int4 (&Q)[kNbrPre],
                                                const int4* __restrict__ region,
                                                uint16_t* __restrict__ nbr, int4* __restrict__ nboxT,
                                                int* __restrict__ ncount,
                                                int* __restrict__ dlist, int* __restrict__ dcount,
                                                int* __restrict__ qual,
                                                int4* __restrict__ nboxU = nullptr,
                                                int* __restrict__ ncountU = nullptr,
                                                int4* lbox = nullptr, int4* ubox = nullptr,
                                                int* cnt2 = nullptr)
{
    __shared__ int cnt, cntU;
    if (threadIdx.x == 0) {
        cnt = 0;
        cntU = 0;
    }
    // the upper neighbours' regions in flight beside the lower ones' tests
    int4 QU[kNbrPre];
#pragma unroll
    for (int q = 0; q < kNbrPre; ++q) {
        const int j = i + 1 + (int)threadIdx.x + q * kBlock;
        QU[q] = nboxU && j < N ? region[j] : make_int4(0x7fffffff, -1, 0x7fffffff, -1);
    }
    __syncthreads();
    if (R.x <= R.y) {
        auto test = [&](int j, const int4& B) {
            if (box_overlap(B, R)) {
                const int p = atomicAdd(&cnt, 1);  // list order is irrelevant (a boolean OR)
                if (p < kPollNbr) {
                    nbr[i * kPollNbr + p] = (uint16_t)j;
                    nboxT[i * kPollNbr + p] = B;   // the neighbour's region box
                    if (lbox) lbox[p] = B;
                }
            }
        };
#pragma unroll
        for (int q = 0; q < kNbrPre; ++q) {
            const int j = threadIdx.x + q * kBlock;
            if (j < i) test(j, Q[q]);
        }
        for (int j = threadIdx.x + kNbrPre * kBlock; j < i; j += kBlock) test(j, region[j]);
        if (nboxU) {
            auto testU = [&](const int4& B) {
                if (box_overlap(B, R)) {
                    const int p = atomicAdd(&cntU, 1);
                    if (p < kPollNbr) {
                        nboxU[i * kPollNbr + p] = B;
                        ubox[p] = B;
                    }
                }
            };
#pragma unroll
            for (int q = 0; q < kNbrPre; ++q) testU(QU[q]);
            for (int j = i + 1 + (int)threadIdx.x + kNbrPre * kBlock; j < N; j += kBlock) testU(region[j]);
        }
    }
    __syncthreads();
    const int nc = cnt;   // (uniform, as R is)
    const bool bad = nc > 0 && (nc > kPollNbr || R.y - R.x + 1 > 64 || R.w - R.z + 1 > 64);
    if (threadIdx.x == 0) {
        ncount[i] = nc;
        qual[i] = nc > 0 && !bad ? 1 : 0;
        if (nc > 0) {
            if (!bad) dlist[atomicAdd(dcount + kDcBits, 1)] = i;
            else dlist[N - 1 - atomicAdd(dcount + kDcOther, 1)] = i;
        }
        if (nboxU) {
            ncountU[i] = cntU;
            if (nc > 0 && cntU > kPollNbr) atomicAdd(dcount + kDcOrBad, 1);
        }
    }
    if (cnt2 && threadIdx.x == 0) {
        cnt2[0] = nc;
        cnt2[1] = cntU;
    }
}

// The device-side walk choice, both costs in one unit (poll-walk tests): the poll walk tests
// every entry of region i against each distinct disk i (A = sum of cost[i].x = U_i * |region i|
// entry visits, broadcast LDS reads); the per-candidate walk visits each candidate's span entries
// (cost[i].y summed) with scattered global loads and tests each covered one against the disks of
// disk i's poll-level neighbour list (ncount[i]; an overflowed list: every lower-index disk, i of
// them, k_walk.h) in fp64 — a visit and a pair test each cost about `ratio` poll-walk tests
// (4: measured) — so B = ratio * sum_i spans_i * (1 + list_i). Poll when A <= B, or `forced`.
// Every block sums in the same fixed order, so every block gets the same choice. Block-uniform
// result. (Round 2's choice, made before the lists existed, priced every pair, K N(N-1)/2: a
// crowded config-5 poll had picked the per-candidate walk on visits alone and rebuilt all pairs
// in every unit, 3.96 ms. Round 3 priced the pairs once per candidate, K * sum_i list_i, not per
// visited entry: the config-5 regression poll at ell 5 then picked the per-candidate walk, 7.1 ms
// against 0.69 ms for the poll walk and the union pass (tools/c5_walks.py); tests/test_gpu_parity.py
// pins both choices.)
__device__ __forceinline__ int walk_choice(int N, int K, const double2* __restrict__ cost,
                                           const int* __restrict__ ncount, double ratio, int forced)
{
    __shared__ double red[kWavesPerBlock];
    __shared__ int smode;
    if (forced) return forced;
    // the per-candidate walk visits every span entry of disk j and tests each covered one
    // against the disk's listed neighbours: span tiles x (1 + list length)
    double a = 0.0, b = 0.0;
    for (int j = threadIdx.x; j < N; j += kBlock) {
        a += cost[j].x;
        const int nc = ncount[j];
        b += cost[j].y * (1.0 + (double)(nc <= kPollNbr ? nc : j));
    }
    (void)K;
    const double A = block_sum_f64(a, red);
    __syncthreads();
    const double B = block_sum_f64(b, red);
    __syncthreads();
    if (threadIdx.x == 0) smode = A <= ratio * B ? kModePoll : kModeTiled;
    __syncthreads();
    return smode;
}

// Entry (tile tx, ty) of region i is shared when it lies in a neighbour's box.
__device__ __forceinline__ bool entry_shared(int nc, const int4* nbox, int tx, int ty)
{
    if (nc > kPollNbr) return true;
    bool s = false;
    for (int m = 0; m < nc; ++m) s |= box_has(nbox[m], tx, ty);
    return s;
}

// Shared-entry pass of the poll kernel (k_poll.h). A job is (disk dlist[job / nsub], candidates
// [kb, kb + C), kb = (job % nsub) * C), C = kShC or kShCWide (the poll kernel picks); the
// workgroup's threads are C candidates x G = 256 / C entry groups. Shared entries are compacted (in
// list order) into LDS round by round; thread (c, eg) decides entries eg, eg + G, ... of each
// round in fp64 for candidate kb + c (the neighbour disks of the candidate preloaded — first four
// — or read once per entry — the rest), and the G group sums are added in group order at the end:
// fixed order. Splitting the entries over groups keeps a heavily overlapped disk from serialising
// one lane per candidate over all of its shared entries; wide jobs re-stage each region fewer
// times when many disks share entries. Writes spart[i*K + k] (the finalize kernel adds the rows of
// the disks with ncount[i] > 0).
constexpr int kShC = 64;                      // candidates per job when few disks share entries
constexpr int kShCWide = kPollThreads;        // ... when many do (one entry group per job)
constexpr int kShG = kPollThreads / kShC;     // the most entry groups
__device__ __forceinline__ void poll_shared_job(
    const double2* __restrict__ xy, const double* __restrict__ w,
    const int32_t* __restrict__ off, const Grid& g, const DiskRec* __restrict__ urec,
    const int* __restrict__ umap, const int4* __restrict__ region, const uint16_t* __restrict__ nbrT,
    const int4* __restrict__ nboxT, const int2* __restrict__ rows,
    const int* __restrict__ ncount, int i, int K, int kb, int C, double* __restrict__ spart,
    int counts)
{
    __shared__ double2 sp[kPollThreads];
    __shared__ double sw[kPollThreads];
    __shared__ int rs[kPollRB], rpre[kPollRB + 1];
    __shared__ int4 nbox[kPollNbr];
    __shared__ uint16_t nbr[kPollNbr];
    __shared__ int wcount[kPollWaves];
    __shared__ double gsum[kPollThreads];     // [group][candidate], C candidates x G groups
    __shared__ int run_s[kPollThreads], run_pre[kPollThreads + 1];
    __shared__ int nruns;

    const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
    const int G = kPollThreads / C;
    const int c = tid % C, eg = tid / C;
    const int k = kb + c;
    const bool valid = k < K;

    const int nc = ncount[i];
    const int ncl = min(nc, kPollNbr);
    const int4 R = region[i];
    const int2 rinfo = tid <= kRowInfo ? rows[(int64_t)i * (kRowInfo + 1) + tid] : make_int2(0, 0);
    const int nrows = R.w - R.z + 1;
    const bool fastrows = nrows <= kRowInfo;   // row runs from the index (k_index.h)
    __syncthreads();  // LDS reuse across jobs
    if (tid < ncl) {
        nbr[tid] = nbrT[i * kPollNbr + tid];
        nbox[tid] = nboxT[i * kPollNbr + tid];
    }
    if (fastrows && tid <= nrows) {
        rs[tid] = rinfo.x;
        rpre[tid] = rinfo.y;
    }
    DiskRec d = DiskRec{0.0, 0.0, -1.0, 0.0};
    DiskRec e[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) e[m] = DiskRec{0.0, 0.0, -1.0, 0.0};
    if (valid) {
        d = rec_of(urec, umap, i, K, k);
#pragma unroll
        for (int m = 0; m < 4; ++m)
            if (m < ncl) e[m] = rec_of(urec, umap, nbrT[i * kPollNbr + m], K, k);
    }
    double acc = 0.0;
    __syncthreads();

    // the fp64 decision of the shared entries in sp/sw[0, ns) for this thread's candidate
    auto decide = [&](int ns) {
        if (valid && d.T >= 0.0) {
            for (int s = eg; s < ns; s += G) {
                const double2 q = sp[s];
                if (!(sqdist(q.x, q.y, d.cx, d.cy) <= d.T)) continue;
                bool stolen = false;
#pragma unroll
                for (int m = 0; m < 4; ++m)
                    if (m < ncl) stolen |= sqdist(q.x, q.y, e[m].cx, e[m].cy) <= e[m].T;
                if (!stolen && nc > 4) {
                    if (nc <= kPollNbr) {
                        for (int m = 4; m < nc && !stolen; ++m) {
                            const DiskRec x = rec_of(urec, umap, nbr[m], K, k);
                            stolen = sqdist(q.x, q.y, x.cx, x.cy) <= x.T;
                        }
                    } else {  // overflowed list: every lower-index overlapping region
                        for (int j = 0; j < i && !stolen; ++j) {
                            if (!box_overlap(region[j], R)) continue;
                            const DiskRec x = rec_of(urec, umap, j, K, k);
                            stolen = sqdist(q.x, q.y, x.cx, x.cy) <= x.T;
                        }
                    }
                }
                if (!stolen) acc += counts ? 1.0 : sw[s];
            }
        }
    };

    // Fast path (regions at most 64 tiles wide and 64 rows high): the shared tiles of each row
    // are runs of a 64-bit tile mask (the union of the neighbour boxes), and a run of tiles is a
    // contiguous run of entries; only those entries are staged, in the same (list) order.
    const int tw = R.y - R.x + 1;
    bool fast = tw <= kWave && nrows <= kWave;
    if (fast) {
        if (tid < kWave) {
            uint64_t mask = 0;
            const int r = R.z + tid;
            if (tid < nrows) {
                const uint64_t all = tw == 64 ? ~0ull : ((1ull << tw) - 1);
                if (nc > kPollNbr) {
                    mask = all;   // overflowed list: every entry is decided here
                } else {
                    for (int m = 0; m < ncl; ++m) {
                        const int4 Q = nbox[m];
                        if (r < Q.z || r > Q.w) continue;
                        const int a = max(R.x, Q.x) - R.x, b = min(R.y, Q.y) - R.x;
                        if (a <= b)   // tiles a..b of the row
                            mask |= (b - a == 63 ? ~0ull : ((1ull << (b - a + 1)) - 1)) << a;
                    }
                }
            }
            const uint64_t starts = mask & ~(mask << 1);
            const int cnt = __popcll(starts);
            const int incl = wave_incl_scan_i32(cnt, tid);
            const int tot = __shfl(incl, kWave - 1, kWave);
            if (tid == 0) nruns = tot;
            if (tot <= kPollThreads) {
                int q = incl - cnt;
                uint64_t m2 = mask;
                const int64_t rowbase = (int64_t)r * g.nTx + R.x;
                while (m2) {
                    const int a = __builtin_ctzll(m2);
                    const uint64_t from = m2 >> a;
                    const int len = ~from ? __builtin_ctzll(~from) : 64 - a;   // tiles in the run
                    const int s0 = off[rowbase + a];
                    run_s[q] = s0;
                    run_pre[q + 1] = off[rowbase + a + len] - s0;
                    ++q;
                    m2 &= len + a >= 64 ? 0ull : (~0ull << (a + len));
                }
            }
        }
        __syncthreads();
        const int nrun = nruns;
        fast = nrun <= kPollThreads;   // uniform
        if (fast) {
            // exclusive prefix of the run lengths (one run per thread)
            const int len = tid < nrun ? run_pre[tid + 1] : 0;
            const int incl = wave_incl_scan_i32(len, lane);
            if (lane == kWave - 1) wcount[wid] = incl;
            __syncthreads();
            int pre = incl - len, total = 0;
            for (int q = 0; q < kPollWaves; ++q) {
                if (q < wid) pre += wcount[q];
                total += wcount[q];
            }
            __syncthreads();
            if (tid < nrun) run_pre[tid] = pre;
            if (tid == 0) run_pre[nrun] = total;
            __syncthreads();
            for (int base = 0; base < total; base += kPollThreads) {
                const int n = min(kPollThreads, total - base);
                if (tid < n) {
                    const int f = base + tid;
                    int lo = 0, hi = nrun - 1;
                    while (lo < hi) {
                        const int mid = (lo + hi + 1) >> 1;
                        if (run_pre[mid] <= f) lo = mid; else hi = mid - 1;
                    }
                    const int j = run_s[lo] + (f - run_pre[lo]);
                    sp[tid] = xy[j];
                    sw[tid] = w[j];
                }
                __syncthreads();
                decide(n);
                __syncthreads();
            }
        }
    }

    for (int rb = R.z; !fast && rb <= R.w; rb += kPollRB) {
        const int nr = min(kPollRB, R.w - rb + 1);
        if (!fastrows) {
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
        for (int base = 0; base < total; base += kPollThreads) {
            // this round's entries (one per thread), shared ones compacted in list order
            const int f = base + tid;
            bool shared = false;
            double2 p = make_double2(0.0, 0.0);
            double ww = 0.0;
            if (f < total) {
                int lo = 0, hi = nr - 1;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (rpre[mid] <= f) lo = mid; else hi = mid - 1;
                }
                const int j = rs[lo] + (f - rpre[lo]);
                p = xy[j];
                ww = w[j];
                shared = entry_shared(nc, nbox, tile_of(p.x, g.gx0, g.invS, g.nTx), rb + lo);
            }
            const uint64_t bal = __ballot(shared);
            if (lane == 0) wcount[wid] = __popcll(bal);
            __syncthreads();
            int pos = __popcll(bal & ((1ull << lane) - 1)), ns = 0;
            for (int q = 0; q < kPollWaves; ++q) {
                if (q < wid) pos += wcount[q];
                ns += wcount[q];
            }
            if (shared) {
                sp[pos] = p;
                sw[pos] = ww;
            }
            __syncthreads();
            decide(ns);
            __syncthreads();
        }
    }
    gsum[eg * C + c] = acc;
    __syncthreads();
    if (eg == 0 && valid) {
        double t = 0.0;
        for (int q = 0; q < G; ++q) t += gsum[q * C + c];
        if (counts) reinterpret_cast<unsigned*>(spart)[(int64_t)i * K + k] = (unsigned)t;
        else spart[(int64_t)i * K + k] = t;
    }
}

}  // namespace mac
