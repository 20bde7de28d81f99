// maxcover.hip — libmaxcover: context, device-resident point list, and the C-ABI declared in
// include/maxcover.h. gfx950 only (hipcc --offload-arch=gfx950).
//
// Reference seam: src/TDM_STATIC_opt.jl:82-100 (AreaMaxObjective / createObjective) and
// src/AreaCoverageCalculation.jl:63-110 (calculateArea). See DESIGN.md.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <dlfcn.h>
#include <sched.h>
#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <hipcub/hipcub.hpp>
#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <new>
#include <string>
#include <type_traits>
#include <thread>
#include <vector>

#include "kernels.h"
#include "maxcover.h"

#pragma clang fp contract(off)

using namespace mac;

static constexpr int kPollMinK = 64;          // below this the per-candidate walk always wins
static constexpr int kTiledMaxN = 2048;       // the per-candidate walk keeps all N disks in LDS;
                                              // more UAVs take the poll walk at any K (one
                                              // workgroup per disk: a per-disk walk for K = 1)
static constexpr double kPollCostRatio = 4.0; // poll walk if its visits <= 4x the other's

// ------------------------------------------------------------------ errors

static thread_local std::string g_last_error;

static int32_t fail(int32_t code, const std::string& msg)
{
    g_last_error = msg;
    return code;
}

struct HipError {
    hipError_t e;
    const char* what;
    int line;
};

#define HCK(expr)                                              \
    do {                                                       \
        hipError_t _e = (expr);                                \
        if (_e != hipSuccess) throw HipError{_e, #expr, __LINE__}; \
    } while (0)

#define ABI_BEGIN try {
#define ABI_END                                                                               \
    }                                                                                         \
    catch (const HipError& he) {                                                              \
        char buf[512];                                                                        \
        snprintf(buf, sizeof buf, "HIP error %d (%s) at maxcover.hip:%d in %s", (int)he.e,     \
                 hipGetErrorString(he.e), he.line, he.what);                                  \
        return fail(he.e == hipErrorOutOfMemory ? MAC_E_NOMEM : MAC_E_HIP, buf);              \
    }                                                                                         \
    catch (const std::bad_alloc&) {                                                           \
        return fail(MAC_E_NOMEM, "host allocation failed");                                   \
    }                                                                                         \
    catch (...) {                                                                             \
        return fail(MAC_E_HIP, "unexpected exception");                                       \
    }

// ------------------------------------------------------------------ device buffers

// hipFree / hipHostFree synchronise the device. While an armed poll's stream wait is enqueued
// ahead of its own launches (mac_poll_arm_dev_f64), a buffer that grows must not be freed there:
// the wait only opens after the arming call returns, so the device would never drain. Frees on
// the arming thread go to this list instead ({pointer, pinned}) and are released at the next
// call that synchronises the device anyway (point-list changes, mac_ctx_destroy).
static thread_local std::vector<std::pair<void*, bool>>* t_defer_free = nullptr;

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    // fine: fine-grained device memory (host-writable through a large BAR: the closure's
    // candidates, closure_launch)
    void reserve(size_t bytes, bool fine = false)
    {
        if (bytes <= cap) return;
        if (p && t_defer_free)
            t_defer_free->push_back({p, false});
        else if (p)
            HCK(hipFree(p));
        p = nullptr;
        cap = 0;
        size_t b = bytes < 256 ? 256 : bytes;
        b = (b + 255) & ~(size_t)255;
        if (fine)
            HCK(hipExtMallocWithFlags(&p, b, hipDeviceMallocFinegrained));
        else
            HCK(hipMalloc(&p, b));
        cap = b;
    }
    // reserve(); true when the buffer was (re)allocated (its contents are then undefined)
    bool grow(size_t bytes)
    {
        if (bytes <= cap) return false;
        reserve(bytes);
        return true;
    }
    void release()
    {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T>
    T* as() const { return (T*)p; }
};

// Page-locked host staging owned by a lane (async copies must not target pageable memory, or
// HIP performs them synchronously).
struct PinnedBuf {
    void* p = nullptr;
    size_t cap = 0;
    void reserve(size_t b, unsigned flags = hipHostMallocDefault)
    {
        if (b <= cap) return;
        if (p && t_defer_free)
            t_defer_free->push_back({p, true});
        else if (p)
            HCK(hipHostFree(p));
        p = nullptr;
        cap = 0;
        HCK(hipHostMalloc(&p, b, flags));
        cap = b;
    }
    void release()
    {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
};

// Per-call scratch + stream ("lane"); lanes are pooled so concurrent host threads each get one.
struct Lane {
    hipStream_t stream = nullptr;
    hipStream_t last = nullptr;   // stream of the most recent use
    hipEvent_t done = nullptr;
    DevBuf cands, disks, partial, area, obj, best, rmax, prev, dlim, region, mode, nbr,
        ncount, dlist, spart, vp, xinc, perm, ucount, umap, keysT, lane4, lanexp, rows, nboxT,
        cnt, dlimraw, finblk, finarrive, c32, p32, qual, nboxU, ncountU, orjobs;
    std::vector<double> h_dlim;
    PinnedBuf h_stage;                         // native MADS driver: best, permutations, incumbent
    PinnedBuf h_io;                            // host-pointer calls: candidates in, results out
    PinnedBuf h_dc;                            // disks with neighbours of the last poll (mapped)
    int* d_dc = nullptr;                       // ... its device address
    int dc_hist[8] = {};                       // ... as read at the last 8 poll enqueues
    PinnedBuf h_cl;                            // closure_kernel's result slot (mapped)
    uint64_t* d_cl = nullptr;                  // ... its device address
    uint64_t cl_seq = 0;
    DevBuf cpart, carrive, ctot;               // closure_kernel: credits, arrivals, packed count
    DevBuf clv;                                // closure candidates written by the host (BAR)
    DevBuf prec, cost;                         // prep launch: per-disk records; walk costs
    int um_hist[8] = {};                       // most distinct positions of a disk, last 8 polls
    int walk_hist[8] = {};                     // the walk AUTO would have chosen, last 8 polls
    // the fused chain (k_fiw.h): displacement partials, failure bytes, credit rows, hint words,
    // the shared entries handed to fin2_kernel
    DevBuf pd, dead8, frows, fwhint, fwlist, fwcount, fwsxy, fwsw;
    int last_chain = 0;                        // the chain of the lane's last poll: 1 five-launch, 2 fused
};

// RCCL's C API, bound at run time from the librccl the process already uses (torch's, or the
// system one): the multi-GPU poll exchange (mac_poll_exchange) issues its all-gather on the poll's
// own stream. The few types it needs, by their published layout (rccl.h): ncclUniqueId is 128
// opaque bytes, ncclComm_t a pointer, ncclUint8 = 1, ncclSuccess = 0.
struct RcclUid {
    char internal[128];
};
struct RcclApi {
    void* lib = nullptr;
    int (*get_unique_id)(RcclUid*) = nullptr;
    int (*comm_init_rank)(void**, int, RcclUid, int) = nullptr;
    int (*all_gather)(const void*, void*, size_t, int, void*, hipStream_t) = nullptr;
    int (*comm_destroy)(void*) = nullptr;
    const char* (*error_string)(int) = nullptr;
};

struct mac_ctx {
    int device = 0;
    int cus = 256;
    std::mutex mu;
    // MAXCOVER_HOST_STATS=1: host time of a device poll call, split at its launches (printed at
    // destroy): [0] entry -> prep launch call, [1] prep launch, [2] fiw launch, [3] fin2 launch
    bool host_stats = false;
    double hs_t[4] = {0, 0, 0, 0};
    int64_t hs_n = 0;
    // the multi-GPU poll exchange (mac_comm_init): an RCCL communicator over the node's ranks and
    // the world x 16-B gather buffer
    RcclApi* rccl = nullptr;
    void* comm = nullptr;
    int comm_rank = 0, comm_world = 0;
    void* d_xrec = nullptr;
    std::mutex xmu;          // mac_exchange_records: its staging
    PinnedBuf h_xrec;        // [own record 256 B][world records]
    void* d_xrec2 = nullptr;
    // the fused chain's routing history over every lane's polls (enqueue_eval): bit q set when the
    // q-th last reported poll did not suit it (a workload property: a MADS stepper or a new lane
    // takes it over from the lanes before it)
    std::atomic<uint64_t> fused_bad{0};
    std::atomic<bool> route_seeded{false};   // the first matrix poll's routing from the poll (seed_route)
    // mac_area_f64's combiner: queued single-candidate requests, one batch launch at a time
    std::mutex cl_mu;
    std::deque<struct ClReq*> cl_q;
    std::atomic<int> cl_busy{0};   // batches being launched (changed under cl_mu; read as a hint)
    std::atomic<int> cl_active{0};   // callers inside mac_area_f64's combiner
    int cl_taken = 0;                // requests in batches in flight (under cl_mu)
    // queued callers sleep on the futex word of their generation (the batches taken since the
    // context began, cl_gen: every request queued between two takes is in the second's batch)
    std::atomic<uint32_t> cl_gen{0};     // (changed under cl_mu)
    std::atomic<int> cl_genw[64] = {};
    int64_t cl_batches = 0, cl_reqs = 0;   // (MAXCOVER_CL_STATS=1: printed at destroy)
    // MAXCOVER_CL_STATS=1 (nanoseconds, relaxed adds: no lock on the combiner's path)
    std::atomic<int64_t> cl_phase_ns[4] = {};   // per batch: staging, copy + launch enqueued, hand-out, lane
    std::atomic<int64_t> cl_req_ns[5] = {};     // per request: queued -> taken -> handed out -> seen ->
                                                // slot read; the call
    std::atomic<int64_t> cl_led{0};             // requests whose own thread led their batch
    std::vector<Lane*> lanes_free;
    std::vector<Lane*> lanes_all;
    hipStream_t setup_stream = nullptr;
    // device polls' result mirror (guarded by mu): one mapped coherent slot {obj bits, index,
    // seq, check} per d_best buffer (k_final.h mirror_check), reassigned least recently used; the
    // finalize of a device poll writes its result into its d_best's slot under a fresh seq
    static constexpr int kMirrorSlots = 64;
    PinnedBuf h_mirror;
    uint64_t* d_mirror = nullptr;
    const void* mirror_key[kMirrorSlots] = {};
    uint64_t mirror_want[kMirrorSlots] = {};
    uint64_t mirror_used[kMirrorSlots] = {};
    uint64_t mirror_seq = 0, mirror_clock = 0;
    // armed polls (mac_poll_arm_dev_f64): the doorbell the streams wait on (coherent host memory), the
    // last ticket armed and the last released (the doorbell's value), tickets voided by a failed
    // arm that are released once every earlier ticket is, and each stream's latest armed ticket
    // (guarded by mu)
    uint64_t* doorbell = nullptr;
    uint64_t armed = 0, fired = 0;
    std::vector<uint64_t> voided;
    std::vector<std::pair<hipStream_t, uint64_t>> armed_on;
    // buffers an arming call replaced (t_defer_free), freed at the next device synchronisation
    std::vector<std::pair<void*, bool>> deferred;

    int algo = MAC_ALGO_AUTO;
    int shared_mode = MAC_SHARED_AUTO;   // MAC_OPT_SHARED
    int chain = MAC_CHAIN_AUTO;          // MAC_OPT_CHAIN
    bool profile = false;
    // In-kernel launch timing (k_common.h ts_begin / ts_end): each profiled walk launch takes
    // nwg consecutive {start, end} slots of `stamps`. a: the scan / tiled launch, b: the poll
    // launch when the device picks the walk (mode != null): the launch that ran is read.
    // c / f: the chain's first launch (the prep) and its last (finalize), whose
    // stamps give the whole poll chain's device span (-1: not stamped)
    // (role stamps, mac_profile_kernels: [r] = {first slot, slots} of launch role r, -1: none)
    struct Prof { int64_t a, na, b, nb; int64_t K; const int* mode; int algo;
                  int64_t c = -1, nc = 0, f = -1, nf = 0;
                  int64_t role[MAC_PROF_ROLES][2] = {{-1, 0}, {-1, 0}, {-1, 0}, {-1, 0}, {-1, 0},
                                                     {-1, 0}, {-1, 0}, {-1, 0}, {-1, 0}}; };
    std::vector<Prof> prof;                          // recorded launches (guarded by mu)
    DevBuf stamps;
    int64_t stamp_cap = 0, stamp_used = 0;           // in workgroup slots (guarded by mu)
    int storage = MAC_STORE_F64;
    int tile_ppt = 4;

    int64_t M = 0;
    bool has_points = false;
    // original (list) order
    DevBuf x, y, w;
    // tile-sorted order
    DevBuf xys, ws, perm, off;
    Grid grid{};
    int64_t nTiles = 1;
    bool w_uniform = false;   // every entry's weight is bit-identical to w0 (build_index)
    // the host writes closure candidates straight into fine-grained device memory (a large-BAR
    // device: no host-to-device copy per closure batch); MAXCOVER_CL_BAR=0 turns it off
    std::atomic<bool> cl_bar{false};
    double w0 = 0.0;
    // setup scratch
    DevBuf keys_in, keys_out, idx_in, tmp, bbox, flags_s, flags_o, keep, sel_count, cx, cy, cw,
        cidx, circ, cdisk;
};

static void set_device(mac_ctx* ctx) { HCK(hipSetDevice(ctx->device)); }

// Free the buffers arming calls replaced; only after the device has been synchronised (every
// armed poll fired and drained).
static void free_deferred(mac_ctx* ctx)
{
    std::vector<std::pair<void*, bool>> v;
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        v.swap(ctx->deferred);
    }
    for (auto& d : v) (void)(d.second ? hipHostFree(d.first) : hipFree(d.first));
}

// A lane's scratch may be reused at once by a call ordered on the SAME stream (stream order
// protects it; `ordered`: the *_dev calls, where `want` may be the null stream 0); on another
// stream only after the lane's last work has completed.
static Lane* acquire_lane(mac_ctx* ctx, hipStream_t want, bool ordered = false)
{
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        if (ordered) {
            for (size_t i = 0; i < ctx->lanes_free.size(); ++i) {
                Lane* l = ctx->lanes_free[i];
                if (l->last == want) {
                    ctx->lanes_free.erase(ctx->lanes_free.begin() + (long)i);
                    return l;
                }
            }
        }
        for (size_t i = 0; i < ctx->lanes_free.size(); ++i) {
            Lane* l = ctx->lanes_free[i];
            if (hipEventQuery(l->done) == hipSuccess) {
                ctx->lanes_free.erase(ctx->lanes_free.begin() + (long)i);
                return l;
            }
        }
    }
    Lane* l = new Lane();
    HCK(hipStreamCreateWithFlags(&l->stream, hipStreamNonBlocking));
    HCK(hipEventCreateWithFlags(&l->done, hipEventDisableTiming));
    HCK(hipEventRecord(l->done, l->stream));
    l->last = l->stream;
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->lanes_all.push_back(l);
    return l;
}

static void release_lane(mac_ctx* ctx, Lane* l, hipStream_t used)
{
    (void)hipEventRecord(l->done, used);
    l->last = used;
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->lanes_free.push_back(l);
}

// Host-pointer calls: a lane on its own stream (synchronised before return).
// Device-pointer calls: the caller's stream; NULL is HIP's null stream, as in every HIP API, so a
// poll is ordered after the caller's default-stream work (torch's default stream is that stream).
// While an armed poll is not fired, no call may free a buffer it outgrows (t_defer_free): the
// free would wait for the device, which waits for the doorbell.
struct DeferFrees {
    mac_ctx* ctx;
    std::vector<std::pair<void*, bool>> v;
    bool on = false;
    explicit DeferFrees(mac_ctx* c) : ctx(c)
    {
        {
            std::lock_guard<std::mutex> lk(ctx->mu);
            on = ctx->armed > ctx->fired && !t_defer_free;
        }
        if (on) t_defer_free = &v;
    }
    ~DeferFrees()
    {
        if (!on) return;
        t_defer_free = nullptr;
        std::lock_guard<std::mutex> lk(ctx->mu);
        ctx->deferred.insert(ctx->deferred.end(), v.begin(), v.end());
    }
};

struct LaneGuard {
    mac_ctx* ctx;
    DeferFrees df;
    Lane* lane;
    hipStream_t used;
    explicit LaneGuard(mac_ctx* c) : ctx(c), df(c), lane(acquire_lane(c, nullptr)), used(lane->stream) {}
    LaneGuard(mac_ctx* c, hipStream_t s) : ctx(c), df(c), lane(acquire_lane(c, s, true)), used(s) {}
    ~LaneGuard() { release_lane(ctx, lane, used); }
};

// A mapped result slot {obj bits, index, seq, check} (k_final.h) read once: true when it holds
// seq `want` and its check word matches (else its stores are still landing, or it is another
// poll's).
static bool mirror_read(const uint64_t* h, uint64_t want, double* obj, int64_t* idx, uint64_t* feas = nullptr)
{
    if (__atomic_load_n(h + 2, __ATOMIC_ACQUIRE) != want) return false;
    const uint64_t o = __atomic_load_n(h + 0, __ATOMIC_ACQUIRE);
    const uint64_t i = __atomic_load_n(h + 1, __ATOMIC_ACQUIRE);
    const uint64_t c = __atomic_load_n(h + 3, __ATOMIC_ACQUIRE);
    const uint64_t f = feas ? __atomic_load_n(h + 4, __ATOMIC_ACQUIRE) : 0;
    if (c != mirror_check(o, i, want, f) || __atomic_load_n(h + 2, __ATOMIC_ACQUIRE) != want) return false;
    *obj = __builtin_bit_cast(double, o);
    *idx = (int64_t)i;
    if (feas) *feas = f;
    return true;
}

// Spin on a slot for up to `ms` milliseconds.
static bool mirror_wait(const uint64_t* h, uint64_t want, double ms, double* obj, int64_t* idx,
                        uint64_t* feas = nullptr)
{
    const auto t0 = std::chrono::steady_clock::now();
    for (int spin = 0;; ++spin) {
        if (mirror_read(h, want, obj, idx, feas)) return true;
        if ((spin & 1023) == 1023 &&
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() > ms)
            return false;
    }
}

static inline unsigned grid1d(int64_t n, int block) { return (unsigned)((n + block - 1) / block); }

// The lane's launch hints, mapped host words the poll kernels write for the next poll's enqueue:
// [0] disks with neighbours, [2] most positions of a disk, [4] the walk AUTO would choose (the
// five-launch chain, k_poll.h); [8..11] the fused chain's report (k_fiw.h kFwHints; -1: none yet)
static void ensure_hints(Lane* L)
{
    if (L->h_dc.p) return;
    L->h_dc.reserve(64, hipHostMallocMapped | hipHostMallocCoherent);
    volatile int* h = (volatile int*)L->h_dc.p;
    for (int q = 0; q < 16; ++q) h[q] = 0;
    h[0] = 1 << 30;   // first poll: launch
    h[8] = -1;
    void* dp = nullptr;
    HCK(hipHostGetDevicePointer(&dp, L->h_dc.p, 0));
    L->d_dc = (int*)dp;
}

// The largest shared-entry work of one disk (entries x lower neighbours) a fused poll may report
// before the lane's next polls take the five-launch chain (its union pass spreads crowded shared
// entries over the whole chip; the fused kernel decides a disk's in its own workgroup).
static constexpr int kFwCrowdWork = 2048;

// fp32 entry points (*_f32): every float is widened to the double of the same value (exact), and
// the fp64 path then evaluates the reference predicate on those doubles.
__global__ void widen_f32_kernel(const float* __restrict__ in, int64_t n, double* __restrict__ out)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) out[t] = (double)in[t];
}

static void widen_async(const float* d_in, int64_t n, double* d_out, hipStream_t s)
{
    if (n <= 0) return;
    hipLaunchKernelGGL(widen_f32_kernel, dim3(grid1d(n, 256)), dim3(256), 0, s, d_in, n, d_out);
    HCK(hipGetLastError());
}

// host floats -> device doubles through the device scratch `stage`
static void upload_widen(const float* h, int64_t n, DevBuf& stage, double* d_out, hipStream_t s)
{
    if (n <= 0) return;
    stage.reserve(sizeof(float) * (size_t)n);
    HCK(hipMemcpyAsync(stage.p, h, sizeof(float) * (size_t)n, hipMemcpyHostToDevice, s));
    widen_async(stage.as<float>(), n, d_out, s);
}

static inline CandSrc matrix_src(const double* d_cands, int N)
{
    CandSrc c{};
    c.cands = d_cands;
    c.ldc = 3 * N;
    return c;
}

// ------------------------------------------------------------------ point list set-up

static Grid choose_grid(double xmn, double xmx, double ymn, double ymx, int64_t M, int ppt)
{
    Grid g{};
    if (!(xmn <= xmx) || !(ymn <= ymx) || M <= 0) {  // no finite point
        g.gx0 = 0.0;
        g.gy0 = 0.0;
        g.S = 1.0;
        g.invS = 1.0;
        g.nTx = 1;
        g.nTy = 1;
        return g;
    }
    const double W = xmx - xmn, H = ymx - ymn;
    double S;
    if (W > 0 && H > 0)
        S = std::sqrt(W * H * (double)ppt / (double)M);
    else if (W > 0 || H > 0)
        S = std::max(W, H) * (double)ppt / (double)M;
    else
        S = 1.0;
    if (!(S > 0) || !std::isfinite(S)) S = 1.0;
    // cap the tile count (int32 keys, offsets memory): at most max(4M, 2^20) tiles, 2^28 total
    const double cap = std::min(268435456.0, std::max(4.0 * (double)M, 1048576.0));
    for (int it = 0; it < 64; ++it) {
        const double nx = std::floor(W / S) + 1.0, ny = std::floor(H / S) + 1.0;
        if (nx * ny <= cap && nx < 1e8 && ny < 1e8) break;
        S *= 1.5;
    }
    {   // still too many tiles (e.g. a bbox of 1e300 m): at most 1024 x 1024
        const double nx = std::floor(W / S) + 1.0, ny = std::floor(H / S) + 1.0;
        if (!(nx * ny <= cap) || !(nx < 1e8) || !(ny < 1e8)) S = std::max(W, H) / 1000.0;
        if (!(S > 0) || !std::isfinite(S)) S = kDblMax;
    }
    g.gx0 = xmn;
    g.gy0 = ymn;
    g.S = S;
    g.invS = 1.0 / S;
    g.nTx = (int)std::min(std::floor(W * g.invS) + 1.0, 1e8);
    g.nTy = (int)std::min(std::floor(H * g.invS) + 1.0, 1e8);
    if (g.nTx < 1) g.nTx = 1;
    if (g.nTy < 1) g.nTy = 1;
    return g;
}

// Build the tile-sorted copy (xys, ws, perm, off) from ctx->x/y/w (list order), on `s`.
static void build_index(mac_ctx* ctx, hipStream_t s)
{
    const int64_t M = ctx->M;
    // bbox, and whether every entry weighs the same (bit for bit)
    const int nb = (int)std::min<int64_t>(std::max<int64_t>(grid1d(M, kBlock), 1), 1024);
    ctx->bbox.reserve(sizeof(double4) * nb + sizeof(int) * nb);
    int* d_wmix = (int*)(ctx->bbox.as<double4>() + nb);
    hipLaunchKernelGGL(bbox_kernel, dim3(nb), dim3(kBlock), 0, s, ctx->x.as<double>(),
                       ctx->y.as<double>(), ctx->w.as<double>(), M, ctx->bbox.as<double4>(), d_wmix);
    HCK(hipGetLastError());
    std::vector<double4> hb(nb);
    std::vector<int> hw(nb);
    double w0 = 0.0;
    HCK(hipMemcpyAsync(hb.data(), ctx->bbox.p, sizeof(double4) * nb, hipMemcpyDeviceToHost, s));
    HCK(hipMemcpyAsync(hw.data(), d_wmix, sizeof(int) * nb, hipMemcpyDeviceToHost, s));
    if (M > 0) HCK(hipMemcpyAsync(&w0, ctx->w.p, sizeof(double), hipMemcpyDeviceToHost, s));
    HCK(hipStreamSynchronize(s));
    ctx->w_uniform = M > 0;
    for (int v : hw) ctx->w_uniform = ctx->w_uniform && v == 0;
    ctx->w0 = w0;
    double xmn = INFINITY, xmx = -INFINITY, ymn = INFINITY, ymx = -INFINITY;
    for (auto& b : hb) {
        xmn = std::min(xmn, b.x);
        xmx = std::max(xmx, b.y);
        ymn = std::min(ymn, b.z);
        ymx = std::max(ymx, b.w);
    }
    ctx->grid = choose_grid(xmn, xmx, ymn, ymx, M, ctx->tile_ppt);
    ctx->nTiles = (int64_t)ctx->grid.nTx * ctx->grid.nTy;

    ctx->xys.reserve(sizeof(double2) * std::max<int64_t>(M, 1));
    ctx->ws.reserve(sizeof(double) * std::max<int64_t>(M, 1));
    ctx->perm.reserve(sizeof(uint32_t) * std::max<int64_t>(M, 1));
    ctx->off.reserve(sizeof(int32_t) * (ctx->nTiles + 1));
    if (M > 0) {
        ctx->keys_in.reserve(sizeof(uint32_t) * M);
        ctx->keys_out.reserve(sizeof(uint32_t) * M);
        ctx->idx_in.reserve(sizeof(uint32_t) * M);
        hipLaunchKernelGGL(tile_key_kernel, dim3(grid1d(M, 256)), dim3(256), 0, s,
                           ctx->x.as<double>(), ctx->y.as<double>(), M, ctx->grid,
                           ctx->keys_in.as<uint32_t>(), ctx->idx_in.as<uint32_t>());
        HCK(hipGetLastError());
        int end_bit = 1;
        while (end_bit < 32 && ((uint64_t)1 << end_bit) < (uint64_t)ctx->nTiles) ++end_bit;
        size_t tb = 0;
        HCK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, ctx->keys_in.as<uint32_t>(),
                                               ctx->keys_out.as<uint32_t>(),
                                               ctx->idx_in.as<uint32_t>(), ctx->perm.as<uint32_t>(),
                                               (int)M, 0, end_bit, s));
        ctx->tmp.reserve(tb);
        HCK(hipcub::DeviceRadixSort::SortPairs(ctx->tmp.p, tb, ctx->keys_in.as<uint32_t>(),
                                               ctx->keys_out.as<uint32_t>(),
                                               ctx->idx_in.as<uint32_t>(), ctx->perm.as<uint32_t>(),
                                               (int)M, 0, end_bit, s));
        hipLaunchKernelGGL(gather_sorted_kernel, dim3(grid1d(M, 256)), dim3(256), 0, s,
                           ctx->x.as<double>(), ctx->y.as<double>(), ctx->w.as<double>(),
                           ctx->perm.as<uint32_t>(), M, ctx->xys.as<double2>(), ctx->ws.as<double>());
        HCK(hipGetLastError());
    }
    hipLaunchKernelGGL(tile_offsets_kernel, dim3(grid1d(ctx->nTiles + 1, 256)), dim3(256), 0, s,
                       ctx->keys_out.as<uint32_t>(), M, ctx->nTiles, ctx->off.as<int32_t>());
    HCK(hipGetLastError());
    HCK(hipStreamSynchronize(s));
    ctx->has_points = true;
}

static int32_t check_M(int64_t M)
{
    if (M < 0) return fail(MAC_E_INVAL, "M < 0");
    if (M >= ((int64_t)1 << 31) - 1) return fail(MAC_E_INVAL, "M must be < 2^31-1");
    return MAC_OK;
}

// ------------------------------------------------------------------ evaluation core

static bool use_tiled(mac_ctx* ctx, int N, const double* h_cands, int64_t three_n)
{
    if (N <= 0 || ctx->algo == MAC_ALGO_SCAN) return false;
    if (ctx->algo == MAC_ALGO_POLL) return true;        // no N limit: fixed LDS footprint
    if (N > kTiledMaxN) return true;                     // the poll walk, whatever K (enqueue_eval)
    if (ctx->algo == MAC_ALGO_TILED) return true;
    if (!h_cands) return true;
    // AUTO with host candidates: compare the tiled walk's point visits for candidate 0 with
    // the scan's M (both per disk); prefer the scan when disks span most of the list.
    const Grid& g = ctx->grid;
    double visits = 0.0;
    for (int i = 0; i < N; ++i) {
        int x0, x1, y0, y1;
        const double r = h_cands[2 * N + i];
        if (!tile_span(h_cands[i], r, g.gx0, g.invS, g.nTx, x0, x1)) continue;
        if (!tile_span(h_cands[N + i], r, g.gy0, g.invS, g.nTy, y0, y1)) continue;
        visits += (double)(x1 - x0 + 1) * (double)(y1 - y0 + 1);
    }
    visits *= (double)ctx->M / (double)std::max<int64_t>(ctx->nTiles, 1);
    (void)three_n;
    return visits < 0.5 * (double)ctx->M * (double)N;
}

// The poll walk's chain (prep keys and records, disk index, walk choice, poll kernel) runs for this
// evaluation: the tiled family, candidates and entries present, and the poll walk allowed.
static bool poll_walk_possible(const mac_ctx* ctx, int N, int K, bool tiled)
{
    return tiled && N > 0 && ctx->M > 0 &&
           (ctx->algo == MAC_ALGO_POLL || N > kTiledMaxN ||
            ((ctx->algo == MAC_ALGO_AUTO || ctx->algo == MAC_ALGO_TILED) && K >= kPollMinK));
}

// Enqueue the prep launch + index + walks + finalize (+ argmin) on stream s. All pointers device.
// area_out/obj_out may be null; best may be null.
// d_dlimT: cons3 thresholds per UAV (host calls), else d_dlim_raw: the raw d_lim, thresholded
// where it is read (device calls).
static thread_local std::chrono::steady_clock::time_point t_poll_entry;   // (MAXCOVER_HOST_STATS)

static void enqueue_eval(mac_ctx* ctx, Lane* L, hipStream_t s, const CandSrc& src, int N,
                         int K, bool tiled, const double* d_rmax, double penalty,
                         const double* d_prev, const double* d_dlimT, const double* d_dlim_raw,
                         double tan_half_fov, double* d_area, double* d_obj, double* d_best,
                         int64_t idx_base, uint64_t* d_mirror = nullptr, uint64_t mirror_seq = 0,
                         const FinBest* fb_mads = nullptr, unsigned long long* d_feas = nullptr)
{
    const int64_t M = ctx->M;
    int n_poll = N, n_other = 1;
    const int* d_mode = nullptr;
    // Profiling: the measured walk launches stamp their own workgroups' start / end times
    // (k_common.h), so measuring adds no packet, event or dependency to the stream.
    int64_t ts_a = -1, ts_na = 0, ts_b = -1, ts_nb = 0, ts_c = -1, ts_nc = 0, ts_f = -1, ts_nf = 0;
    int64_t ts_i = -1, ts_ni = 0, ts_s = -1, ts_ns = 0, ts_g = -1, ts_ng = 0;   // index, set-up, bits
    int64_t ts_w = -1, ts_nw = 0;                                               // the fused kernel
    auto take_ts = [&](int64_t nwg, int64_t& base, int64_t& n) -> uint64_t* {
        if (!ctx->profile) return nullptr;
        std::lock_guard<std::mutex> lk(ctx->mu);
        if (ctx->stamp_used + nwg > ctx->stamp_cap) return nullptr;   // full: not recorded
        base = ctx->stamp_used;
        n = nwg;
        ctx->stamp_used += nwg;
        return ctx->stamps.as<uint64_t>() + 2 * base;
    };
    // the objective's penalty and cons3 (the prep launch: one sequential chain per candidate)
    const PenArgs pa{d_rmax, d_prev, d_dlimT, d_dlim_raw, tan_half_fov};
    double* d_vp = nullptr;            // per-candidate penalty (or +inf: cons3)
    const double* d_spart = nullptr;   // poll walk: shared-entry rows
    const int* d_umap = nullptr;       // poll walk: candidate -> distinct-disk position
    const int* d_ncount = nullptr;
    int counts = 0;                    // poll walk with equal weights: integer count rows
    int bits_on = 0;                   // the shared-entry pass's launch hint (walk set-up)
    if (d_obj) {
        L->vp.reserve(sizeof(double) * (size_t)std::max(K, 1));
        d_vp = L->vp.as<double>();
    }
    const bool big = N > kTiledMaxN;
    // the poll chain's walk: forced by the algorithm option (or N past the per-candidate walk's
    // LDS limit), else 0 = the device's choice (k_poll_shared.h walk_choice)
    const int walk_forced = (ctx->algo == MAC_ALGO_POLL || big) ? kModePoll
                          : ctx->algo == MAC_ALGO_TILED ? kModeTiled : 0;
    const bool poll_possible = poll_walk_possible(ctx, N, K, tiled);
    // candidates per index thread: 3 (K <= 3073), 6 (K <= 6145); larger: identity map
    const int iper = K <= kIndexMaxK + 1 ? kIdxPer : K <= kIndexMaxKWide + 1 ? kIdxPerWide : 0;
    const bool want_keys = poll_possible && iper;   // the index hashes the prep's fp32 keys
    auto prof_end = [&]() {
        if (!ctx->profile || (ts_a < 0 && ts_b < 0)) return;
        std::lock_guard<std::mutex> lk(ctx->mu);
        mac_ctx::Prof p{ts_a, ts_na, ts_b, ts_nb, (int64_t)K, d_mode,
                        ts_w >= 0 ? MAC_ALGO_POLL : tiled ? MAC_ALGO_TILED : MAC_ALGO_SCAN, ts_c, ts_nc,
                        ts_f, ts_nf};
        if (ts_c >= 0) {   // a poll chain: every launch's stamps by role (mac_profile_kernels)
            const int64_t r[MAC_PROF_ROLES][2] = {{ts_c, ts_nc}, {ts_i, ts_ni}, {ts_s, ts_ns},
                                                  {ts_w >= 0 ? -1 : ts_a, ts_w >= 0 ? 0 : ts_na},
                                                  {ts_b, ts_nb}, {ts_g, ts_ng},
                                                  {ts_w >= 0 ? -1 : ts_f, ts_w >= 0 ? 0 : ts_nf},
                                                  {ts_w, ts_nw},
                                                  {ts_w >= 0 ? ts_f : -1, ts_w >= 0 ? ts_nf : 0}};
            for (int q = 0; q < MAC_PROF_ROLES; ++q) {
                p.role[q][0] = r[q][0];
                p.role[q][1] = r[q][1];
            }
        }
        ctx->prof.push_back(p);
    };

    CandSrc isrc = src;
    const int target = 8 * ctx->cus;
    const int G = (int)std::max<int64_t>(
        1, std::min<int64_t>((target + K - 1) / K, std::max(1, N / kWavesPerBlock)));
    const int64_t units = (int64_t)K * G;
    // generated complete polls (the native MADS loop: K = 2n): the prep draws each B entry once
    // for its plus and minus candidates (k_prep.h PrepArgs.pair)
    const bool pair = !src.cands && src.k0 == 0 && K == 6 * N && (3 * N) % 4 == 0 && kPrepC == 8;
    // ... or, with one block of UAVs, prep_x_kernel's layout (k_prep.h prep_block_x<true>): a column
    // triple of B per workgroup (its plus and minus candidates: 6), N workgroups, a ninth wave
    // folding the penalty chains beside the keys and the records
    const bool gen_x = !src.cands && src.k0 == 0 && K == 6 * N && N >= 1 && N <= kPrepU;
    const int nchain = pair ? (3 * N) / 4 : (K + kPrepC - 1) / kPrepC;

    // The fused chain (k_fiw.h: prep -> fiw -> fin2) whenever the poll walk runs on packed keys of at
    // most kFwMaxK + 1 candidates, unless one of the context's last 64 polls did not suit it: a crowded
    // poll (many shared entries: the five-launch chain's union pass), a scattered batch (the
    // per-candidate walk) or escaped keys (fp32 keys). Either chain gives the same results. The
    // history is long because a wrong choice costs asymmetrically: a crowded poll in the fused
    // chain decides its shared entries per candidate in place (0.4-2 ms at configs 5 and 4
    // clustered), an uncrowded one in the five-launch chain costs ~20 us more.
    // A generated poll whose step the host knows (a stepper's, not the pipelined loop's) at
    // 2^ell > 8 goes to the five-launch chain under AUTO: its disks spread over more than the
    // index's direct-mapped box (ell <= 3) and its superset boxes overlap widely (config 5's first
    // poll of an MPC step: 0.5 ms fused against ~0.11 ms).
    const bool wide_gen = !src.cands && !src.mst &&
                          (src.ltri ? (double)src.b * __builtin_fabs(src.delta) > 8.0 : src.b > 8);
    if (poll_possible && want_keys && N > 0 && M > 0 && K > 0 && K <= kFwMaxK + 1 &&
        ctx->chain != MAC_CHAIN_FIVE && walk_forced != kModeTiled &&
        (ctx->chain == MAC_CHAIN_FUSED || (!wide_gen && !src.route_five))) {
        ensure_hints(L);
        volatile int* hw = (volatile int*)L->h_dc.p;
        int bad_now = -1;   // the lane's last poll's report (a hint: it may be an older poll's)
        if (L->last_chain == 2 && hw[8] >= 0)
            bad_now = hw[8] > kFwCrowdWork || hw[9] > 0 || hw[11] > 0 ? 1 : 0;   // (k_fiw.h kFwHints)
        else if (L->last_chain == 1 && hw[0] < (1 << 30))
            bad_now = hw[0] > kBitsMinDisks || hw[4] == kModeTiled ? 1 : 0;
        if (bad_now >= 0) {
            uint64_t o = ctx->fused_bad.load(std::memory_order_relaxed);
            while (!ctx->fused_bad.compare_exchange_weak(o, (o << 1) | (uint64_t)bad_now,
                                                         std::memory_order_relaxed)) {
            }
        }
        const bool fused = ctx->fused_bad.load(std::memory_order_relaxed) == 0;
        if (fused || ctx->chain == MAC_CHAIN_FUSED) {
            const int ldk = keys_ld(K);
            counts = ctx->w_uniform ? 1 : 0;
            L->keysT.reserve(sizeof(float) * (size_t)4 * N * ldk);
            // a matrix source: kPrepCX (+1) candidates per workgroup (k_prep.h prep_x_kernel)
            const int gx = K / kPrepCX;
            const bool xk = (src.cands && !pair && N <= kPrepU && gx >= 1 && K - gx * kPrepCX <= gx) || gen_x;
            const int nprep = gen_x ? N : xk ? gx : nchain;
            L->pd.reserve(sizeof(double4) * (size_t)nprep);
            L->frows.reserve((counts ? sizeof(unsigned) : sizeof(double)) * (size_t)N * ldk);
            if (L->fwhint.grow(sizeof(int) * kFwHints)) HCK(hipMemsetAsync(L->fwhint.p, 0, L->fwhint.cap, s));
            // cons3 failures are left out of the walk when only objectives are asked for
            const bool excl = d_obj && d_prev && !d_area && N <= kPrepU;
            if (excl) L->dead8.reserve((size_t)ldk + 16);   // (the fused kernel reads 4-B words)
            L->fwlist.reserve(sizeof(int4) * (size_t)std::max(N, kF2Pre));
            if (L->fwcount.grow(sizeof(int))) HCK(hipMemsetAsync(L->fwcount.p, 0, L->fwcount.cap, s));
            L->fwsxy.reserve(sizeof(double2) * (size_t)N * kFwShCap);
            L->fwsw.reserve(sizeof(double) * (size_t)N * kFwShCap);
            PrepArgs pr{};
            pr.src = src;
            pr.N = N;
            pr.K = K;
            pr.pa = pa;
            pr.penalty = penalty;
            pr.vp = d_vp;
            pr.nchain = nprep;
            pr.xbase = gx * kPrepCX;
            pr.skip_failed = d_area ? 0 : 1;
            pr.pair = pair ? 1 : 0;
            pr.g = ctx->grid;
            pr.keysP = L->keysT.as<uint32_t>();
            pr.keysT = L->keysT.as<float>() + (size_t)N * ldk;
            pr.ldk = ldk;
            pr.pd = L->pd.as<double4>();
            pr.dead8 = excl ? L->dead8.as<uint8_t>() : nullptr;
            pr.mst_w = excl && fb_mads ? fb_mads->st : nullptr;
            pr.feas = d_feas;
            pr.lreset = L->fwcount.as<int>();
            uint64_t* tsk = take_ts(nprep, ts_c, ts_nc);
            using hclk = std::chrono::steady_clock;
            hclk::time_point h1, h2, h3;
            if (ctx->host_stats) h1 = hclk::now();
            if (xk && gen_x)
                hipLaunchKernelGGL(prep_x_kernel<true>, dim3((unsigned)nprep), dim3(kPrepU + kWave), 0, s, tsk, pr);
            else if (xk)
                hipLaunchKernelGGL(prep_x_kernel<false>, dim3((unsigned)nprep), dim3(kPrepU + kWave), 0, s, tsk, pr);
            else hipLaunchKernelGGL(prep_kernel, dim3((unsigned)nprep), dim3(kPrepU), 0, s, tsk, pr);
            HCK(hipGetLastError());
            if (ctx->host_stats) h2 = hclk::now();
            FwArgs fa{};
            fa.src = src;
            fa.src.keysP = pr.keysP;
            fa.src.keysT = pr.keysT;
            fa.src.ldk = ldk;
            fa.N = N;
            fa.K = K;
            fa.g = ctx->grid;
            fa.dead = pr.dead8;
            fa.pd = pr.pd;
            fa.npd = nprep;
            fa.xy = ctx->xys.as<double2>();
            fa.w = ctx->ws.as<double>();
            fa.off = ctx->off.as<int32_t>();
            fa.counts = counts;
            fa.crow = L->frows.as<unsigned>();
            fa.frow = L->frows.as<double>();
            fa.ldk = ldk;
            fa.hint = L->fwhint.as<int>();
            fa.sh = FwShared{L->fwcount.as<int>(), L->fwlist.as<int4>(), L->fwsxy.as<double2>(),
                             L->fwsw.as<double>()};
            const F2Shared f2s{fa.src, L->fwcount.as<int>(), L->fwlist.as<int4>(), L->fwsxy.as<double2>(),
                               L->fwsw.as<double>(), fa.dead};
            const unsigned nfw = 8 * (unsigned)((N + 7) / 8);
            uint64_t* tsw = take_ts(nfw, ts_w, ts_nw);
            ts_a = ts_w;   // (mac_profile_read: the walk launch)
            ts_na = ts_nw;
            if (counts) hipLaunchKernelGGL(fiw_kernel<true>, dim3(nfw), dim3(kFwThreads), 0, s, tsw, fa);
            else hipLaunchKernelGGL(fiw_kernel<false>, dim3(nfw), dim3(kFwThreads), 0, s, tsw, fa);
            HCK(hipGetLastError());
            if (ctx->host_stats) h3 = hclk::now();
            const unsigned nfin = 8 * (unsigned)((K + 8 * kF2C - 1) / (8 * kF2C));
            FinBest fb{};
            if (d_best) {
                L->finblk.reserve(2 * sizeof(unsigned long long) * nfin);
                if (L->finarrive.grow(sizeof(unsigned)))
                    HCK(hipMemsetAsync(L->finarrive.p, 0, L->finarrive.cap, s));
                if (fb_mads) fb = *fb_mads;
                fb.best = d_best;
                fb.mirror = d_mirror;
                fb.seq = mirror_seq;
                fb.idx_base = idx_base;
                fb.blk = L->finblk.as<unsigned long long>();
                fb.arrive = L->finarrive.as<unsigned>();
                fb.hint = L->fwhint.as<int>();   // (read and cleared by the argmin's last block)
                fb.hint_host = L->d_dc + 8;
                fb.nhint = kFwHints;
                fb.feas = d_mirror ? d_feas : nullptr;
            }
            uint64_t* tsf = take_ts(nfin, ts_f, ts_nf);
            if (counts)
                hipLaunchKernelGGL(fin2_kernel<true>, dim3(nfin), dim3(kF2Threads), 0, s, L->frows.as<unsigned>(),
                                   nullptr, ldk, N, K, ctx->w0, d_vp, d_area, d_obj, fb, f2s, tsf);
            else
                hipLaunchKernelGGL(fin2_kernel<false>, dim3(nfin), dim3(kF2Threads), 0, s, nullptr,
                                   L->frows.as<double>(), ldk, N, K, ctx->w0, d_vp, d_area, d_obj, fb, f2s, tsf);
            HCK(hipGetLastError());
            if (ctx->host_stats) {
                const auto h4 = hclk::now();
                std::lock_guard<std::mutex> lk(ctx->mu);
                ctx->hs_t[0] += std::chrono::duration<double>(h1 - t_poll_entry).count();
                ctx->hs_t[1] += std::chrono::duration<double>(h2 - h1).count();
                ctx->hs_t[2] += std::chrono::duration<double>(h3 - h2).count();
                ctx->hs_t[3] += std::chrono::duration<double>(h4 - h3).count();
                ++ctx->hs_n;
            }
            L->last_chain = 2;
            prof_end();
            return;
        }
    }
    if (poll_possible) L->last_chain = 1;
    int nrec = nchain;   // the prep's records per disk (workgroups of the prep launch)

    if ((d_obj || poll_possible) && K > 0) {
        // the prep launch (k_prep.h): penalty chains + cons3 into vp, the poll walk's partial
        // regions, and the index's fp32 keys
        // a generated complete poll with the index's keys: prep_x_kernel's column-triple layout
        const bool gx5 = gen_x && poll_possible && want_keys;
        nrec = gx5 ? N : nchain;
        PrepArgs pr{};
        pr.src = src;
        pr.N = N;
        pr.K = K;
        pr.pa = pa;
        pr.penalty = penalty;
        pr.vp = d_vp;
        pr.nchain = nrec;
        pr.skip_failed = d_area ? 0 : 1;   // (the index maps them to an inert position likewise)
        pr.pair = pair ? 1 : 0;
        pr.g = ctx->grid;
        pr.feas = d_feas;
        // the pipelined MADS loop: a poll cons3 rejects whole is decided by the prep (k_prep.h
        // MadsState.skip) when its failures are left out of the walk (the prep's excl)
        pr.mst_w = fb_mads && poll_possible && d_obj && d_prev && !d_area && N <= kPrepU ? fb_mads->st
                                                                                           : nullptr;
        if (poll_possible) {
            L->prec.reserve(sizeof(int4) * (size_t)nrec * N);
            pr.prec = L->prec.as<int4>();
        }
        if (want_keys) {
            const int ldk = keys_ld(K);
            // packed keys (one row per disk), then the fp32 rows of escaped values (k_prep.h)
            L->keysT.reserve(sizeof(float) * (size_t)4 * N * ldk);
            pr.keysP = L->keysT.as<uint32_t>();
            pr.keysT = L->keysT.as<float>() + (size_t)N * ldk;
            pr.ldk = ldk;
            isrc.keysP = pr.keysP;
            isrc.keysT = pr.keysT;
            isrc.ldk = ldk;
        }
        uint64_t* tsk = poll_possible ? take_ts(nrec, ts_c, ts_nc) : nullptr;
        if (gx5) hipLaunchKernelGGL(prep_x_kernel<true>, dim3((unsigned)nrec), dim3(kPrepU + kWave), 0, s, tsk, pr);
        else hipLaunchKernelGGL(prep_kernel, dim3((unsigned)nchain), dim3(kPrepU), 0, s, tsk, pr);
        HCK(hipGetLastError());
    }

    if (N == 0 || M == 0) {  // no UAV or no entry: every area is 0 (the loops never run)
        L->partial.reserve(sizeof(double) * (size_t)K);
        HCK(hipMemsetAsync(L->partial.p, 0, sizeof(double) * (size_t)K, s));
    } else if (!tiled) {
        L->disks.reserve(sizeof(DiskRec) * (size_t)N * K);
        hipLaunchKernelGGL(disk_prep_kernel, dim3(grid1d((int64_t)N * K, 256)), dim3(256), 0, s,
                           src, N, K, L->disks.as<DiskRec>());
        HCK(hipGetLastError());
        constexpr int KB = 4, PPT = 4;
        const int64_t per_pass = (int64_t)kBlock * PPT;
        int64_t nblk = std::max<int64_t>(1, (M + per_pass - 1) / per_pass);
        const int kgroups = (K + KB - 1) / KB;
        const int64_t want = std::max<int64_t>(1, (int64_t)(8 * ctx->cus) / kgroups);
        nblk = std::min(nblk, want);
        int64_t chunk = (M + nblk - 1) / nblk;
        chunk = ((chunk + per_pass - 1) / per_pass) * per_pass;
        nblk = std::max<int64_t>(1, (M + chunk - 1) / chunk);
        n_other = (int)nblk;
        L->partial.reserve(sizeof(double) * (size_t)K * nblk);
        uint64_t* ts = take_ts(nblk * kgroups, ts_a, ts_na);
        hipLaunchKernelGGL((coverage_scan_kernel<KB, PPT>), dim3((unsigned)nblk, (unsigned)kgroups),
                           dim3(kBlock), 0, s, ts, ctx->xys.as<double2>(), ctx->ws.as<double>(), M,
                           L->disks.as<DiskRec>(), N, K, chunk, L->partial.as<double>());
        HCK(hipGetLastError());
    } else {
        // the disk index: distinct disks per UAV, their records, the map and the poll walk's lane
        // constants (k_index.h)
        L->disks.reserve(sizeof(DiskRec) * (size_t)N * K);
        L->umap.reserve(sizeof(int) * (size_t)N * K);
        L->ucount.reserve(sizeof(int) * (size_t)N);
        if (poll_possible) {  // the poll walk's lane constants and row descriptors
            L->lane4.reserve(sizeof(float4) * (size_t)N * K);
            L->lanexp.reserve(sizeof(float) * (size_t)N * K);
            L->rows.reserve(sizeof(int2) * (size_t)N * (kRowInfo + 1));
        }
        counts = poll_possible && ctx->w_uniform ? 1 : 0;   // equal weights: the walks count
        n_other = G;
        const DiskRec* d_urec = L->disks.as<DiskRec>();
        const int* d_map = L->umap.as<int>();
        if (!poll_possible) {
            // the per-candidate walk alone (small batches, the single-candidate closure): the
            // identity map, one thread per (disk, candidate), no key pass
            const int64_t nk = (int64_t)N * K;
            hipLaunchKernelGGL(disk_index_identity_kernel, dim3(grid1d(nk, 256)), dim3(256), 0, s,
                               src, N, K, L->disks.as<DiskRec>(), L->umap.as<int>());
            HCK(hipGetLastError());
            L->partial.reserve(sizeof(double) * (size_t)K * G);
            uint64_t* ts = take_ts(units, ts_a, ts_na);
            hipLaunchKernelGGL(coverage_tiled_kernel, dim3((unsigned)units), dim3(kBlock),
                               (uint32_t)tiled_lds_bytes(N), s, ts, ctx->xys.as<double2>(),
                               ctx->ws.as<double>(), ctx->off.as<int32_t>(), ctx->grid, d_urec, d_map,
                               N, K, G, nullptr, L->partial.as<double>());
            HCK(hipGetLastError());
        } else {
            L->region.reserve(sizeof(int4) * N);
            L->cost.reserve(sizeof(double2) * N);
            L->mode.reserve((1 + kDcCount) * sizeof(int));  // [0] walk, [1..kDcCount] the poll walk's counters (k_common.h)
            const IndexOut io{L->disks.as<DiskRec>(), L->umap.as<int>(), L->ucount.as<int>(),
                              L->region.as<int4>(), L->cost.as<double2>(), L->mode.as<int>() + 1,
                              L->prec.as<int4>(), nrec,
                              L->lane4.as<float4>(), L->lanexp.as<float>(), L->rows.as<int2>(),
                              ctx->off.as<int32_t>(),
                              // cons3 failures are not evaluated (objective +inf) unless the caller
                              // also wants every candidate's area
                              d_area ? nullptr : d_vp};
            const unsigned nidx = 8 * ((N + 7) / 8);
            const int dedup = iper ? 1 : 0;
            uint64_t* tsi = ts_c >= 0 ? take_ts(nidx, ts_i, ts_ni) : nullptr;
            if (isrc.keysT && iper == kIdxPerWide)
                hipLaunchKernelGGL((disk_index_kernel<true, kIdxPerWide>), dim3(nidx), dim3(kIdxThreads),
                                   0, s, tsi, isrc, N, K, ctx->grid, dedup, io);
            else if (isrc.keysT)
                hipLaunchKernelGGL((disk_index_kernel<true, kIdxPer>), dim3(nidx), dim3(kIdxThreads), 0, s,
                                   tsi, isrc, N, K, ctx->grid, dedup, io);
            else if (iper == kIdxPerWide)
                hipLaunchKernelGGL((disk_index_kernel<false, kIdxPerWide>), dim3(nidx), dim3(kIdxThreads),
                                   0, s, tsi, isrc, N, K, ctx->grid, dedup, io);
            else
                hipLaunchKernelGGL((disk_index_kernel<false, kIdxPer>), dim3(nidx), dim3(kIdxThreads), 0,
                                   s, tsi, isrc, N, K, ctx->grid, dedup, io);
            HCK(hipGetLastError());
            // launch hints from the lane's previous polls (mapped host memory the poll kernel
            // writes): disks with neighbours, most positions of a disk, the walk AUTO would choose
            ensure_hints(L);
            // neighbour lists (k_walk.h walk_setup_kernel), then — when the per-candidate walk is
            // forced, or AUTO chose it on one of the lane's last 8 polls — the walk choice and that
            // walk (coverage_tiled_poll_kernel). Otherwise the poll walk runs; its kernel records
            // the choice AUTO would have made, so a batch that favours the per-candidate walk gets
            // it from the lane's next poll on (the choice only changes speed, never results).
            // (a lane's first poll has no report yet: it launches the kernel once, and the
            // sentinel stays out of the history)
            const int walk_now = ((volatile int*)L->h_dc.p)[4];
            bool hinted = walk_now == 0;
            if (!hinted) {
                for (int q = 7; q > 0; --q) L->walk_hist[q] = L->walk_hist[q - 1];
                L->walk_hist[0] = walk_now;
            }
            for (int q = 0; q < 8; ++q) hinted |= L->walk_hist[q] == kModeTiled;
            const bool run_tiled = walk_forced == kModeTiled || (walk_forced == 0 && hinted);
            L->nbr.reserve(sizeof(uint16_t) * (size_t)N * kPollNbr);
            L->ncount.reserve(sizeof(int) * (size_t)N);
            L->dlist.reserve(sizeof(int) * (size_t)N);
            L->qual.reserve(sizeof(int) * (size_t)N);
            L->nboxT.reserve(sizeof(int4) * (size_t)N * kPollNbr);
            L->partial.reserve(sizeof(double) * (size_t)K * std::max(G, N));
            // the shared-entry pass of crowded polls, launched when one of the lane's last 8 polls
            // had more than kBitsMinDisks disks with neighbours (the poll kernel writes the count to
            // mapped host memory): a hint only, the poll kernel takes every disk when it is not
            // launched (MADS alternates crowded and quiet polls, and a crowded poll without the
            // pass costs several times its launch)
            const int dc_now = *(volatile int*)L->h_dc.p;   // 1 << 30 until a poll wrote it
            int dc_max = dc_now;
            if (dc_now < (1 << 30)) {
                for (int q = 7; q > 0; --q) L->dc_hist[q] = L->dc_hist[q - 1];
                L->dc_hist[0] = dc_now;
                for (int q = 0; q < 8; ++q) dc_max = std::max(dc_max, L->dc_hist[q]);
            }
            // 0: fp64 jobs; 1: above kBitsMinDisks disks with neighbours; 2: always
            bits_on = ctx->shared_mode == MAC_SHARED_BITS ? 2
                    : ctx->shared_mode == MAC_SHARED_FP64 ? 0
                    : dc_max > kBitsMinDisks ? 1 : 0;
            // equal weights: the union pass (k_or.h), whose jobs walk_setup lists with the upper
            // neighbour boxes; weighted lists: the bit-word kernel (k_bits.h)
            OrSetup orj{};
            if (bits_on && counts) {
                L->nboxU.reserve(sizeof(int4) * (size_t)N * kPollNbr);
                L->ncountU.reserve(sizeof(int) * (size_t)N);
                const int64_t cap = M / kOrE + N + 64;   // the owned sets are disjoint
                L->orjobs.reserve(sizeof(int2) * (size_t)cap * kOrBuckets);   // a list per bucket
                orj = OrSetup{L->nboxU.as<int4>(), L->ncountU.as<int>(), L->orjobs.as<int2>(), (int)cap,
                              ctx->off.as<int32_t>(), ctx->grid, L->ucount.as<int>()};
            }
            uint64_t* tss = ts_c >= 0 ? take_ts(N, ts_s, ts_ns) : nullptr;
            hipLaunchKernelGGL(walk_setup_kernel, dim3((unsigned)N), dim3(kBlock), 0, s, tss, N,
                               L->region.as<int4>(), L->nbr.as<uint16_t>(), L->nboxT.as<int4>(),
                               L->ncount.as<int>(), L->dlist.as<int>(), L->mode.as<int>() + 1,
                               L->mode.as<int>(), L->qual.as<int>(), src.mst, orj);
            HCK(hipGetLastError());
            if (run_tiled) {
                // one workgroup per CU at most, grid-striding over the (candidate, slice) units
                const unsigned nwg = (unsigned)std::max<int64_t>(1, std::min<int64_t>(units, ctx->cus));
                uint64_t* ts = take_ts(nwg, ts_a, ts_na);
                hipLaunchKernelGGL(coverage_tiled_poll_kernel, dim3(nwg), dim3(kBlock),
                                   (uint32_t)tiled_lds_bytes(N), s, ts, ctx->xys.as<double2>(),
                                   ctx->ws.as<double>(), ctx->off.as<int32_t>(), ctx->grid, d_urec, d_map,
                                   N, K, G, L->mode.as<int>(), L->partial.as<double>(),
                                   L->nbr.as<uint16_t>(), L->ncount.as<int>(), L->cost.as<double2>(),
                                   kPollCostRatio, walk_forced, L->d_dc + 4);
                HCK(hipGetLastError());
            }
            d_mode = L->mode.as<int>();
            d_umap = d_map;
        }
        if (poll_possible) {
            // walk rows: the lane's last 8 polls' most distinct positions of a disk (poll kernel
            // hint), one row per kPollKPB-position slice up to 4 (further slices loop)
            const int um_now = ((volatile int*)L->h_dc.p)[2];
            for (int q = 7; q > 0; --q) L->um_hist[q] = L->um_hist[q - 1];
            L->um_hist[0] = um_now;
            int um_max = 0;
            for (int q = 0; q < 8; ++q) um_max = std::max(um_max, L->um_hist[q]);
            const int gy = std::max(1, std::min(4, (um_max + kPollKPB - 1) / kPollKPB));
            L->spart.reserve(sizeof(double) * (size_t)N * K);
            const int n_shared = kSharedWG;
            const dim3 pgrid(8 * ((N + 7) / 8) + n_shared, gy);   // walk workgroups, then shared
            uint64_t* ts = take_ts((int64_t)pgrid.x * pgrid.y, ts_b, ts_nb);
            hipLaunchKernelGGL(coverage_poll_kernel, pgrid, dim3(kPollThreads), 0, s, ts,
                               ctx->xys.as<double2>(), ctx->ws.as<double>(),
                               ctx->off.as<int32_t>(), ctx->grid, d_urec, d_map,
                               L->ucount.as<int>(), L->region.as<int4>(), L->nbr.as<uint16_t>(),
                               L->nboxT.as<int4>(), L->lane4.as<float4>(), L->lanexp.as<float>(),
                               L->rows.as<int2>(),
                               L->ncount.as<int>(), L->dlist.as<int>(), L->mode.as<int>() + 1,
                               L->mode.as<int>() + 2, N, K,
                               d_mode, L->partial.as<double>(), L->spart.as<double>(), n_shared, counts,
                               bits_on, L->d_dc, L->qual.as<int>(),
                               walk_forced == 0 ? L->cost.as<double2>() : nullptr, kPollCostRatio);
            HCK(hipGetLastError());
            // the shared entries of crowded polls: the union pass (equal weights, k_or.h) or
            // bit-words per distinct position (k_bits.h); both return at once when few disks have
            // neighbours (the poll kernel took them)
            const unsigned nbits = (unsigned)std::max(1, std::min(N, ctx->cus));
            const unsigned nor = (unsigned)(2 * ctx->cus);   // grid-strides over the listed jobs
            uint64_t* tsg = bits_on && ts_c >= 0 ? take_ts(counts ? nor : nbits, ts_g, ts_ng) : nullptr;
            if (!bits_on)
                ;
            else if (counts) {
                OrArgs oa{};
                oa.xy = ctx->xys.as<double2>();
                oa.off = ctx->off.as<int32_t>();
                oa.g = ctx->grid;
                oa.urec = d_urec;
                oa.umap = d_map;
                oa.ucount = L->ucount.as<int>();
                oa.region = L->region.as<int4>();
                oa.nbrT = L->nbr.as<uint16_t>();
                oa.nboxT = L->nboxT.as<int4>();
                oa.ncount = L->ncount.as<int>();
                oa.nboxU = L->nboxU.as<int4>();
                oa.ncountU = L->ncountU.as<int>();
                oa.lane4 = L->lane4.as<float4>();
                oa.lanexp = L->lanexp.as<float>();
                oa.jobs = L->orjobs.as<int2>();
                oa.dcount = L->mode.as<int>() + 1;
                oa.mode = d_mode;
                oa.spart = L->spart.as<unsigned>();
                oa.N = N;
                oa.K = K;
                oa.bits_on = bits_on;
                oa.cap = (int)(M / kOrE + N + 64);
                hipLaunchKernelGGL(shared_or_kernel, dim3(nor), dim3(kOrThreads), 0, s, tsg, oa);
            } else
                hipLaunchKernelGGL(shared_bits_kernel<false>, dim3(nbits), dim3(kBitsThreads), 0, s,
                                   tsg, ctx->xys.as<double2>(), ctx->ws.as<double>(), ctx->off.as<int32_t>(),
                                   ctx->grid, d_urec, d_map, L->ucount.as<int>(), L->region.as<int4>(),
                                   L->nbr.as<uint16_t>(), L->lane4.as<float4>(), L->lanexp.as<float>(),
                                   L->ncount.as<int>(), L->qual.as<int>(), L->mode.as<int>() + 1, d_mode,
                                   N, K, L->spart.as<double>(), bits_on == 2 ? 0 : kBitsMinDisks);
            HCK(hipGetLastError());
            d_spart = L->spart.as<double>();
            d_ncount = L->ncount.as<int>();
        }
    }
    // finalize, with the poll argmin taken by its last-arriving block (k_final.h)
    const unsigned nfin = 8 * (unsigned)((K + 8 * kFinC - 1) / (8 * kFinC));   // k_final.h: XCD map
    FinBest fb{};
    if (d_best) {
        L->finblk.reserve(2 * sizeof(unsigned long long) * nfin);
        if (L->finarrive.grow(sizeof(unsigned)))   // zero once; the last block of each launch resets it
            HCK(hipMemsetAsync(L->finarrive.p, 0, L->finarrive.cap, s));
        if (fb_mads) fb = *fb_mads;   // the pipelined MADS loop's update fields
        fb.best = d_best;
        fb.mirror = d_mirror;
        fb.seq = mirror_seq;
        fb.idx_base = idx_base;
        fb.blk = L->finblk.as<unsigned long long>();
        fb.arrive = L->finarrive.as<unsigned>();
        fb.feas = d_mirror ? d_feas : nullptr;
    }
    uint64_t* tsf = ts_c >= 0 ? take_ts(nfin, ts_f, ts_nf) : nullptr;
    hipLaunchKernelGGL(finalize_kernel, dim3(nfin), dim3(kFinThreads), 0, s,
                       L->partial.as<double>(), d_mode, n_poll, n_other, K, N, d_umap, d_spart, d_ncount,
                       counts, ctx->w0, d_vp, d_area, d_obj, fb, tsf);
    HCK(hipGetLastError());
    prof_end();
}

static double dlim_threshold(double d) { return mac::dlim_threshold(d); }

static int32_t check_common(mac_ctx* ctx, int64_t three_n, int64_t K)
{
    if (!ctx) return fail(MAC_E_INVAL, "null context");
    if (three_n < 0 || K < 0) return fail(MAC_E_INVAL, "negative size");
    if (three_n % 3 != 0)
        return fail(MAC_E_SIZE, "InexactError: Int64(" + std::to_string(three_n) + "/3)");
    if (!ctx->has_points) return fail(MAC_E_NOPOINTS, "no point list set");
    if (three_n / 3 > 65535) return fail(MAC_E_INVAL, "N > 65535 UAVs");
    if (K > (int64_t)1 << 30) return fail(MAC_E_INVAL, "K too large");
    return MAC_OK;
}

// Host-pointer batch: upload, evaluate, download.
static int host_crowded_disks(const double* x, int N, double b, double S);

// A context's first matrix poll routes from the poll, before any chain has reported to the history
// above: its candidate 0 (a DirectSearch poll's incumbent) overlap-tested as host_crowded_disks
// does for generated polls, with no displacement (the matrix's spread is unknown here). A crowded
// incumbent starts the history all "unsuited" (the five-launch chain; the fused chain again after
// 64 polls that suit it), so a crowded poll does not pay the fused chain's in-place shared
// decisions on its first call (clustered config 4: 2.7 ms against 0.17). Not from an arming call
// (its stream waits on the doorbell: no synchronous copy there).
static void seed_route(mac_ctx* ctx, const double* x0, int N)
{
    if (N > 0 && host_crowded_disks(x0, N, 0.0, ctx->grid.S) > kBitsMinDisks)
        ctx->fused_bad.store(~(uint64_t)0, std::memory_order_relaxed);
}

// A large host buffer into device memory through the lane's pinned staging: host threads copy
// chunks into the staging while this thread enqueues each chunk's async copy as soon as it has
// landed (a single-threaded memcpy of config 4's 37.7-MB matrix took ~3 ms before the first byte
// moved; MAXCOVER_STAGE_THREADS sets the threads, 1 = the plain copy). Returns once every copy is
// enqueued and every host thread has finished (the staging may then be reused after the stream).
static const int kStageThreads = [] {
    const char* e = std::getenv("MAXCOVER_STAGE_THREADS");
    const int v = e ? std::atoi(e) : 8;
    return std::max(1, std::min(v, 32));
}();

static void staged_upload(const void* src, void* pinned, void* dev, size_t bytes, hipStream_t s)
{
    constexpr size_t kChunk = (size_t)4 << 20;
    const int T = (int)std::min<size_t>((size_t)kStageThreads, (bytes + kChunk - 1) / kChunk);
    if (T <= 1 || bytes < 2 * kChunk) {
        std::memcpy(pinned, src, bytes);
        HCK(hipMemcpyAsync(dev, pinned, bytes, hipMemcpyHostToDevice, s));
        return;
    }
    const size_t nc = (bytes + kChunk - 1) / kChunk;
    std::vector<std::atomic<int>> done(nc);
    for (auto& d : done) d.store(0, std::memory_order_relaxed);
    auto work = [&](int t) {   // chunks t, t + T, ...: the early chunks land first
        for (size_t c = (size_t)t; c < nc; c += (size_t)T) {
            const size_t o = c * kChunk, n = std::min(kChunk, bytes - o);
            std::memcpy((char*)pinned + o, (const char*)src + o, n);
            done[c].store(1, std::memory_order_release);
        }
    };
    std::vector<std::thread> th;
    int started = 1;   // workers 1 .. started-1 run on their own threads; the rest on this one
    try {
        th.reserve((size_t)T - 1);
        for (int t = 1; t < T; ++t, ++started) th.emplace_back(work, t);
    } catch (...) {   // (no thread to spare: this thread copies their chunks too)
    }
    for (int t = started; t < T; ++t) work(t);
    work(0);
    HipError err{hipSuccess, "", 0};
    for (size_t c = 0; c < nc; ++c) {   // (every thread is joined before an error leaves)
        while (!done[c].load(std::memory_order_acquire)) std::this_thread::yield();
        const size_t o = c * kChunk, n = std::min(kChunk, bytes - o);
        if (err.e == hipSuccess) {
            const hipError_t e = hipMemcpyAsync((char*)dev + o, (const char*)pinned + o, n, hipMemcpyHostToDevice, s);
            if (e != hipSuccess) err = HipError{e, "hipMemcpyAsync (staged_upload)", __LINE__};
        }
    }
    for (auto& t : th) t.join();
    if (err.e != hipSuccess) throw err;
}

template <class T>
static int32_t host_eval(mac_ctx* ctx, const T* cands, int64_t three_n, int64_t K,
                         const double* r_max, double penalty, const T* prev,
                         const double* d_lim, double tan_half_fov, double* area_out,
                         double* obj_out, double* best_obj, int64_t* best_idx)
{
    constexpr bool f32 = std::is_same<T, float>::value;
    int32_t rc = check_common(ctx, three_n, K);
    if (rc) return rc;
    if (K == 0) {
        if (best_idx) *best_idx = -1;
        if (best_obj) *best_obj = INFINITY;
        return MAC_OK;
    }
    if (!cands) return fail(MAC_E_INVAL, "null candidates");
    const int N = (int)(three_n / 3);
    set_device(ctx);
    LaneGuard lg(ctx);
    Lane* L = lg.lane;
    hipStream_t s = L->stream;
    L->cands.reserve(sizeof(double) * (size_t)std::max<int64_t>(three_n * K, 1));
    L->area.reserve(sizeof(double) * K);
    L->obj.reserve(sizeof(double) * K);
    L->best.reserve(16);
    // pinned staging (up to 64 MB): from pageable memory HIP would stage each copy
    // synchronously; one host memcpy into the lane's pinned buffer keeps the copies async
    const size_t in_bytes = sizeof(T) * (size_t)(three_n * K);
    const size_t out_bytes = sizeof(double) * (size_t)K * ((area_out ? 1 : 0) + (obj_out ? 1 : 0)) + 16;
    const bool staged = std::max(in_bytes, out_bytes) <= ((size_t)64 << 20);
    if (staged) L->h_io.reserve(std::max<size_t>(std::max(in_bytes, out_bytes), 64));
    const T* src_in = cands;
    if constexpr (!f32) {
        if (staged && in_bytes)
            staged_upload(cands, L->h_io.p, L->cands.p, in_bytes, s);
        else if (in_bytes)
            HCK(hipMemcpyAsync(L->cands.p, cands, in_bytes, hipMemcpyHostToDevice, s));
    } else {
        if (staged && in_bytes) {
            std::memcpy(L->h_io.p, cands, in_bytes);
            src_in = (const T*)L->h_io.p;
        }
        if (three_n * K > 0) upload_widen(src_in, three_n * K, L->c32, L->cands.as<double>(), s);
    }
    const bool want_obj = obj_out || best_obj || best_idx;
    double* d_rmax = nullptr;
    if (want_obj && r_max && N > 0) {
        L->rmax.reserve(sizeof(double) * N);
        HCK(hipMemcpyAsync(L->rmax.p, r_max, sizeof(double) * N, hipMemcpyHostToDevice, s));
        d_rmax = L->rmax.as<double>();
    }
    double* d_prev = nullptr;
    double* d_dlimT = nullptr;
    if (want_obj && prev && N > 0) {
        if (!d_lim) return fail(MAC_E_INVAL, "prev given without d_lim");
        L->prev.reserve(sizeof(double) * three_n);
        L->dlim.reserve(sizeof(double) * N);
        L->dlimraw.reserve(sizeof(double) * N);
        L->h_dlim.resize(N);
        for (int i = 0; i < N; ++i) L->h_dlim[i] = dlim_threshold(d_lim[i]);
        if constexpr (f32)
            upload_widen(prev, three_n, L->p32, L->prev.as<double>(), s);
        else
            HCK(hipMemcpyAsync(L->prev.p, prev, sizeof(double) * three_n, hipMemcpyHostToDevice, s));
        HCK(hipMemcpyAsync(L->dlim.p, L->h_dlim.data(), sizeof(double) * N, hipMemcpyHostToDevice,
                           s));
        HCK(hipMemcpyAsync(L->dlimraw.p, d_lim, sizeof(double) * N, hipMemcpyHostToDevice, s));
        d_prev = L->prev.as<double>();
        d_dlimT = L->dlim.as<double>();
    }
    const double* hc = nullptr;
    if constexpr (!f32) hc = cands;   // (AUTO's host-side walk estimate reads fp64 candidates)
    if (K > 1 && !t_defer_free && !ctx->route_seeded.exchange(true)) {
        if constexpr (f32) {
            std::vector<double> x0(cands, cands + three_n);
            seed_route(ctx, x0.data(), N);
        } else {
            seed_route(ctx, cands, N);
        }
    }
    const bool tiled = use_tiled(ctx, N, hc, three_n);
    enqueue_eval(ctx, L, s, matrix_src(L->cands.as<double>(), N), N, (int)K, tiled, d_rmax, penalty, d_prev,
                 d_dlimT, d_prev ? L->dlimraw.as<double>() : nullptr, tan_half_fov,
                 area_out ? L->area.as<double>() : nullptr,
                 want_obj ? L->obj.as<double>() : nullptr,
                 (best_obj || best_idx) ? L->best.as<double>() : nullptr, 0);
    // results: into the pinned buffer (the upload has completed before the kernels ran), then
    // one host copy each after the sync
    double* ho = staged ? (double*)L->h_io.p : nullptr;
    double* h_area = area_out ? (staged ? ho : area_out) : nullptr;
    double* h_obj = obj_out ? (staged ? ho + (area_out ? K : 0) : obj_out) : nullptr;
    double hb_local[2] = {0, 0};
    double* hb = staged ? ho + (size_t)K * ((area_out ? 1 : 0) + (obj_out ? 1 : 0)) : hb_local;
    if (h_area) HCK(hipMemcpyAsync(h_area, L->area.p, sizeof(double) * K, hipMemcpyDeviceToHost, s));
    if (h_obj) HCK(hipMemcpyAsync(h_obj, L->obj.p, sizeof(double) * K, hipMemcpyDeviceToHost, s));
    if (best_obj || best_idx) HCK(hipMemcpyAsync(hb, L->best.p, 16, hipMemcpyDeviceToHost, s));
    HCK(hipStreamSynchronize(s));
    if (staged && area_out) std::memcpy(area_out, h_area, sizeof(double) * K);
    if (staged && obj_out) std::memcpy(obj_out, h_obj, sizeof(double) * K);
    if (best_obj) *best_obj = hb[0];
    if (best_idx) *best_idx = __builtin_bit_cast(int64_t, hb[1]);
    return MAC_OK;
}


// The basis form of a caller-owned poll (mac_poll_basis_f64): the incumbent, B = L[rp][:, cp] as L's
// packed lower triangle (int16) with the two permutations, and delta; the 2n candidates
// x + delta B[:, k], x - delta B[:, k] are expanded on the device (k_prep.h CandSrc.entry), so the
// host ships n(n+1) + 16n bytes instead of the 3N x 2n matrix's 16 n^2.
static int32_t host_eval_basis(mac_ctx* ctx, const double* x_inc, int64_t three_n, const int16_t* ltri,
                               const int32_t* rp, const int32_t* cp, double delta, const double* r_max,
                               double penalty, const double* prev, const double* d_lim,
                               double tan_half_fov, double* obj_out, double* best_obj, int64_t* best_idx)
{
    const int64_t n = three_n;
    const int64_t K = 2 * n;
    int32_t rc = check_common(ctx, three_n, K);
    if (rc) return rc;
    if (n == 0) {
        if (best_idx) *best_idx = -1;
        if (best_obj) *best_obj = INFINITY;
        return MAC_OK;
    }
    if (!x_inc || !ltri || !rp || !cp || !r_max) return fail(MAC_E_INVAL, "null argument");
    if (!std::isfinite(delta)) return fail(MAC_E_INVAL, "delta not finite");
    // the permutations index L on the device: every value must lie in [0, n)
    for (int64_t v = 0; v < n; ++v)
        if (rp[v] < 0 || rp[v] >= n || cp[v] < 0 || cp[v] >= n)
            return fail(MAC_E_INVAL, "rp / cp entry outside [0, n)");
    if (prev && !d_lim) return fail(MAC_E_INVAL, "prev given without d_lim");
    const int N = (int)(three_n / 3);
    int64_t bmax = 1;   // the largest |diagonal| (LTMADS: the step 2^ell): the chain's routing hint
    for (int64_t r = 0; r < n; ++r) bmax = std::max<int64_t>(bmax, std::abs((int)ltri[r * (r + 1) / 2 + r]));
    set_device(ctx);
    LaneGuard lg(ctx);
    Lane* L = lg.lane;
    hipStream_t s = L->stream;
    const size_t tri = (size_t)n * (size_t)(n + 1) / 2;
    const size_t in_bytes = sizeof(double) * n + sizeof(int32_t) * 2 * n + sizeof(int16_t) * tri;
    const size_t out_bytes = (obj_out ? sizeof(double) * K : 0) + 16;
    L->cands.reserve(in_bytes);
    L->obj.reserve(sizeof(double) * K);
    L->best.reserve(16);
    // one pinned staging area and one copy: [x 8n][rp 4n][cp 4n][L 2 tri]
    L->h_io.reserve(std::max(in_bytes, out_bytes));
    unsigned char* h = (unsigned char*)L->h_io.p;
    std::memcpy(h, x_inc, sizeof(double) * n);
    std::memcpy(h + 8 * n, rp, sizeof(int32_t) * n);
    std::memcpy(h + 12 * n, cp, sizeof(int32_t) * n);
    std::memcpy(h + 16 * n, ltri, sizeof(int16_t) * tri);
    HCK(hipMemcpyAsync(L->cands.p, h, in_bytes, hipMemcpyHostToDevice, s));
    L->rmax.reserve(sizeof(double) * N);
    HCK(hipMemcpyAsync(L->rmax.p, r_max, sizeof(double) * N, hipMemcpyHostToDevice, s));
    double* d_prev = nullptr;
    double* d_dlimT = nullptr;
    if (prev) {
        L->prev.reserve(sizeof(double) * three_n);
        L->dlim.reserve(sizeof(double) * N);
        L->dlimraw.reserve(sizeof(double) * N);
        L->h_dlim.resize(N);
        for (int i = 0; i < N; ++i) L->h_dlim[i] = dlim_threshold(d_lim[i]);
        HCK(hipMemcpyAsync(L->prev.p, prev, sizeof(double) * three_n, hipMemcpyHostToDevice, s));
        HCK(hipMemcpyAsync(L->dlim.p, L->h_dlim.data(), sizeof(double) * N, hipMemcpyHostToDevice, s));
        HCK(hipMemcpyAsync(L->dlimraw.p, d_lim, sizeof(double) * N, hipMemcpyHostToDevice, s));
        d_prev = L->prev.as<double>();
        d_dlimT = L->dlim.as<double>();
    }
    unsigned char* d = (unsigned char*)L->cands.p;
    CandSrc src{};
    src.xinc = (const double*)d;
    src.rp = (const int*)(d + 8 * n);
    src.cp = (const int*)(d + 12 * n);
    src.ltri = (const int16_t*)(d + 16 * n);
    src.delta = delta;
    src.b = bmax;
    src.k0 = 0;
    src.route_five = host_crowded_disks(x_inc, N, (double)bmax * std::fabs(delta), ctx->grid.S) > kBitsMinDisks;
    enqueue_eval(ctx, L, s, src, N, (int)K, use_tiled(ctx, N, nullptr, three_n), L->rmax.as<double>(),
                 penalty, d_prev, d_dlimT, d_prev ? L->dlimraw.as<double>() : nullptr, tan_half_fov,
                 nullptr, L->obj.as<double>(), L->best.as<double>(), 0);
    // (the upload completed before the kernels ran: the staging takes the results)
    double* ho = (double*)L->h_io.p;
    double* hb = ho + (obj_out ? K : 0);
    if (obj_out) HCK(hipMemcpyAsync(ho, L->obj.p, sizeof(double) * K, hipMemcpyDeviceToHost, s));
    HCK(hipMemcpyAsync(hb, L->best.p, 16, hipMemcpyDeviceToHost, s));
    HCK(hipStreamSynchronize(s));
    if (obj_out) std::memcpy(obj_out, ho, sizeof(double) * K);
    if (best_obj) *best_obj = hb[0];
    if (best_idx) *best_idx = __builtin_bit_cast(int64_t, hb[1]);
    return MAC_OK;
}

// ------------------------------------------------------------------ C-ABI

extern "C" {

#ifdef MAC_DIAG
// diagnostic build only (not declared in maxcover.h): per-workgroup poll-walk stamps
int32_t mac_diag_index_read(uint64_t* out, int64_t n)
{
    if (n > (int64_t)(8 * 65536)) n = 8 * 65536;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_diag_index), sizeof(uint64_t) * n, 0,
                            hipMemcpyDeviceToHost) != hipSuccess)
        return MAC_E_HIP;
    return MAC_OK;
}

int32_t mac_diag_walk_read(uint64_t* out, int64_t n)
{
    if (n > (int64_t)(8 * 65536)) n = 8 * 65536;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_diag_walk), sizeof(uint64_t) * n, 0,
                            hipMemcpyDeviceToHost) != hipSuccess)
        return MAC_E_HIP;
    return MAC_OK;
}

// diagnostic build only: per-disk phase stamps of the fused kernel (k_fiw.h)
int32_t mac_diag_fiw_read(uint64_t* out, int64_t n)
{
    if (n > (int64_t)(16 * 65536)) n = 16 * 65536;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_diag_fiw), sizeof(uint64_t) * n, 0,
                            hipMemcpyDeviceToHost) != hipSuccess)
        return MAC_E_HIP;
    return MAC_OK;
}

// diagnostic build only: per-block phase stamps of fin2_kernel (k_fiw.h)
int32_t mac_diag_f2_read(uint64_t* out, int64_t n)
{
    if (n > (int64_t)(8 * 4096)) n = 8 * 4096;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_diag_f2), sizeof(uint64_t) * n, 0,
                            hipMemcpyDeviceToHost) != hipSuccess)
        return MAC_E_HIP;
    return MAC_OK;
}

// diagnostic build only: phase stamps of the prep launch's first 64 chain workgroups (k_prep.h)
int32_t mac_diag_prep_read(uint64_t* out, int64_t n)
{
    if (n > 64 * 16) n = 64 * 16;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_diag_prep), sizeof(uint64_t) * n, 0,
                            hipMemcpyDeviceToHost) != hipSuccess)
        return MAC_E_HIP;
    return MAC_OK;
}

// diagnostic build only: per-workgroup phase ticks of shared_bits_kernel (k_bits.h)
int32_t mac_diag_bits_read(uint64_t* out, int64_t n)
{
    if (n > 256 * 16) n = 256 * 16;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_diag_bits), sizeof(uint64_t) * n, 0,
                            hipMemcpyDeviceToHost) != hipSuccess)
        return MAC_E_HIP;
    return MAC_OK;
}

// diagnostic build only: per-workgroup phase ticks of shared_or_kernel (k_or.h)
int32_t mac_diag_or_read(uint64_t* out, int64_t n)
{
    if (n > 1024 * 16) n = 1024 * 16;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_diag_or), sizeof(uint64_t) * n, 0,
                            hipMemcpyDeviceToHost) != hipSuccess)
        return MAC_E_HIP;
    return MAC_OK;
}

// diagnostic build only: the raw profiling stamps ({start, end} per workgroup slot, in launch
// order) and how many slots are used
int32_t mac_diag_stamps(mac_ctx* ctx, uint64_t* out, int64_t n, int64_t* used)
{
    if (!ctx) return MAC_E_INVAL;
    if (hipDeviceSynchronize() != hipSuccess) return MAC_E_HIP;
    std::lock_guard<std::mutex> lk(ctx->mu);
    *used = ctx->stamp_used;
    n = std::min<int64_t>(n, 2 * ctx->stamp_used);
    if (n > 0 && hipMemcpy(out, ctx->stamps.p, sizeof(uint64_t) * n, hipMemcpyDeviceToHost) != hipSuccess)
        return MAC_E_HIP;
    return MAC_OK;
}

int32_t mac_diag_read(uint64_t* out, int64_t n)
{
    if (n > (int64_t)(4 * kDiagMax)) n = 4 * kDiagMax;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_diag), sizeof(uint64_t) * n, 0, hipMemcpyDeviceToHost) != hipSuccess)
        return MAC_E_HIP;
    return MAC_OK;
}
#endif

const char* mac_last_error(void) { return g_last_error.c_str(); }

const char* mac_version(void) { return "maxcover 0.1.0 gfx950"; }

double mac_cover_threshold(double r) { return cover_threshold(r); }

int32_t mac_profile_read(mac_ctx* ctx, double* kernel_ms, int64_t* launches,
                         int64_t* candidates, int32_t* last_algo, int32_t reset)
{
    ABI_BEGIN
    if (!ctx) return fail(MAC_E_INVAL, "null context");
    set_device(ctx);
    HCK(hipDeviceSynchronize());   // every recorded launch has completed
    std::lock_guard<std::mutex> lk(ctx->mu);
    std::vector<uint64_t> st((size_t)(2 * ctx->stamp_used));
    if (!st.empty())
        HCK(hipMemcpy(st.data(), ctx->stamps.p, sizeof(uint64_t) * st.size(), hipMemcpyDeviceToHost));
    double ms = 0.0;
    int64_t n = 0, kc = 0;
    int algo = 0;
    // launch time = last wave end - first workgroup start over the launch's workgroups
    auto span_ms = [&](int64_t base, int64_t nwg) {
        uint64_t t0 = ~(uint64_t)0, t1 = 0;
        for (int64_t q = base; q < base + nwg; ++q) {
            t0 = std::min(t0, st[(size_t)(2 * q)]);
            t1 = std::max(t1, st[(size_t)(2 * q + 1)]);
        }
        return t1 > t0 ? (double)(t1 - t0) / kRealtimeHz * 1e3 : 0.0;
    };
    for (auto& p : ctx->prof) {
        algo = p.algo;
        int64_t a = p.a, na = p.na;
        if (p.mode) {  // the device's choice (the lane's mode word holds its latest decision)
            int m = 0;
            HCK(hipMemcpy(&m, p.mode, sizeof(int), hipMemcpyDeviceToHost));
            algo = m == kModePoll ? MAC_ALGO_POLL : MAC_ALGO_TILED;
            if (m == kModePoll) {
                a = p.b;
                na = p.nb;
            }
        }
        if (a < 0) continue;
        ms += span_ms(a, na);
        ++n;
        kc += p.K;
    }
    if (kernel_ms) *kernel_ms = ms;
    if (launches) *launches = n;
    if (candidates) *candidates = kc;
    if (last_algo) *last_algo = algo;
    if (reset) {
        ctx->prof.clear();
        if (ctx->stamp_used) HCK(hipMemset(ctx->stamps.p, 0, sizeof(uint64_t) * 2 * ctx->stamp_used));
        ctx->stamp_used = 0;
    }
    return MAC_OK;
    ABI_END
}

int32_t mac_profile_split(mac_ctx* ctx, double* prep_ms, double* walk_ms, double* gap_ms,
                          int64_t* polls)
{
    ABI_BEGIN
    if (!ctx) return fail(MAC_E_INVAL, "null context");
    set_device(ctx);
    HCK(hipDeviceSynchronize());
    std::lock_guard<std::mutex> lk(ctx->mu);
    std::vector<uint64_t> st((size_t)(2 * ctx->stamp_used));
    if (!st.empty())
        HCK(hipMemcpy(st.data(), ctx->stamps.p, sizeof(uint64_t) * st.size(), hipMemcpyDeviceToHost));
    double a1 = 0.0, a2 = 0.0, gap = 0.0;
    int64_t n = 0;
    for (auto& p : ctx->prof) {
        // the launch chain: prep = first launch's start .. the walk's start, walk = the walk
        // launch, gap = the walk's end .. finalize's end (the argmin included)
        if (p.c < 0 || p.f < 0) continue;
        int64_t wa = p.a, wn = p.na;
        if (p.mode) {
            int m = 0;
            HCK(hipMemcpy(&m, p.mode, sizeof(int), hipMemcpyDeviceToHost));
            if (m == kModePoll) {
                wa = p.b;
                wn = p.nb;
            }
        }
        uint64_t s0 = ~(uint64_t)0, sw = ~(uint64_t)0, ew = 0, ef = 0;
        for (int64_t q = p.c; q < p.c + p.nc; ++q) s0 = std::min(s0, st[(size_t)(2 * q)]);
        for (int64_t q = wa; wa >= 0 && q < wa + wn; ++q) {
            sw = std::min(sw, st[(size_t)(2 * q)]);
            ew = std::max(ew, st[(size_t)(2 * q + 1)]);
        }
        for (int64_t q = p.f; q < p.f + p.nf; ++q) ef = std::max(ef, st[(size_t)(2 * q + 1)]);
        if (!(ef > s0) || !(ew > sw) || sw < s0) continue;
        a1 += (double)(sw - s0) / kRealtimeHz * 1e3;
        a2 += (double)(ew - sw) / kRealtimeHz * 1e3;
        gap += (double)(ef - ew) / kRealtimeHz * 1e3;
        ++n;
    }
    if (prep_ms) *prep_ms = a1;
    if (walk_ms) *walk_ms = a2;
    if (gap_ms) *gap_ms = gap;
    if (polls) *polls = n;
    return MAC_OK;
    ABI_END
}

int32_t mac_profile_kernels(mac_ctx* ctx, double* ms_out, int64_t* launches_out, int32_t n_roles)
{
    ABI_BEGIN
    if (!ctx) return fail(MAC_E_INVAL, "null context");
    if (n_roles < 0 || (n_roles > 0 && (!ms_out || !launches_out)))
        return fail(MAC_E_INVAL, "null output / negative role count");
    set_device(ctx);
    HCK(hipDeviceSynchronize());
    std::lock_guard<std::mutex> lk(ctx->mu);
    std::vector<uint64_t> st((size_t)(2 * ctx->stamp_used));
    if (!st.empty())
        HCK(hipMemcpy(st.data(), ctx->stamps.p, sizeof(uint64_t) * st.size(), hipMemcpyDeviceToHost));
    const int nr = std::min<int32_t>(n_roles, MAC_PROF_ROLES);
    for (int r = 0; r < n_roles; ++r) {
        ms_out[r] = 0.0;
        launches_out[r] = 0;
    }
    for (auto& p : ctx->prof) {
        for (int r = 0; r < nr; ++r) {
            const int64_t base = p.role[r][0], nwg = p.role[r][1];
            if (base < 0 || nwg <= 0) continue;
            uint64_t t0 = ~(uint64_t)0, t1 = 0;
            for (int64_t q = base; q < base + nwg; ++q) {
                t0 = std::min(t0, st[(size_t)(2 * q)]);
                t1 = std::max(t1, st[(size_t)(2 * q + 1)]);
            }
            if (!(t1 > t0)) continue;
            ms_out[r] += (double)(t1 - t0) / kRealtimeHz * 1e3;
            ++launches_out[r];
        }
    }
    return MAC_OK;
    ABI_END
}

int32_t mac_device_count(int32_t* count_out)
{
    ABI_BEGIN
    if (!count_out) return fail(MAC_E_INVAL, "null count_out");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *count_out = n;
    return MAC_OK;
    ABI_END
}

int32_t mac_ctx_create(mac_ctx** out, int32_t device)
{
    ABI_BEGIN
    if (!out) return fail(MAC_E_INVAL, "null out");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return fail(MAC_E_NODEVICE, "no HIP device visible");
    if (device < 0 || device >= n) return fail(MAC_E_NODEVICE, "device index out of range");
    HCK(hipSetDevice(device));
    mac_ctx* ctx = new mac_ctx();
    if (const char* e = std::getenv("MAXCOVER_HOST_STATS"); e && *e == '1') ctx->host_stats = true;
    ctx->device = device;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
        ctx->cus = prop.multiProcessorCount;
    int bar = 0;
    const char* eb = std::getenv("MAXCOVER_CL_BAR");
    ctx->cl_bar = hipDeviceGetAttribute(&bar, hipDeviceAttributeIsLargeBar, device) == hipSuccess && bar == 1 &&
                  !(eb && *eb == '0');
    HCK(hipStreamCreateWithFlags(&ctx->setup_stream, hipStreamNonBlocking));
    *out = ctx;
    return MAC_OK;
    ABI_END
}

void mac_ctx_destroy(mac_ctx* ctx)
{
    if (!ctx) return;
    if (const char* e = std::getenv("MAXCOVER_CL_STATS"); e && *e == '1' && ctx->cl_batches) {
        std::fprintf(stderr, "maxcover: closure batches %lld, requests %lld (%.2f per batch); per batch (us): "
                     "lane %.1f, staging %.1f, copy+launch %.1f, hand-out %.1f\n",
                     (long long)ctx->cl_batches, (long long)ctx->cl_reqs, (double)ctx->cl_reqs / (double)ctx->cl_batches,
                     ctx->cl_phase_ns[3] * 1e-3 / ctx->cl_batches, ctx->cl_phase_ns[0] * 1e-3 / ctx->cl_batches,
                     ctx->cl_phase_ns[1] * 1e-3 / ctx->cl_batches, ctx->cl_phase_ns[2] * 1e-3 / ctx->cl_batches);
        const double u = 1e-3 / (double)ctx->cl_reqs;
        std::fprintf(stderr, "maxcover: closure per request (us): queued %.1f, taken -> handed out %.1f, "
                     "-> seen %.1f, -> slot read %.1f; call %.1f; led by own thread %.0f%%\n",
                     ctx->cl_req_ns[0] * u, ctx->cl_req_ns[1] * u, ctx->cl_req_ns[2] * u, ctx->cl_req_ns[3] * u,
                     ctx->cl_req_ns[4] * u, 100.0 * ctx->cl_led / ctx->cl_reqs);
    }
    if (ctx->host_stats && ctx->hs_n)
        std::fprintf(stderr, "maxcover: fused polls %lld, host us per poll: to prep launch %.2f, prep launch %.2f, "
                     "fiw launch %.2f, fin2 launch %.2f\n", (long long)ctx->hs_n, ctx->hs_t[0] / ctx->hs_n * 1e6,
                     ctx->hs_t[1] / ctx->hs_n * 1e6, ctx->hs_t[2] / ctx->hs_n * 1e6, ctx->hs_t[3] / ctx->hs_n * 1e6);
    (void)hipSetDevice(ctx->device);
    if (ctx->doorbell) {   // every armed poll released first (else the synchronisation would wait)
        __atomic_store_n(ctx->doorbell, ~(uint64_t)0 >> 1, __ATOMIC_RELEASE);
        ctx->fired = ctx->armed;
    }
    (void)hipDeviceSynchronize();
    if (ctx->comm) (void)ctx->rccl->comm_destroy(ctx->comm);
    if (ctx->d_xrec) (void)hipFree(ctx->d_xrec);
    if (ctx->d_xrec2) (void)hipFree(ctx->d_xrec2);
    ctx->h_xrec.release();
    free_deferred(ctx);
    if (ctx->doorbell) (void)hipHostFree(ctx->doorbell);
    ctx->h_mirror.release();
    for (Lane* l : ctx->lanes_all) {
        l->h_stage.release();
        l->h_io.release();
        l->h_dc.release();
        l->h_cl.release();
        for (DevBuf* b : {&l->cands, &l->disks, &l->partial, &l->area, &l->obj, &l->best,
                          &l->rmax, &l->prev, &l->dlim, &l->region, &l->mode, &l->nbr,
                          &l->ncount, &l->dlist, &l->qual, &l->spart, &l->vp, &l->xinc,
                          &l->perm, &l->ucount, &l->umap, &l->keysT, &l->lane4,
                          &l->lanexp, &l->rows, &l->nboxT, &l->cnt, &l->dlimraw, &l->finblk, &l->finarrive, &l->c32, &l->p32,
                          &l->cpart, &l->carrive, &l->ctot, &l->clv, &l->prec, &l->cost, &l->nboxU,
                          &l->ncountU, &l->orjobs, &l->pd, &l->dead8, &l->frows, &l->fwhint, &l->fwlist, &l->fwcount,
                          &l->fwsxy, &l->fwsw})
            b->release();
        if (l->done) (void)hipEventDestroy(l->done);

        if (l->stream) (void)hipStreamDestroy(l->stream);
        delete l;
    }
    for (DevBuf* b : {&ctx->x, &ctx->y, &ctx->w, &ctx->xys, &ctx->ws, &ctx->perm, &ctx->off,
                      &ctx->keys_in, &ctx->keys_out, &ctx->idx_in, &ctx->tmp, &ctx->bbox,
                      &ctx->flags_s, &ctx->flags_o, &ctx->keep, &ctx->sel_count, &ctx->cx,
                      &ctx->cy, &ctx->cw, &ctx->cidx, &ctx->circ, &ctx->cdisk})
        b->release();
    ctx->stamps.release();
    if (ctx->setup_stream) (void)hipStreamDestroy(ctx->setup_stream);
    delete ctx;
}

int32_t mac_set_option(mac_ctx* ctx, int32_t option, int64_t value)
{
    if (!ctx) return fail(MAC_E_INVAL, "null context");
    switch (option) {
    case MAC_OPT_ALGO:
        if (value < MAC_ALGO_AUTO || value > MAC_ALGO_POLL) return fail(MAC_E_INVAL, "bad algo");
        ctx->algo = (int)value;
        return MAC_OK;
    case MAC_OPT_STORAGE:
        if (value != MAC_STORE_F64 && value != MAC_STORE_F32)
            return fail(MAC_E_INVAL, "bad storage");
        // the list stays fp64 in HBM: the walks' band decisions re-read exact coordinates, and
        // fp32 inputs arrive through the *_f32 entry points, widened losslessly
        if (value == MAC_STORE_F32) return fail(MAC_E_INVAL, "storage is fp64 (use the *_f32 entry points)");
        ctx->storage = (int)value;
        return MAC_OK;
    case MAC_OPT_PROFILE: {
        ABI_BEGIN
        std::lock_guard<std::mutex> lk(ctx->mu);
        if (value && !ctx->profile) {  // fresh, zeroed stamp slots (outside any timed region)
            set_device(ctx);
            constexpr int64_t kSlots = (int64_t)1 << 21;   // 32 MB: ~800 config-4 poll chains
            ctx->stamps.reserve(sizeof(uint64_t) * 2 * kSlots);
            HCK(hipDeviceSynchronize());
            HCK(hipMemset(ctx->stamps.p, 0, sizeof(uint64_t) * 2 * kSlots));
            ctx->stamp_cap = kSlots;
            ctx->stamp_used = 0;
            ctx->prof.clear();
        }
        ctx->profile = value != 0;
        return MAC_OK;
        ABI_END
    }
    case MAC_OPT_SHARED:
        if (value < MAC_SHARED_AUTO || value > MAC_SHARED_BITS) return fail(MAC_E_INVAL, "bad shared mode");
        ctx->shared_mode = (int)value;
        return MAC_OK;
    case MAC_OPT_CHAIN:
        if (value < MAC_CHAIN_AUTO || value > MAC_CHAIN_FUSED) return fail(MAC_E_INVAL, "bad chain");
        ctx->chain = (int)value;
        return MAC_OK;
    case MAC_OPT_TILE_POINTS:
        if (value < 1 || value > 4096) return fail(MAC_E_INVAL, "tile points out of range");
        ctx->tile_ppt = (int)value;
        return MAC_OK;
    default:
        return fail(MAC_E_INVAL, "unknown option");
    }
}

static int32_t set_points_common(mac_ctx* ctx, int64_t M)
{
    if (!ctx) return fail(MAC_E_INVAL, "null context");
    int32_t rc = check_M(M);
    if (rc) return rc;
    set_device(ctx);
    HCK(hipDeviceSynchronize());  // no evaluation may overlap a point-list change
    free_deferred(ctx);
    ctx->M = M;
    ctx->has_points = false;
    const size_t b = sizeof(double) * (size_t)std::max<int64_t>(M, 1);
    ctx->x.reserve(b);
    ctx->y.reserve(b);
    ctx->w.reserve(b);
    return MAC_OK;
}

int32_t mac_set_points_f64(mac_ctx* ctx, const double* x, const double* y, const double* w,
                           int64_t M)
{
    ABI_BEGIN
    if (M > 0 && (!x || !y || !w)) return fail(MAC_E_INVAL, "null point array");
    int32_t rc = set_points_common(ctx, M);
    if (rc) return rc;
    hipStream_t s = ctx->setup_stream;
    if (M > 0) {
        HCK(hipMemcpyAsync(ctx->x.p, x, sizeof(double) * M, hipMemcpyHostToDevice, s));
        HCK(hipMemcpyAsync(ctx->y.p, y, sizeof(double) * M, hipMemcpyHostToDevice, s));
        HCK(hipMemcpyAsync(ctx->w.p, w, sizeof(double) * M, hipMemcpyHostToDevice, s));
    }
    build_index(ctx, s);
    return MAC_OK;
    ABI_END
}

int32_t mac_set_points_f32(mac_ctx* ctx, const float* x, const float* y, const float* w, int64_t M)
{
    ABI_BEGIN
    if (M > 0 && (!x || !y || !w)) return fail(MAC_E_INVAL, "null point array");
    int32_t rc = set_points_common(ctx, M);
    if (rc) return rc;
    hipStream_t s = ctx->setup_stream;
    upload_widen(x, M, ctx->tmp, ctx->x.as<double>(), s);
    HCK(hipStreamSynchronize(s));   // (one staging buffer, reused per coordinate)
    upload_widen(y, M, ctx->tmp, ctx->y.as<double>(), s);
    HCK(hipStreamSynchronize(s));
    upload_widen(w, M, ctx->tmp, ctx->w.as<double>(), s);
    build_index(ctx, s);
    return MAC_OK;
    ABI_END
}

int32_t mac_set_points_dev_f32(mac_ctx* ctx, const float* d_x, const float* d_y, const float* d_w,
                               int64_t M)
{
    ABI_BEGIN
    if (M > 0 && (!d_x || !d_y || !d_w)) return fail(MAC_E_INVAL, "null point array");
    int32_t rc = set_points_common(ctx, M);
    if (rc) return rc;
    hipStream_t s = ctx->setup_stream;
    widen_async(d_x, M, ctx->x.as<double>(), s);
    widen_async(d_y, M, ctx->y.as<double>(), s);
    widen_async(d_w, M, ctx->w.as<double>(), s);
    build_index(ctx, s);
    return MAC_OK;
    ABI_END
}

int32_t mac_set_points_records_f64(mac_ctx* ctx, const double* rec, int64_t M, int64_t stride)
{
    ABI_BEGIN
    if (M > 0 && !rec) return fail(MAC_E_INVAL, "null records");
    if (stride < 4) return fail(MAC_E_INVAL, "record stride < 4");
    std::vector<double> hx(std::max<int64_t>(M, 0)), hy(hx.size()), hw(hx.size());
    for (int64_t i = 0; i < M; ++i) {
        hx[i] = rec[i * stride + 0];
        hy[i] = rec[i * stride + 1];
        hw[i] = rec[i * stride + 3];  // column 4, src/AreaCoverageCalculation.jl:72
    }
    return mac_set_points_f64(ctx, hx.data(), hy.data(), hw.data(), M);
    ABI_END
}

int32_t mac_set_points_dev_f64(mac_ctx* ctx, const double* d_x, const double* d_y,
                               const double* d_w, int64_t M)
{
    ABI_BEGIN
    if (M > 0 && (!d_x || !d_y || !d_w)) return fail(MAC_E_INVAL, "null point array");
    int32_t rc = set_points_common(ctx, M);
    if (rc) return rc;
    hipStream_t s = ctx->setup_stream;
    if (M > 0) {
        HCK(hipMemcpyAsync(ctx->x.p, d_x, sizeof(double) * M, hipMemcpyDeviceToDevice, s));
        HCK(hipMemcpyAsync(ctx->y.p, d_y, sizeof(double) * M, hipMemcpyDeviceToDevice, s));
        HCK(hipMemcpyAsync(ctx->w.p, d_w, sizeof(double) * M, hipMemcpyDeviceToDevice, s));
    }
    build_index(ctx, s);
    return MAC_OK;
    ABI_END
}

// update_POI (src/CellFunctions.jl:59-79): the list grows at its end; the existing entries keep
// their positions (list order = summation order), then the tile index is rebuilt.
static int32_t append_common(mac_ctx* ctx, const void* x, const void* y, const void* w, int64_t m,
                             hipMemcpyKind kind)
{
    if (!ctx) return fail(MAC_E_INVAL, "null context");
    if (m < 0) return fail(MAC_E_INVAL, "m < 0");
    if (m > 0 && (!x || !y || !w)) return fail(MAC_E_INVAL, "null point array");
    const int64_t M0 = ctx->has_points ? ctx->M : 0;
    int32_t rc = check_M(M0 + m);
    if (rc) return rc;
    set_device(ctx);
    HCK(hipDeviceSynchronize());  // no evaluation may overlap a point-list change
    free_deferred(ctx);
    hipStream_t s = ctx->setup_stream;
    const size_t need = sizeof(double) * (size_t)std::max<int64_t>(M0 + m, 1);
    if (need > ctx->x.cap) {      // grow by 1.5x, keeping the existing entries
        const size_t b = std::max(need, ctx->x.cap + ctx->x.cap / 2);
        for (DevBuf* d : {&ctx->x, &ctx->y, &ctx->w}) {
            DevBuf nb;
            nb.reserve(b);
            if (M0 > 0) HCK(hipMemcpyAsync(nb.p, d->p, sizeof(double) * M0, hipMemcpyDeviceToDevice, s));
            HCK(hipStreamSynchronize(s));
            d->release();
            *d = nb;
            nb.p = nullptr;
            nb.cap = 0;
        }
    }
    if (m > 0) {
        HCK(hipMemcpyAsync(ctx->x.as<double>() + M0, x, sizeof(double) * m, kind, s));
        HCK(hipMemcpyAsync(ctx->y.as<double>() + M0, y, sizeof(double) * m, kind, s));
        HCK(hipMemcpyAsync(ctx->w.as<double>() + M0, w, sizeof(double) * m, kind, s));
    }
    ctx->M = M0 + m;
    build_index(ctx, s);
    return MAC_OK;
}

int32_t mac_append_points_f64(mac_ctx* ctx, const double* x, const double* y, const double* w,
                              int64_t m)
{
    ABI_BEGIN
    return append_common(ctx, x, y, w, m, hipMemcpyHostToDevice);
    ABI_END
}

int32_t mac_append_points_dev_f64(mac_ctx* ctx, const double* d_x, const double* d_y,
                                  const double* d_w, int64_t m)
{
    ABI_BEGIN
    return append_common(ctx, d_x, d_y, d_w, m, hipMemcpyDeviceToDevice);
    ABI_END
}

int32_t mac_num_points(mac_ctx* ctx, int64_t* M_out)
{
    if (!ctx || !M_out) return fail(MAC_E_INVAL, "null argument");
    *M_out = ctx->has_points ? ctx->M : 0;
    return MAC_OK;
}

int32_t mac_get_points_f64(mac_ctx* ctx, double* x, double* y, double* w)
{
    ABI_BEGIN
    if (!ctx) return fail(MAC_E_INVAL, "null context");
    if (!ctx->has_points) return fail(MAC_E_NOPOINTS, "no point list set");
    set_device(ctx);
    hipStream_t s = ctx->setup_stream;
    const size_t b = sizeof(double) * ctx->M;
    if (ctx->M > 0) {
        if (x) HCK(hipMemcpyAsync(x, ctx->x.p, b, hipMemcpyDeviceToHost, s));
        if (y) HCK(hipMemcpyAsync(y, ctx->y.p, b, hipMemcpyDeviceToHost, s));
        if (w) HCK(hipMemcpyAsync(w, ctx->w.p, b, hipMemcpyDeviceToHost, s));
    }
    HCK(hipStreamSynchronize(s));
    return MAC_OK;
    ABI_END
}

// covered flags (list order) into ctx->flags_o for one candidate; returns on stream s.
static void compute_flags(mac_ctx* ctx, hipStream_t s, const double* circles, int N)
{
    const int64_t M = ctx->M;
    ctx->flags_s.reserve(std::max<int64_t>(M, 1));
    ctx->flags_o.reserve(std::max<int64_t>(M, 1));
    ctx->circ.reserve(sizeof(double) * std::max(3 * N, 1));
    ctx->cdisk.reserve(sizeof(DiskRec) * std::max(N, 1));
    if (M == 0) return;
    HCK(hipMemsetAsync(ctx->flags_s.p, 0, M, s));
    if (N > 0) {
        HCK(hipMemcpyAsync(ctx->circ.p, circles, sizeof(double) * 3 * N, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(disk_prep_kernel, dim3(grid1d(N, 256)), dim3(256), 0, s,
                           matrix_src(ctx->circ.as<double>(), N), N, 1, ctx->cdisk.as<DiskRec>());
        HCK(hipGetLastError());
        const unsigned nb = (unsigned)std::max(1, std::min((N + kWavesPerBlock - 1) / kWavesPerBlock,
                                                           8 * ctx->cus));
        hipLaunchKernelGGL(covered_flags_tiled_kernel, dim3(nb), dim3(kBlock), 0, s,
                           ctx->xys.as<double2>(), ctx->off.as<int32_t>(), ctx->grid,
                           ctx->cdisk.as<DiskRec>(), N, ctx->flags_s.as<uint8_t>());
        HCK(hipGetLastError());
    }
    hipLaunchKernelGGL(scatter_flags_kernel, dim3(grid1d(M, 256)), dim3(256), 0, s,
                       ctx->flags_s.as<uint8_t>(), ctx->perm.as<uint32_t>(), M,
                       ctx->flags_o.as<uint8_t>());
    HCK(hipGetLastError());
}

int32_t mac_covered_flags_f64(mac_ctx* ctx, const double* circles, int64_t three_n,
                              uint8_t* flags_out)
{
    ABI_BEGIN
    int32_t rc = check_common(ctx, three_n, 0);
    if (rc) return rc;
    if (three_n > 0 && !circles) return fail(MAC_E_INVAL, "null circles");
    set_device(ctx);
    hipStream_t s = ctx->setup_stream;
    HCK(hipDeviceSynchronize());
    free_deferred(ctx);
    compute_flags(ctx, s, circles, (int)(three_n / 3));
    if (ctx->M > 0 && flags_out)
        HCK(hipMemcpyAsync(flags_out, ctx->flags_o.p, ctx->M, hipMemcpyDeviceToHost, s));
    HCK(hipStreamSynchronize(s));
    return MAC_OK;
    ABI_END
}

int32_t mac_remove_covered_f64(mac_ctx* ctx, const double* circles, int64_t three_n,
                               int64_t* kept_idx, int64_t* M_out)
{
    ABI_BEGIN
    int32_t rc = check_common(ctx, three_n, 0);
    if (rc) return rc;
    if (three_n > 0 && !circles) return fail(MAC_E_INVAL, "null circles");
    set_device(ctx);
    hipStream_t s = ctx->setup_stream;
    HCK(hipDeviceSynchronize());
    free_deferred(ctx);
    const int64_t M = ctx->M;
    compute_flags(ctx, s, circles, (int)(three_n / 3));
    int64_t kept = M;
    if (M > 0) {
        ctx->keep.reserve(M);
        hipLaunchKernelGGL(invert_flags_kernel, dim3(grid1d(M, 256)), dim3(256), 0, s,
                           ctx->flags_o.as<uint8_t>(), M, ctx->keep.as<uint8_t>());
        HCK(hipGetLastError());
        ctx->sel_count.reserve(sizeof(int64_t) * 4);
        const size_t b = sizeof(double) * M;
        ctx->cx.reserve(b);
        ctx->cy.reserve(b);
        ctx->cw.reserve(b);
        ctx->cidx.reserve(sizeof(int64_t) * M);
        size_t tb = 0, tb2 = 0;
        HCK(hipcub::DeviceSelect::Flagged(nullptr, tb, ctx->x.as<double>(), ctx->keep.as<uint8_t>(),
                                          ctx->cx.as<double>(), ctx->sel_count.as<int64_t>(), M, s));
        hipcub::CountingInputIterator<int64_t> it(0);
        HCK(hipcub::DeviceSelect::Flagged(nullptr, tb2, it, ctx->keep.as<uint8_t>(),
                                          ctx->cidx.as<int64_t>(), ctx->sel_count.as<int64_t>(), M,
                                          s));
        ctx->tmp.reserve(std::max(tb, tb2));
        HCK(hipcub::DeviceSelect::Flagged(ctx->tmp.p, tb, ctx->x.as<double>(), ctx->keep.as<uint8_t>(),
                                          ctx->cx.as<double>(), ctx->sel_count.as<int64_t>(), M, s));
        HCK(hipcub::DeviceSelect::Flagged(ctx->tmp.p, tb, ctx->y.as<double>(), ctx->keep.as<uint8_t>(),
                                          ctx->cy.as<double>(), ctx->sel_count.as<int64_t>(), M, s));
        HCK(hipcub::DeviceSelect::Flagged(ctx->tmp.p, tb, ctx->w.as<double>(), ctx->keep.as<uint8_t>(),
                                          ctx->cw.as<double>(), ctx->sel_count.as<int64_t>(), M, s));
        HCK(hipcub::DeviceSelect::Flagged(ctx->tmp.p, tb2, it, ctx->keep.as<uint8_t>(),
                                          ctx->cidx.as<int64_t>(), ctx->sel_count.as<int64_t>(), M,
                                          s));
        HCK(hipMemcpyAsync(&kept, ctx->sel_count.p, sizeof(int64_t), hipMemcpyDeviceToHost, s));
        HCK(hipStreamSynchronize(s));
        std::swap(ctx->x, ctx->cx);
        std::swap(ctx->y, ctx->cy);
        std::swap(ctx->w, ctx->cw);
        if (kept_idx && kept > 0)
            HCK(hipMemcpyAsync(kept_idx, ctx->cidx.p, sizeof(int64_t) * kept, hipMemcpyDeviceToHost,
                               s));
        ctx->M = kept;
        build_index(ctx, s);
    }
    if (M_out) *M_out = kept;
    return MAC_OK;
    ABI_END
}

// ------------------------------------------------------------------ native MADS driver

// Stable argsort of the next n stream values after stream position `first` - 1 (numpy
// argsort(kind="stable") of SplitMix64.next_u64(n)).
static void stream_permutation(uint64_t state, uint64_t first, int n, std::vector<int>& out)
{
    // A stable argsort of the keys, i.e. the order of the (key, index) pairs: bucketed by the
    // keys' top bits (uniform keys: O(n)), then insertion-sorted inside each bucket.
    int bits = 1;
    while ((1 << bits) < n && bits < 20) ++bits;
    const int nb = 1 << bits;
    std::vector<uint64_t> keys(n);
    std::vector<int> start(nb + 1, 0);
    for (int q = 0; q < n; ++q) {
        keys[q] = splitmix_at(state, first + (uint64_t)q);
        ++start[(keys[q] >> (64 - bits)) + 1];
    }
    for (int b = 0; b < nb; ++b) start[b + 1] += start[b];
    out.assign(n, 0);
    std::vector<int> fill(start.begin(), start.end() - 1);
    for (int q = 0; q < n; ++q) out[fill[keys[q] >> (64 - bits)]++] = q;  // ascending q per bucket
    for (int b = 0; b < nb; ++b) {
        for (int a = start[b] + 1; a < start[b + 1]; ++a) {
            const int v = out[a];
            int c = a - 1;
            while (c >= start[b] && keys[out[c]] > keys[v]) {  // strict: equal keys keep q order
                out[c + 1] = out[c];
                --c;
            }
            out[c + 1] = v;
        }
    }
}



// The native MADS loop as a stepper (mac_mads_begin / _poll / _update / _result): one
// iteration = one complete LTMADS poll generated on the device. A stepper may own a shard
// [lo, hi) of every poll's 2n candidates: the ranks of a multi-GPU run poll their shards, combine
// their local bests (16 B each, lexicographic (objective, index) minimum) and all apply the same
// update, so they stay in lock step with the single-GPU loop (mac_mads_run = one stepper owning
// the whole poll).
struct mac_mads {
    mac_ctx* ctx = nullptr;
    Lane* L = nullptr;
    hipStream_t s = nullptr;
    int N = 0, n = 0, K = 0;
    int64_t lo = 0, hi = 0;
    mac_mads_params prm{};
    double penalty = 1e5, tan_half_fov = 1.0;
    const double* d_prev = nullptr;
    const double* d_dlimT = nullptr;
    std::vector<double> x;
    double f = INFINITY;
    int64_t evals = 0, it = 0, rejected = 0, succ = 0;
    int ell = 0;
    std::vector<double> h_prev;   // cons3's prev (host copy: whole-poll rejection, poll_rejected)
    DevBuf d_feas;                // candidates that passed cons3 (the prep launches count them)
    uint64_t feas_seen = 0;       // d_feas as the last mac_mads_poll_ahead read it
    uint64_t state = 0, T = 0, per_iter = 0;
    std::vector<int> rp, cp, rp_next, cp_next;
    double* hb = nullptr;
    double* hx = nullptr;
    int* hperm = nullptr;
    // the poll's best, written by finalize's last block into a mapped slot {obj bits, index,
    // seq, check} (k_final.h): read here without a copy or a stream synchronisation
    PinnedBuf hslot;
    uint64_t* d_slot = nullptr;
    uint64_t seq = 0;
    bool slotted = false;
    int64_t slot_fallbacks = 0;   // slot waits that timed out (copy + sync instead)
    int route_five = 0;           // the polls are crowded (host_crowded_disks at begin): five-launch chain
    double* ext_best = nullptr;   // mac_mads_best_buffer: the polls' best goes here
    int64_t polled_b = 0;        // 2^ell of the poll awaiting its update (0: none)
    double h_enq = 0, h_perm = 0, h_wait = 0, h_post = 0;
    std::chrono::steady_clock::time_point t0;
    // the pipelined loop (mads_run_pipelined): incumbent double buffer, device state, permutation
    // rings
    DevBuf d_x, d_st, d_ring;
    PinnedBuf h_ring;
    ~mac_mads()
    {
        d_x.release();
        d_feas.release();
        d_st.release();
        d_ring.release();
        h_ring.release();
    }
};

static double* mads_best_ptr(mac_mads* m) { return m->ext_best ? m->ext_best : m->L->best.as<double>(); }

// Whether cons3 rejects every candidate of the poll at mesh step b around x (k_prep.h
// diag_rejects for each of the 3N variables: each is the diagonal of one column of B, so each
// candidate carries one such step). Exact: the prep's cons3 would mark every candidate failed,
// and the poll's result would be (+inf, -1).
// Routing a generated poll from the poll itself (the native MADS driver knows its incumbent and mesh
// step): the fused chain's superset boxes (k_fiw.h sup_box: every candidate's disk i lies within b of
// the incumbent's per coordinate, so box i is within 2b + r_i of its centre, plus a tile of
// rounding) overlap-tested by a sweep over the boxes sorted by their x start. More than
// kBitsMinDisks disks with a lower-index neighbour is a crowded poll (the five-launch chain's
// union pass decides its shared entries once; the fused chain would decide them per candidate in
// place, 5-20x slower: tools/c5_route.py). Returns that count.
static int host_crowded_disks(const double* x, int N, double b, double S)
{
    struct Bx {
        double x0, x1, y0, y1;
        int i;
    };
    std::vector<Bx> v;
    v.reserve(N);
    for (int i = 0; i < N; ++i) {
        const double r = x[2 * N + i];
        if (!(r + b > 0.0)) continue;   // covers nothing at any candidate
        const double h = 2.0 * b + std::fabs(r) + S;
        if (!std::isfinite(h) || !std::isfinite(x[i]) || !std::isfinite(x[N + i])) return N;   // (unknown)
        v.push_back({x[i] - h, x[i] + h, x[N + i] - h, x[N + i] + h, i});
    }
    std::sort(v.begin(), v.end(), [](const Bx& a, const Bx& c) { return a.x0 < c.x0; });
    std::vector<char> has(N, 0);
    std::vector<int> act;   // boxes whose x range may still reach later starts
    for (int q = 0; q < (int)v.size(); ++q) {
        const Bx& c = v[q];
        int w = 0;
        for (int a : act) {
            const Bx& o = v[a];
            if (o.x1 < c.x0) continue;   // (dropped: no later box starts before it ends)
            act[w++] = a;
            if (o.y0 <= c.y1 && c.y0 <= o.y1) has[std::max(o.i, c.i)] = 1;
        }
        act.resize(w);
        act.push_back(q);
    }
    int n = 0;
    for (char h : has) n += h;
    return n;
}

static bool poll_rejected(const mac_mads* m, int64_t b)
{
    if (!m->d_prev) return false;
    const int N = m->N;
    const std::vector<double>& T3 = m->L->h_dlim;
    for (int v = 0; v < m->n; ++v) {
        const int q = v / N, i = v % N;
        if (!diag_rejects(m->x[v], (double)b, m->h_prev[v], q, m->tan_half_fov, T3[i])) return false;
    }
    return true;
}

// slot: the poll's best through the mapped slot finalize's last block writes (mads_wait_best),
// else a 16-B copy
static void mads_make_slot(mac_mads* m)
{
    if (m->d_slot) return;
    m->hslot.reserve(64, hipHostMallocMapped | hipHostMallocCoherent);
    std::memset(m->hslot.p, 0, 64);
    void* dp = nullptr;
    HCK(hipHostGetDevicePointer(&dp, m->hslot.p, 0));
    m->d_slot = (uint64_t*)dp;
}

static void mads_best_of(mac_mads* m, const CandSrc& src, int Kc, int64_t idx_base, bool slot = false)
{
    if (slot) mads_make_slot(m);
    m->slotted = slot;
    enqueue_eval(m->ctx, m->L, m->s, src, m->N, Kc, use_tiled(m->ctx, m->N, nullptr, m->n),
                 m->L->rmax.as<double>(), m->penalty, m->d_prev, m->d_dlimT,
                 m->d_prev ? m->L->dlimraw.as<double>() : nullptr, m->tan_half_fov,
                 nullptr, m->L->obj.as<double>(), mads_best_ptr(m), idx_base,
                 slot ? m->d_slot : nullptr, slot ? ++m->seq : 0, nullptr,
                 slot ? m->d_feas.as<unsigned long long>() : nullptr);
    if (!slot) HCK(hipMemcpyAsync(m->hb, mads_best_ptr(m), 16, hipMemcpyDeviceToHost, m->s));
}

// The best {objective, global index} of the poll mads_best_of enqueued: from the mapped slot once
// it holds this poll's seq and a matching check word, or, after 50 ms (a failed launch) or
// without a slot, the stream synchronised and the copy.
static void mads_wait_best(mac_mads* m, double* obj, int64_t* idx, uint64_t* feas_cum = nullptr)
{
    if (m->slotted) {
        // a slotted poll always hands finalize the stepper's d_feas (mads_best_of), so the check
        // word folds in the feasible count of word 4: read it whether or not the caller wants it
        // (with f = 0 the check never matched once a candidate had passed cons3, and every wait
        // ran into the 50-ms limit: round 5's sharded-loop stall)
        uint64_t fe = 0;
        if (mirror_wait((const uint64_t*)m->hslot.p, m->seq, 50.0, obj, idx, &fe)) {
            if (feas_cum) *feas_cum = fe;
            return;
        }
        ++m->slot_fallbacks;
        HCK(hipMemcpyAsync(m->hb, mads_best_ptr(m), 16, hipMemcpyDeviceToHost, m->s));
    }
    HCK(hipStreamSynchronize(m->s));
    *obj = m->hb[0];
    *idx = __builtin_bit_cast(int64_t, m->hb[1]);
    if (feas_cum) {
        unsigned long long fe = 0;
        HCK(hipMemcpy(&fe, m->d_feas.p, sizeof(fe), hipMemcpyDeviceToHost));
        *feas_cum = fe;
    }
}

static void mads_free(mac_mads* m)
{
    if (!m) return;
    if (m->L) release_lane(m->ctx, m->L, m->s);
    delete m;
}

int32_t mac_mads_begin(mac_ctx* ctx, const double* x0, int64_t three_n, const double* r_max,
                       double penalty, const double* prev, const double* d_lim, double tan_half_fov,
                       const mac_mads_params* prm, int64_t shard_lo, int64_t shard_hi,
                       mac_mads** out)
{
    ABI_BEGIN
    if (!out) return fail(MAC_E_INVAL, "null out");
    *out = nullptr;
    int32_t rc = check_common(ctx, three_n, 1);
    if (rc) return rc;
    if (!x0 || !r_max || !prm) return fail(MAC_E_INVAL, "null argument");
    if (prev && !d_lim) return fail(MAC_E_INVAL, "prev given without d_lim");
    if (prm->ell0 < 0 || prm->ell_max < prm->ell0 || prm->ell_max > 52)
        return fail(MAC_E_INVAL, "need 0 <= ell0 <= ell_max <= 52");
    const int N = (int)(three_n / 3);
    if (N == 0) return fail(MAC_E_INVAL, "no UAV");
    const int n = (int)three_n, K = 2 * n;
    if (shard_lo < 0 || shard_hi > K || shard_lo > shard_hi)
        return fail(MAC_E_INVAL, "shard outside [0, 2n)");
    set_device(ctx);
    mac_mads* m = new mac_mads();
    m->t0 = std::chrono::steady_clock::now();
    m->ctx = ctx;
    try {
        m->L = acquire_lane(ctx, nullptr);
        m->s = m->L->stream;
        Lane* L = m->L;
        hipStream_t s = m->s;
        m->N = N;
        m->n = n;
        m->K = K;
        m->lo = shard_lo;
        m->hi = shard_hi;
        m->prm = *prm;
        m->penalty = penalty;
        m->tan_half_fov = tan_half_fov;
        L->cands.reserve(sizeof(double) * three_n);
        L->xinc.reserve(sizeof(double) * three_n);
        L->perm.reserve(sizeof(int) * 2 * n);
        L->area.reserve(sizeof(double) * K);
        L->obj.reserve(sizeof(double) * K);
        L->best.reserve(16);
        L->rmax.reserve(sizeof(double) * N);
        HCK(hipMemcpyAsync(L->rmax.p, r_max, sizeof(double) * N, hipMemcpyHostToDevice, s));
        m->d_feas.reserve(sizeof(unsigned long long));
        HCK(hipMemsetAsync(m->d_feas.p, 0, sizeof(unsigned long long), s));
        if (prev) {
            m->h_prev.assign(prev, prev + three_n);
            L->prev.reserve(sizeof(double) * three_n);
            L->dlim.reserve(sizeof(double) * N);
            L->dlimraw.reserve(sizeof(double) * N);
            L->h_dlim.resize(N);
            for (int i = 0; i < N; ++i) L->h_dlim[i] = dlim_threshold(d_lim[i]);
            HCK(hipMemcpyAsync(L->prev.p, prev, sizeof(double) * three_n, hipMemcpyHostToDevice, s));
            HCK(hipMemcpyAsync(L->dlim.p, L->h_dlim.data(), sizeof(double) * N,
                               hipMemcpyHostToDevice, s));
            HCK(hipMemcpyAsync(L->dlimraw.p, d_lim, sizeof(double) * N, hipMemcpyHostToDevice, s));
            m->d_prev = L->prev.as<double>();
            m->d_dlimT = L->dlim.as<double>();
        }
        m->x.assign(x0, x0 + three_n);
        // pinned staging: [best 16 B][incumbent 8*3N][permutations 4*2n]
        L->h_stage.reserve(16 + sizeof(double) * three_n + sizeof(int) * 2 * n);
        m->hb = (double*)L->h_stage.p;
        m->hx = m->hb + 2;
        m->hperm = (int*)(m->hx + three_n);
        // f(x0): the objective, +inf when x0 itself violates cons3 (every rank evaluates it)
        std::copy(m->x.begin(), m->x.end(), m->hx);
        HCK(hipMemcpyAsync(L->cands.p, m->hx, sizeof(double) * three_n, hipMemcpyHostToDevice, s));
        mads_best_of(m, matrix_src(L->cands.as<double>(), N), 1, 0);
        HCK(hipStreamSynchronize(s));
        m->f = __builtin_bit_cast(int64_t, m->hb[1]) >= 0 ? m->hb[0] : INFINITY;
        m->evals = 1;
        m->ell = prm->ell0;
        // the run's chain, from its first poll: x0 at mesh step 2^ell0 (the incumbent moves by a few
        // steps over a run; crowding is a property of the UAVs' layout)
        m->route_five = host_crowded_disks(x0, N, std::ldexp(1.0, prm->ell0), ctx->grid.S) > kBitsMinDisks ? 1 : 0;
        m->state = prm->seed;
        m->T = (uint64_t)n * (uint64_t)(n - 1) / 2;
        m->per_iter = (uint64_t)n + m->T + 2 * (uint64_t)n;   // ltmads_basis's draws
        // the permutations do not depend on the poll outcomes: the next iteration's are
        // computed on the host while the device evaluates the current poll
        stream_permutation(m->state, (uint64_t)n + m->T + 1, n, m->rp_next);
        stream_permutation(m->state, (uint64_t)n + m->T + n + 1, n, m->cp_next);
    } catch (...) {
        mads_free(m);
        throw;
    }
    *out = m;
    return MAC_OK;
    ABI_END
}

int32_t mac_mads_poll(mac_mads* m, int32_t* done, double* best_obj, int64_t* best_idx)
{
    ABI_BEGIN
    if (!m || !done || !best_obj || !best_idx) return fail(MAC_E_INVAL, "null argument");
    if (m->polled_b) return fail(MAC_E_INVAL, "mac_mads_poll twice without mac_mads_update");
    *done = 0;
    if (m->it >= m->prm.n_iter || m->ell < 0) {
        *done = 1;
        return MAC_OK;
    }
    set_device(m->ctx);
    using clk = std::chrono::steady_clock;
    const auto ta = clk::now();
    ++m->it;
    const int n = m->n;
    const int64_t b = (int64_t)1 << m->ell;
    m->rp.swap(m->rp_next);
    m->cp.swap(m->cp_next);
    const int Kc = (int)(m->hi - m->lo);
    // a poll cons3 rejects whole: no launch, its result (+inf, -1) (every rank decides alike)
    const bool rejected = Kc > 0 && poll_rejected(m, b);
    if (rejected) {
        ++m->rejected;
        if (m->ext_best) {   // the buffer holds this poll's best once the call returns
            m->hb[0] = INFINITY;
            m->hb[1] = __builtin_bit_cast(double, (int64_t)-1);
            HCK(hipMemcpyAsync(m->ext_best, m->hb, 16, hipMemcpyHostToDevice, m->s));
            HCK(hipStreamSynchronize(m->s));
        }
    }
    if (Kc > 0 && !rejected) {
        // (the staging is free: the previous iteration's copies completed at its sync)
        // one copy of the contiguous staging [incumbent 8n][permutations 4*2n] (n = 3N); the
        // staging is free: the previous poll's copy preceded its finalize, whose results were read
        std::copy(m->rp.begin(), m->rp.end(), m->hperm);
        std::copy(m->cp.begin(), m->cp.end(), m->hperm + n);
        std::copy(m->x.begin(), m->x.end(), m->hx);
        m->L->xinc.reserve(sizeof(double) * n + sizeof(int) * 2 * n);
        HCK(hipMemcpyAsync(m->L->xinc.p, m->hx, sizeof(double) * n + sizeof(int) * 2 * n,
                           hipMemcpyHostToDevice, m->s));
        CandSrc src{};
        src.xinc = m->L->xinc.as<double>();
        src.rp = reinterpret_cast<int*>(m->L->xinc.as<double>() + n);
        src.cp = src.rp + n;
        src.state = m->state;
        src.b = b;
        src.k0 = (int)m->lo;
        src.route_five = m->route_five;
        mads_best_of(m, src, Kc, m->lo, true);
    }
    const auto tb = clk::now();
    if (m->it < m->prm.n_iter) {
        const uint64_t ns = m->state + m->per_iter * 0x9E3779B97F4A7C15ull;
        stream_permutation(ns, (uint64_t)n + m->T + 1, n, m->rp_next);
        stream_permutation(ns, (uint64_t)n + m->T + n + 1, n, m->cp_next);
    }
    const auto tc = clk::now();
    if (Kc > 0 && !rejected) {
        mads_wait_best(m, best_obj, best_idx);
    } else {
        *best_obj = INFINITY;
        *best_idx = -1;
    }
    const auto td = clk::now();
    m->polled_b = b;
    m->h_enq += std::chrono::duration<double>(tb - ta).count();
    m->h_perm += std::chrono::duration<double>(tc - tb).count();
    m->h_wait += std::chrono::duration<double>(td - tc).count();
    return MAC_OK;
    ABI_END
}

int32_t mac_mads_update(mac_mads* m, double best_obj, int64_t best_idx)
{
    ABI_BEGIN
    if (!m) return fail(MAC_E_INVAL, "null stepper");
    if (!m->polled_b) return fail(MAC_E_INVAL, "mac_mads_update without a poll");
    if (best_idx >= m->K) return fail(MAC_E_INVAL, "best index outside the poll");
    const auto te0 = std::chrono::steady_clock::now();
    const int n = m->n;
    const int64_t b = m->polled_b;
    m->polled_b = 0;
    m->evals += m->K;
    if (best_idx >= 0 && best_obj < m->f) {
        const int kk = best_idx < n ? (int)best_idx : (int)best_idx - n;
        for (int v = 0; v < n; ++v) {
            const double d = ltmads_entry(m->state, n, b, m->rp[v], m->cp[kk]);
            m->x[v] = best_idx < n ? m->x[v] + d : m->x[v] - d;
        }
        m->f = best_obj;
        m->ell = std::min(m->ell + 1, (int)m->prm.ell_max);
        ++m->succ;
    } else {
        --m->ell;
    }
    m->state += m->per_iter * 0x9E3779B97F4A7C15ull;
    m->h_post += std::chrono::duration<double>(std::chrono::steady_clock::now() - te0).count();
    return MAC_OK;
    ABI_END
}

// Speculation over failure branches (the sharded loop's other mode, dist.mads_loop speculate):
// a failed iteration's next poll is fully determined — the same incumbent, ell - 1 and the next
// stream position — so rank j can evaluate, beside rank 0's real poll, the poll that follows j
// consecutive failures. mac_mads_poll_ahead evaluates it (the whole poll, this stepper's shard)
// without advancing the stepper; mac_mads_advance then applies the gathered results in order, one
// iteration each, up to the first success. Same iterates as the sequential loop.
int32_t mac_mads_poll_ahead(mac_mads* m, int32_t ahead, int32_t* done, double* best_obj, int64_t* best_idx,
                            int64_t* feasible)
{
    ABI_BEGIN
    if (!m || !done || !best_obj || !best_idx) return fail(MAC_E_INVAL, "null argument");
    if (feasible) *feasible = 0;
    if (ahead < 0) return fail(MAC_E_INVAL, "negative ahead");
    if (m->polled_b) return fail(MAC_E_INVAL, "mac_mads_poll_ahead with a mac_mads_poll pending");
    *done = 0;
    *best_obj = INFINITY;
    *best_idx = -1;
    if (m->it + ahead >= m->prm.n_iter || m->ell - ahead < 0) {
        *done = 1;
        return MAC_OK;
    }
    set_device(m->ctx);
    const int n = m->n;
    const int ell = m->ell - ahead;
    const int64_t b = (int64_t)1 << ell;
    const uint64_t state = m->state + (uint64_t)ahead * m->per_iter * 0x9E3779B97F4A7C15ull;
    const int Kc = (int)(m->hi - m->lo);
    if (Kc == 0) return MAC_OK;
    if (poll_rejected(m, b)) return MAC_OK;   // (counted by mac_mads_advance once applied)
    if (ahead == 0) {   // the current iteration's permutations are computed already
        std::copy(m->rp_next.begin(), m->rp_next.end(), m->hperm);
        std::copy(m->cp_next.begin(), m->cp_next.end(), m->hperm + n);
    } else {
        std::vector<int> rp, cp;
        stream_permutation(state, (uint64_t)n + m->T + 1, n, rp);
        stream_permutation(state, (uint64_t)n + m->T + n + 1, n, cp);
        std::copy(rp.begin(), rp.end(), m->hperm);
        std::copy(cp.begin(), cp.end(), m->hperm + n);
    }
    std::copy(m->x.begin(), m->x.end(), m->hx);
    m->L->xinc.reserve(sizeof(double) * n + sizeof(int) * 2 * n);
    HCK(hipMemcpyAsync(m->L->xinc.p, m->hx, sizeof(double) * n + sizeof(int) * 2 * n,
                       hipMemcpyHostToDevice, m->s));
    CandSrc src{};
    src.xinc = m->L->xinc.as<double>();
    src.rp = reinterpret_cast<int*>(m->L->xinc.as<double>() + n);
    src.cp = src.rp + n;
    src.state = state;
    src.b = b;
    src.k0 = (int)m->lo;
    src.route_five = m->route_five;
    mads_best_of(m, src, Kc, m->lo, true);
    uint64_t fe = 0;
    mads_wait_best(m, best_obj, best_idx, &fe);
    if (feasible) *feasible = (int64_t)(fe - m->feas_seen);
    m->feas_seen = fe;
    return MAC_OK;
    ABI_END
}

int32_t mac_mads_advance(mac_mads* m, double best_obj, int64_t best_idx, int32_t* moved)
{
    ABI_BEGIN
    if (!m) return fail(MAC_E_INVAL, "null stepper");
    if (m->polled_b) return fail(MAC_E_INVAL, "mac_mads_advance with a mac_mads_poll pending (use mac_mads_update)");
    if (best_idx >= m->K) return fail(MAC_E_INVAL, "best index outside the poll");
    if (m->it >= m->prm.n_iter || m->ell < 0) return fail(MAC_E_INVAL, "mac_mads_advance past the loop's end");
    const int n = m->n;
    const int64_t b = (int64_t)1 << m->ell;
    // the applied poll's whole-poll rejection, decided as mac_mads_poll does (the speculating ranks'
    // own polls ahead are not counted: they may never be applied)
    if (m->hi > m->lo && poll_rejected(m, b)) ++m->rejected;
    ++m->it;
    m->evals += m->K;
    const bool better = best_idx >= 0 && best_obj < m->f;
    if (better) {   // the current iteration's permutations (rp_next / cp_next)
        const int kk = best_idx < n ? (int)best_idx : (int)best_idx - n;
        for (int v = 0; v < n; ++v) {
            const double d = ltmads_entry(m->state, n, b, m->rp_next[v], m->cp_next[kk]);
            m->x[v] = best_idx < n ? m->x[v] + d : m->x[v] - d;
        }
        m->f = best_obj;
        m->ell = std::min(m->ell + 1, (int)m->prm.ell_max);
        ++m->succ;
    } else {
        --m->ell;
    }
    m->state += m->per_iter * 0x9E3779B97F4A7C15ull;
    if (m->it < m->prm.n_iter) {
        stream_permutation(m->state, (uint64_t)n + m->T + 1, n, m->rp_next);
        stream_permutation(m->state, (uint64_t)n + m->T + n + 1, n, m->cp_next);
    }
    if (moved) *moved = better ? 1 : 0;
    return MAC_OK;
    ABI_END
}

int32_t mac_mads_result(mac_mads* m, double* x_out, mac_mads_stats* st)
{
    ABI_BEGIN
    if (!m) return fail(MAC_E_INVAL, "null stepper");
    if (x_out) std::copy(m->x.begin(), m->x.end(), x_out);
    if (st) {
        st->f = m->f;
        st->iterations = m->it;
        st->evaluations = m->evals;
        st->status = m->ell < 0 ? 0 : 1;
        st->feasible = std::isfinite(m->f) ? 1 : 0;
        st->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - m->t0).count();
        st->host_enqueue_s = m->h_enq;
        st->host_perm_s = m->h_perm;
        st->wait_s = m->h_wait;
        st->host_post_s = m->h_post;
        unsigned long long fe = 0;
        set_device(m->ctx);
        HCK(hipMemcpyAsync(&fe, m->d_feas.p, sizeof(fe), hipMemcpyDeviceToHost, m->s));
        HCK(hipStreamSynchronize(m->s));
        st->feasible_evaluations = (int64_t)fe;
        st->rejected_polls = m->rejected;
        st->successes = m->succ;
        st->slot_fallbacks = m->slot_fallbacks;
    }
    return MAC_OK;
    ABI_END
}

int32_t mac_mads_best_buffer(mac_mads* m, void* d_best16)
{
    if (!m) return fail(MAC_E_INVAL, "null stepper");
    ABI_BEGIN
    if (((uintptr_t)d_best16 & 7) != 0) return fail(MAC_E_INVAL, "d_best16 not 8-byte aligned");
    m->ext_best = (double*)d_best16;
    if (d_best16 && m->hi == m->lo) {   // an empty shard never polls: it offers {+inf, -1}
        set_device(m->ctx);
        const double none[2] = {INFINITY, __builtin_bit_cast(double, (int64_t)-1)};
        HCK(hipMemcpy(d_best16, none, 16, hipMemcpyHostToDevice));
    }
    return MAC_OK;
    ABI_END
}

void mac_mads_destroy(mac_mads* m)
{
    if (!m) return;
    (void)hipSetDevice(m->ctx->device);
    (void)hipStreamSynchronize(m->s);
    mads_free(m);
}

// ------------------------------------------------------------------ pipelined MADS loop
// mac_mads_run on one GPU when the poll walk runs: every poll's finalize applies the poll's update on
// the device (k_final.h mads_step) and the next poll's launches read the mesh index from the device
// state (k_prep.h MadsState), so the host enqueues poll t + kMadsWindow - 1 while poll t runs and
// waits only to bound that window (on the mapped slot's seq word). The permutations do not depend
// on the outcomes: computed kMadsAhead iterations ahead into a pinned ring and uploaded kMadsChunk
// iterations per copy. Same incumbents, objective and counts as the stepper loop, bit for bit (the
// same arithmetic, only where it runs differs): tests/test_gpu_parity.py
// test_native_mads_pipelined_matches_stepper.
static constexpr int kMadsWindow = 3;   // polls in flight
static constexpr int kMadsAhead = 16;   // permutations computed ahead of the enqueued poll
static constexpr int kMadsChunk = 8;    // iterations per permutation upload
static constexpr int kMadsRing = 32;    // permutation slots (device and pinned)
static constexpr uint64_t kMadsDoneSeq = 1ull << 62;   // seq word of a stopped loop

static bool mads_pipelinable(const mac_mads* m)
{
    return m->lo == 0 && m->hi == m->K && !m->ext_best && m->prm.n_iter > 0 &&
           poll_walk_possible(m->ctx, m->N, m->K, use_tiled(m->ctx, m->N, nullptr, m->n));
}

static void mads_run_pipelined(mac_mads* m)
{
    using clk = std::chrono::steady_clock;
    const int n = m->n;
    const int64_t n_iter = m->prm.n_iter;
    const size_t slot_ints = 2 * (size_t)n;
    hipStream_t s = m->s;
    mads_make_slot(m);
    m->d_x.reserve(sizeof(double) * 2 * n);
    m->d_st.reserve(sizeof(MadsState));
    m->d_ring.reserve(sizeof(int) * slot_ints * kMadsRing);
    m->h_ring.reserve(sizeof(int) * slot_ints * kMadsRing);
    double* dx = m->d_x.as<double>();
    MadsState* dst = m->d_st.as<MadsState>();
    int* dring = m->d_ring.as<int>();
    int* hring = (int*)m->h_ring.p;
    const uint64_t step = m->per_iter * 0x9E3779B97F4A7C15ull;
    const uint64_t seed_state = m->state;   // iteration t's stream state: seed + (t - 1) * step
    auto state_of = [&](int64_t t) { return seed_state + (uint64_t)(t - 1) * step; };
    auto perms_of = [&](int64_t t) {   // into the pinned ring
        int* h = hring + (size_t)((t - 1) % kMadsRing) * slot_ints;
        stream_permutation(state_of(t), (uint64_t)n + m->T + 1, n, m->rp_next);
        stream_permutation(state_of(t), (uint64_t)n + m->T + n + 1, n, m->cp_next);
        std::memcpy(h, m->rp_next.data(), sizeof(int) * n);
        std::memcpy(h + n, m->cp_next.data(), sizeof(int) * n);
    };
    int64_t uploaded = 0;   // iterations [1, uploaded] on the device
    auto upload_to = [&](int64_t t1) {   // [uploaded + 1, t1]: contiguous slots (chunk aligned)
        const int64_t t0 = uploaded + 1;
        if (t1 < t0) return;
        const size_t q0 = (size_t)((t0 - 1) % kMadsRing);
        HCK(hipMemcpyAsync(dring + q0 * slot_ints, hring + q0 * slot_ints,
                           sizeof(int) * slot_ints * (size_t)(t1 - t0 + 1), hipMemcpyHostToDevice, s));
        uploaded = t1;
    };
    // the incumbent and the state: x0 (begin's pinned staging holds it), f(x0), ell0
    const auto ta = clk::now();
    HCK(hipMemcpyAsync(dx, m->hx, sizeof(double) * n, hipMemcpyHostToDevice, s));
    const MadsState st0{m->f, 0, m->ell, 0, 0ull, 0, 0};
    HCK(hipMemcpy(dst, &st0, sizeof(st0), hipMemcpyHostToDevice));
    int64_t computed = std::min<int64_t>(n_iter, kMadsAhead);
    for (int64_t t = 1; t <= computed; ++t) perms_of(t);
    for (int64_t t = kMadsChunk; t <= computed; t += kMadsChunk) upload_to(t);
    upload_to(computed);
    m->h_perm += std::chrono::duration<double>(clk::now() - ta).count();

    const volatile uint64_t* seqw = (const volatile uint64_t*)m->hslot.p + 2;
    bool stopped = false;
    for (int64_t t = 1; t <= n_iter && !stopped; ++t) {
        const auto t1 = clk::now();
        if (t > kMadsWindow) {   // poll t - kMadsWindow finished (or the loop stopped)
            const uint64_t want = (uint64_t)(t - kMadsWindow);
            for (int spin = 0; *seqw < want; ++spin) {
                if ((spin & 1023) == 1023 &&
                    std::chrono::duration<double, std::milli>(clk::now() - t1).count() > 50.0) {
                    HCK(hipStreamSynchronize(s));   // a failed launch surfaces here
                    if (*seqw < want) throw HipError{hipErrorUnknown, "pipelined MADS poll lost", __LINE__};
                }
            }
            stopped = *seqw >= kMadsDoneSeq;
            if (stopped) break;
        }
        const auto t2 = clk::now();
        const int* rp = dring + (size_t)((t - 1) % kMadsRing) * slot_ints;
        CandSrc src{};
        src.xinc = dx + (size_t)((t - 1) & 1) * n;
        src.rp = rp;
        src.cp = rp + n;
        src.state = state_of(t);
        src.b = 0;   // from the device state
        src.k0 = 0;
        src.mst = dst;
        src.route_five = m->route_five;
        FinBest fbm{};
        fbm.st = dst;
        fbm.x = src.xinc;
        fbm.x_next = dx + (size_t)(t & 1) * n;
        fbm.rp = src.rp;
        fbm.cp = src.cp;
        fbm.state = src.state;
        fbm.n = n;
        fbm.ell_max = (int)m->prm.ell_max;
        fbm.done_seq = kMadsDoneSeq;
        enqueue_eval(m->ctx, m->L, s, src, m->N, m->K, true, m->L->rmax.as<double>(), m->penalty,
                     m->d_prev, m->d_dlimT, m->d_prev ? m->L->dlimraw.as<double>() : nullptr,
                     m->tan_half_fov, nullptr, m->L->obj.as<double>(),
                     m->L->best.as<double>(), 0, m->d_slot, (uint64_t)t, &fbm, &dst->feas);
        const auto t3 = clk::now();
        if (computed < n_iter) {   // one iteration's permutations per poll, uploaded per chunk
            perms_of(++computed);
            if (computed % kMadsChunk == 0 || computed == n_iter) upload_to(computed);
        }
        const auto t4 = clk::now();
        m->h_wait += std::chrono::duration<double>(t2 - t1).count();
        m->h_enq += std::chrono::duration<double>(t3 - t2).count();
        m->h_perm += std::chrono::duration<double>(t4 - t3).count();
    }
    const auto t5 = clk::now();
    HCK(hipStreamSynchronize(s));
    MadsState st{};
    HCK(hipMemcpy(&st, dst, sizeof(st), hipMemcpyDeviceToHost));
    HCK(hipMemcpy(m->x.data(), dx + (size_t)(st.it & 1) * n, sizeof(double) * n, hipMemcpyDeviceToHost));
    m->f = st.f;
    m->it = st.it;
    m->ell = st.ell;
    m->evals = 1 + st.it * (int64_t)m->K;
    m->rejected += st.skipped;
    m->succ += st.succ;
    if (st.feas) {   // (the stepper's counter holds the polls' evaluations: none before this loop)
        const unsigned long long fe = st.feas;
        HCK(hipMemcpy(m->d_feas.p, &fe, sizeof(fe), hipMemcpyHostToDevice));
    }
    m->state = state_of(st.it + 1);
    m->h_wait += std::chrono::duration<double>(clk::now() - t5).count();
}

int32_t mac_mads_run(mac_ctx* ctx, const double* x0, int64_t three_n, const double* r_max,
                     double penalty, const double* prev, const double* d_lim, double tan_half_fov,
                     const mac_mads_params* prm, double* x_out, mac_mads_stats* st)
{
    ABI_BEGIN
    if (!x_out) return fail(MAC_E_INVAL, "null argument");
    mac_mads* m = nullptr;
    int32_t rc = mac_mads_begin(ctx, x0, three_n, r_max, penalty, prev, d_lim, tan_half_fov, prm,
                                0, 2 * three_n, &m);
    if (rc) return rc;
    if (mads_pipelinable(m)) {
        try {
            set_device(ctx);
            mads_run_pipelined(m);
        } catch (...) {
            mac_mads_destroy(m);
            throw;
        }
    } else {
        for (;;) {
            int32_t done = 0;
            double bo = 0.0;
            int64_t bi = -1;
            rc = mac_mads_poll(m, &done, &bo, &bi);
            if (rc || done) break;
            rc = mac_mads_update(m, bo, bi);
            if (rc) break;
        }
    }
    if (!rc) rc = mac_mads_result(m, x_out, st);
    mac_mads_destroy(m);
    return rc;
    ABI_END
}

// The single-candidate closure (k_closure.h): the candidates written by the host straight into the
// lane's fine-grained device buffer through the BAR (a large-BAR device; else pinned staging and a
// copy), one kernel (grid.y = the batch), each area from its own mapped slot (no copy either way,
// no stream synchronisation). AUTO / TILED walks, N <= kClosureMaxN; if a slot has not landed within 2 ms (a
// failed launch) a stream synchronisation reports it.
static constexpr int kClBatch = 64;   // concurrent mac_area_f64 calls evaluated by one launch
// slot reads spun with a pause before a reader starts yielding its CPU (MAXCOVER_CL_READSPIN overrides)
static const int kClReadSpin = [] {
    const char* e = std::getenv("MAXCOVER_CL_READSPIN");
    return e ? std::max(0, std::atoi(e)) : 64;
}();

static bool closure_path(const mac_ctx* ctx, int64_t three_n)
{
    return (ctx->algo == MAC_ALGO_AUTO || ctx->algo == MAC_ALGO_TILED) && three_n / 3 <= kClosureMaxN;
}

static const bool kClStats = [] {
    const char* e = std::getenv("MAXCOVER_CL_STATS");
    return e && *e == '1';
}();static void cl_add(std::atomic<int64_t>& a, std::chrono::steady_clock::duration d)
{
    a.fetch_add(std::chrono::duration_cast<std::chrono::nanoseconds>(d).count(), std::memory_order_relaxed);
}

// A launched batch of closure candidates: its lane (stream, staging, result slots) stays with the
// batch until every one of its callers has read its slot (the last returns the lane to the pool),
// so a later batch can neither overwrite a slot nor the staging before they are consumed.
struct ClBatch {
    Lane* L = nullptr;
    uint64_t seq = 0;
    std::atomic<int> readers{0};
};

// Write the B candidates into the lane's device buffer (through the BAR, or pinned staging and a
// copy) and launch one closure_kernel (grid.y = B) whose candidate b writes its area into the lane's mapped slot b under `seq`. Returns
// after enqueueing: the launching caller does not wait for the results.
static uint64_t closure_launch(mac_ctx* ctx, Lane* L, int64_t three_n, const double* const* cands, int B)
{
    const int N = (int)(three_n / 3);
    hipStream_t s = L->stream;
    const size_t one = sizeof(double) * (size_t)three_n;
    const auto t0 = std::chrono::steady_clock::now();
    const double* dc;
    bool bar = ctx->cl_bar.load(std::memory_order_relaxed);
    if (bar) {
        try {
            L->clv.reserve(one * kClBatch, true);
        } catch (const HipError&) {   // no fine-grained device memory to spare: the copy path from now on
            (void)hipGetLastError();
            ctx->cl_bar.store(false, std::memory_order_relaxed);
            bar = false;
        }
    }
    if (bar) {   // straight into device memory through the BAR; the fence drains the
                 // write-combining buffers before the launch's doorbell
        for (int b = 0; b < B; ++b) std::memcpy((char*)L->clv.p + one * b, cands[b], one);
        _mm_sfence();
        dc = L->clv.as<double>();
    } else {
        L->h_io.reserve(std::max<size_t>(one * B, 64));
        for (int b = 0; b < B; ++b) std::memcpy((char*)L->h_io.p + one * b, cands[b], one);
        L->cands.reserve(one * B);
        dc = L->cands.as<double>();
    }
    const auto t1 = std::chrono::steady_clock::now();
    L->area.reserve(sizeof(double) * B);
    L->cpart.reserve(sizeof(unsigned long long) * (size_t)N * B);
    // zero once; the last block of each candidate resets its words
    if (L->carrive.grow(sizeof(unsigned) * kClBatch)) HCK(hipMemsetAsync(L->carrive.p, 0, L->carrive.cap, s));
    if (L->ctot.grow(sizeof(uint64_t) * kClBatch)) HCK(hipMemsetAsync(L->ctot.p, 0, L->ctot.cap, s));
    if (!L->h_cl.p) {   // a 32-B slot per batch candidate
        L->h_cl.reserve(32 * kClBatch, hipHostMallocMapped | hipHostMallocCoherent);
        std::memset(L->h_cl.p, 0, 32 * kClBatch);
        void* dp = nullptr;
        HCK(hipHostGetDevicePointer(&dp, L->h_cl.p, 0));
        L->d_cl = (uint64_t*)dp;
    }
    const uint64_t seq = ++L->cl_seq;
    if (!bar) HCK(hipMemcpyAsync(L->cands.p, L->h_io.p, one * B, hipMemcpyHostToDevice, s));
    const int nwg = (N + kClosureDisksPerWG - 1) / kClosureDisksPerWG;   // a wave per disk
    int64_t ts_a = -1;
    uint64_t* ts = nullptr;
    if (ctx->profile) {
        std::lock_guard<std::mutex> lk(ctx->mu);
        if (ctx->stamp_used + (int64_t)nwg * B <= ctx->stamp_cap) {
            ts_a = ctx->stamp_used;
            ctx->stamp_used += (int64_t)nwg * B;
            ts = ctx->stamps.as<uint64_t>() + 2 * ts_a;
        }
    }
    const ClosureOut co{L->cpart.as<unsigned long long>(), L->ctot.as<unsigned long long>(),
                        L->carrive.as<unsigned>(), L->area.as<double>(), L->d_cl, seq};
    hipLaunchKernelGGL(closure_kernel, dim3((unsigned)nwg, (unsigned)B), dim3(kBlock),
                       (uint32_t)closure_lds_bytes(N), s, ts, dc, N, ctx->grid,
                       ctx->xys.as<double2>(), ctx->ws.as<double>(), ctx->off.as<int32_t>(),
                       ctx->w_uniform ? 1 : 0, ctx->w0, co);
    HCK(hipGetLastError());
    if (ts) {
        std::lock_guard<std::mutex> lk(ctx->mu);
        ctx->prof.push_back({ts_a, (int64_t)nwg * B, -1, 0, (int64_t)B, nullptr, MAC_ALGO_TILED});
    }
    if (kClStats) {
        const auto t2 = std::chrono::steady_clock::now();
        cl_add(ctx->cl_phase_ns[0], t1 - t0);
        cl_add(ctx->cl_phase_ns[1], t2 - t1);
    }
    return seq;
}

// Candidate b's area of a launched batch, from its mapped slot (spinning with pauses: the other
// callers' threads lead batches meanwhile); after 2 ms (a failed launch) the lane's stream is
// synchronised, which reports the error, then the slot or the device word is read.
static double closure_read(mac_ctx* ctx, ClBatch* bt, int b)
{
    const uint64_t* slot = (const uint64_t*)bt->L->h_cl.p + 4 * b;
    double a = 0.0;
    int64_t unused = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (int spin = 0;; ++spin) {
        if (mirror_read(slot, bt->seq, &a, &unused)) return a;
        // past a short spin, yield the CPU between reads: under many concurrent callers the
        // threads launching the next batches need it more than the spinning readers (the call's
        // HIP enqueue time doubles when every CPU of the share spins)
        if (spin < kClReadSpin) __builtin_ia32_pause();
        else sched_yield();
        if ((spin & 255) == 255 &&
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() > 2.0)
            break;
    }
    set_device(ctx);
    HCK(hipStreamSynchronize(bt->L->stream));
    if (!mirror_read(slot, bt->seq, &a, &unused))
        HCK(hipMemcpy(&a, bt->L->area.as<double>() + b, sizeof(double), hipMemcpyDeviceToHost));
    return a;
}

// One caller is done with the batch; the last returns the lane (its stream holds nothing unread:
// every slot has landed, so the kernel that wrote them is ending, and later work on the stream is
// ordered after it).
static void closure_done(mac_ctx* ctx, ClBatch* bt)
{
    if (bt->readers.fetch_sub(1, std::memory_order_acq_rel) != 1) return;
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        bt->L->last = bt->L->stream;
        ctx->lanes_free.push_back(bt->L);
    }
    delete bt;
}

// Concurrent callers (DirectSearch's threaded poll, src/TDM_STATIC_opt.jl:129: one objective call
// per trial point per thread) are combined: a caller queues its request; while fewer than
// kClLeaders batches are being launched, a caller whose request is still queued takes every queued
// request of the same size (up to kClBatch), launches them as one batch on a lane of its own and
// goes back to waiting for its own result like every other caller: no thread waits for a batch's
// results but the threads whose requests it holds, each on its own mapped slot, so the next batch
// can be formed and launched while earlier ones run (round 5's leaders waited for their whole batch
// before another could start). A lone caller launches its own request at once. Results per call are
// exactly the single-candidate kernel's (the batch dimension only selects the candidate).
#ifndef MAC_CL_LEADERS
#define MAC_CL_LEADERS 2
#endif
// batches being launched at once (MAXCOVER_CL_LEADERS overrides, for measurements)
static const int kClLeaders = [] {
    const char* e = std::getenv("MAXCOVER_CL_LEADERS");
    const int v = e ? std::atoi(e) : 0;
    return v >= 1 && v <= 16 ? v : MAC_CL_LEADERS;
}();
// pause iterations before a waiter sleeps on its futex (MAXCOVER_CL_SPIN overrides, for measurements)
static const int kClSpin = [] {
    const char* e = std::getenv("MAXCOVER_CL_SPIN");
    return e ? std::max(0, std::atoi(e)) : 64;
}();

static constexpr int kClGather = 0;        // pauses a would-be leader waits for every caller to queue (0: none)
// batches one thread launches in a row while requests are queued (MAXCOVER_CL_LEAD overrides): the
// launching thread is awake on a CPU, a queued caller woken to lead instead takes tens of
// microseconds to run; the cap bounds how long the leader's own call waits behind others' batches
static const int kClLead = [] {
    const char* e = std::getenv("MAXCOVER_CL_LEAD");
    const int v = e ? std::atoi(e) : 0;
    return v >= 1 ? v : 16;
}();

// Waiting while queued: a short spin, then a futex sleep (no CPU taken from the threads that lead
// batches) on the word of the request's generation, or 1 ms. A leader that launches generation g's
// batch bumps g's word and wakes ONE sleeper (a futex wake costs the waker microseconds per thread;
// the launching thread is the combiner's bottleneck); a thread woken with its request launched
// passes the wake on to the rest of its generation. A leader that frees a launch slot with requests
// still queued wakes one of them to lead.
static std::atomic<int>& cl_word(mac_ctx* ctx, uint32_t gen) { return ctx->cl_genw[gen & 63]; }

static void cl_wake(std::atomic<int>& w, int n)
{
    w.fetch_add(1, std::memory_order_seq_cst);
    syscall(SYS_futex, reinterpret_cast<int*>(&w), FUTEX_WAKE_PRIVATE, n, nullptr, nullptr, 0);
}

struct ClReq {
    const double* c;
    int64_t three_n;
    double* out;
    std::atomic<int> state{0};   // 0 queued, 1 taken by a batch, 2 failed, 3 launched (read the slot)
    std::atomic<int> released{0};   // 1 once the leader no longer touches the request (after its
                                    // futex wake): the owner's stack object may then go
    uint32_t gen = 0;            // the generation whose futex word this request sleeps on (cl_mu)
    std::chrono::steady_clock::time_point t_taken, t_handed;   // (MAXCOVER_CL_STATS=1)
    ClBatch* bt = nullptr;       // (state 3) the batch and this request's slot in it
    int b = 0;
    int32_t rc = MAC_OK;
    std::string err;
};

static void cl_wait(mac_ctx* ctx, ClReq& r, int spin)
{
    if (spin < kClSpin) {
        __builtin_ia32_pause();
        return;
    }
    uint32_t g = r.gen;   // (written by this thread only)
    if (r.state.load(std::memory_order_relaxed) == 0 && g != ctx->cl_gen.load(std::memory_order_relaxed)) {
        // still queued past an earlier take (a batch of another size): join the current generation
        std::lock_guard<std::mutex> lk(ctx->cl_mu);
        if (r.state.load(std::memory_order_relaxed) == 0) r.gen = ctx->cl_gen.load(std::memory_order_relaxed);
        g = r.gen;
    }
    std::atomic<int>& w = cl_word(ctx, g);
    const int v = w.load(std::memory_order_seq_cst);
    const int st = r.state.load(std::memory_order_seq_cst);
    if (st == 2 || st == 3) return;
    struct timespec ts{0, 1000000};
    syscall(SYS_futex, reinterpret_cast<int*>(&w), FUTEX_WAIT_PRIVATE, v, &ts, nullptr, 0);
    const int now = r.state.load(std::memory_order_acquire);
    if (now == 2 || now == 3) cl_wake(w, INT_MAX);   // the rest of the generation's sleepers
}

int32_t mac_area_f64(mac_ctx* ctx, const double* circles, int64_t three_n, double* area_out)
{
    ABI_BEGIN
    if (!area_out) return fail(MAC_E_INVAL, "null area_out");
    int32_t rc = check_common(ctx, three_n, 1);
    if (rc) return rc;
    if (!circles) return fail(MAC_E_INVAL, "null circles");
    if (!closure_path(ctx, three_n))
        return host_eval<double>(ctx, circles, three_n, 1, nullptr, 0.0, nullptr, nullptr, 1.0, area_out,
                                 nullptr, nullptr, nullptr);
    if (three_n == 0 || ctx->M == 0) {
        *area_out = 0.0;
        return MAC_OK;
    }
    ClReq r;
    r.c = circles;
    r.three_n = three_n;
    r.out = area_out;
    using clk = std::chrono::steady_clock;
    const auto tq = kClStats ? clk::now() : clk::time_point{};
    bool led = false;
    ctx->cl_active.fetch_add(1);
    {
        std::lock_guard<std::mutex> lk(ctx->cl_mu);
        r.gen = ctx->cl_gen.load(std::memory_order_relaxed);
        ctx->cl_q.push_back(&r);
    }
    // take every queued request of the front request's size (up to kClBatch) as a batch, if a
    // launch slot is free (under cl_mu)
    auto take = [&](std::vector<ClReq*>& batch, bool& mixed) {
        if (ctx->cl_busy >= kClLeaders || ctx->cl_q.empty()) return;
        ++ctx->cl_busy;
        ++ctx->cl_batches;
        const uint32_t g = ctx->cl_gen.fetch_add(1, std::memory_order_relaxed);   // requests queued from
                                                                                  // now on: the next batch's
        const int64_t tn = ctx->cl_q.front()->three_n;
        for (auto it = ctx->cl_q.begin(); it != ctx->cl_q.end() && (int)batch.size() < kClBatch;) {
            if ((*it)->three_n == tn) {
                if (kClStats) (*it)->t_taken = clk::now();
                (*it)->state.store(1, std::memory_order_relaxed);
                batch.push_back(*it);
                ++ctx->cl_reqs;
                ++ctx->cl_taken;
                it = ctx->cl_q.erase(it);
            } else {
                ++it;
            }
        }
        // a request of this generation left queued (another size, or past kClBatch) sleeps on the
        // same word: the batch's wake must then reach every sleeper, not one
        mixed = false;
        for (ClReq* q : ctx->cl_q) mixed |= q->gen == g;
    };
    std::vector<ClReq*> batch;
    bool mixed = false;
    for (int spin = 0, led_batches = 0;; ++spin) {
        const int st = r.state.load(std::memory_order_acquire);
        const bool mine = st == 2 || st == 3;   // this request is launched (or failed)
        if (mine && (batch.empty() || led_batches >= kClLead)) break;
        if (!mine && batch.empty() && ctx->cl_busy.load(std::memory_order_relaxed) < kClLeaders) {
            std::lock_guard<std::mutex> lk(ctx->cl_mu);
            // lead once every caller in the combiner has queued (the whole convoy in one launch),
            // or after a short wait
            const bool all_in = (int)ctx->cl_q.size() + ctx->cl_taken >= ctx->cl_active.load() ||
                                spin >= kClGather;
            if (r.state.load(std::memory_order_relaxed) == 0 && all_in) take(batch, mixed);
        }
        if (batch.empty()) {
            const int seen = r.state.load(std::memory_order_acquire);
            if (seen != 2 && seen != 3) cl_wait(ctx, r, spin);
            continue;
        }
        // lead: launch the batch, hand every request its slot; then, while requests are queued and
        // up to kClLead batches, lead again (this thread is awake on a CPU: a queued caller woken
        // to lead takes tens of microseconds to run under load), else wait for our own slot
        for (ClReq* q : batch) led |= q == &r;
        ++led_batches;
        const bool again = led_batches < kClLead;
        const auto tp = kClStats ? clk::now() : clk::time_point{};
        ClBatch* bt = new ClBatch();
        bt->readers.store((int)batch.size(), std::memory_order_relaxed);
        int32_t brc = MAC_OK;
        std::string msg;
        try {
            std::vector<const double*> cs(batch.size());
            for (size_t q = 0; q < batch.size(); ++q) cs[q] = batch[q]->c;
            set_device(ctx);
            bt->L = acquire_lane(ctx, nullptr);
            if (kClStats) cl_add(ctx->cl_phase_ns[3], clk::now() - tp);
            bt->seq = closure_launch(ctx, bt->L, batch[0]->three_n, cs.data(), (int)batch.size());
        } catch (const HipError& he) {
            brc = he.e == hipErrorOutOfMemory ? MAC_E_NOMEM : MAC_E_HIP;
            char buf[512];
            snprintf(buf, sizeof buf, "HIP error %d (%s) at maxcover.hip:%d in %s", (int)he.e,
                     hipGetErrorString(he.e), he.line, he.what);
            msg = buf;
        } catch (const std::bad_alloc&) {
            brc = MAC_E_NOMEM;
            msg = "host allocation failed";
        } catch (...) {
            brc = MAC_E_HIP;
            msg = "unexpected exception";
        }
        if (brc != MAC_OK) {   // nothing was launched: the lane back, the requests failed
            if (bt->L) {
                std::lock_guard<std::mutex> lk(ctx->mu);
                ctx->lanes_free.push_back(bt->L);
            }
            delete bt;
            bt = nullptr;
        }
        const auto th = kClStats ? clk::now() : clk::time_point{};
        std::vector<uint32_t> wake_gens;
        std::vector<ClReq*> handed;
        handed.swap(batch);
        const int wake_n = mixed ? INT_MAX : 1;
        {
            std::lock_guard<std::mutex> lk(ctx->cl_mu);
            --ctx->cl_busy;
            ctx->cl_taken -= (int)handed.size();
            if (again && brc == MAC_OK) {
                take(batch, mixed);   // the next batch, taken before this one's callers run
            } else {   // a queued request whose thread may lead the freed launch slot
                for (ClReq* q : ctx->cl_q)
                    if (q != &r) {
                        cl_wake(cl_word(ctx, q->gen), 1);
                        break;
                    }
            }
            // the generations of the handed-out requests (one, but for requests of another size
            // queued past an earlier take)
            for (ClReq* q : handed) wake_gens.push_back(q->gen);
        }
        for (size_t q = 0; q < handed.size(); ++q) {   // (a request lives until its released word reads 1)
            ClReq* rq = handed[q];
            rq->bt = bt;
            rq->b = (int)q;
            rq->rc = brc;
            rq->err = msg;
            if (kClStats) rq->t_handed = clk::now();
            rq->state.store(bt ? 3 : 2, std::memory_order_seq_cst);
            rq->released.store(1, std::memory_order_release);
        }
        // one sleeper per generation woken here; it wakes the others (cl_wait)
        std::sort(wake_gens.begin(), wake_gens.end());
        for (size_t q = 0; q < wake_gens.size(); ++q)
            if (q == 0 || wake_gens[q] != wake_gens[q - 1])
                cl_wake(cl_word(ctx, wake_gens[q]), wake_gens.front() == wake_gens.back() ? wake_n : INT_MAX);
        if (kClStats) cl_add(ctx->cl_phase_ns[2], clk::now() - th);
        spin = 0;
    }
    // the leader that launched this request may still be between its state store and its wake (the
    // futex word is this stack object): wait for its release, a few instructions away
    while (r.released.load(std::memory_order_acquire) == 0) __builtin_ia32_pause();
    const auto tl = kClStats ? clk::now() : clk::time_point{};
    if (r.state.load(std::memory_order_acquire) == 3) {
        try {
            *area_out = closure_read(ctx, r.bt, r.b);
        } catch (...) {
            closure_done(ctx, r.bt);
            ctx->cl_active.fetch_sub(1);
            throw;
        }
        closure_done(ctx, r.bt);
    }
    if (kClStats) {
        const auto te = clk::now();
        cl_add(ctx->cl_req_ns[0], r.t_taken - tq);
        cl_add(ctx->cl_req_ns[1], r.t_handed - r.t_taken);
        cl_add(ctx->cl_req_ns[2], tl - r.t_handed);
        cl_add(ctx->cl_req_ns[3], te - tl);
        cl_add(ctx->cl_req_ns[4], te - tq);
        ctx->cl_led.fetch_add(led, std::memory_order_relaxed);
    }
    ctx->cl_active.fetch_sub(1);
    if (r.rc) return fail(r.rc, r.err);
    return MAC_OK;
    ABI_END
}

int32_t mac_area_batch_f64(mac_ctx* ctx, const double* cands, int64_t three_n, int64_t K,
                           double* area_out)
{
    ABI_BEGIN
    if (!area_out && K > 0) return fail(MAC_E_INVAL, "null area_out");
    return host_eval<double>(ctx, cands, three_n, K, nullptr, 0.0, nullptr, nullptr, 1.0, area_out,
                     nullptr, nullptr, nullptr);
    ABI_END
}

int32_t mac_objective_batch_f64(mac_ctx* ctx, const double* cands, int64_t three_n, int64_t K,
                                const double* r_max, double penalty, double* obj_out)
{
    ABI_BEGIN
    if (!obj_out && K > 0) return fail(MAC_E_INVAL, "null obj_out");
    if (!r_max && three_n > 0) return fail(MAC_E_INVAL, "null r_max");
    return host_eval<double>(ctx, cands, three_n, K, r_max, penalty, nullptr, nullptr, 1.0, nullptr,
                     obj_out, nullptr, nullptr);
    ABI_END
}

int32_t mac_poll_best_f64(mac_ctx* ctx, const double* cands, int64_t three_n, int64_t K,
                          const double* r_max, double penalty, const double* prev,
                          const double* d_lim, double tan_half_fov, double* obj_out,
                          double* best_obj, int64_t* best_idx)
{
    ABI_BEGIN
    if (!best_obj || !best_idx) return fail(MAC_E_INVAL, "null best output");
    if (!r_max && three_n > 0) return fail(MAC_E_INVAL, "null r_max");
    return host_eval<double>(ctx, cands, three_n, K, r_max, penalty, prev, d_lim, tan_half_fov, nullptr,
                     obj_out, best_obj, best_idx);
    ABI_END
}

int32_t mac_area_f32(mac_ctx* ctx, const float* circles, int64_t three_n, double* area_out)
{
    ABI_BEGIN
    if (!area_out) return fail(MAC_E_INVAL, "null area_out");
    return host_eval<float>(ctx, circles, three_n, 1, nullptr, 0.0, nullptr, nullptr, 1.0, area_out,
                            nullptr, nullptr, nullptr);
    ABI_END
}

int32_t mac_area_batch_f32(mac_ctx* ctx, const float* cands, int64_t three_n, int64_t K,
                           double* area_out)
{
    ABI_BEGIN
    if (!area_out && K > 0) return fail(MAC_E_INVAL, "null area_out");
    return host_eval<float>(ctx, cands, three_n, K, nullptr, 0.0, nullptr, nullptr, 1.0, area_out,
                            nullptr, nullptr, nullptr);
    ABI_END
}

int32_t mac_poll_best_f32(mac_ctx* ctx, const float* cands, int64_t three_n, int64_t K,
                          const double* r_max, double penalty, const float* prev,
                          const double* d_lim, double tan_half_fov, double* obj_out,
                          double* best_obj, int64_t* best_idx)
{
    ABI_BEGIN
    if (!best_obj || !best_idx) return fail(MAC_E_INVAL, "null best output");
    if (!r_max && three_n > 0) return fail(MAC_E_INVAL, "null r_max");
    return host_eval<float>(ctx, cands, three_n, K, r_max, penalty, prev, d_lim, tan_half_fov,
                            nullptr, obj_out, best_obj, best_idx);
    ABI_END
}

int32_t mac_area_batch_dev_f64(mac_ctx* ctx, const double* d_cands, int64_t three_n, int64_t K,
                               double* d_area, void* stream)
{
    ABI_BEGIN
    int32_t rc = check_common(ctx, three_n, K);
    if (rc) return rc;
    if (K == 0) return MAC_OK;
    if (!d_cands || !d_area) return fail(MAC_E_INVAL, "null device pointer");
    set_device(ctx);
    hipStream_t s = (hipStream_t)stream;   // NULL: HIP's null stream
    LaneGuard lg(ctx, s);
    const int N = (int)(three_n / 3);
    enqueue_eval(ctx, lg.lane, s, matrix_src(d_cands, N), N, (int)K, use_tiled(ctx, N, nullptr, three_n), nullptr,
                 0.0, nullptr, nullptr, nullptr, 1.0, d_area, nullptr, nullptr, 0);
    return MAC_OK;
    ABI_END
}

}  // extern "C" (the template below has C++ linkage)

// The argument checks of a device poll (every failure a device poll can report before it
// enqueues anything but a HIP error): an armed poll runs them before its stream wait goes in.
static int32_t poll_dev_check(mac_ctx* ctx, const void* d_cands, int64_t three_n, int64_t K,
                              const void* d_prev, const double* d_dlim, const void* d_best)
{
    int32_t rc = check_common(ctx, three_n, K);
    if (rc) return rc;
    if (!d_best) return fail(MAC_E_INVAL, "null d_best");
    if (K > 0 && !d_cands) return fail(MAC_E_INVAL, "null d_cands");
    if (d_prev && !d_dlim) return fail(MAC_E_INVAL, "d_prev given without d_dlim");
    return MAC_OK;
}

// d_best's mapped result slot {obj, idx, seq, check} (k_final.h): its own, else the least recently
// used one (a fetch still waiting on a reassigned slot sees another seq and falls back to the
// stream + copy). Returns the slot's device address and the seq the next write carries.
static uint64_t* assign_mirror(mac_ctx* ctx, const void* d_best, uint64_t* seq)
{
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (!ctx->d_mirror) {
        const size_t b = sizeof(uint64_t) * 4 * mac_ctx::kMirrorSlots;
        ctx->h_mirror.reserve(b, hipHostMallocMapped | hipHostMallocCoherent);
        std::memset(ctx->h_mirror.p, 0, b);
        void* dp = nullptr;
        HCK(hipHostGetDevicePointer(&dp, ctx->h_mirror.p, 0));
        ctx->d_mirror = (uint64_t*)dp;
    }
    int q = 0;
    for (int j = 0; j < mac_ctx::kMirrorSlots; ++j) {
        if (ctx->mirror_key[j] == d_best) {
            q = j;
            break;
        }
        if (ctx->mirror_used[j] < ctx->mirror_used[q]) q = j;
    }
    ctx->mirror_key[q] = d_best;
    ctx->mirror_used[q] = ++ctx->mirror_clock;
    *seq = ctx->mirror_want[q] = ++ctx->mirror_seq;
    return ctx->d_mirror + 4 * q;
}

template <class T>
static int32_t poll_best_dev(mac_ctx* ctx, const T* d_cands_in, int64_t three_n, int64_t K,
                             const double* d_rmax, double penalty, const T* d_prev_in,
                             const double* d_dlim, double tan_half_fov, int64_t idx_base,
                             double* d_obj, void* d_best, void* stream)
{
    if (ctx && ctx->host_stats) t_poll_entry = std::chrono::steady_clock::now();
    constexpr bool f32 = std::is_same<T, float>::value;
    int32_t rc = poll_dev_check(ctx, d_cands_in, three_n, K, d_prev_in, d_dlim, d_best);
    if (rc) return rc;
    set_device(ctx);
    hipStream_t s = (hipStream_t)stream;   // NULL: HIP's null stream
    LaneGuard lg(ctx, s);
    Lane* L = lg.lane;
    const int N = (int)(three_n / 3);
    const double* d_cands;
    const double* d_prev;
    if constexpr (f32) {   // widened into the lane's scratch, stream-ordered before the chain
        L->cands.reserve(sizeof(double) * (size_t)std::max<int64_t>(three_n * K, 1));
        widen_async(d_cands_in, three_n * K, L->cands.as<double>(), s);
        d_cands = L->cands.as<double>();
        d_prev = nullptr;
        if (d_prev_in) {
            L->prev.reserve(sizeof(double) * (size_t)std::max<int64_t>(three_n, 1));
            widen_async(d_prev_in, three_n, L->prev.as<double>(), s);
            d_prev = L->prev.as<double>();
        }
    } else {
        d_cands = d_cands_in;
        d_prev = d_prev_in;
    }
    if (K == 0) {
        {
            std::lock_guard<std::mutex> lk(ctx->mu);
            for (int q = 0; q < mac_ctx::kMirrorSlots; ++q)
                if (ctx->mirror_key[q] == d_best) ctx->mirror_key[q] = nullptr;   // fetch: copy
        }
        double hb[2] = {INFINITY, __builtin_bit_cast(double, (int64_t)-1)};
        L->best.reserve(16);
        HCK(hipMemcpyAsync(d_best, hb, 16, hipMemcpyHostToDevice, s));
        HCK(hipStreamSynchronize(s));
        return MAC_OK;
    }
    // cons3: the raw d_lim goes down the chain; the kernels that read it threshold it once per
    // UAV (k_prep.h pen_threshold)
    const double* d_dlimT = nullptr;
    double* d_o = d_obj;
    if (!d_o) {
        L->obj.reserve(sizeof(double) * K);
        d_o = L->obj.as<double>();
    }
    if (K > 1 && !t_defer_free && !ctx->route_seeded.exchange(true)) {   // (seed_route)
        std::vector<double> x0((size_t)three_n);
        HCK(hipMemcpyAsync(x0.data(), d_cands, sizeof(double) * (size_t)three_n, hipMemcpyDeviceToHost, s));
        HCK(hipStreamSynchronize(s));
        seed_route(ctx, x0.data(), N);
    }
    uint64_t seq = 0;
    uint64_t* d_mirror = assign_mirror(ctx, d_best, &seq);
    enqueue_eval(ctx, L, s, matrix_src(d_cands, N), N, (int)K, use_tiled(ctx, N, nullptr, three_n), d_rmax,
                 penalty, d_prev, d_dlimT, d_dlim, tan_half_fov, nullptr, d_o, (double*)d_best, idx_base,
                 d_mirror, seq);
    return MAC_OK;
}

extern "C" {

int32_t mac_poll_best_dev_f64(mac_ctx* ctx, const double* d_cands, int64_t three_n, int64_t K,
                              const double* d_rmax, double penalty, const double* d_prev,
                              const double* d_dlim, double tan_half_fov, int64_t idx_base,
                              double* d_obj, void* d_best, void* stream)
{
    ABI_BEGIN
    return poll_best_dev<double>(ctx, d_cands, three_n, K, d_rmax, penalty, d_prev, d_dlim,
                                 tan_half_fov, idx_base, d_obj, d_best, stream);
    ABI_END
}

// Release tickets up to t (the doorbell's value), then every voided ticket that follows
// (guarded by mu).
static void release_tickets(mac_ctx* ctx, uint64_t t)
{
    if (t > ctx->fired) ctx->fired = t;
    for (bool more = true; more;) {
        more = false;
        for (size_t q = 0; q < ctx->voided.size(); ++q)
            if (ctx->voided[q] <= ctx->fired + 1) {
                ctx->fired = std::max(ctx->fired, ctx->voided[q]);
                ctx->voided.erase(ctx->voided.begin() + (long)q);
                more = true;
                break;
            }
    }
    __atomic_store_n(ctx->doorbell, ctx->fired, __ATOMIC_RELEASE);
}

int32_t mac_poll_arm_dev_f64(mac_ctx* ctx, const double* d_cands, int64_t three_n, int64_t K,
                             const double* d_rmax, double penalty, const double* d_prev,
                             const double* d_dlim, double tan_half_fov, int64_t idx_base,
                             double* d_obj, void* d_best, void* stream, uint64_t* ticket)
{
    ABI_BEGIN
    if (!ctx || !ticket) return fail(MAC_E_INVAL, "null context / ticket");
    if (K <= 0) return fail(MAC_E_INVAL, "an armed poll needs K > 0");   // (K = 0 synchronises)
    // every argument failure is reported before the wait goes into the stream
    int32_t rc = poll_dev_check(ctx, d_cands, three_n, K, d_prev, d_dlim, d_best);
    if (rc) return rc;
    // not on HIP's null stream: until the fire, a wait there would block every blocking-stream
    // operation of the process (the library's own synchronous copies, torch's .item() / .cpu())
    if (!stream) return fail(MAC_E_INVAL, "an armed poll needs a stream (not HIP's null stream)");
    set_device(ctx);
    hipStream_t s = (hipStream_t)stream;
    uint64_t t = 0;
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        if (!ctx->doorbell) {
            int ok = 0;
            HCK(hipDeviceGetAttribute(&ok, hipDeviceAttributeCanUseStreamWaitValue, ctx->device));
            if (!ok) return fail(MAC_E_HIP, "the device cannot wait on stream values");
            // coherent host memory: the host rings it with a plain atomic store, the stream's
            // wait polls it (a signal-memory doorbell would need the HSA signal API to wake it)
            void* p = nullptr;
            HCK(hipHostMalloc(&p, 64, hipHostMallocCoherent | hipHostMallocMapped));
            ctx->doorbell = (uint64_t*)p;
            __atomic_store_n(ctx->doorbell, (uint64_t)0, __ATOMIC_RELEASE);
            ctx->armed = ctx->fired = 0;
        }
        t = ++ctx->armed;
        bool found = false;
        for (auto& a : ctx->armed_on)
            if (a.first == s) {
                a.second = t;
                found = true;
            }
        if (!found) ctx->armed_on.push_back({s, t});
    }
    *ticket = t;
    // buffers the poll grows are not freed here (hipFree would wait for the device, which waits
    // for this ticket): they are kept until the next device synchronisation
    std::vector<std::pair<void*, bool>> defer;
    t_defer_free = &defer;
    bool ok = false;
    try {
        HCK(hipStreamWaitValue64(s, ctx->doorbell, t, hipStreamWaitValueGte, ~(uint64_t)0));
        rc = poll_best_dev<double>(ctx, d_cands, three_n, K, d_rmax, penalty, d_prev, d_dlim,
                                   tan_half_fov, idx_base, d_obj, d_best, stream);
        ok = rc == MAC_OK;
    } catch (...) {
        rc = -1;
    }
    t_defer_free = nullptr;
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->deferred.insert(ctx->deferred.end(), defer.begin(), defer.end());
    if (!ok) {
        // the poll did not go in: only its own ticket is released (now if every earlier one is,
        // else together with the last of them), never an earlier armed poll's
        if (t == ctx->fired + 1)
            release_tickets(ctx, t);
        else
            ctx->voided.push_back(t);
        if (rc < 0) return fail(MAC_E_HIP, "arming the poll failed");
    }
    return rc;
    ABI_END
}

int32_t mac_poll_fire(mac_ctx* ctx, uint64_t ticket)
{
    if (!ctx) return fail(MAC_E_INVAL, "null context");
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (!ctx->doorbell || ticket > ctx->armed) return fail(MAC_E_INVAL, "ticket was not armed");
    if (ticket > ctx->fired) release_tickets(ctx, ticket);
    return MAC_OK;
}

int32_t mac_poll_best_dev_f32(mac_ctx* ctx, const float* d_cands, int64_t three_n, int64_t K,
                              const double* d_rmax, double penalty, const float* d_prev,
                              const double* d_dlim, double tan_half_fov, int64_t idx_base,
                              double* d_obj, void* d_best, void* stream)
{
    ABI_BEGIN
    return poll_best_dev<float>(ctx, d_cands, three_n, K, d_rmax, penalty, d_prev, d_dlim,
                                tan_half_fov, idx_base, d_obj, d_best, stream);
    ABI_END
}

int32_t mac_poll_basis_f64(mac_ctx* ctx, const double* x_inc, int64_t three_n, const int16_t* ltri,
                           const int32_t* rp, const int32_t* cp, double delta, const double* r_max,
                           double penalty, const double* prev, const double* d_lim, double tan_half_fov,
                           double* obj_out, double* best_obj, int64_t* best_idx)
{
    ABI_BEGIN
    return host_eval_basis(ctx, x_inc, three_n, ltri, rp, cp, delta, r_max, penalty, prev, d_lim,
                           tan_half_fov, obj_out, best_obj, best_idx);
    ABI_END
}

int32_t mac_best_reduce_dev(mac_ctx* ctx, const void* d_records, int32_t n_records, void* d_best,
                            void* stream)
{
    ABI_BEGIN
    if (!ctx) return fail(MAC_E_INVAL, "null context");
    if (!d_best || (!d_records && n_records > 0)) return fail(MAC_E_INVAL, "null d_best / d_records");
    if (n_records < 0) return fail(MAC_E_INVAL, "negative record count");
    if ((((uintptr_t)d_records) | ((uintptr_t)d_best)) & 7)
        return fail(MAC_E_INVAL, "records / d_best not 8-byte aligned");
    set_device(ctx);
    uint64_t seq = 0;
    uint64_t* d_mirror = assign_mirror(ctx, d_best, &seq);
    hipLaunchKernelGGL(best_reduce_kernel, dim3(1), dim3(kWave), 0, (hipStream_t)stream,
                       (const unsigned long long*)d_records, (int)n_records, (unsigned long long*)d_best,
                       d_mirror, seq);
    HCK(hipGetLastError());
    return MAC_OK;
    ABI_END
}

// librccl bound once per path (the process keeps it: RCCL is never unloaded under live comms)
static RcclApi* rccl_api(const char* path)
{
    static std::mutex mu;
    static std::vector<std::pair<std::string, RcclApi*>> apis;
    std::lock_guard<std::mutex> lk(mu);
    const std::string key = path ? path : "";
    for (auto& a : apis)
        if (a.first == key) return a.second;
    void* h = nullptr;
    if (path && *path) {
        h = dlopen(path, RTLD_NOW | RTLD_LOCAL | RTLD_NOLOAD);   // the copy already loaded (torch's)
        if (!h) h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    } else {
        h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    }
    if (!h) return nullptr;
    RcclApi* a = new RcclApi();
    a->lib = h;
    a->get_unique_id = (int (*)(RcclUid*))dlsym(h, "ncclGetUniqueId");
    a->comm_init_rank = (int (*)(void**, int, RcclUid, int))dlsym(h, "ncclCommInitRank");
    a->all_gather = (int (*)(const void*, void*, size_t, int, void*, hipStream_t))dlsym(h, "ncclAllGather");
    a->comm_destroy = (int (*)(void*))dlsym(h, "ncclCommDestroy");
    a->error_string = (const char* (*)(int))dlsym(h, "ncclGetErrorString");
    if (!a->get_unique_id || !a->comm_init_rank || !a->all_gather || !a->comm_destroy) {
        delete a;
        return nullptr;
    }
    apis.push_back({key, a});
    return a;
}

static int32_t rccl_fail(RcclApi* a, int r, const char* what)
{
    std::string m = std::string(what) + ": RCCL error " + std::to_string(r);
    if (a && a->error_string) m += std::string(" (") + a->error_string(r) + ")";
    return fail(MAC_E_HIP, m.c_str());
}

int32_t mac_comm_unique_id(const char* rccl_path, void* id_out)
{
    ABI_BEGIN
    if (!id_out) return fail(MAC_E_INVAL, "null id");
    RcclApi* a = rccl_api(rccl_path);
    if (!a) return fail(MAC_E_HIP, "cannot load librccl");
    RcclUid id{};
    const int r = a->get_unique_id(&id);
    if (r) return rccl_fail(a, r, "ncclGetUniqueId");
    std::memcpy(id_out, &id, sizeof(id));
    return MAC_OK;
    ABI_END
}

int32_t mac_comm_init(mac_ctx* ctx, const char* rccl_path, const void* id, int32_t rank, int32_t world)
{
    ABI_BEGIN
    if (!ctx || !id) return fail(MAC_E_INVAL, "null context / id");
    if (world < 1 || rank < 0 || rank >= world) return fail(MAC_E_INVAL, "bad rank / world");
    if (ctx->comm) return fail(MAC_E_INVAL, "communicator already set");
    RcclApi* a = rccl_api(rccl_path);
    if (!a) return fail(MAC_E_HIP, "cannot load librccl");
    set_device(ctx);
    RcclUid uid;
    std::memcpy(&uid, id, sizeof(uid));
    void* comm = nullptr;
    const int r = a->comm_init_rank(&comm, world, uid, rank);   // (collective: every rank calls it)
    if (r) return rccl_fail(a, r, "ncclCommInitRank");
    void* buf = nullptr;
    if (hipMalloc(&buf, 16 * (size_t)world) != hipSuccess) {
        (void)a->comm_destroy(comm);
        return fail(MAC_E_NOMEM, "exchange buffer");
    }
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->rccl = a;
    ctx->comm = comm;
    ctx->comm_rank = rank;
    ctx->comm_world = world;
    ctx->d_xrec = buf;
    return MAC_OK;
    ABI_END
}

int32_t mac_exchange_records(mac_ctx* ctx, const void* rec, int32_t bytes, void* out, void* stream)
{
    ABI_BEGIN
    if (!ctx || !rec || !out) return fail(MAC_E_INVAL, "null argument");
    if (!ctx->comm) return fail(MAC_E_INVAL, "no communicator (mac_comm_init)");
    if (bytes <= 0 || bytes > 256 || bytes % 8) return fail(MAC_E_INVAL, "record size: a multiple of 8 up to 256");
    set_device(ctx);
    hipStream_t s = (hipStream_t)stream;
    const size_t W = (size_t)ctx->comm_world;
    std::lock_guard<std::mutex> xl(ctx->xmu);   // (one exchange at a time: the buffers are the context's)
    if (!ctx->h_xrec.p) {
        ctx->h_xrec.reserve(256 * (W + 1));
        HCK(hipMalloc(&ctx->d_xrec2, 256 * (W + 1)));
    }
    // this rank's record up, every rank's gathered on the stream, then down: one synchronisation
    unsigned char* h = (unsigned char*)ctx->h_xrec.p;
    unsigned char* d = (unsigned char*)ctx->d_xrec2;
    std::memcpy(h, rec, (size_t)bytes);
    HCK(hipMemcpyAsync(d, h, (size_t)bytes, hipMemcpyHostToDevice, s));
    const int r = ctx->rccl->all_gather(d, d + 256, (size_t)bytes, 1 /* ncclUint8 */, ctx->comm, s);
    if (r) return rccl_fail(ctx->rccl, r, "ncclAllGather");
    HCK(hipMemcpyAsync(h + 256, d + 256, (size_t)bytes * W, hipMemcpyDeviceToHost, s));
    HCK(hipStreamSynchronize(s));
    std::memcpy(out, h + 256, (size_t)bytes * W);
    return MAC_OK;
    ABI_END
}

int32_t mac_poll_exchange(mac_ctx* ctx, const void* d_best, void* d_out, void* stream, double* best_obj,
                          int64_t* best_idx)
{
    ABI_BEGIN
    if (!ctx || !d_best || !d_out) return fail(MAC_E_INVAL, "null argument");
    if (!ctx->comm) return fail(MAC_E_INVAL, "no communicator (mac_comm_init)");
    if ((((uintptr_t)d_best) | ((uintptr_t)d_out)) & 7) return fail(MAC_E_INVAL, "records not 8-byte aligned");
    set_device(ctx);
    hipStream_t s = (hipStream_t)stream;
    // every rank's 16-B record into the gather buffer, on the poll's stream (RCCL over xGMI), then
    // one wave's argmin into d_out and its mapped slot, then the slot read (mac_best_fetch)
    const int r = ctx->rccl->all_gather(d_best, ctx->d_xrec, 16, 1 /* ncclUint8 */, ctx->comm, s);
    if (r) return rccl_fail(ctx->rccl, r, "ncclAllGather");
    uint64_t seq = 0;
    uint64_t* d_mirror = assign_mirror(ctx, d_out, &seq);
    hipLaunchKernelGGL(best_reduce_kernel, dim3(1), dim3(kWave), 0, s, (const unsigned long long*)ctx->d_xrec,
                       ctx->comm_world, (unsigned long long*)d_out, d_mirror, seq);
    HCK(hipGetLastError());
    if (!best_obj && !best_idx) return MAC_OK;
    return mac_best_fetch(ctx, d_out, stream, best_obj, best_idx);
    ABI_END
}

int32_t mac_best_fetch(mac_ctx* ctx, const void* d_best, void* stream, double* best_obj,
                       int64_t* best_idx)
{
    ABI_BEGIN
    if (!ctx) return fail(MAC_E_INVAL, "null context");
    if (!d_best) return fail(MAC_E_INVAL, "null d_best");
    set_device(ctx);
    hipStream_t s = (hipStream_t)stream;   // NULL: HIP's null stream
    const uint64_t* slot = nullptr;
    uint64_t want = 0;
    bool pending = false;   // an armed poll on `stream` is not fired: it must not be waited for
    {
        std::lock_guard<std::mutex> lk(ctx->mu);   // (released before any wait)
        for (int q = 0; q < mac_ctx::kMirrorSlots; ++q)
            if (ctx->mirror_key[q] == d_best && ctx->h_mirror.p) {
                slot = (const uint64_t*)ctx->h_mirror.p + 4 * q;
                want = ctx->mirror_want[q];
                break;
            }
        for (auto& a : ctx->armed_on)   // an armed poll on THIS stream is not fired
            pending = pending || (a.first == s && a.second > ctx->fired);
    }
    if (slot) {
        // the latest device poll on d_best writes its result into this slot (the poll takes
        // ~0.1 ms); after 2 ms wait for the stream (which also reports a failed launch), then
        // read the slot once more, else copy d_best
        double o = 0.0;
        int64_t i = -1;
        bool ok = mirror_wait(slot, want, pending ? 2000.0 : 2.0, &o, &i);
        if (!ok && pending)
            return fail(MAC_E_HIP, "poll result not written within 2 s (armed polls pending)");
        if (!ok) {
            HCK(hipStreamSynchronize(s));
            ok = mirror_read(slot, want, &o, &i);
        }
        if (ok) {
            if (best_obj) *best_obj = o;
            if (best_idx) *best_idx = i;
            return MAC_OK;
        }
    }
    double tmp[2];
    HCK(hipMemcpyAsync(tmp, d_best, 16, hipMemcpyDeviceToHost, s));
    HCK(hipStreamSynchronize(s));
    if (best_obj) *best_obj = tmp[0];
    if (best_idx) *best_idx = __builtin_bit_cast(int64_t, tmp[1]);
    return MAC_OK;
    ABI_END
}

}  // extern "C"
