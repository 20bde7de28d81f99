/*
 * maxcover.h — C-ABI of libmaxcover, the MI355X (gfx950) implementation of the
 * MADS area-coverage objective of Gabisanth/MaximumAreaCoverageOptimization.jl.
 *
 * Plain C, no C++ exceptions cross it, no torch types: it is what a Julia
 * `ccall`, a Python `ctypes` stub or any other FFI binds.
 *
 * Reference seam this replaces (paths relative to the reference repo root):
 *   - AreaCoverageCalculation.calculateArea(circles, points)
 *         src/AreaCoverageCalculation.jl:63-110 (live loop :67-78)
 *   - the AreaMaxObjective closure built by TDM_STATIC_opt.createObjective
 *         src/TDM_STATIC_opt.jl:82-100 (penalty :89-97)
 *   - the extreme constraint cons3 built by create_cons3
 *         src/TDM_Constraints.jl:54-75
 *   - CellFunctions.rmvCoveredPOI (order-preserving deletion)
 *         src/CellFunctions.jl:81-108 (predicate :90, deleteat! :101)
 *   - DirectSearch's poll step (evaluate every trial point, keep the best)
 *         called at src/TDM_STATIC_opt.jl:162 (third-party, not vendored)
 *
 * Semantics kept bit-for-bit:
 *   covered(p) = exists c: sqrt((px-cx)^2 + (py-cy)^2) < r_c     (fp64, ^2 = x*x, no FMA,
 *                                                                 correctly rounded sqrt, strict <)
 *   area       = sum of w_p over covered p, w = record column 4   (duplicates counted per entry)
 *   objective  = -area + 1e5 * sum_i |x[2N+i] - r_max[i]|        (sequential sum over i)
 * Candidates use the reference layout [x_1..x_N; y_1..y_N; r_1..r_N] (3N doubles).
 *
 * Ownership: host arrays are borrowed read-only for the duration of a call; the library
 * copies what it keeps into device buffers it owns. Outputs are written before return
 * (synchronous API) except for the *_dev entry points, which are stream-ordered.
 * Threading: mac_area_* / mac_objective_* / mac_poll_* may be called concurrently on one
 * context from several host threads (DirectSearch SetMaxEvals, src/TDM_STATIC_opt.jl:129);
 * mac_set_points_* / mac_remove_covered_* must not overlap evaluations (points only
 * change between MADS calls, src/FullSimulation.jl:50-61).
 */
#ifndef MAXCOVER_H
#define MAXCOVER_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes --------------------------------------------------------------- */
#define MAC_OK            0
#define MAC_E_INVAL       1  /* null pointer / negative size / bad option                    */
#define MAC_E_SIZE        2  /* three_n % 3 != 0: the reference's Int(length/3) InexactError,
                                src/AreaCoverageCalculation.jl:65                            */
#define MAC_E_NOPOINTS    3  /* no point list set on the context                             */
#define MAC_E_HIP         4  /* a HIP runtime call failed (see mac_last_error)               */
#define MAC_E_NOMEM       5  /* device allocation failed                                     */
#define MAC_E_LOSSY       6  /* reserved                                                      */
#define MAC_E_NODEVICE    7  /* no HIP device / bad device index                             */

/* ---- options (mac_set_option) --------------------------------------------------- */
#define MAC_OPT_ALGO         1  /* MAC_ALGO_AUTO (default) | _SCAN | _TILED | _POLL             */
#define MAC_OPT_STORAGE      2  /* MAC_STORE_F64 only: the list is kept in fp64 (fp32 inputs go
                                   through the *_f32 entry points, widened exactly); _F32 fails */
#define MAC_OPT_TILE_POINTS  3  /* target points per spatial tile (default 4), set before points */
#define MAC_OPT_PROFILE      4  /* 1: the timed launches stamp their workgroups' start / end     */
#define MAC_OPT_SHARED       5  /* poll walk, entries two disks' regions share:
                                   MAC_SHARED_AUTO (default) | _FP64 | _BITS                      */

#define MAC_OPT_CHAIN        6  /* the poll chain: MAC_CHAIN_AUTO (default) | _FIVE | _FUSED */

#define MAC_CHAIN_AUTO   0  /* the fused three-launch chain unless one of the context's last 64 polls was crowded,
                               scattered or off the packed-key grid (then the five-launch chain)  */
#define MAC_CHAIN_FIVE   1  /* always the five-launch chain (prep, index, set-up, walk, finalize)   */
#define MAC_CHAIN_FUSED  2  /* the fused chain whenever it applies (K <= 3073, packed keys possible) */

#define MAC_SHARED_AUTO  0  /* bit-word kernel when one of the lane's last 8 polls had more than 16
                               disks with neighbours, else fp64 jobs in the poll kernel         */
#define MAC_SHARED_FP64  1  /* always the poll kernel's fp64 jobs                                */
#define MAC_SHARED_BITS  2  /* always the bit-word kernel (every disk it takes, any count)       */

#define MAC_ALGO_AUTO   0
#define MAC_ALGO_SCAN   1  /* streaming brute-force scan: every point against every disk     */
#define MAC_ALGO_TILED  2  /* per-candidate walk over the tile-binned point list (exact culling) */
#define MAC_ALGO_POLL   3  /* per-disk walk over the whole poll: region entries staged in LDS,
                              one candidate per lane (the six-launch chain; weighted lists) */
/* (4 was an opt-in two-launch poll, measured slower than the chain and removed: refused) */

#define MAC_STORE_F64   0
#define MAC_STORE_F32   1

typedef struct mac_ctx mac_ctx;

/* Thread-local message for the last non-zero status returned on this thread. */
const char* mac_last_error(void);
/* Library version string, e.g. "maxcover 0.1.0 gfx950". */
const char* mac_version(void);

int32_t mac_device_count(int32_t* count_out);
int32_t mac_ctx_create(mac_ctx** out, int32_t device);
void    mac_ctx_destroy(mac_ctx* ctx);
int32_t mac_set_option(mac_ctx* ctx, int32_t option, int64_t value);

/* ---- point list (per MPC step) -------------------------------------------------- */
/* SoA host arrays, M entries each; weight w = the reference's column 4 ("importance"). */
int32_t mac_set_points_f64(mac_ctx* ctx, const double* x, const double* y, const double* w,
                           int64_t M);
/* Reference records: M rows of `stride` doubles, [x, y, area, importance, covered, ...];
 * x = col 1, y = col 2, weight = col 4 (src/AreaCoverageCalculation.jl:16,72). stride >= 4. */
int32_t mac_set_points_records_f64(mac_ctx* ctx, const double* rec, int64_t M, int64_t stride);
/* Same, from device-resident SoA arrays (borrowed for the call, copied). */
int32_t mac_set_points_dev_f64(mac_ctx* ctx, const double* d_x, const double* d_y,
                               const double* d_w, int64_t M);
/* fp32 point lists (SURVEY 8(b) *_f32): each float is widened to the double of the same value
 * on the device and the list is then exactly the fp64 list of those values (the reference's
 * Vector{Float64} would hold the same doubles after Float64(::Float32)). */
int32_t mac_set_points_f32(mac_ctx* ctx, const float* x, const float* y, const float* w,
                           int64_t M);
int32_t mac_set_points_dev_f32(mac_ctx* ctx, const float* d_x, const float* d_y, const float* d_w,
                               int64_t M);
int32_t mac_num_points(mac_ctx* ctx, int64_t* M_out);
/* Copy the current list (original order) back to host SoA arrays (each M_out entries). */
int32_t mac_get_points_f64(mac_ctx* ctx, double* x, double* y, double* w);

/* rmvCoveredPOI (src/CellFunctions.jl:81-108): delete, in place and order-preserving, every
 * entry covered by `circles` ([x;y;r], three_n doubles). kept_idx (nullable, capacity M)
 * receives the 0-based original indices of the kept entries; *M_out the new length. */
int32_t mac_remove_covered_f64(mac_ctx* ctx, const double* circles, int64_t three_n,
                               int64_t* kept_idx, int64_t* M_out);
/* Covered flags for the current list (original order), one byte per entry. */
int32_t mac_covered_flags_f64(mac_ctx* ctx, const double* circles, int64_t three_n,
                              uint8_t* flags_out);
/* update_POI (src/CellFunctions.jl:59-79): append m entries at the END of the list (list order
 * = summation order), then re-index. Host SoA arrays / device-resident SoA arrays. */
int32_t mac_append_points_f64(mac_ctx* ctx, const double* x, const double* y, const double* w,
                              int64_t m);
int32_t mac_append_points_dev_f64(mac_ctx* ctx, const double* d_x, const double* d_y,
                                  const double* d_w, int64_t m);

/* ---- objective ------------------------------------------------------------------ */
/* calculateArea(circles, points): one candidate. */
int32_t mac_area_f64(mac_ctx* ctx, const double* circles, int64_t three_n, double* area_out);
/* K candidates, column-major 3N x K (each candidate contiguous, as a Julia Matrix(3N,K)). */
int32_t mac_area_batch_f64(mac_ctx* ctx, const double* cands, int64_t three_n, int64_t K,
                           double* area_out);
/* AreaMaxObjective for K candidates: obj_k = -area_k + penalty * sum_i |x[2N+i] - r_max[i]|
 * (penalty = 1e5 in the reference). r_max: N doubles. */
int32_t mac_objective_batch_f64(mac_ctx* ctx, const double* cands, int64_t three_n, int64_t K,
                                const double* r_max, double penalty, double* obj_out);

/* Poll step: evaluate K candidates, reject those failing cons3 (3-D displacement from
 * `prev` [x;y;r] > d_lim[i], z = R / tan_half_fov; src/TDM_Constraints.jl:54-75) when prev
 * is non-null, and return the lowest-index minimiser (ties -> lowest index, the order a
 * sequential poll keeps its first best). best_idx = -1 when no candidate is feasible.
 * obj_out (nullable, K doubles) receives every objective (+inf for infeasible). As in
 * DirectSearch's extreme barrier, an infeasible candidate is not evaluated: its coverage is never
 * computed (the walks leave it out when N <= 512), only its +inf objective reported. */
int32_t mac_poll_best_f64(mac_ctx* ctx, const double* cands, int64_t three_n, int64_t K,
                          const double* r_max, double penalty,
                          const double* prev, const double* d_lim, double tan_half_fov,
                          double* obj_out, double* best_obj, int64_t* best_idx);

/* Basis form of a caller-owned poll (DirectSearch's poll, src/TDM_STATIC_opt.jl:22-44 CustomPoll
 * b / i / maximal_basis; :162): the 2n candidates (n = three_n) x_inc + delta * B[:, k] (index k)
 * and x_inc - delta * B[:, k] (index n + k), k < n, with B = L[rp][:, cp]: B[v][k] =
 * L[rp[v]][cp[k]], L lower triangular, passed as its lower triangle packed by rows (int16, entry
 * (r, c <= r) at r(r+1)/2 + c; n(n+1)/2 entries), rp / cp permutations of [0, n) (any values in
 * [0, n) are accepted). B's entry is delta * L exactly as the double product, so the candidates
 * equal the matrix a caller would build with the same arithmetic, and the results equal
 * mac_poll_best_f64 on that 3N x 2n matrix bit for bit. Ships 16n + n(n+1) bytes instead of 16n^2
 * (config 4: 2.4 MB instead of 37.7 MB). obj_out nullable (2n doubles). */
int32_t mac_poll_basis_f64(mac_ctx* ctx, const double* x_inc, int64_t three_n, const int16_t* ltri,
                           const int32_t* rp, const int32_t* cp, double delta, const double* r_max,
                           double penalty, const double* prev, const double* d_lim, double tan_half_fov,
                           double* obj_out, double* best_obj, int64_t* best_idx);

/* ---- native MADS driver ------------------------------------------ */
/* A granular MADS with a complete LTMADS poll, the restatement of DirectSearch's Optimize!
 * (src/TDM_STATIC_opt.jl:118-169; the third-party algorithm is not vendored, so this is the
 * build's own, parity-tested against maximumareacoverageoptimization.jl_amd/TDM_STATIC_opt.mads):
 *   f = objective(x0) (+inf if x0 fails cons3); ell = ell0; per iteration (at most n_iter,
 *   while ell >= 0): B = L[rp][:, cp] with L lower triangular (diagonal +-2^ell, strictly lower
 *   uniform integers in [-(2^ell-1), 2^ell-1]) and random row / column permutations, all drawn
 *   from a splitmix64 stream seeded with `seed`; the 2n candidates x + B[:,k], x - B[:,k] are
 *   generated ON THE DEVICE (no candidate matrix), evaluated with the objective and cons3 as an
 *   extreme barrier; success (best < f): x, f <- best, ell <- min(ell + 1, ell_max); else
 *   ell <- ell - 1. One 16-byte read-back per iteration. */
typedef struct mac_mads_params {
    int64_t n_iter;        /* iteration limit (SetIterationLimit, 100 in the reference)      */
    int32_t ell0, ell_max; /* initial / largest mesh exponent (0 <= ell0 <= ell_max <= 52)    */
    uint64_t seed;
} mac_mads_params;
typedef struct mac_mads_stats {
    double f;              /* objective at x_out (+inf: no feasible point found)              */
    int64_t iterations;
    int64_t evaluations;   /* 1 + 2n per iteration                                            */
    int32_t status;        /* 0: mesh precision limit (ell < 0); 1: iteration limit           */
    int32_t feasible;
    double seconds;        /* wall time inside the call                                       */
    double host_enqueue_s; /* of which: enqueueing the polls (uploads + kernel launches)       */
    double host_perm_s;    /*           next iteration's permutations (overlaps the device)    */
    double wait_s;         /*           waiting for the device                                 */
    double host_post_s;    /*           incumbent update after each poll                       */
    int64_t feasible_evaluations; /* poll candidates that passed cons3 and were evaluated (this
                                     stepper's shard; the start point's evaluation not counted) */
    int64_t rejected_polls;       /* iterations cons3 rejected whole with no evaluation: every
                                     variable's diagonal step +-2^ell alone breaks its UAV's d_lim
                                     (src/TDM_Constraints.jl:67), so no candidate passes — a
                                     failure (ell - 1), as the extreme barrier makes it         */
    int64_t successes;            /* iterations whose poll moved the incumbent (the rest failed) */
    int64_t slot_fallbacks;       /* polls whose result did not arrive through the mapped slot within
                                     50 ms (read by a copy after a stream synchronisation instead):
                                     0 in a healthy run                                           */
} mac_mads_stats;
int32_t mac_mads_run(mac_ctx* ctx, const double* x0, int64_t three_n, const double* r_max,
                     double penalty, const double* prev, const double* d_lim, double tan_half_fov,
                     const mac_mads_params* params, double* x_out, mac_mads_stats* stats);

/* The same loop one iteration at a time, for the multi-GPU poll (BASELINE config 5 "8 GPUs";
 * src/TDM_STATIC_opt.jl:129, SetMaxEvals's poll-level parallelism). A stepper owns the shard
 * [shard_lo, shard_hi) of every poll's 2n candidates (0, 2n: the whole poll, as mac_mads_run):
 *   mac_mads_poll    done = 1 once the iteration limit or ell < 0 is reached; otherwise evaluates
 *                    this iteration's shard (generated on the device) and returns its best
 *                    (objective, poll-wide index) (+inf, -1 for an empty shard or no feasible
 *                    candidate);
 *   mac_mads_update  applies the poll's best over ALL shards (the lexicographic (objective,
 *                    index) minimum of the ranks' results, e.g. a 16-B all-gather): the
 *                    incumbent, ell and the stream position advance exactly as in mac_mads_run,
 *                    so every rank stays in lock step with the single-GPU loop;
 *   mac_mads_result  x and the statistics (evaluations count whole polls). */
typedef struct mac_mads mac_mads;
int32_t mac_mads_begin(mac_ctx* ctx, const double* x0, int64_t three_n, const double* r_max,
                       double penalty, const double* prev, const double* d_lim, double tan_half_fov,
                       const mac_mads_params* params, int64_t shard_lo, int64_t shard_hi,
                       mac_mads** out);
int32_t mac_mads_poll(mac_mads* m, int32_t* done, double* best_obj, int64_t* best_idx);
int32_t mac_mads_update(mac_mads* m, double best_obj, int64_t best_idx);
int32_t mac_mads_result(mac_mads* m, double* x_out, mac_mads_stats* stats);
/* Speculation over failure branches (src/TDM_STATIC_opt.jl:162: the MADS iterations are
 * serial, but a failed iteration's next poll is fully determined: the same incumbent, ell - 1, the
 * stream's next position). Rank j of a P-GPU loop evaluates, beside rank 0's real poll, the poll
 * that follows j consecutive failures; after one exchange every rank applies the results in
 * order up to the first success, so a run of failures advances up to P iterations per round:
 *   mac_mads_poll_ahead  evaluates (this stepper's shard of) the poll of the iteration `ahead`
 *                        failures past the current one, without advancing; done = 1 when that
 *                        poll does not exist (iteration limit or ell - ahead < 0); feasible (may be
 *                        NULL): its candidates that passed cons3 (evaluated);
 *   mac_mads_advance     applies one iteration's result (the poll at ahead = 0) as
 *                        mac_mads_update does, without a prior mac_mads_poll; moved = 1 when the
 *                        incumbent moved (success). Same iterates as the sequential loop. */
int32_t mac_mads_poll_ahead(mac_mads* m, int32_t ahead, int32_t* done, double* best_obj, int64_t* best_idx,
                            int64_t* feasible);
int32_t mac_mads_advance(mac_mads* m, double best_obj, int64_t best_idx, int32_t* moved);
void mac_mads_destroy(mac_mads* m);
/* Every later poll of the stepper also writes its 16-byte shard best {objective, index as
 * int64 bits} to d_best16 (device memory of the context's device, 8-byte aligned; NULL: stop):
 * once mac_mads_poll has returned, the buffer holds that poll's best for device work on any
 * stream (mac_best_fetch's ordering), so a multi-GPU loop all-gathers straight from it with no
 * host-to-device copy per iteration (dist.DeviceGather). */
int32_t mac_mads_best_buffer(mac_mads* m, void* d_best16);

/* fp32 candidates (config 3's "fp32" caller path; SURVEY 8(b) "*_f32: coords f32, accum f64"):
 * the candidate matrix (and prev) are uploaded as floats and widened exactly on the device;
 * coverage is then the reference's fp64 predicate on those doubles, areas accumulate in fp64 /
 * integer counts, and the outputs equal the *_f64 calls on the widened inputs bit for bit.
 * r_max and d_lim stay fp64 (model parameters, not coordinates). */
int32_t mac_area_f32(mac_ctx* ctx, const float* circles, int64_t three_n, double* area_out);
int32_t mac_area_batch_f32(mac_ctx* ctx, const float* cands, int64_t three_n, int64_t K,
                           double* area_out);
int32_t mac_poll_best_f32(mac_ctx* ctx, const float* cands, int64_t three_n, int64_t K,
                          const double* r_max, double penalty, const float* prev,
                          const double* d_lim, double tan_half_fov, double* obj_out,
                          double* best_obj, int64_t* best_idx);

/* ---- device-pointer, stream-ordered variants (inputs already resident in HBM) ----- */
/* d_cands: 3N x K column-major on the context's device; d_area: K doubles. `stream` is a
 * hipStream_t; NULL is HIP's null stream (as in every HIP API: the work is ordered after the
 * caller's default-stream work, e.g. torch's default stream, which produced d_cands). Returns
 * after enqueueing. */
int32_t mac_area_batch_dev_f64(mac_ctx* ctx, const double* d_cands, int64_t three_n, int64_t K,
                               double* d_area, void* stream);
/* Device poll: d_best receives {best_obj (double), best_idx (int64 stored as double bits)}
 * as 16 bytes; d_obj (nullable) K objectives. d_prev/d_dlim nullable (no cons3). */
int32_t mac_poll_best_dev_f64(mac_ctx* ctx, const double* d_cands, int64_t three_n, int64_t K,
                              const double* d_rmax, double penalty,
                              const double* d_prev, const double* d_dlim, double tan_half_fov,
                              int64_t idx_base, double* d_obj, void* d_best, void* stream);
/* Same with fp32 d_cands / d_prev (widened into the call's scratch on `stream` first). */
int32_t mac_poll_best_dev_f32(mac_ctx* ctx, const float* d_cands, int64_t three_n, int64_t K,
                              const double* d_rmax, double penalty,
                              const float* d_prev, const double* d_dlim, double tan_half_fov,
                              int64_t idx_base, double* d_obj, void* d_best, void* stream);
/* The host side of one MADS poll step: returns the {objective, index} the latest
 * mac_poll_best_dev_* on d_best wrote. Each d_best buffer gets a mapped host slot that the
 * poll's last finalize block fills (after its d_best stores have reached the device's L2), so
 * the call returns as soon as the result exists, without a copy: at that point d_best holds the
 * result for device work, but the poll's launch may still be retiring on `stream` — order later
 * work that reads d_best or reuses the poll's inputs on `stream`, or synchronise it first.
 * Without a slot (a K = 0 poll, or the slot taken by 64 newer d_best buffers) or after 2 ms,
 * it waits for `stream` (NULL: HIP's null stream) and copies d_best. Polls on different
 * d_best buffers may be issued and fetched concurrently from several host threads. */
int32_t mac_best_fetch(mac_ctx* ctx, const void* d_best, void* stream, double* best_obj,
                       int64_t* best_idx);

/* The multi-GPU poll's exchange, reduced on the device: d_records holds n_records 16-B records
 * {objective, index as int64 bits} (the ranks' d_best, e.g. one RCCL all-gather into one buffer
 * ordered on `stream`); one wave writes their lexicographic minimum to d_best (a record with
 * index < 0 or an objective not < +inf never wins; ties to the lowest index; none: {+inf, -1})
 * and to d_best's mapped result slot, so mac_best_fetch(d_best) returns the node's argmin without
 * a copy or a stream synchronisation. Stream-ordered; returns after enqueueing. */
int32_t mac_best_reduce_dev(mac_ctx* ctx, const void* d_records, int32_t n_records, void* d_best,
                            void* stream);

/* The multi-GPU poll exchange over RCCL (xGMI) on the poll's own stream. librccl is bound at run
 * time from rccl_path (the copy the process already loaded when it is loaded, e.g. torch's; NULL:
 * librccl.so.1 from the library path).
 *   mac_comm_unique_id  rank 0 makes the communicator id (128 bytes) the ranks share out of band;
 *   mac_comm_init       every rank (collective) joins with its rank and the world size;
 *   mac_poll_exchange   all-gathers every rank's 16-B {objective, index} record d_best into the
 *                       context's buffer (ncclAllGather on `stream`, ordered after the rank's poll),
 *                       reduces it on the device as mac_best_reduce_dev into d_out and its mapped
 *                       slot, and (best_obj / best_idx non-null) returns the node's argmin from the
 *                       slot as mac_best_fetch does. Collective: every rank calls it per poll.
 * The communicator is destroyed with the context. */
int32_t mac_comm_unique_id(const char* rccl_path, void* id_out);
int32_t mac_comm_init(mac_ctx* ctx, const char* rccl_path, const void* id, int32_t rank, int32_t world);
int32_t mac_poll_exchange(mac_ctx* ctx, const void* d_best, void* d_out, void* stream, double* best_obj,
                          int64_t* best_idx);
/* Every rank's host record of `bytes` bytes (a multiple of 8, at most 256) gathered into `out`
 * (world x bytes, rank order) over the context's communicator: one upload, the all-gather and one
 * download on `stream`, then its synchronisation (the speculative MADS loop's per-round exchange:
 * {done, objective, index, feasible} of every rank's poll). Collective. */
int32_t mac_exchange_records(mac_ctx* ctx, const void* rec, int32_t bytes, void* out, void* stream);

/* Armed device polls: the host turnaround between dependent polls of a MADS loop (the next poll
 * is known only after the previous one's result) taken off the device's critical path. The
 * chain of mac_poll_best_dev_f64 is enqueued ahead of time behind a stream wait on the context's
 * doorbell (a coherent host word the stream waits on), so its launches are already queued
 * when the host decides; mac_poll_fire rings the doorbell and the chain starts without a launch.
 * Its inputs (d_cands, d_prev, ...) may be written until the fire (device writes on other
 * streams must have completed). Rules: tickets are fired in arming order (a fire releases every
 * armed poll with a ticket <= it); a poll and the armed poll after it use different d_best
 * buffers (each buffer's mapped slot follows its latest poll); nothing may wait for the stream
 * (or the device) while an armed poll on it is not fired — mac_best_fetch of a fired poll never
 * does, and mac_ctx_destroy fires every outstanding ticket first. Argument errors are reported
 * before anything is enqueued; a poll that fails after its wait went in voids only its own ticket
 * (released together with the earlier tickets, never ahead of them). `stream` must be a created
 * stream, not NULL (MAC_E_INVAL): an unfired wait on HIP's null stream would block every
 * blocking-stream operation of the process. Buffers an armed poll grows
 * are released at the next device synchronisation (point-list changes, mac_ctx_destroy), since
 * freeing them would wait for the unfired poll. MAC_E_HIP when the device cannot wait on stream
 * values (hipDeviceAttributeCanUseStreamWaitValue). */
int32_t mac_poll_arm_dev_f64(mac_ctx* ctx, const double* d_cands, int64_t three_n, int64_t K,
                             const double* d_rmax, double penalty,
                             const double* d_prev, const double* d_dlim, double tan_half_fov,
                             int64_t idx_base, double* d_obj, void* d_best, void* stream,
                             uint64_t* ticket);
int32_t mac_poll_fire(mac_ctx* ctx, uint64_t ticket);

/* ---- measurement ----------------------------------------------------------------- */
/* With MAC_OPT_PROFILE = 1, the coverage-kernel launches (and the first and last launch of
 * each poll chain) stamp their workgroups' start / end times (s_memrealtime, k_common.h): no
 * packet or dependency is added to the stream. Reads (after a device sync) the summed coverage-
 * kernel time in ms (last end - first start per launch), the launch count and the candidates
 * evaluated by those launches, and the walk the LAST of them used (MAC_ALGO_SCAN / _TILED /
 * _POLL, 0 = none); reset != 0 clears the record. */
int32_t mac_profile_read(mac_ctx* ctx, double* kernel_ms, int64_t* launches,
                         int64_t* candidates, int32_t* last_algo, int32_t reset);

/* Split of the poll chains recorded since the last reset (call before mac_profile_read with
 * reset), summed: launch chain: prep = first launch's first start .. the walk's first start,
 * walk = the walk launch, gap = the walk's last end .. finalize's (+ argmin) last end.
 * polls = chains counted. */
int32_t mac_profile_split(mac_ctx* ctx, double* prep_ms, double* walk_ms, double* gap_ms,
                          int64_t* polls);

/* Per-kernel split of the same poll chains (call before mac_profile_read with reset): for each
 * launch role r < n_roles, the summed launch spans (last workgroup end - first workgroup start,
 * in-kernel stamps) in ms_out[r] and the launches counted in launches_out[r]. Roles:
 *   0 prep_kernel, 1 disk_index_kernel, 2 walk_setup_kernel, 3 coverage_tiled_poll_kernel,
 *   4 coverage_poll_kernel, 5 the crowded-poll shared-entry pass (shared_or_kernel on equal
 *   weights, shared_bits_kernel otherwise), 6 finalize_kernel (five-launch chain), 7 fiw_kernel and
 *   8 fin2_kernel (the fused chain) (MAC_PROF_ROLES = 9). */
#define MAC_PROF_ROLES 9
int32_t mac_profile_kernels(mac_ctx* ctx, double* ms_out, int64_t* launches_out, int32_t n_roles);

/* ---- fire generator (src/DynamicArea.jl, config 5) ------------------------------ */
/* Cellular-automaton forest fire on an nx x ny grid of dx x dy cells, cell (i, j) 1-based with
 * i the row (x index) and j the column (y index), as the reference indexes grid[i, j].
 *   init (:26-35): TREE with probability forest_density else EMPTY; the block
 *                  [ix0, ix1] x [iy0, iy1] (inclusive, 1-based) set to FIRE.
 *   step (:52-72): every interior TREE cell tests each FIRE cell of its 3x3 block, in column-major
 *                  block order, with wind_speed*cos(wind_direction - atan(2-c, 2-r))*prob_spread
 *                  > u; each success makes it FIRE in the new grid and emits one point
 *                  (i*dx - dx/2, j*dy - dy/2, dx*dy, dx*dy, 0) — duplicates per igniting
 *                  neighbour, cells in i-outer/j-inner order (the reference's push order).
 * u is a counter-based hash of (seed, step, cell, neighbour) instead of the reference's unseeded
 * rand(), so runs are reproducible and identical to the CPU restatement. */
typedef struct mac_fire mac_fire;
typedef struct mac_fire_params {
    int64_t nx, ny;                 /* grid size in cells (>= 3 each)                          */
    double dx, dy;                  /* cell pitch (m): 5, 5 in the reference (:6-7)            */
    double forest_density;          /* 0.7 (:20)                                               */
    double prob_spread;             /* 0.5 (:21)                                               */
    double wind_speed;              /* 4 (:47)                                                 */
    double wind_direction;          /* radians; deg2rad(270) (:48)                             */
    int64_t ix0, ix1, iy0, iy1;     /* ignition block, 1-based inclusive (:35)                 */
    uint64_t seed;
} mac_fire_params;
const char* mac_fire_last_error(void);
/* the nine spread thresholds, slot q = (c-1)*3 + (r-1) (column-major block position) */
void    mac_fire_thresholds(const mac_fire_params* p, double* out9);
int32_t mac_fire_create(mac_fire** out, int32_t device, const mac_fire_params* p);
void    mac_fire_destroy(mac_fire* f);
/* :37-42: the initial points (y outer, x inner) as records of 5 doubles; *n_out = count
 * (records written up to cap; rec nullable to query the count). */
int32_t mac_fire_initial_points(mac_fire* f, double* rec, int64_t cap, int64_t* n_out);
/* One update_grid step; *n_new = number of points pushed. They are appended to `append_to`'s
 * list (device to device, update_POI) when non-null. */
int32_t mac_fire_step(mac_fire* f, mac_ctx* append_to, int64_t* n_new);
/* The last step's points as records of 5 doubles (up to cap); *n_out = their count. */
int32_t mac_fire_last_points(mac_fire* f, double* rec, int64_t cap, int64_t* n_out);
/* The current grid, nx*ny bytes, row-major in (i, j): 0 EMPTY, 1 TREE, 2 FIRE. */
int32_t mac_fire_get_grid(mac_fire* f, uint8_t* out);
int32_t mac_fire_set_grid(mac_fire* f, const uint8_t* in);

/* ---- exact predicate helpers (host) --------------------------------------------- */
/* Largest double T with: for every double a >= 0, (sqrt(a) < r) <=> (a <= T), where sqrt is
 * the correctly rounded fp64 sqrt. -1.0 when nothing can be covered (r <= 0 or NaN). */
double mac_cover_threshold(double r);

#ifdef __cplusplus
}
#endif

#endif /* MAXCOVER_H */
