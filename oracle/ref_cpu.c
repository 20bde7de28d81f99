/*
 * oracle/ref_cpu.c — TEST INFRASTRUCTURE ONLY. Never linked into, loaded by or called from
 * the product path (libmaxcover); only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, as the checker / the CPU baseline.
 *
 * A plain-C restatement of the reference's hot path, following the cited Julia lines
 * statement by statement (the reference is Julia; Julia is not installed here, so the
 * reference itself cannot be run — see DESIGN.md "Oracle"). Parity is pinned by integer
 * lattice known-answer tests and by the FirePoints.xlsx data converted to
 * tests/golden/firepoints.csv; the reference's own tests pin nothing on this path
 * (test/runtests.jl:4-6).
 *
 * Build: -O2 -ffp-contract=off, no fast-math (Julia neither contracts a*b+c into an FMA
 * nor reorders the sum; x^2 on Float64 lowers to x*x).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define REF_OK 0
#define REF_E_SIZE 2  /* Int(length(circles)/3) InexactError, src/AreaCoverageCalculation.jl:65 */

/* src/AreaCoverageCalculation.jl:63-78 — calculateArea(circles::Vector{Float64},
 * points::Vector{Vector{Float64}}). `points` mirrors Vector{Vector{Float64}}: an array of
 * pointers to per-entry records [x, y, area, importance, covered]. */
int ref_calculate_area_ptrs(const double* circles, int64_t three_n,
                            const double* const* points, int64_t M, double* out)
{
    if (three_n % 3 != 0) return REF_E_SIZE;                 /* :65 */
    const int64_t Nc = three_n / 3;
    double area_covered = 0.0;                               /* :64 */
    for (int64_t p = 0; p < M; ++p) {                        /* :67 */
        const double* pt = points[p];
        for (int64_t c = 0; c < Nc; ++c) {                   /* :68 */
            const double dx = pt[0] - circles[c];
            const double dy = pt[1] - circles[Nc + c];
            if (sqrt(dx * dx + dy * dy) < circles[2 * Nc + c]) {  /* :70 */
                area_covered += pt[3];                       /* :72 (column 4) */
                break;                                       /* :74 */
            }
        }
    }
    *out = area_covered;                                     /* :109 */
    return REF_OK;
}

/* Flat-record convenience: rows of `stride` doubles. Same loop as above. */
int ref_calculate_area_rec(const double* circles, int64_t three_n, const double* rec,
                           int64_t M, int64_t stride, double* out)
{
    if (three_n % 3 != 0) return REF_E_SIZE;
    const int64_t Nc = three_n / 3;
    double area_covered = 0.0;
    for (int64_t p = 0; p < M; ++p) {
        const double* pt = rec + p * stride;
        for (int64_t c = 0; c < Nc; ++c) {
            const double dx = pt[0] - circles[c];
            const double dy = pt[1] - circles[Nc + c];
            if (sqrt(dx * dx + dy * dy) < circles[2 * Nc + c]) {
                area_covered += pt[3];
                break;
            }
        }
    }
    *out = area_covered;
    return REF_OK;
}

/* src/TDM_STATIC_opt.jl:82-100 — AreaMaxObjective(x) = -calculateArea(x, pts) + 1e5*violation,
 * violation = sum_{i=1..N} abs(x[i+2N] - r_max[i]) accumulated sequentially (:89-93, :97).
 * make_circles/make_MADS (src/AreaCoverageCalculation.jl:33-59) are the identity on values. */
int ref_objective_ptrs(const double* x, int64_t three_n, const double* const* points, int64_t M,
                       const double* r_max, double penalty, double* out)
{
    double area;
    int rc = ref_calculate_area_ptrs(x, three_n, points, M, &area);
    if (rc) return rc;
    const int64_t N = three_n / 3;
    double violation = 0.0;                                  /* :89 */
    for (int64_t i = 0; i < N; ++i)                          /* :90 */
        violation += fabs(x[i + 2 * N] - r_max[i]);          /* :92 */
    *out = -area + violation * penalty;                      /* :97 */
    return REF_OK;
}

/* Pointer-per-entry point list, mirroring Julia's Vector{Vector{Float64}} (one heap block of
 * `stride` doubles per entry). Used for the CPU baseline so its memory behaviour matches. */
double** ref_points_alloc(const double* rec, int64_t M, int64_t stride)
{
    double** pts = (double**)malloc((size_t)(M > 0 ? M : 1) * sizeof(double*));
    if (!pts) return NULL;
    for (int64_t p = 0; p < M; ++p) {
        pts[p] = (double*)malloc((size_t)stride * sizeof(double));
        memcpy(pts[p], rec + p * stride, (size_t)stride * sizeof(double));
    }
    return pts;
}

void ref_points_free(double** pts, int64_t M)
{
    if (!pts) return;
    for (int64_t p = 0; p < M; ++p) free(pts[p]);
    free(pts);
}

/* K candidates (3N x K column-major), OpenMP over candidates — mirrors DirectSearch's
 * SetMaxEvals poll-level threading (src/TDM_STATIC_opt.jl:129). nthreads <= 0: default. */
int ref_area_batch_ptrs(const double* cands, int64_t three_n, int64_t K,
                        const double* const* points, int64_t M, double* out, int nthreads)
{
    if (three_n % 3 != 0) return REF_E_SIZE;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int64_t k = 0; k < K; ++k)
        ref_calculate_area_ptrs(cands + k * three_n, three_n, points, M, &out[k]);
    (void)nthreads;
    return REF_OK;
}

int ref_max_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* src/CellFunctions.jl:81-108 — rmvCoveredPOI: same predicate (:90), first hit breaks (:95),
 * indices collected in list order and deleted with the order-preserving deleteat! (:101).
 * Writes the kept 0-based indices to kept_idx and returns their count via *M_out. */
int ref_remove_covered_rec(const double* circles, int64_t three_n, const double* rec, int64_t M,
                           int64_t stride, int64_t* kept_idx, int64_t* M_out)
{
    if (three_n % 3 != 0) return REF_E_SIZE;
    const int64_t Nc = three_n / 3;
    int64_t kept = 0;
    for (int64_t p = 0; p < M; ++p) {
        const double* pt = rec + p * stride;
        int covered = 0;
        for (int64_t c = 0; c < Nc; ++c) {
            const double dx = pt[0] - circles[c];
            const double dy = pt[1] - circles[Nc + c];
            if (sqrt(dx * dx + dy * dy) < circles[2 * Nc + c]) { covered = 1; break; }
        }
        if (!covered) kept_idx[kept++] = p;
    }
    *M_out = kept;
    return REF_OK;
}

/* src/AreaCoverageCalculation.jl:11-21 — createPOI(dx, dy, x_length, y_length): i outer over
 * 1:x_length, j inner over 1:y_length, entry [i*dx-dx/2, j*dy-dy/2, dx*dy, dx*dy, false].
 * `out` receives nx*ny rows of 5 doubles (covered = 0.0). Julia's `1:x_length` on a Float64
 * end runs i = 1.0, 2.0, ... while i <= x_length. */
int64_t ref_create_poi(double dx, double dy, double x_length, double y_length, double* out)
{
    int64_t n = 0;
    for (double i = 1.0; i <= x_length; i += 1.0) {
        for (double j = 1.0; j <= y_length; j += 1.0) {
            if (out) {
                double* r = out + 5 * n;
                r[0] = i * dx - dx / 2;
                r[1] = j * dy - dy / 2;
                r[2] = dx * dy;
                r[3] = dx * dy;
                r[4] = 0.0;
            }
            ++n;
        }
    }
    return n;
}

/* src/TDM_Constraints.jl:54-75 — cons3(x): for every UAV i, reject if the 3-D displacement
 * sqrt((x1-x2)^2+(y1-y2)^2+(z1-z2)^2) > d_lim[i], z = R / tan(FOV/2) (:60,:65,:67).
 * `prev` is pre_optimized_circles_MADS as [x;y;R]. Returns 1 feasible, 0 infeasible. */
int ref_cons3(const double* prev, const double* x, int64_t three_n, const double* d_lim,
              double tan_half_fov)
{
    const int64_t N = three_n / 3;
    for (int64_t i = 0; i < N; ++i) {
        const double x1 = prev[i], y1 = prev[N + i], z1 = prev[2 * N + i] / tan_half_fov;
        const double x2 = x[i], y2 = x[N + i], z2 = x[2 * N + i] / tan_half_fov;
        const double ddx = x1 - x2, ddy = y1 - y2, ddz = z1 - z2;
        if (sqrt(ddx * ddx + ddy * ddy + ddz * ddz) > d_lim[i]) return 0;
    }
    return 1;
}

/* src/Base_Functions.jl:44-65 — allocate_even_circles(r_centering_cir, N, r_uav, cx, cy):
 * angle 2*pi/N*(i-1), x = r*cos + cx, y = r*sin + cy, R = r_uav; returns [x;y;R]. */
void ref_allocate_even_circles(double r_centering, int64_t N, double r_uav, double center_x,
                               double center_y, double* out)
{
    const double two_pi = 2.0 * 3.14159265358979323846;
    for (int64_t i = 0; i < N; ++i) {
        const double ang = two_pi / (double)N * (double)i;
        out[i] = r_centering * cos(ang) + center_x;
        out[N + i] = r_centering * sin(ang) + center_y;
        out[2 * N + i] = r_uav;
    }
}

/* ---- src/DynamicArea.jl: cellular-automaton fire (config 5 point stream) ----------------
 * The reference draws with an unseeded rand(); the restatement (and the GPU generator) draw
 * u = hash(seed, step t, cell, neighbour slot q) so that runs are reproducible. The hash is
 * part of this build's specification (splitmix64 finaliser over a keyed counter). */
static uint64_t ref_mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

double ref_fire_uniform(uint64_t seed, uint64_t t, uint64_t cell, uint64_t q)
{
    uint64_t z = seed ^ (t * 0xD1B54A32D192ED03ull);
    z ^= (cell * 9ull + q) * 0x9E3779B97F4A7C15ull;
    return (double)(ref_mix64(z) >> 11) * 0x1p-53;
}

/* :63 — the spread threshold of block position (r, c), 1-based: slot q = (c-1)*3 + (r-1)
 * (findall's column-major order over grid[i-1:i+1, j-1:j+1]). */
void ref_fire_thresholds(double wind_speed, double wind_direction, double prob_spread, double* p9)
{
    for (int c = 1; c <= 3; ++c)
        for (int r = 1; r <= 3; ++r)
            p9[(c - 1) * 3 + (r - 1)] =
                wind_speed * cos(wind_direction - atan2((double)(2 - c), (double)(2 - r))) * prob_spread;
}

/* :26-35 — grid[i,j] (1-based, row-major storage (i-1)*ny + (j-1)): TREE (1) when
 * u(seed, 0, cell, 0) < density else EMPTY (0); the ignition block set to FIRE (2). */
void ref_fire_init(uint8_t* g, int64_t nx, int64_t ny, double density, uint64_t seed, int64_t ix0,
                   int64_t ix1, int64_t iy0, int64_t iy1)
{
    for (int64_t i = 1; i <= nx; ++i)
        for (int64_t j = 1; j <= ny; ++j) {
            const int64_t cell = (i - 1) * ny + (j - 1);
            g[cell] = ref_fire_uniform(seed, 0, (uint64_t)cell, 0) < density ? 1 : 0;
        }
    for (int64_t i = ix0; i <= ix1; ++i)
        for (int64_t j = iy0; j <= iy1; ++j) g[(i - 1) * ny + (j - 1)] = 2;
}

/* :52-72 — update_grid: new_grid = copy(grid); for i in 2:nx-1, j in 2:ny-1 (i outer): a TREE
 * cell with FIRE in its 3x3 block tests each FIRE position in column-major order; success ->
 * new_grid[i,j] = FIRE and push!(points, i*dx - dx/2, j*dy - dy/2, dx*dy, dx*dy, false).
 * `gn` receives the new grid; rec (nullable) up to cap records of 5 doubles. Returns the number
 * of points pushed. */
int64_t ref_fire_step(const uint8_t* g, uint8_t* gn, int64_t nx, int64_t ny, const double* p9,
                      double dx, double dy, uint64_t seed, uint64_t t, double* rec, int64_t cap)
{
    int64_t n = 0;
    memcpy(gn, g, (size_t)(nx * ny));
    for (int64_t i = 2; i <= nx - 1; ++i) {
        for (int64_t j = 2; j <= ny - 1; ++j) {
            const int64_t cell = (i - 1) * ny + (j - 1);
            if (g[cell] != 1) continue;
            for (int c = 1; c <= 3; ++c) {           /* findall: column-major over the block */
                for (int r = 1; r <= 3; ++r) {
                    if (g[(i - 3 + r) * ny + (j - 3 + c)] != 2) continue;  /* grid[i-2+r, j-2+c], 1-based */
                    const int q = (c - 1) * 3 + (r - 1);
                    if (p9[q] > ref_fire_uniform(seed, t, (uint64_t)cell, (uint64_t)q)) {
                        gn[cell] = 2;
                        if (rec && n < cap) {
                            double* o = rec + 5 * n;
                            o[0] = (double)i * dx - dx / 2;
                            o[1] = (double)j * dy - dy / 2;
                            o[2] = dx * dy;
                            o[3] = dx * dy;
                            o[4] = 0.0;
                        }
                        ++n;
                    }
                }
            }
        }
    }
    return n;
}

/* ---------------------------------------------------------------------------------------
 * Known-answer counts (independent of floating point), for full-size parity checks.
 * On the half-integer lattice of createPOI(pitch, pitch, G, G) (src/AreaCoverageCalculation.jl
 * :11-21: entry (i - 1/2)*pitch, (j - 1/2)*pitch) with integer disk centres and radii, entry
 * (i, j) lies strictly inside disk (cx, cy, R) iff ((2i-1)p - 2cx)^2 + ((2j-1)p - 2cy)^2 < 4R^2
 * in exact int64 arithmetic. out[k] = number of entries covered by the union of candidate k's
 * disks (cands: K x 3N, integer-valued doubles; R <= 0 covers nothing). One G x G byte mask per
 * thread; only the disks' bounding windows are touched and cleared. */
int ref_lattice_count_batch(const double* cands, int64_t three_n, int64_t K, int64_t G,
                            int64_t pitch, int64_t* out, int nthreads)
{
    if (three_n % 3 != 0) return REF_E_SIZE;
    const int64_t N = three_n / 3;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    int rc = REF_OK;
#ifdef _OPENMP
#pragma omp parallel
#endif
    {
        uint8_t* cov = (uint8_t*)calloc((size_t)(G * G), 1);
        if (!cov) rc = -1;
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 4)
#endif
        for (int64_t k = 0; k < K; ++k) {
            if (!cov) continue;
            const double* c = cands + k * three_n;
            int64_t n = 0;
            for (int pass = 0; pass < 2; ++pass) {   /* 0: mark and count, 1: clear windows */
                for (int64_t d = 0; d < N; ++d) {
                    const int64_t cx = (int64_t)c[d], cy = (int64_t)c[N + d], R = (int64_t)c[2 * N + d];
                    if (R <= 0) continue;
                    int64_t i0 = (2 * (cx - R)) / (2 * pitch) - 1, i1 = (2 * (cx + R)) / (2 * pitch) + 2;
                    int64_t j0 = (2 * (cy - R)) / (2 * pitch) - 1, j1 = (2 * (cy + R)) / (2 * pitch) + 2;
                    if (i0 < 1) i0 = 1;
                    if (j0 < 1) j0 = 1;
                    if (i1 > G) i1 = G;
                    if (j1 > G) j1 = G;
                    for (int64_t i = i0; i <= i1; ++i) {
                        const int64_t dx = (2 * i - 1) * pitch - 2 * cx;
                        for (int64_t j = j0; j <= j1; ++j) {
                            uint8_t* m = cov + (i - 1) * G + (j - 1);
                            if (pass) { *m = 0; continue; }
                            const int64_t dy = (2 * j - 1) * pitch - 2 * cy;
                            if (dx * dx + dy * dy < 4 * R * R && !*m) { *m = 1; ++n; }
                        }
                    }
                }
            }
            out[k] = n;
        }
        free(cov);
    }
    return rc;
}

/* The objective penalty of src/TDM_STATIC_opt.jl:89-93 for K candidates (K x 3N rows):
 * violation_k = sum_{i=1..N} abs(x[i+2N] - r_max[i]) accumulated sequentially from 0.0. */
void ref_violation_batch(const double* cands, int64_t three_n, int64_t K, const double* r_max,
                         double* out)
{
    const int64_t N = three_n / 3;
    for (int64_t k = 0; k < K; ++k) {
        const double* x = cands + k * three_n;
        double v = 0.0;
        for (int64_t i = 0; i < N; ++i) v += fabs(x[i + 2 * N] - r_max[i]);
        out[k] = v;
    }
}

/* cons3 (ref_cons3) for K candidates: feas[k] = 1 feasible, 0 infeasible. */
void ref_cons3_batch(const double* prev, const double* cands, int64_t three_n, int64_t K,
                     const double* d_lim, double tan_half_fov, uint8_t* feas)
{
    for (int64_t k = 0; k < K; ++k)
        feas[k] = (uint8_t)ref_cons3(prev, cands + k * three_n, three_n, d_lim, tan_half_fov);
}
