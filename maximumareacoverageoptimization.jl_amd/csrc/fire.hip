// fire.hip — the cellular-automaton fire generator of src/DynamicArea.jl on the GPU, and the
// stream of new fire points it feeds into a context's point list (config 5).
//
// Reference (src/DynamicArea.jl):
//   :26-33  grid cell (i, j) = TREE with probability forest_density, else EMPTY
//   :35     cells [round(x_start1/dx) : round(x_start2/dx)] x [round(y_start1/dy) :
//           round(y_start2/dy)] set to FIRE
//   :37-42  initial points: for y in that y range, x in that x range (y outer):
//           (x*dx - dx/2, y*dy - dy/2, dx*dy, dx*dy, false)
//   :52-72  update_grid: for i in 2:nx-1, j in 2:ny-1 (i outer): a TREE cell with any FIRE cell
//           in its 3x3 block tests every FIRE neighbour, in findall's column-major order over
//           the block, with  wind_speed * cos(wind_direction - atan(2 - c, 2 - r)) *
//           prob_spread > rand()  ((r, c) the 1-based position in the block); each success sets
//           the cell to FIRE in the NEW grid and pushes (i*dx - dx/2, j*dy - dy/2, dx*dy, dx*dy,
//           false) — one point per igniting neighbour, hence the duplicates. FIRE never burns
//           out; border cells never change.
// The reference's rand() is unseeded (not reproducible); here every draw is a counter-based
// hash of (seed, step, cell, neighbour) — identical on the CPU restatement (oracle/ref_cpu.c
// ref_fire_*) — and the nine thresholds are computed once on the host, so the GPU compares
// the same doubles as the CPU.
//
// Per step: count kernel (new state + ignitions per cell) -> exclusive scan -> emit kernel
// (points in cell order: the reference's push order) -> append to the context (re-index).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "maxcover.h"

namespace {

constexpr uint8_t kEmpty = 0, kTree = 1, kFire = 2;

thread_local std::string g_fire_err;

int32_t ffail(int32_t code, const std::string& m)
{
    g_fire_err = m;
    return code;
}

#define FCK(expr)                                                                              \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess) return ffail(MAC_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

__host__ __device__ inline uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// uniform double in [0, 1) for (seed, step t, cell, neighbour slot q)
__host__ __device__ inline double fire_uniform(uint64_t seed, uint64_t t, uint64_t cell, uint64_t q)
{
    uint64_t z = seed ^ (t * 0xD1B54A32D192ED03ull);
    z ^= (cell * 9ull + q) * 0x9E3779B97F4A7C15ull;
    return (double)(mix64(z) >> 11) * 0x1p-53;
}

struct FireConst {
    double p[9];      // column-major slot q = (c-1)*3 + (r-1)
    double dx, dy;
    uint64_t seed;
    int64_t nx, ny;
};

__global__ void fire_init_kernel(uint8_t* __restrict__ g, FireConst fc, double density,
                                 int64_t ix0, int64_t ix1, int64_t iy0, int64_t iy1)
{
    const int64_t cell = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (cell >= fc.nx * fc.ny) return;
    const int64_t i = cell / fc.ny + 1, j = cell % fc.ny + 1;   // 1-based (row i, column j)
    uint8_t s = fire_uniform(fc.seed, 0, (uint64_t)cell, 0) < density ? kTree : kEmpty;
    if (i >= ix0 && i <= ix1 && j >= iy0 && j <= iy1) s = kFire;
    g[cell] = s;
}

__global__ void fire_count_kernel(const uint8_t* __restrict__ g, uint8_t* __restrict__ gn,
                                  uint32_t* __restrict__ cnt, FireConst fc, uint64_t t)
{
    const int64_t cell = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (cell >= fc.nx * fc.ny) return;
    const int64_t i = cell / fc.ny, j = cell % fc.ny;           // 0-based
    const uint8_t s = g[cell];
    uint32_t c = 0;
    if (s == kTree && i >= 1 && i <= fc.nx - 2 && j >= 1 && j <= fc.ny - 2) {
#pragma unroll
        for (int cc = 0; cc < 3; ++cc) {       // block column (j offset), column-major order
#pragma unroll
            for (int rr = 0; rr < 3; ++rr) {   // block row (i offset)
                const uint8_t v = g[(i - 1 + rr) * fc.ny + (j - 1 + cc)];
                if (v == kFire) {
                    const int q = cc * 3 + rr;
                    if (fc.p[q] > fire_uniform(fc.seed, t, (uint64_t)cell, (uint64_t)q)) ++c;
                }
            }
        }
    }
    gn[cell] = c ? kFire : s;
    cnt[cell] = c;
}

__global__ void fire_emit_kernel(const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ off,
                                 FireConst fc, double* __restrict__ x, double* __restrict__ y,
                                 double* __restrict__ w)
{
    const int64_t cell = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (cell >= fc.nx * fc.ny) return;
    const uint32_t c = cnt[cell];
    if (!c) return;
    const int64_t i = cell / fc.ny + 1, j = cell % fc.ny + 1;
    const double px = (double)i * fc.dx - fc.dx / 2, py = (double)j * fc.dy - fc.dy / 2;
    const double wt = fc.dx * fc.dy;
    for (uint32_t m = 0; m < c; ++m) {
        x[off[cell] + m] = px;
        y[off[cell] + m] = py;
        w[off[cell] + m] = wt;
    }
}

}  // namespace

struct mac_fire {
    int device = 0;
    hipStream_t s = nullptr;
    FireConst fc{};
    mac_fire_params p{};
    uint64_t step = 0;
    uint8_t* g = nullptr;
    uint8_t* gn = nullptr;
    uint32_t* cnt = nullptr;
    uint32_t* off = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    double* px = nullptr;
    double* py = nullptr;
    double* pw = nullptr;
    int64_t pcap = 0;
    int64_t last_n = 0;
};

static inline unsigned blocks(int64_t n) { return (unsigned)((n + 255) / 256); }

extern "C" {

const char* mac_fire_last_error(void) { return g_fire_err.c_str(); }

// Reference thresholds: wind_speed * cos(wind_direction - atan(2 - c, 2 - r)) * prob_spread.
void mac_fire_thresholds(const mac_fire_params* p, double* out9)
{
    for (int c = 1; c <= 3; ++c)
        for (int r = 1; r <= 3; ++r)
            out9[(c - 1) * 3 + (r - 1)] =
                p->wind_speed * std::cos(p->wind_direction - std::atan2((double)(2 - c), (double)(2 - r))) *
                p->prob_spread;
}

int32_t mac_fire_create(mac_fire** out, int32_t device, const mac_fire_params* p)
{
    try {
        if (!out || !p) return ffail(MAC_E_INVAL, "null argument");
        *out = nullptr;
        // <= 2^28 cells: at most 8 points per cell keeps the per-step offsets in uint32
        if (p->nx < 3 || p->ny < 3 || p->nx > ((int64_t)1 << 28) || p->ny > ((int64_t)1 << 28) ||
            p->nx * p->ny > ((int64_t)1 << 28))
            return ffail(MAC_E_INVAL, "grid must be >= 3 x 3 and at most 2^28 cells");
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n)
            return ffail(MAC_E_NODEVICE, "no such HIP device");
        FCK(hipSetDevice(device));
        mac_fire* f = new mac_fire();
        f->device = device;
        f->p = *p;
        mac_fire_thresholds(p, f->fc.p);
        f->fc.dx = p->dx;
        f->fc.dy = p->dy;
        f->fc.seed = p->seed;
        f->fc.nx = p->nx;
        f->fc.ny = p->ny;
        const int64_t C = p->nx * p->ny;
        if (hipStreamCreateWithFlags(&f->s, hipStreamNonBlocking) != hipSuccess ||
            hipMalloc(&f->g, C) != hipSuccess || hipMalloc(&f->gn, C) != hipSuccess ||
            hipMalloc(&f->cnt, sizeof(uint32_t) * C) != hipSuccess ||
            hipMalloc(&f->off, sizeof(uint32_t) * C) != hipSuccess) {
            mac_fire_destroy(f);
            return ffail(MAC_E_NOMEM, "fire grid allocation failed");
        }
        (void)hipcub::DeviceScan::ExclusiveSum(nullptr, f->tmp_bytes, f->cnt, f->off, (int)C, f->s);
        if (hipMalloc(&f->tmp, std::max<size_t>(f->tmp_bytes, 256)) != hipSuccess) {
            mac_fire_destroy(f);
            return ffail(MAC_E_NOMEM, "scan scratch allocation failed");
        }
        hipLaunchKernelGGL(fire_init_kernel, dim3(blocks(C)), dim3(256), 0, f->s, f->g, f->fc,
                           p->forest_density, p->ix0, p->ix1, p->iy0, p->iy1);
        FCK(hipGetLastError());
        FCK(hipStreamSynchronize(f->s));
        *out = f;
        return MAC_OK;
    } catch (...) {
        return ffail(MAC_E_HIP, "unexpected exception");
    }
}

void mac_fire_destroy(mac_fire* f)
{
    if (!f) return;
    (void)hipSetDevice(f->device);
    if (f->s) (void)hipStreamSynchronize(f->s);
    for (void* q : {(void*)f->g, (void*)f->gn, (void*)f->cnt, (void*)f->off, f->tmp, (void*)f->px,
                    (void*)f->py, (void*)f->pw})
        if (q) (void)hipFree(q);
    if (f->s) (void)hipStreamDestroy(f->s);
    delete f;
}

int32_t mac_fire_initial_points(mac_fire* f, double* rec, int64_t cap, int64_t* n_out)
{
    if (!f || !n_out) return ffail(MAC_E_INVAL, "null argument");
    const mac_fire_params& p = f->p;
    int64_t n = 0;
    for (int64_t yy = p.iy0; yy <= p.iy1; ++yy)        // :38 y outer
        for (int64_t xx = p.ix0; xx <= p.ix1; ++xx) {  // :39 x inner
            if (rec && n < cap) {
                double* r = rec + 5 * n;
                r[0] = (double)xx * p.dx - p.dx / 2;
                r[1] = (double)yy * p.dy - p.dy / 2;
                r[2] = p.dx * p.dy;
                r[3] = p.dx * p.dy;
                r[4] = 0.0;
            }
            ++n;
        }
    *n_out = n;
    return MAC_OK;
}

int32_t mac_fire_step(mac_fire* f, mac_ctx* append_to, int64_t* n_new)
{
    try {
        if (!f || !n_new) return ffail(MAC_E_INVAL, "null argument");
        FCK(hipSetDevice(f->device));
        const int64_t C = f->fc.nx * f->fc.ny;
        const uint64_t t = ++f->step;
        hipLaunchKernelGGL(fire_count_kernel, dim3(blocks(C)), dim3(256), 0, f->s, f->g, f->gn,
                           f->cnt, f->fc, t);
        FCK(hipGetLastError());
        FCK(hipcub::DeviceScan::ExclusiveSum(f->tmp, f->tmp_bytes, f->cnt, f->off, (int)C, f->s));
        uint32_t last_off = 0, last_cnt = 0;
        FCK(hipMemcpyAsync(&last_off, f->off + C - 1, 4, hipMemcpyDeviceToHost, f->s));
        FCK(hipMemcpyAsync(&last_cnt, f->cnt + C - 1, 4, hipMemcpyDeviceToHost, f->s));
        FCK(hipStreamSynchronize(f->s));
        std::swap(f->g, f->gn);
        const int64_t n = (int64_t)last_off + last_cnt;
        f->last_n = n;
        *n_new = n;
        if (n == 0) return MAC_OK;
        if (n > f->pcap) {
            for (double** q : {&f->px, &f->py, &f->pw}) {
                if (*q) FCK(hipFree(*q));
                *q = nullptr;
            }
            const int64_t c2 = std::max<int64_t>(n, f->pcap + f->pcap / 2);
            f->pcap = 0;
            if (hipMalloc(&f->px, 8 * c2) != hipSuccess || hipMalloc(&f->py, 8 * c2) != hipSuccess ||
                hipMalloc(&f->pw, 8 * c2) != hipSuccess)
                return ffail(MAC_E_NOMEM, "fire point allocation failed");
            f->pcap = c2;
        }
        hipLaunchKernelGGL(fire_emit_kernel, dim3(blocks(C)), dim3(256), 0, f->s, f->cnt, f->off,
                           f->fc, f->px, f->py, f->pw);
        FCK(hipGetLastError());
        FCK(hipStreamSynchronize(f->s));
        if (append_to) {
            const int32_t rc = mac_append_points_dev_f64(append_to, f->px, f->py, f->pw, n);
            if (rc) return ffail(rc, std::string("append: ") + mac_last_error());
        }
        return MAC_OK;
    } catch (...) {
        return ffail(MAC_E_HIP, "unexpected exception");
    }
}

int32_t mac_fire_last_points(mac_fire* f, double* rec, int64_t cap, int64_t* n_out)
{
    if (!f || !n_out) return ffail(MAC_E_INVAL, "null argument");
    *n_out = f->last_n;
    const int64_t m = std::min(f->last_n, cap);
    if (!rec || m <= 0) return MAC_OK;
    FCK(hipSetDevice(f->device));
    std::vector<double> hx(m), hy(m), hw(m);
    FCK(hipMemcpy(hx.data(), f->px, 8 * m, hipMemcpyDeviceToHost));
    FCK(hipMemcpy(hy.data(), f->py, 8 * m, hipMemcpyDeviceToHost));
    FCK(hipMemcpy(hw.data(), f->pw, 8 * m, hipMemcpyDeviceToHost));
    for (int64_t q = 0; q < m; ++q) {
        rec[5 * q + 0] = hx[q];
        rec[5 * q + 1] = hy[q];
        rec[5 * q + 2] = hw[q];
        rec[5 * q + 3] = hw[q];
        rec[5 * q + 4] = 0.0;
    }
    return MAC_OK;
}

int32_t mac_fire_get_grid(mac_fire* f, uint8_t* out)
{
    if (!f || !out) return ffail(MAC_E_INVAL, "null argument");
    FCK(hipSetDevice(f->device));
    FCK(hipMemcpy(out, f->g, f->fc.nx * f->fc.ny, hipMemcpyDeviceToHost));
    return MAC_OK;
}

int32_t mac_fire_set_grid(mac_fire* f, const uint8_t* in)
{
    if (!f || !in) return ffail(MAC_E_INVAL, "null argument");
    FCK(hipSetDevice(f->device));
    FCK(hipMemcpy(f->g, in, f->fc.nx * f->fc.ny, hipMemcpyHostToDevice));
    return MAC_OK;
}

}  // extern "C"
