// Probe: can one launch carry a 12-KB candidate (N = 512 disks, 3N doubles) as its kernel
// arguments on this ROCm / gfx950, and what does a dependent launch cost that way against the
// pinned copy + launch the closure path uses? Prints one JSON line.
//   hipcc --offload-arch=gfx950 -O2 kernarg_probe.hip -o kernarg_probe && ./kernarg_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>

struct Cand { double v[1536]; };

// every workgroup reads the whole argument block (as the closure kernel stages the candidate)
__global__ void from_args(Cand c, double* out, unsigned long long* slot, unsigned long long seq)
{
    __shared__ double s[1536];
    for (int j = threadIdx.x; j < 1536; j += blockDim.x) s[j] = c.v[j];
    __syncthreads();
    double a = 0.0;
    for (int j = threadIdx.x; j < 1536; j += blockDim.x) a += s[j];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        out[0] = s[1535] + s[0];
        slot[0] = seq;
    }
    if (a == -1.0) out[1] = a;
}

__global__ void from_buf(const double* __restrict__ c, double* out, unsigned long long* slot,
                         unsigned long long seq)
{
    __shared__ double s[1536];
    for (int j = threadIdx.x; j < 1536; j += blockDim.x) s[j] = c[j];
    __syncthreads();
    double a = 0.0;
    for (int j = threadIdx.x; j < 1536; j += blockDim.x) a += s[j];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        out[0] = s[1535] + s[0];
        slot[0] = seq;
    }
    if (a == -1.0) out[1] = a;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("{\"error\": \"%s at %d\"}\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main()
{
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    double* out;
    double* dbuf;
    CK(hipMalloc(&out, 64));
    CK(hipMalloc(&dbuf, sizeof(Cand)));
    unsigned long long* hslot;
    CK(hipHostMalloc((void**)&hslot, 64, hipHostMallocMapped | hipHostMallocCoherent));
    unsigned long long* dslot;
    CK(hipHostGetDevicePointer((void**)&dslot, hslot, 0));
    Cand* hc;
    CK(hipHostMalloc((void**)&hc, sizeof(Cand), hipHostMallocDefault));
    Cand c;
    bool ok = true;
    auto wait = [&](unsigned long long seq) {
        while (__atomic_load_n(hslot, __ATOMIC_ACQUIRE) != seq) {}
    };
    const int iters = 2000;
    unsigned long long seq = 0;
    // correctness of the argument path
    for (int t = 0; t < 16; ++t) {
        for (int j = 0; j < 1536; ++j) c.v[j] = t * 1000.0 + j;
        hipLaunchKernelGGL(from_args, dim3(512), dim3(256), 0, s, c, out, dslot, ++seq);
        CK(hipGetLastError());
        CK(hipStreamSynchronize(s));
        double o = 0;
        CK(hipMemcpy(&o, out, 8, hipMemcpyDeviceToHost));
        ok = ok && o == c.v[1535] + c.v[0];
    }
    auto t0 = std::chrono::steady_clock::now();
    for (int t = 0; t < iters; ++t) {
        c.v[0] = t;
        hipLaunchKernelGGL(from_args, dim3(512), dim3(256), 0, s, c, out, dslot, ++seq);
        wait(seq);
    }
    auto t1 = std::chrono::steady_clock::now();
    for (int t = 0; t < iters; ++t) {
        hc->v[0] = t;
        CK(hipMemcpyAsync(dbuf, hc, sizeof(Cand), hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(from_buf, dim3(512), dim3(256), 0, s, (const double*)dbuf, out, dslot, ++seq);
        wait(seq);
    }
    auto t2 = std::chrono::steady_clock::now();
    CK(hipStreamSynchronize(s));
    const double a_us = std::chrono::duration<double, std::micro>(t1 - t0).count() / iters;
    const double b_us = std::chrono::duration<double, std::micro>(t2 - t1).count() / iters;
    printf("{\"args_12kb_ok\": %s, \"launch_with_args_us\": %.2f, \"copy_then_launch_us\": %.2f}\n",
           ok ? "true" : "false", a_us, b_us);
    return 0;
}
