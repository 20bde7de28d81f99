// Probe: cycles per dependent v_add_f64 on gfx950, from registers and from LDS (the prep fold's
// shape: batches of 12 terms read as pairs). One workgroup of 64 threads, 8 lanes folding.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void chain_regs(const double* in, double* out, long long* cyc, int n)
{
    double t[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) t[j] = in[threadIdx.x * 16 + j];
    double acc = 0.0;
    const long long c0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int r = 0; r < n / 16; ++r) {
#pragma unroll
        for (int j = 0; j < 16; ++j) acc += t[j];
    }
    const long long c1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = c1 - c0;
}

template <int kB>
__global__ void chain_lds(const double* in, double* out, long long* cyc, int n)
{
    __shared__ __attribute__((aligned(16))) double term[8][512 + 2];
    for (int q = threadIdx.x; q < 8 * 512; q += blockDim.x) term[q / 512][q % 512] = in[q];
    __syncthreads();
    double acc = 0.0;
    const int u = threadIdx.x;
    long long c0 = 0, c1 = 0;
    if (u < 8) {
        c0 = __builtin_amdgcn_s_memtime();
        const double2* row2 = reinterpret_cast<const double2*>(&term[u][0]);
        const int nfull = n / (2 * kB);
        auto batch = [&](double2 (&buf)[kB], int bt) {
            const int at = (bt < nfull ? bt : nfull - 1) * kB;
#pragma unroll
            for (int j = 0; j < kB; ++j) buf[j] = row2[at + j];
        };
        auto add = [&](const double2 (&buf)[kB]) {
#pragma unroll
            for (int j = 0; j < kB; ++j) { acc += buf[j].x; acc += buf[j].y; }
        };
        double2 A[kB], B[kB];
        batch(A, 0);
#pragma unroll 1
        for (int bt = 0; bt < nfull; bt += 2) {
            batch(B, bt + 1);
            __builtin_amdgcn_sched_barrier(0);
            add(A);
            if (bt + 1 >= nfull) break;
            batch(A, bt + 2);
            __builtin_amdgcn_sched_barrier(0);
            add(B);
        }
        c1 = __builtin_amdgcn_s_memtime();
    }
    if (u < 8) out[u] = acc;
    if (u == 0) cyc[0] = c1 - c0;
}

int main()
{
    const int n = 504;  // 42 batches of 12
    double *in, *out;
    long long* cyc;
    hipMalloc(&in, sizeof(double) * 8 * 512);
    hipMalloc(&out, sizeof(double) * 64);
    hipMalloc(&cyc, sizeof(long long) * 4);
    double h[8 * 512];
    for (int i = 0; i < 8 * 512; ++i) h[i] = 0.001 * (i % 97) + 1e-7 * i;
    hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
    long long c = 0;
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(chain_regs, dim3(1), dim3(64), 0, 0, in, out, cyc, 512);
        hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("regs: %lld cycles for 512 adds = %.2f cyc/add\n", c, c / 512.0);
        hipLaunchKernelGGL(chain_lds<6>, dim3(1), dim3(64), 0, 0, in, out, cyc, n);
        hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("lds kB=6: %lld cycles for %d adds = %.2f cyc/add\n", c, n, c / (double)n);
        hipLaunchKernelGGL(chain_lds<12>, dim3(1), dim3(64), 0, 0, in, out, cyc, n);
        hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("lds kB=12: %lld cycles for %d adds = %.2f cyc/add\n", c, n, c / (double)n);
    }
    return 0;
}
