// Probe: can the host write a closure candidate (N = 512 disks, 3N doubles = 12 KB) straight into
// device memory (fine-grained VRAM through the BAR), so that a closure call is one launch with no
// host-to-device copy? For each allocation kind: its pointer attributes; where the host can reach
// it, R rounds of {host writes the candidate with a round-dependent pattern, fence, launch a
// 128-workgroup kernel whose every workgroup checks the whole candidate, wait for its mapped slot}
// against the pinned staging + hipMemcpyAsync + launch the closure path uses. Prints JSON lines;
// a nonzero "mismatches" means the device saw stale data (then the kind is unusable).
//   hipcc --offload-arch=gfx950 -O2 vram_probe.hip -o vram_probe && ./vram_probe
#include <hip/hip_runtime.h>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <immintrin.h>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    std::printf("{\"error\": \"%s\", \"at\": %d}\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int kN = 1536;   // 3N doubles, N = 512
constexpr int kWG = 128;   // the closure kernel's workgroups for N = 512

__device__ inline double pat(unsigned long long r, int j) { return (double)((r * 2654435761ull + j) & 0xfffff); }

// every workgroup stages the whole candidate in LDS and counts entries that differ from round r's
// pattern; the last workgroup to arrive writes {mismatches, r} to the mapped host slot
__global__ __launch_bounds__(256) void check(const double* c, unsigned long long r, unsigned* arrive,
                                             unsigned* bad, volatile unsigned long long* slot)
{
    __shared__ double s[kN];
    __shared__ unsigned wbad;
    if (threadIdx.x == 0) wbad = 0;
    for (int j = threadIdx.x; j < kN; j += blockDim.x) s[j] = c[j];
    __syncthreads();
    unsigned b = 0;
    for (int j = threadIdx.x; j < kN; j += blockDim.x) b += s[j] != pat(r, j);
    if (b) atomicAdd(&wbad, b);
    __syncthreads();
    if (threadIdx.x == 0) {
        if (wbad) atomicAdd(bad, wbad);
        __threadfence();
        if (atomicAdd(arrive, 1u) == gridDim.x - 1) {
            const unsigned tb = atomicAdd(bad, 0u);
            *arrive = 0;
            *bad = 0;
            __threadfence_system();
            slot[0] = tb;
            __threadfence_system();
            slot[1] = r;
        }
    }
}

static void host_fill(double* h, unsigned long long r)
{
    for (int j = 0; j < kN; ++j) h[j] = (double)((r * 2654435761ull + j) & 0xfffff);
}

int main(int argc, char** argv)
{
    const int R = argc > 1 ? std::atoi(argv[1]) : 20000;
    CK(hipSetDevice(0));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    unsigned *arrive, *bad;
    CK(hipMalloc(&arrive, 4));
    CK(hipMalloc(&bad, 4));
    CK(hipMemset(arrive, 0, 4));
    CK(hipMemset(bad, 0, 4));
    unsigned long long* hslot;
    CK(hipHostMalloc(&hslot, 64, hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(hslot, 0, 64);
    unsigned long long* dslot;
    CK(hipHostGetDevicePointer((void**)&dslot, hslot, 0));
    const size_t bytes = sizeof(double) * kN;

    auto wait = [&](unsigned long long r) {
        const auto t0 = std::chrono::steady_clock::now();
        while (__atomic_load_n(&hslot[1], __ATOMIC_ACQUIRE) != r) {
            _mm_pause();
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > 0.5) return false;
        }
        return true;
    };

    // the closure path's way: pinned staging, hipMemcpyAsync, launch
    {
        double* h;
        double* d;
        CK(hipHostMalloc(&h, bytes, 0));
        CK(hipMalloc(&d, bytes));
        unsigned long long mism = 0, lost = 0;
        double t_enq = 0;
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 1; i <= R; ++i) {
            host_fill(h, (unsigned long long)i);
            const auto a = std::chrono::steady_clock::now();
            CK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s));
            hipLaunchKernelGGL(check, dim3(kWG), dim3(256), 0, s, d, (unsigned long long)i, arrive, bad, dslot);
            t_enq += std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count();
            if (!wait((unsigned long long)i)) { ++lost; CK(hipStreamSynchronize(s)); }
            mism += hslot[0] != 0;
        }
        const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        std::printf("{\"kind\": \"pinned+memcpyAsync\", \"rounds\": %d, \"us_per_round\": %.2f, \"enqueue_us\": %.2f, "
                    "\"mismatches\": %llu, \"lost\": %llu}\n", R, dt / R * 1e6, t_enq / R * 1e6, mism, lost);
        CK(hipHostFree(h));
        CK(hipFree(d));
    }

    struct Kind { const char* name; int how; };
    const Kind kinds[] = {{"hipExtMallocWithFlags(fine-grained)", 0}, {"hipMalloc", 1},
                          {"hipExtMallocWithFlags(uncached)", 2}};
    for (const Kind& k : kinds) {
        void* d = nullptr;
        hipError_t e = k.how == 0 ? hipExtMallocWithFlags(&d, bytes, hipDeviceMallocFinegrained)
                     : k.how == 1 ? hipMalloc(&d, bytes)
                                  : hipExtMallocWithFlags(&d, bytes, hipDeviceMallocUncached);
        if (e != hipSuccess) {
            std::printf("{\"kind\": \"%s\", \"alloc\": \"%s\"}\n", k.name, hipGetErrorString(e));
            continue;
        }
        hipPointerAttribute_t at{};
        e = hipPointerGetAttributes(&at, d);
        std::printf("{\"kind\": \"%s\", \"attr\": \"%s\", \"type\": %d, \"device_ptr\": \"%p\", \"host_ptr\": \"%p\", "
                    "\"is_managed\": %d}\n", k.name, hipGetErrorString(e), (int)at.type, at.devicePointer,
                    at.hostPointer, (int)at.isManaged);
        double* h = (double*)at.hostPointer;
        // "touch": try the device address itself from the host (unified addressing over a large
        // BAR); a segfault here answers "no" (run this mode last, nothing after it on the GPU)
        if (!h && k.how == 0 && std::getenv("VRAM_TOUCH")) {
            std::printf("{\"touch\": \"writing %p from the host\"}\n", d);
            std::fflush(stdout);
            ((volatile double*)d)[0] = 42.0;
            _mm_sfence();
            double back = 0.0;
            CK(hipMemcpy(&back, d, sizeof(double), hipMemcpyDeviceToHost));
            std::printf("{\"touch\": \"ok\", \"read_back\": %g}\n", back);
            h = (double*)d;
        }
        if (e != hipSuccess || !h) {
            CK(hipFree(d));
            continue;
        }
        unsigned long long mism = 0, lost = 0;
        double t_fill = 0, t_enq = 0;
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 1; i <= R; ++i) {
            const auto a = std::chrono::steady_clock::now();
            host_fill(h, (unsigned long long)i);   // straight into device memory
            _mm_sfence();
            const auto b = std::chrono::steady_clock::now();
            hipLaunchKernelGGL(check, dim3(kWG), dim3(256), 0, s, (const double*)d, (unsigned long long)i, arrive,
                               bad, dslot);
            t_fill += std::chrono::duration<double>(b - a).count();
            t_enq += std::chrono::duration<double>(std::chrono::steady_clock::now() - b).count();
            if (!wait((unsigned long long)i)) { ++lost; CK(hipStreamSynchronize(s)); }
            mism += hslot[0] != 0;
        }
        const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        std::printf("{\"kind\": \"%s\", \"rounds\": %d, \"us_per_round\": %.2f, \"host_fill_us\": %.2f, "
                    "\"enqueue_us\": %.2f, \"mismatches\": %llu, \"lost\": %llu}\n", k.name, R, dt / R * 1e6,
                    t_fill / R * 1e6, t_enq / R * 1e6, mism, lost);
        CK(hipFree(d));
    }
    CK(hipStreamSynchronize(s));
    return 0;
}
