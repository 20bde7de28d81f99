// closure_threads.cpp — measurement helper (not part of the C-ABI): T native host threads call
// the single-candidate closure mac_area_f64 at once for a fixed time, as DirectSearch's threaded
// poll does (src/TDM_STATIC_opt.jl:129: one objective call per trial point per thread). Python
// threads cannot measure this (ctypes re-takes the GIL around every call), so bench.py loads this
// library and passes it libmaxcover's mac_area_f64. Thread t evaluates candidates t, t + T, ...
// (column-major 3N x K, candidate k at cands + k * three_n) and counts results that differ from
// want[k].
#include <atomic>
#include <chrono>
#include <cstdint>
#include <thread>
#include <vector>

typedef int32_t (*area_fn)(void* ctx, const double* circles, int64_t three_n, double* area_out);

extern "C" double mac_closure_threads(void* fn, void* ctx, const double* cands, int64_t K,
                                      int64_t three_n, const double* want, int32_t threads,
                                      double seconds, int64_t* calls, int64_t* mismatches,
                                      int64_t* failures)
{
    area_fn f = reinterpret_cast<area_fn>(fn);
    std::atomic<int64_t> ncall{0}, nbad{0}, nfail{0};
    std::atomic<int> ready{0};
    std::atomic<bool> go{false}, stop{false};
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t) {
        th.emplace_back([&, t]() {
            ready.fetch_add(1);
            while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
            int64_t k = t % K, n = 0, bad = 0, fail = 0;
            while (!stop.load(std::memory_order_relaxed)) {
                double a = 0.0;
                if (f(ctx, cands + k * three_n, three_n, &a) != 0) ++fail;
                else if (a != want[k]) ++bad;
                ++n;
                k += threads;
                if (k >= K) k = t % K;
            }
            ncall.fetch_add(n);
            nbad.fetch_add(bad);
            nfail.fetch_add(fail);
        });
    }
    while (ready.load() < threads) std::this_thread::yield();
    const auto t0 = std::chrono::steady_clock::now();
    go.store(true, std::memory_order_release);
    std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
    stop.store(true);
    for (auto& h : th) h.join();
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    *calls = ncall.load();
    *mismatches = nbad.load();
    *failures = nfail.load();
    return dt;
}
