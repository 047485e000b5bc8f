// Stress test of the host work pool (approx_counter_amd/csrc/host_pack.cpp), CPU only:
// many back-to-back run() / begin-help-finish calls of varying sizes, every task must run exactly once per
// call, with the workers' spin time short enough that they also sleep and wake.
//   pool_stress THREADS CALLS [CALLERS] [HOGS] [PIN]
// CALLERS threads drive the one pool at once (contexts on several threads share host_pool(); a call
// must hold the pool for its whole begin .. finish), HOGS threads spin on the same CPUs to stand in for
// other tenants' load (workers get descheduled mid-task), PIN = 1 pins worker i to CPU i % ncpu as the
// library's plan does.  Built and run by tests/test_host_pool.py; exit status 0 = every check passed.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "host_pack.h"

int main(int argc, char** argv) {
    const unsigned threads = argc > 1 ? (unsigned)std::atoi(argv[1]) : 8;
    const int calls = argc > 2 ? std::atoi(argv[2]) : 20000;
    const unsigned callers = argc > 3 ? (unsigned)std::max(1, std::atoi(argv[3])) : 1u;
    const unsigned hogs = argc > 4 ? (unsigned)std::atoi(argv[4]) : 0u;
    const bool pin = argc > 5 && std::atoi(argv[5]) != 0;
    std::vector<int> cpus;
    if (pin) {
        const unsigned ncpu = std::max(1u, std::thread::hardware_concurrency());
        for (unsigned i = 0; i < threads; ++i) cpus.push_back((int)(i % ncpu));
    }
    acamd::WorkPool pool(threads, cpus, true);
    std::atomic<bool> stop{false};
    std::vector<std::thread> hog;
    for (unsigned h = 0; h < hogs; ++h)
        hog.emplace_back([&] {
            volatile uint64_t x = 0;
            while (!stop.load(std::memory_order_relaxed)) x = x + 1;
        });
    std::atomic<int> bad{0};
    std::atomic<uint64_t> total{0};
    auto drive = [&](unsigned who) {
        std::vector<std::atomic<uint32_t>> hits(4096);
        for (int c = 0; c < calls && !bad.load(std::memory_order_relaxed); ++c) {
            const uint32_t n = (uint32_t)(((c + 7 * who) * 2654435761u) % 257u);  // 0..256 tasks, 0 and 1 included
            for (uint32_t i = 0; i < n; ++i) hits[i].store(0, std::memory_order_relaxed);
            const std::function<void(uint32_t)> fn = [&](uint32_t i) { hits[i].fetch_add(1, std::memory_order_relaxed); };
            if (c % 3 == 0) {
                pool.run(n, fn);
            } else {  // the stepwise form, as the host-buffer stage uses it: help with prefixes, then finish
                pool.begin(n, fn);
                pool.help(n / 3);
                pool.help(n / 2);
                pool.finish();
            }
            for (uint32_t i = 0; i < n; ++i)
                if (hits[i].load(std::memory_order_relaxed) != 1) {
                    std::fprintf(stderr, "caller %u call %d: task %u ran %u times (n = %u)\n", who, c, i, hits[i].load(), n);
                    bad.store(1);
                    return;
                }
            total.fetch_add(n, std::memory_order_relaxed);
        }
    };
    std::vector<std::thread> drivers;
    for (unsigned w = 1; w < callers; ++w) drivers.emplace_back(drive, w);
    drive(0);
    for (std::thread& t : drivers) t.join();
    stop.store(true);
    for (std::thread& t : hog) t.join();
    if (bad.load()) return 1;
    std::printf("ok: %d calls x %u callers, %llu tasks, %u participants, %u hogs%s\n", calls, callers,
                (unsigned long long)total.load(), pool.size(), hogs, pin ? ", pinned" : "");
    return 0;
}
