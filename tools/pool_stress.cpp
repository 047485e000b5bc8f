// Stress test of the host work pool (approx_counter_amd/csrc/host_pack.cpp), CPU only:
// many back-to-back run() / begin-help-finish calls of varying sizes, every task must run exactly once per
// call, with the workers' spin time short enough that they also sleep and wake.
// Built and run by tests/test_host_pool.py; exit status 0 = every check passed.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "host_pack.h"

int main(int argc, char** argv) {
    const unsigned threads = argc > 1 ? (unsigned)std::atoi(argv[1]) : 8;
    const int calls = argc > 2 ? std::atoi(argv[2]) : 20000;
    acamd::WorkPool pool(threads);
    std::vector<std::atomic<uint32_t>> hits(4096);
    uint64_t total = 0;
    for (int c = 0; c < calls; ++c) {
        const uint32_t n = (uint32_t)((c * 2654435761u) % 257u);  // 0..256 tasks, 0 and 1 included
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
                std::fprintf(stderr, "call %d: task %u ran %u times (n = %u)\n", c, i, hits[i].load(), n);
                return 1;
            }
        total += n;
    }
    std::printf("ok: %d calls, %llu tasks, %u participants\n", calls, (unsigned long long)total, pool.size());
    return 0;
}
