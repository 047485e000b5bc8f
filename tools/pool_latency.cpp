// Call latency of the host work pool under CPU contention (CPU only): `threads`
// participants run calls of 64 tasks of ~task_us each (the cfg2 stage's packing:
// ~4 tasks per participant, 2-4 us each), while `hogs` busy threads compete for the
// first CPUs of the pool's set.  Pin modes: "each" (worker i on one CPU, round 2),
// "set" (every worker on the whole set), "none".  Prints the per-call latency
// distribution; a worker descheduled while it holds a task shows as max >> p50.
//   g++ -O2 -std=c++17 -pthread -Iapprox_counter_amd/csrc tools/pool_latency.cpp \
//       approx_counter_amd/csrc/host_pack.cpp -o /tmp/pool_latency
//   /tmp/pool_latency <threads> <calls> <each|set|none> <hogs> [task_us]
#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "host_pack.h"

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const unsigned threads = argc > 1 ? (unsigned)std::atoi(argv[1]) : 8;
    const int calls = argc > 2 ? std::atoi(argv[2]) : 5000;
    const char* mode = argc > 3 ? argv[3] : "each";
    const int hogs = argc > 4 ? std::atoi(argv[4]) : 0;
    const double task_us = argc > 5 ? std::atof(argv[5]) : 3.0;
    std::vector<int> cpus;
    for (unsigned c = 0; c < threads; ++c) cpus.push_back((int)c);
    const bool none = std::strcmp(mode, "none") == 0;
    acamd::WorkPool pool(threads, none ? std::vector<int>{} : cpus, std::strcmp(mode, "each") == 0);
    // the caller on the last CPU of the set (as the stage's calling thread is unpinned, leave it)
    std::atomic<bool> stop{false};
    std::vector<std::thread> hog;
    for (int h = 0; h < hogs; ++h) {
        hog.emplace_back([&] {
            while (!stop.load(std::memory_order_relaxed)) {
            }
        });
        cpu_set_t s;
        CPU_ZERO(&s);
        CPU_SET(h % threads, &s);  // the first CPUs of the pool's set
        pthread_setaffinity_np(hog.back().native_handle(), sizeof s, &s);
    }
    const std::function<void(uint32_t)> fn = [&](uint32_t) {
        const double t = now_us();
        while (now_us() - t < task_us) {
        }
    };
    std::vector<double> lat;
    for (int c = 0; c < calls; ++c) {
        const double t = now_us();
        pool.run(64, fn);
        lat.push_back(now_us() - t);
        const double g = now_us();
        while (now_us() - g < 100.0) {
        }
    }
    stop = true;
    for (auto& h : hog) h.join();
    std::sort(lat.begin(), lat.end());
    auto q = [&](double f) { return lat[(size_t)(f * (lat.size() - 1))]; };
    std::printf("%s pin, %u participants, %d hogs: p50 %.1f p99 %.1f p99.9 %.1f max %.1f us (max/p50 %.1f)\n", mode,
                threads, hogs, q(.5), q(.99), q(.999), lat.back(), lat.back() / q(.5));
    return 0;
}
