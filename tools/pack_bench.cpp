// Host-side latency of the stage's packing (host_pack.cpp), CPU only: two jobs (read ends)
// of n Dna5 windows (100 / 101 bases) packed by the pool the way ac_error_count_jobs does
// (tasks in job order, the caller helping), timing when job 0 and job 1 are complete.
//   g++ -O3 -std=c++17 -pthread -Iapprox_counter_amd/csrc tools/pack_bench.cpp \
//       approx_counter_amd/csrc/host_pack.cpp -o /tmp/pack_bench && /tmp/pack_bench [n] [iters] [per] [records]
// AC_PACK_CPUS=<cpulist> pins the pool to those CPUs (a rank's share of the host, as ac_plan_host_cpus
// plans it; tools/pack8.py runs eight such processes at once); AC_HOST_THREADS sizes the pool.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "host_pack.h"

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 10000;
    const int iters = argc > 2 ? std::atoi(argv[2]) : 2000;
    const uint32_t per_arg = argc > 3 ? (uint32_t)std::atoi(argv[3]) : 0;
    // records = 1: the stage's equal-window form (inline N records, no descriptors), 0.1 % N bases
    const bool records = argc > 4 ? std::atoi(argv[4]) != 0 : true;
    if (const char* c = std::getenv("AC_PACK_CPUS")) {
        acamd::HostPlan plan;
        plan.cpus = acamd::parse_cpulist(c);
        (void)acamd::set_host_plan(plan);
    }
    acamd::WorkPool& pool = acamd::host_pool();
    std::mt19937 rng(1);
    struct Job {
        std::vector<uint8_t> bases;
        std::vector<uint64_t> off;
        std::vector<uint32_t> len;
        std::vector<uint32_t> codes, nmask;
        std::vector<uint64_t> st;
        std::vector<uint32_t> ln;
    } job[2];
    for (int j = 0; j < 2; ++j) {
        const uint32_t L = 100 + j;
        job[j].bases.resize((size_t)n * L);
        for (auto& b : job[j].bases) b = (rng() % 1000u == 0u) ? 4u : (uint8_t)(rng() & 3u);
        for (uint32_t i = 0; i < n; ++i) {
            job[j].off.push_back((uint64_t)i * L);
            job[j].len.push_back(L);
        }
        job[j].codes.assign((size_t)n * 128 / 16, 0);
        job[j].nmask.assign((size_t)n * 128 / 32, 0);
        job[j].st.assign(n, 0);
        job[j].ln.assign(n, 0);
    }
    const uint32_t per = per_arg ? per_arg : std::max<uint32_t>(256, 2 * n / (4 * pool.size()) + 1);
    struct Task {
        uint32_t j, w0, w1;
    };
    std::vector<Task> tasks;
    for (uint32_t j = 0; j < 2; ++j)
        for (uint32_t w = 0; w < n; w += per) tasks.push_back({j, w, std::min(n, w + per)});
    const uint32_t t_split = (uint32_t)std::count_if(tasks.begin(), tasks.end(), [](const Task& t) { return t.j == 0; });
    std::vector<double> d0, d1;
    for (int it = 0; it < iters; ++it) {
        std::atomic<uint32_t> left[2];
        left[0] = t_split;
        left[1] = (uint32_t)tasks.size() - t_split;
        const std::function<void(uint32_t)> fn = [&](uint32_t t) {
            const Task& x = tasks[t];
            Job& b = job[x.j];
            acamd::pack_dna5_range(b.bases.data(), b.off.data(), b.len.data(), x.w0, x.w1, (uint64_t)x.w0 * 128,
                                   b.codes.data(), b.nmask.data(), b.st.data() + x.w0, b.ln.data() + x.w0, records);
            left[x.j].fetch_sub(1, std::memory_order_release);
        };
        const double t0 = now_us();
        pool.begin((uint32_t)tasks.size(), fn);
        pool.help(t_split);
        while (left[0].load(std::memory_order_acquire)) __builtin_ia32_pause();
        const double t1 = now_us();
        pool.help((uint32_t)tasks.size());
        while (left[1].load(std::memory_order_acquire)) __builtin_ia32_pause();
        pool.finish();
        const double t2 = now_us();
        if (it >= iters / 10) {
            d0.push_back(t1 - t0);
            d1.push_back(t2 - t0);
        }
        // a GPU-stage-like gap between calls
        const double g = now_us();
        while (now_us() - g < 120.0) __builtin_ia32_pause();
    }
    std::sort(d0.begin(), d0.end());
    std::sort(d1.begin(), d1.end());
    auto q = [](const std::vector<double>& v, double f) { return v[(size_t)(f * (v.size() - 1))]; };
    std::printf("participants %u, %zu tasks of %u windows, n=%u per job, records %d\n", pool.size(), tasks.size(), per,
                n, (int)records);
    std::printf("job 0 packed: p10 %.1f p50 %.1f p90 %.1f max %.1f us\n", q(d0, .1), q(d0, .5), q(d0, .9), d0.back());
    std::printf("both packed:  p10 %.1f p50 %.1f p90 %.1f max %.1f us\n", q(d1, .1), q(d1, .5), q(d1, .9), d1.back());
    std::printf("{\"participants\": %u, \"n\": %u, \"both_p50_us\": %.2f, \"both_p90_us\": %.2f, \"both_max_us\": %.2f, "
                "\"job0_p50_us\": %.2f}\n", pool.size(), n, q(d1, .5), q(d1, .9), d1.back(), q(d0, .5));
    return 0;
}
