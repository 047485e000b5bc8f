// Probe (GPU box, one-off measurement): can the host pack straight into device memory?
// A fine-grained device allocation (hipExtMallocWithFlags, hipDeviceMallocFinegrained) is
// mapped into the host through the PCIe BAR; host stores to it are posted PCIe writes (no
// round trip), unlike the count kernel's staging copy, whose PCIe reads of the pinned block
// move ~320 KB in 13-19 us (profiles/r03_m1/stamps.log).  Measures (1) host write bandwidth
// into it, 1 and 8 threads; (2) whether a kernel that already read the region (lines in its
// L2) sees the host's new data after a host flag, with plain loads, after an acquire fence at
// system scope, and with nontemporal loads; (3) the kernel's read time of that memory against
// ordinary device memory.  Build: hipcc -O2 --offload-arch=gfx950 -Xarch_host -mavx512f tools/bar_probe.hip -o bar_probe
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <signal.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                              \
        }                                                                              \
    } while (0)

static const size_t WORDS = 160 * 1024;  // 640 KB: one cfg2 read end is ~324 KB, both ~650 KB

static void on_segv(int) {
    const char m[] = "host access to the fine-grained device allocation: SIGSEGV\n";
    (void)!write(2, m, sizeof(m) - 1);
    _exit(3);
}

// mode 0: plain loads; 1: system-scope acquire fence after the flag; 2: nontemporal loads (modes 0-2
// read the region before waiting, so their L2 holds the old lines); 3: plain loads, no read of the
// region in this launch before the flag (an earlier launch read it) -- the early-launch stage's case
__global__ void check_kernel(const uint32_t* buf, uint32_t n, const uint32_t* flag, uint32_t want, uint32_t* bad,
                             uint32_t* seen_ticks, int mode) {
    const uint32_t i0 = blockIdx.x * blockDim.x + threadIdx.x, stride = gridDim.x * blockDim.x;
    uint32_t sink = 0;
    if (mode != 3)
        for (uint32_t i = i0; i < n; i += stride) sink += buf[i];  // pull the old lines into L2 / L1
    if (sink == 0xfffffffeu) bad[1] = sink;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t f = 0;
    while ((f = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) != want) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {  // 1 s
            if (threadIdx.x == 0) atomicAdd(bad + 2, 1u);
            return;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    if (mode == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    uint32_t wrong = 0;
    for (uint32_t i = i0; i < n; i += stride) {
        const uint32_t v = mode == 2 ? __builtin_nontemporal_load(buf + i) : buf[i];
        wrong += v != want + i;
    }
    if (wrong) atomicAdd(bad, wrong);
    if (i0 == 0) *seen_ticks = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t0);
}

__global__ void read_kernel(const uint32_t* buf, uint32_t n, uint32_t passes, uint32_t* out) {
    uint32_t s = 0;
    for (uint32_t p = 0; p < passes; ++p)
        for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) s += buf[i] ^ p;
    if (s == 0x12345u) *out = s;
}

static void host_fill(uint32_t* dst, uint32_t v, size_t lo, size_t hi) {
    // 64-byte streaming stores, as the packer would write (full PCIe write requests)
    size_t i = lo;
    for (; i + 16 <= hi; i += 16) {
        __m512i x = _mm512_add_epi32(_mm512_set1_epi32((int)(v + i)), _mm512_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15));
        _mm512_stream_si512((__m512i*)(dst + i), x);
    }
    for (; i < hi; ++i) dst[i] = v + (uint32_t)i;
    _mm_sfence();
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    signal(SIGSEGV, on_segv);
    signal(SIGBUS, on_segv);
    uint32_t *fg = nullptr, *cg = nullptr;
    CK(hipExtMallocWithFlags((void**)&fg, WORDS * 4, hipDeviceMallocFinegrained));
    CK(hipMalloc((void**)&cg, WORDS * 4));
    uint32_t *flag = nullptr, *bad = nullptr;
    CK(hipHostMalloc((void**)&flag, 4096, hipHostMallocCoherent | hipHostMallocMapped));
    CK(hipHostMalloc((void**)&bad, 4096, hipHostMallocCoherent | hipHostMallocMapped));
    uint32_t *flag_d = nullptr, *bad_d = nullptr;
    CK(hipHostGetDevicePointer((void**)&flag_d, flag, 0));
    CK(hipHostGetDevicePointer((void**)&bad_d, bad, 0));
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, fg) != hipSuccess) {
        std::printf("fine-grained allocation: no pointer attributes; not probing host stores\n");
        return 0;
    }
    std::printf("fine-grained allocation: type %d device %d host pointer %p device pointer %p\n", (int)at.type,
                at.device, at.hostPointer, at.devicePointer);
    // Refuse rather than fault: without a host mapping of the allocation (hostPointer NULL,
    // as on some boxes of this pool, profiles/r03_bar_probe.log) a host store to it is not a BAR write.
    if (!at.hostPointer) {
        std::printf("no host mapping of the device allocation on this box: host writes into device memory "
                    "are not available here; nothing probed\n");
        return 0;
    }

    // (1) host write bandwidth
    fg[0] = 7;
    std::printf("host store + load back: %u\n", fg[0]);
    for (int threads : {1, 4, 8}) {
        std::vector<double> t;
        for (int r = 0; r < 50; ++r) {
            const double a = now_us();
            std::vector<std::thread> th;
            for (int q = 0; q < threads; ++q)
                th.emplace_back(host_fill, fg, (uint32_t)r, WORDS * q / threads, WORDS * (q + 1) / threads);
            for (auto& x : th) x.join();
            t.push_back(now_us() - a);
        }
        std::sort(t.begin(), t.end());
        std::printf("host write %zu KB into device memory, %d thread(s): p50 %.1f us (%.1f GB/s), p10 %.1f us\n",
                    WORDS * 4 / 1024, threads, t[t.size() / 2], WORDS * 4 / t[t.size() / 2] / 1e3, t[t.size() / 10]);
    }
    {  // persistent threads (no spawn inside the timed region), 1-16 writers, 64-B streaming stores
        for (int threads : {1, 2, 4, 8, 12}) {
            std::atomic<int> go{0}, done{0};
            std::atomic<bool> quit{false};
            std::vector<std::thread> th;
            for (int q = 0; q < threads; ++q)
                th.emplace_back([&, q] {
                    int seen = 0;
                    for (;;) {
                        int g;
                        while ((g = go.load(std::memory_order_acquire)) == seen)
                            if (quit.load(std::memory_order_relaxed)) return;
                        seen = g;
                        host_fill(fg, (uint32_t)g, WORDS * q / threads, WORDS * (q + 1) / threads);
                        done.fetch_add(1, std::memory_order_acq_rel);
                    }
                });
            std::vector<double> t;
            for (int r = 1; r <= 60; ++r) {
                done.store(0);
                const double a = now_us();
                go.store(r, std::memory_order_release);
                while (done.load(std::memory_order_acquire) != threads) {}
                t.push_back(now_us() - a);
            }
            quit.store(true);
            for (auto& x : th) x.join();
            std::sort(t.begin() + 10, t.end());
            const double p50 = t[10 + (t.size() - 10) / 2];
            std::printf("persistent writers: %2d thread(s), %zu KB into device memory: p50 %.1f us (%.1f GB/s), best %.1f us\n",
                        threads, WORDS * 4 / 1024, p50, WORDS * 4 / p50 / 1e3, t[10]);
        }
    }
    {  // the same into pinned host memory, for scale
        uint32_t* hp = nullptr;
        CK(hipHostMalloc((void**)&hp, WORDS * 4, hipHostMallocDefault));
        std::vector<double> t;
        for (int r = 0; r < 50; ++r) {
            const double a = now_us();
            host_fill(hp, (uint32_t)r, 0, WORDS);
            t.push_back(now_us() - a);
        }
        std::sort(t.begin(), t.end());
        std::printf("host write %zu KB into pinned host memory, 1 thread: p50 %.1f us\n", WORDS * 4 / 1024, t[t.size() / 2]);
        CK(hipHostFree(hp));
    }

    // (2) visibility of host writes to a kernel that has the old lines cached
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint32_t* ticks = bad + 16;
    for (int mode = 0; mode < 4; ++mode) {
        uint32_t total_bad = 0, timeouts = 0;
        double tick_sum = 0;
        const int iters = mode == 3 ? 1000 : 200;
        for (int it = 1; it <= iters; ++it) {
            const uint32_t want = (uint32_t)(mode * 100000 + it * 1000);
            __atomic_store_n(bad, 0u, __ATOMIC_RELEASE);
            __atomic_store_n(bad + 2, 0u, __ATOMIC_RELEASE);
            __atomic_store_n(flag, 0u, __ATOMIC_RELEASE);
            if (mode == 3)  // the lines pulled into L2 by an earlier launch; the checking launch reads only after the flag
                hipLaunchKernelGGL(read_kernel, dim3(512), dim3(256), 0, s, fg, (uint32_t)WORDS, 2u, bad_d + 32);
            hipLaunchKernelGGL(check_kernel, dim3(512), dim3(256), 0, s, fg, (uint32_t)WORDS, flag_d, want, bad_d,
                               ticks, mode);
            CK(hipGetLastError());
            const double a = now_us();
            while (now_us() - a < 40.0) {}  // let the kernel pull the old lines in
            std::vector<std::thread> th;
            for (int q = 0; q < 8; ++q) th.emplace_back(host_fill, fg, want, WORDS * q / 8, WORDS * (q + 1) / 8);
            for (auto& x : th) x.join();
            __atomic_store_n(flag, want, __ATOMIC_RELEASE);
            CK(hipStreamSynchronize(s));
            total_bad += __atomic_load_n(bad, __ATOMIC_ACQUIRE);
            timeouts += __atomic_load_n(bad + 2, __ATOMIC_ACQUIRE);
            tick_sum += __atomic_load_n(ticks, __ATOMIC_ACQUIRE);
        }
        std::printf("visibility mode %d (%s): %u stale words over %d iterations, %u timeouts, flag wait %.1f us avg\n",
                    mode, mode == 0 ? "plain loads" : mode == 1 ? "system acquire" : mode == 2 ? "nontemporal loads" : "no read before the flag in this launch, plain loads", total_bad,
                    iters, timeouts, tick_sum / iters / 100.0);
    }

    // (3) kernel read time: fine-grained vs ordinary device memory
    uint32_t* out = nullptr;
    CK(hipMalloc((void**)&out, 64));
    CK(hipMemset(cg, 1, WORDS * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int rep = 0; rep < 2; ++rep)
        for (int which = 0; which < 2; ++which) {
            const uint32_t* b = which ? fg : cg;
            hipLaunchKernelGGL(read_kernel, dim3(2048), dim3(256), 0, s, b, (uint32_t)WORDS, 64u, out);
            CK(hipEventRecord(e0, s));
            for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(read_kernel, dim3(2048), dim3(256), 0, s, b, (uint32_t)WORDS, 64u, out);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            std::printf("read 64 x %zu KB from %s memory: %.1f us per launch\n", WORDS * 4 / 1024,
                        which ? "fine-grained" : "ordinary device", ms * 100.0);
        }
    std::printf("done\n");
    return 0;
}
