// Probe: how large may a kernel's by-value argument be on this HIP runtime, what does the host pay
// to enqueue it, and how soon after launch does a kernel have it?  For the idea of passing a staged
// launch's candidate k-mers (cfg2: 2 x 500 x 4 B) in the kernel arguments instead of staging them.
//   hipcc -O3 --offload-arch=gfx950 tools/kernarg_probe.hip -o /tmp/kernarg_probe && /tmp/kernarg_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdint>

template <int N>
struct Arg {
    uint32_t v[N];
};

template <int N>
__global__ void sum_arg(Arg<N> a, uint32_t* out, uint64_t* t) {
    if (threadIdx.x == 0 && blockIdx.x == 0) t[0] = __builtin_amdgcn_s_memrealtime();
    uint32_t s = 0;
    for (int i = threadIdx.x; i < N; i += blockDim.x) s += a.v[i];
    atomicAdd(out, s);
    if (threadIdx.x == 0 && blockIdx.x == 0) t[1] = __builtin_amdgcn_s_memrealtime();
}

template <int N>
void run(uint32_t* d_out, uint64_t* d_t, hipStream_t st) {
    static Arg<N> a;
    uint64_t want = 0;
    for (int i = 0; i < N; ++i) {
        a.v[i] = (uint32_t)(i * 2654435761u);
        want += a.v[i];
    }
    const int reps = 200;
    double enq = 0;
    for (int r = 0; r < reps + 10; ++r) {
        (void)hipMemsetAsync(d_out, 0, 4, st);
        auto t0 = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(sum_arg<N>, dim3(1024), dim3(256), 0, st, a, d_out, d_t);
        auto t1 = std::chrono::steady_clock::now();
        if (r >= 10) enq += std::chrono::duration<double, std::micro>(t1 - t0).count();
        (void)hipStreamSynchronize(st);
    }
    hipError_t e = hipGetLastError();
    uint32_t got = 0;
    uint64_t tt[2];
    (void)hipMemcpy(&got, d_out, 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(tt, d_t, 16, hipMemcpyDeviceToHost);
    std::printf("arg %6zu B: %s, enqueue %.2f us, sum %s, first wave in-kernel %.2f us\n", sizeof(Arg<N>),
                hipGetErrorString(e), enq / reps, got == (uint32_t)(want * 1024) ? "ok" : "WRONG",
                (tt[1] - tt[0]) / 100.0);
}

int main() {
    uint32_t* d_out;
    uint64_t* d_t;
    hipStream_t st;
    (void)hipMalloc(&d_out, 4);
    (void)hipMalloc(&d_t, 16);
    (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    run<16>(d_out, d_t, st);
    run<256>(d_out, d_t, st);
    run<512>(d_out, d_t, st);
    run<1000>(d_out, d_t, st);
    run<1024>(d_out, d_t, st);
    run<2048>(d_out, d_t, st);
    run<4096>(d_out, d_t, st);
    return 0;
}
