// ubench_chain.hip -- dependent-issue cost of full-rate VALU ops on gfx950.
//
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_chain.hip -o build/ubench_chain && build/ubench_chain
//
// Each wave runs C independent chains of v_bitop3_b32 (each instruction reads
// the previous result of its chain), interleaved round-robin, at W waves per
// SIMD.  cycles/instr per SIMD (in-kernel clock) shows how many waves x chains
// it takes to hide the dependent-issue latency.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e = (x);                                                               \
        if (e != hipSuccess) {                                                            \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            std::exit(1);                                                                 \
        }                                                                                 \
    } while (0)

constexpr int N_INSTR = 16384;  // instructions per wave

template <int C>
__global__ __launch_bounds__(256) void chain(uint32_t* out, unsigned long long* clk, uint32_t seed) {
    uint32_t r[C];
    uint32_t a = seed ^ threadIdx.x, b = seed * 7u + blockIdx.x;
#pragma unroll
    for (int c = 0; c < C; ++c) r[c] = a + c;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long w0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < N_INSTR / (C * 8); ++i) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
#pragma unroll
            for (int c = 0; c < C; ++c)
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(r[c]) : "v"(a), "v"(b));
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long w1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = w1 - w0;
    }
    uint32_t x = 0;
#pragma unroll
    for (int c = 0; c < C; ++c) x ^= r[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

typedef void (*kfn)(uint32_t*, unsigned long long*, uint32_t);

int main() {
    CHECK(hipSetDevice(0));
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    uint32_t* out;
    unsigned long long* clk;
    CHECK(hipMalloc(&out, sizeof(uint32_t) * cus * 8 * 256));
    CHECK(hipMalloc(&clk, sizeof(unsigned long long) * cus * 8 * 2));
    std::vector<unsigned long long> h(cus * 8 * 2);
    struct K { int c; kfn f; };
    K ks[] = {{1, chain<1>}, {2, chain<2>}, {3, chain<3>}, {4, chain<4>}, {8, chain<8>}};
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::printf("%8s %8s %10s %10s %12s\n", "chains", "w/SIMD", "ms", "clk GHz", "cyc/instr");
    for (int w : {1, 2, 4, 8}) {
        for (const K& k : ks) {
            const int blocks = cus * w;
            for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, clk, 3u);
            CHECK(hipEventRecord(e0));
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, clk, 5u);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            CHECK(hipMemcpy(h.data(), clk, sizeof(unsigned long long) * blocks * 2, hipMemcpyDeviceToHost));
            double ghz = 0, cyc = 0;
            for (int i = 0; i < blocks; ++i) {
                ghz += (double)h[2 * i] / (double)h[2 * i + 1] * 0.1;
                cyc += (double)h[2 * i];
            }
            ghz /= blocks;
            cyc /= blocks;  // in-kernel cycles per wave
            // per SIMD: w waves x N_INSTR instructions in `cyc` cycles
            std::printf("%8d %8d %10.3f %10.3f %12.2f\n", k.c, w, ms, ghz, cyc / ((double)N_INSTR * w));
        }
    }
    return 0;
}
