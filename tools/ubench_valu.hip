// ubench_valu.hip -- issue rate of the VALU instructions the count kernel uses (gfx950).
//
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_valu.hip -o build/ubench_valu && build/ubench_valu
//
// Every wave runs a long unrolled stream of ONE instruction over 8 independent
// register chains (no dependency stalls), 8 waves per SIMD on every CU.  Prints
// wave-instructions per SIMD per clock, with the clock measured in-kernel
// (s_memtime / s_memrealtime, 100 MHz reference), so the result is the
// instruction's issue cost in cycles per wave64 instruction on one SIMD.
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

constexpr int ITERS = 2048;  // loop trips
constexpr int UNROLL = 8;    // instructions per chain per trip (x 8 chains)

#define OP8(OPSTR)                                                                              \
    asm volatile(OPSTR : "+v"(r0) : "v"(a), "v"(b));                                            \
    asm volatile(OPSTR : "+v"(r1) : "v"(a), "v"(b));                                            \
    asm volatile(OPSTR : "+v"(r2) : "v"(a), "v"(b));                                            \
    asm volatile(OPSTR : "+v"(r3) : "v"(a), "v"(b));                                            \
    asm volatile(OPSTR : "+v"(r4) : "v"(a), "v"(b));                                            \
    asm volatile(OPSTR : "+v"(r5) : "v"(a), "v"(b));                                            \
    asm volatile(OPSTR : "+v"(r6) : "v"(a), "v"(b));                                            \
    asm volatile(OPSTR : "+v"(r7) : "v"(a), "v"(b));

#define KERNEL(NAME, OPSTR)                                                                      \
    __global__ __launch_bounds__(256) void NAME(uint32_t* out, unsigned long long* clk, uint32_t seed) { \
        uint32_t a = seed ^ threadIdx.x, b = seed * 3u + blockIdx.x;                             \
        uint32_t r0 = a, r1 = b, r2 = a + 1, r3 = b + 1, r4 = a + 2, r5 = b + 2, r6 = a + 3, r7 = b + 3; \
        unsigned long long t0 = __builtin_amdgcn_s_memtime();                                    \
        unsigned long long w0 = __builtin_amdgcn_s_memrealtime();                                \
        for (int i = 0; i < ITERS; ++i) {                                                        \
            for (int u = 0; u < UNROLL; ++u) { OP8(OPSTR) }                                      \
        }                                                                                        \
        unsigned long long t1 = __builtin_amdgcn_s_memtime();                                    \
        unsigned long long w1 = __builtin_amdgcn_s_memrealtime();                                \
        if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = w1 - w0; } \
        out[blockIdx.x * blockDim.x + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7;      \
    }

KERNEL(k_and, "v_and_b32 %0, %0, %1")
KERNEL(k_xor, "v_xor_b32 %0, %0, %1")
KERNEL(k_add, "v_add_u32 %0, %0, %1")
KERNEL(k_lshl, "v_lshlrev_b32 %0, 1, %0")
KERNEL(k_or3, "v_or3_b32 %0, %0, %1, %2")
KERNEL(k_and_or, "v_and_or_b32 %0, %0, %1, %2")
KERNEL(k_lshl_or, "v_lshl_or_b32 %0, %0, 1, %1")
KERNEL(k_bitop3, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0xdc")
KERNEL(k_min, "v_min_u32 %0, %0, %1")
KERNEL(k_fma, "v_fma_f32 %0, %0, %1, %2")
KERNEL(k_mov, "v_mov_b32 %0, %1")
KERNEL(k_or, "v_or_b32 %0, %0, %1")
KERNEL(k_sub, "v_sub_u32 %0, %0, %1")
KERNEL(k_addc, "v_addc_co_u32 %0, vcc, %1, %0, vcc")
KERNEL(k_bfi, "v_bfi_b32 %0, %0, %1, %2")
KERNEL(k_alignbit, "v_alignbit_b32 %0, %0, %1, 31")
KERNEL(k_cndmask, "v_cndmask_b32 %0, %0, %1, vcc")
KERNEL(k_add3, "v_add3_u32 %0, %0, %1, %2")
KERNEL(k_lshl_add, "v_lshl_add_u32 %0, %0, 1, %1")
KERNEL(k_xad, "v_xad_u32 %0, %0, %1, %2")
KERNEL(k_mad24, "v_mad_u32_u24 %0, %0, %1, %2")
KERNEL(k_perm, "v_perm_b32 %0, %0, %1, %2")
KERNEL(k_bfe, "v_bfe_u32 %0, %0, 1, 7")
KERNEL(k_not, "v_not_b32 %0, %0")
KERNEL(k_lshr, "v_lshrrev_b32 %0, 1, %0")
KERNEL(k_max3, "v_max3_u32 %0, %0, %1, %2")
KERNEL(k_bcnt, "v_bcnt_u32_b32 %0, %0, %1")
KERNEL(k_addlit, "v_add_u32 %0, 0x12345, %0")
KERNEL(k_andsg, "v_and_b32 %0, s4, %0")
// 64-bit ops: operands are register pairs; use the 32-bit chain as the low half
#define KERNEL64(NAME, OPSTR)                                                                    \
    __global__ __launch_bounds__(256) void NAME(uint32_t* out, unsigned long long* clk, uint32_t seed) { \
        uint64_t a = seed ^ threadIdx.x, b = seed * 3ull + blockIdx.x;                           \
        uint64_t r0 = a, r1 = b, r2 = a + 1, r3 = b + 1, r4 = a + 2, r5 = b + 2, r6 = a + 3, r7 = b + 3; \
        unsigned long long t0 = __builtin_amdgcn_s_memtime();                                    \
        unsigned long long w0 = __builtin_amdgcn_s_memrealtime();                                \
        for (int i = 0; i < ITERS; ++i) {                                                        \
            for (int u = 0; u < UNROLL; ++u) { OP8(OPSTR) }                                      \
        }                                                                                        \
        unsigned long long t1 = __builtin_amdgcn_s_memtime();                                    \
        unsigned long long w1 = __builtin_amdgcn_s_memrealtime();                                \
        if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = w1 - w0; } \
        out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7); \
    }
KERNEL64(k_lshl64, "v_lshlrev_b64 %0, 1, %0")
KERNEL64(k_pk_fma, "v_pk_fma_f32 %0, %0, %1, %2")
KERNEL64(k_pk_add, "v_pk_add_f32 %0, %0, %1")
KERNEL64(k_pk_mov, "v_pk_mov_b32 %0, %0, %1 op_sel:[0,1]")

typedef void (*kfn)(uint32_t*, unsigned long long*, uint32_t);

int main(int argc, char** argv) {
    int dev = 0;
    CHECK(hipSetDevice(dev));
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, dev));
    const int cus = prop.multiProcessorCount;
    const int waves_per_simd = argc > 1 ? std::atoi(argv[1]) : 8;
    const int blocks = cus * waves_per_simd;  // 256-thread block = 4 waves = 1 per SIMD
    uint32_t* out;
    unsigned long long* clk;
    CHECK(hipMalloc(&out, sizeof(uint32_t) * blocks * 256));
    CHECK(hipMalloc(&clk, sizeof(unsigned long long) * blocks * 2));
    struct K { const char* name; kfn f; };
    K ks[] = {{"v_and_b32", k_and},     {"v_xor_b32", k_xor},       {"v_add_u32", k_add},
              {"v_lshlrev_b32", k_lshl}, {"v_or3_b32", k_or3},       {"v_and_or_b32", k_and_or},
              {"v_lshl_or_b32", k_lshl_or}, {"v_bitop3_b32", k_bitop3}, {"v_min_u32", k_min},
              {"v_fma_f32", k_fma},     {"v_mov_b32", k_mov},       {"v_lshlrev_b64", k_lshl64},
              {"v_pk_fma_f32", k_pk_fma}, {"v_pk_add_f32", k_pk_add}, {"v_pk_mov_b32", k_pk_mov},
              {"v_or_b32", k_or}, {"v_sub_u32", k_sub}, {"v_addc_co_u32", k_addc}, {"v_bfi_b32", k_bfi},
              {"v_alignbit_b32", k_alignbit}, {"v_cndmask_b32", k_cndmask}, {"v_add3_u32", k_add3},
              {"v_lshl_add_u32", k_lshl_add}, {"v_xad_u32", k_xad}, {"v_mad_u32_u24", k_mad24},
              {"v_perm_b32", k_perm}, {"v_bfe_u32", k_bfe}, {"v_not_b32", k_not},
              {"v_lshrrev_b32", k_lshr}, {"v_max3_u32", k_max3}, {"v_bcnt_u32_b32", k_bcnt},
              {"v_add_u32 lit", k_addlit}, {"v_and_b32 sgpr", k_andsg}};
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::vector<unsigned long long> h(blocks * 2);
    std::printf("CUs=%d waves/SIMD=%d blocks=%d\n", cus, waves_per_simd, blocks);
    std::printf("%-16s %10s %12s %14s %12s\n", "instr", "ms", "clk GHz", "lane-op/s", "cyc/instr");
    for (const K& k : ks) {
        for (int rep = 0; rep < 3; ++rep) {  // warm the clock
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, clk, 7u);
        }
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, clk, 11u);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        CHECK(hipMemcpy(h.data(), clk, sizeof(unsigned long long) * blocks * 2, hipMemcpyDeviceToHost));
        double ghz = 0;
        for (int i = 0; i < blocks; ++i) ghz += (double)h[2 * i] / (double)h[2 * i + 1] * 0.1;
        ghz /= blocks;
        const double instrs = (double)ITERS * UNROLL * 8;           // per wave
        const double lane_ops = instrs * 64.0 * blocks * 4;         // all waves
        const double rate = lane_ops / (ms * 1e-3);
        // cycles per wave-instruction on one SIMD = SIMD cycles / instructions issued to it
        const double simd_instrs = instrs * waves_per_simd;
        const double cyc = (ms * 1e-3) * ghz * 1e9 / simd_instrs;
        std::printf("%-16s %10.3f %12.3f %14.4g %12.2f\n", k.name, ms, ghz, rate, cyc);
    }
    return 0;
}
