// Probe (GPU box, one-off measurement): how fast can kernel waves pull a packed read end from
// pinned host memory into device memory?  The early-launch stage moves ~324 KB
// per cfg2 read end with one 4 KB chunk per wave (4 x 16-B nontemporal loads per lane) and
// measures 13-19 us per end (~20 GB/s, profiles/r03_m1/stamps.log), against ~37 GB/s for the
// copy engine.  This sweeps the pinned allocation's flags, the chunk per wave, the loads in
// flight per lane and the loads' cache policy, timing each launch alone with events (the host
// rewrites the block between launches, so no cache holds it).  The copy engine for scale.
// Build: hipcc -O2 --offload-arch=gfx950 tools/pull_probe.hip -o pull_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                                          \
        }                                                                                          \
    } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

// One wave per chunk of 1024 * U bytes: each lane U loads of 16 B (aux = cache policy bits), then stores.
template <int U, int AUX>
__global__ void pull_kernel(const uint8_t* src, uint8_t* dst, uint32_t bytes) {
    const uint32_t wave = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64, lane = threadIdx.x & 63u;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, (int)bytes, 0x00020000);
    __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)dst, 0, (int)bytes, 0x00020000);
    const uint32_t o = wave * (1024u * U) + lane * 16u;
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, o + u * 1024u, 0, AUX);
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_amdgcn_raw_buffer_store_b128(v[u], rd, o + u * 1024u, 0, 16);
}

template <int U, int AUX>
static float run(const uint8_t* src_d, uint8_t* src_h, uint8_t* dst, uint32_t bytes, int waves_per_block, hipStream_t s,
                 hipEvent_t e0, hipEvent_t e1) {
    const uint32_t chunk = 1024u * U, waves = (bytes + chunk - 1) / chunk;
    const uint32_t blocks = (waves + waves_per_block - 1) / waves_per_block;
    std::vector<float> t;
    for (int r = 0; r < 25; ++r) {
        std::memset(src_h, r, bytes);  // fresh data: nothing cached from the last launch
        CK(hipEventRecord(e0, s));
        hipLaunchKernelGGL((pull_kernel<U, AUX>), dim3(blocks), dim3(64 * waves_per_block), 0, s, src_d, dst, bytes);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 5) t.push_back(ms * 1000.f);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const size_t MAXB = 2u << 20;
    uint8_t* dst = nullptr;
    CK(hipMalloc((void**)&dst, MAXB));
    struct Kind {
        const char* name;
        unsigned flags;
    } kinds[] = {{"default", hipHostMallocDefault},
                 {"coherent", hipHostMallocCoherent | hipHostMallocMapped},
                 {"noncoherent", hipHostMallocNonCoherent | hipHostMallocMapped},
                 {"writecombined", hipHostMallocWriteCombined | hipHostMallocMapped}};
    // empty launch, for the fixed cost inside the event pair
    {
        uint8_t* h = nullptr;
        CK(hipHostMalloc((void**)&h, 4096, hipHostMallocDefault));
        uint8_t* hd = nullptr;
        CK(hipHostGetDevicePointer((void**)&hd, h, 0));
        std::printf("one-wave 1 KB launch: %.1f us\n", run<1, 2>(hd, h, dst, 1024, 1, s, e0, e1));
        CK(hipHostFree(h));
    }
    for (const Kind& k : kinds) {
        uint8_t* h = nullptr;
        CK(hipHostMalloc((void**)&h, MAXB, k.flags));
        uint8_t* hd = nullptr;
        CK(hipHostGetDevicePointer((void**)&hd, h, 0));
        for (uint32_t bytes : {324u * 1024u, 648u * 1024u, 2048u * 1024u}) {
            std::printf("%-13s %5u KB:", k.name, bytes / 1024);
            struct R {
                const char* n;
                float us;
            } r[] = {
                {"4KBx1w nt", run<4, 2>(hd, h, dst, bytes, 1, s, e0, e1)},
                {"4KBx1w plain", run<4, 0>(hd, h, dst, bytes, 1, s, e0, e1)},
                {"4KBx1w sc0sc1", run<4, 17>(hd, h, dst, bytes, 1, s, e0, e1)},
                {"1KBx1w nt", run<1, 2>(hd, h, dst, bytes, 1, s, e0, e1)},
                {"1KBx4w nt", run<1, 2>(hd, h, dst, bytes, 4, s, e0, e1)},
                {"8KBx1w nt", run<8, 2>(hd, h, dst, bytes, 1, s, e0, e1)},
                {"16KBx1w nt", run<16, 2>(hd, h, dst, bytes, 1, s, e0, e1)},
            };
            for (const R& x : r) std::printf("  %s %.1f us (%.0f GB/s)", x.n, x.us, bytes / x.us / 1e3);
            std::printf("\n");
        }
        // the copy engine
        for (uint32_t bytes : {324u * 1024u, 648u * 1024u, 2048u * 1024u}) {
            std::vector<float> t;
            for (int r = 0; r < 25; ++r) {
                std::memset(h, r, bytes);
                CK(hipEventRecord(e0, s));
                CK(hipMemcpyAsync(dst, h, bytes, hipMemcpyHostToDevice, s));
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r >= 5) t.push_back(ms * 1000.f);
            }
            std::sort(t.begin(), t.end());
            std::printf("%-13s %5u KB: copy engine %.1f us (%.0f GB/s)\n", k.name, bytes / 1024, t[t.size() / 2],
                        bytes / t[t.size() / 2] / 1e3);
        }
        CK(hipHostFree(h));
    }
    std::printf("done\n");
    return 0;
}
