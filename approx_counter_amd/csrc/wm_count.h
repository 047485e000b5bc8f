// wm_count.h -- launch descriptor shared by the kernel and the C-ABI layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define AC_MAX_SEGS 4    // segments fused into one launch (start + end ends, shards)
#define AC_MAX_PACK 4    // candidates interleaved per 32-bit lane word (P = min(32/k, 4))
#ifndef AC_WAVE_WORDS
#define AC_WAVE_WORDS 1  // lane words (independent NFAs) per lane (2 measured slower: profiles/r01_kernel_log.md)
#endif
#ifndef AC_MIN_WAVES_PER_SIMD
#define AC_MIN_WAVES_PER_SIMD 8  // occupancy the register budget is sized for (<= 64 VGPRs)
#endif

namespace acamd {

struct SegDev {
    const uint64_t* kmers;
    const uint32_t* codes;
    const uint32_t* nmask;
    const uint64_t* start;
    const uint32_t* length;
    uint32_t* counts;
    uint64_t wave_begin;  // first global wave of this segment
    uint64_t n_bases;     // image size (bases); windows outside it are skipped
    uint32_t n_kmers;
    uint32_t n_windows;
    uint32_t groups;      // candidate groups of cands_per_wave(P) candidates
    uint32_t wpw;         // windows per wave
};

struct LaunchArgs {
    SegDev seg[AC_MAX_SEGS];
    uint64_t total_waves;
    uint32_t n_segs;
    uint32_t m;  // k-mer length
    uint32_t P;  // candidates per lane word
};

inline uint32_t pack_factor(uint32_t k) { return (32u / k) < AC_MAX_PACK ? (32u / k) : AC_MAX_PACK; }
inline uint32_t cands_per_wave(uint32_t P) { return 64u * P * AC_WAVE_WORDS; }

// Waves of the count kernel for pattern pack P that fit on the device at once.
hipError_t resident_waves(uint32_t P, int cu_count, uint32_t* waves);

#ifdef AC_STAMPS
hipError_t debug_stamps(void* host, size_t bytes);
#endif

hipError_t launch_wm2_count(const LaunchArgs& args, hipStream_t stream);

}  // namespace acamd
