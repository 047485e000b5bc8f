// wm_count.h -- launch descriptor shared by the kernel and the C-ABI layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define AC_MAX_SEGS 4  // segments fused into one launch (start + end ends, shards)
#define AC_MAX_PACK 4  // candidates packed per 32-bit lane word (P = min(32/k, 4))

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
    uint32_t groups;      // candidate groups of 64*P candidates
    uint32_t wpw;         // windows per wave
};

struct LaunchArgs {
    SegDev seg[AC_MAX_SEGS];
    uint64_t total_waves;
    uint32_t n_segs;
    uint32_t m;  // k-mer length
    uint32_t P;  // candidates per lane
};

hipError_t launch_wm2_count(const LaunchArgs& args, hipStream_t stream);

}  // namespace acamd
