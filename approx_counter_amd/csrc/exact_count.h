// exact_count.h -- launch descriptor of the exact-count kernels (exact_count.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define EXACT_WINDOWS_PER_BLOCK 16  // windows aggregated per workgroup in LDS
#define EXACT_HIST_BINS 4096        // count histogram (last bin collects larger counts)

namespace acamd {

struct ExactArgs {
    // window image (device)
    const uint32_t* codes;
    const uint32_t* nmask;
    const uint64_t* start;
    const uint32_t* length;
    uint64_t n_bases;
    uint32_t n_windows;
    uint32_t k;
    // hash table: `slots` (a power of two) keys + counts; slot index `slots`
    // (past the table) stands for the all-T 32-mer, counted in special[0]
    uint64_t* keys;
    uint32_t* cnts;
    uint64_t slots;
    uint64_t mask;
    uint32_t* special;
    unsigned long long* had_n;
    // filters
    float lc_threshold;
    const uint64_t* forbidden;  // sorted
    uint32_t n_forbidden;
    // scan / gather
    uint32_t* hist;  // EXACT_HIST_BINS
    uint32_t threshold;
    uint64_t* out_keys;
    uint32_t* out_cnts;
    unsigned long long* n_out;
    uint64_t out_cap;
};

hipError_t launch_exact_insert(const ExactArgs& a, hipStream_t stream);
hipError_t launch_exact_scan(const ExactArgs& a, hipStream_t stream);
hipError_t launch_exact_gather(const ExactArgs& a, hipStream_t stream);

}  // namespace acamd
