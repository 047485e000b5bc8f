// exact_count.h -- launch descriptor of the exact-count kernels (exact_count.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "wm_count.h"  // AC_DEVERR_*

#ifndef EXACT_WINDOWS_PER_BLOCK
#define EXACT_WINDOWS_PER_BLOCK 16  // windows aggregated per workgroup in LDS
#endif
#define EXACT_HIST_BINS 4096        // count histogram (last bin collects larger counts)
#define EXACT_LIST_MIN 2            // the scan compacts kept entries with at least this count

namespace acamd {

// Wide slot (k > 16): 16 bytes, claimed with a CAS on the key, counted with an
// add on cnt.
struct alignas(16) ExactSlot {
    uint64_t key;  // k-mer + 1; 0 = empty
    uint32_t cnt;
    uint32_t pad;
};
// Compact slot (k <= 16): one u64 = (uint32)(k-mer + 1) << 32 | count.  A new
// key is claimed AND counted by one CAS (most k-mers of a sample occur once);
// a repeated key takes one 64-bit add on the same word.
constexpr uint32_t EXACT_COMPACT_MAX_K = 16;

struct ExactArgs {
    // window image (device)
    const uint32_t* codes;
    const uint32_t* nmask;
    const uint64_t* start;
    const uint32_t* length;
    uint64_t n_bases;
    uint32_t n_windows;
    uint32_t k;
    // hash table: `slots` (a power of two) slots, ExactSlot {k-mer + 1, count}
    // or, when `compact`, u64 (k-mer + 1) << 32 | count; stored key 0 = empty,
    // so a zero memset clears it.  Slot index `slots` (past the table) stands
    // for the all-T k-mer whose stored key wraps to 0 (the 32-mer in the wide
    // layout, the 16-mer in the compact one), counted in special[0].
    ExactSlot* table;
    unsigned long long* ctable;
    uint32_t compact;
    uint64_t slots;
    uint64_t mask;
    uint32_t* special;
    unsigned long long* had_n;
    uint32_t* err;  // AC_DEVERR_* bits (wm_count.h), read back by the host
    // filters
    float lc_threshold;
    const uint64_t* forbidden;  // sorted
    uint32_t n_forbidden;
    // scan: count histogram of the kept entries, and the kept entries with
    // count >= EXACT_LIST_MIN compacted into list_keys/list_cnts
    uint32_t* hist;  // EXACT_HIST_BINS
    uint64_t* list_keys;
    uint32_t* list_cnts;
    unsigned long long* n_list;
    uint64_t list_cap;
    // gather: entries with count >= threshold, from the list (threshold >=
    // EXACT_LIST_MIN) or from the whole table
    uint32_t threshold;
    uint64_t* out_keys;
    uint32_t* out_cnts;
    unsigned long long* n_out;
    uint64_t out_cap;
};

hipError_t launch_exact_insert(const ExactArgs& a, hipStream_t stream);
hipError_t launch_exact_scan(const ExactArgs& a, hipStream_t stream);
// from_list: gather from the scan's compacted list of n_list entries, else from the table
hipError_t launch_exact_gather(const ExactArgs& a, bool from_list, uint64_t n_list, hipStream_t stream);

}  // namespace acamd
