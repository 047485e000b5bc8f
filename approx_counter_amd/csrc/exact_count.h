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
    // partitioned path: the forbidden k-mers sorted by (bucket, k-mer), bucket b's at
    // [fb_start[b], fb_start[b + 1]) (NULL when the set is empty)
    const uint64_t* fb_bucketed;
    const uint32_t* fb_start;
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
    // Partitioned path: every k-mer position's key
    // written densely (`keys`, n_keys of them), moved into 2^s_log2
    // super-buckets (`tmp`; per-chunk histogram h1 [chunk][super], sizes
    // stot), then into the 2^nb_log2 buckets (`parts`; per level-2 chunk
    // histogram h2 [chunk][sub]; bucket starts bstart, nb + 1 of them); one
    // workgroup per bucket counts its keys in LDS.  No global hash table.
    void* keys;   // uint32_t keys for k <= 16, uint64_t above
    void* tmp;
    void* parts;
    unsigned long long* n_keys;
    uint32_t* h1;
    uint32_t* h2;
    uint32_t* stot;
    uint32_t* slab;    // [slab][super]: h1's column sums over EXACT_SCAN_SLAB rows (the level-1 scan)
    uint32_t* bstart;  // nb + 1
    uint32_t nb_log2;
    uint32_t s_log2;    // super-buckets: nb_log2 - s_log2 <= 6
    uint32_t n_chunks;  // level-1 grid: ceil(key capacity / exact_part_chunk(k))
    uint32_t n_chunks2; // level-2 grid bound: n_chunks + 2^s_log2
    uint64_t key_cap;
    uint32_t list_min;   // the count kernel lists kept entries with count >= list_min
    uint32_t emit_only;  // 1: list only (the histogram and distinct count were taken by an earlier pass)
    uint32_t* overflow;  // set when a bucket outgrows the count kernel's LDS table
    uint32_t* phist;     // [bucket][EXACT_PHIST] partial histograms of the count kernel (counts 1..EXACT_PHIST)
};

#define EXACT_PHIST 32  // per-bucket partial histogram bins (counts 1..32; larger counts go straight to hist)

#define EXACT_SCAN_SLAB 128   // level-1 histogram rows (chunks) per workgroup of the column scan
#define EXACT_MAX_SUPER 1024  // level-1 super-buckets (at most)
#ifndef AC_SUB_LOG2
// log2 buckets per super-bucket at 2^16 buckets: 512 super-buckets of 128 (round 6; 1024 of 64 before):
// the level-1 scatter writes runs of ~16 keys per chunk and super-bucket instead of ~8 (partial
// lines), cfg4 2.14-2.17 ms against 2.26-2.27 (profiles/r06_m14, r06_m15)
#define AC_SUB_LOG2 7
#endif
#define EXACT_MAX_SUB (1 << AC_SUB_LOG2)  // buckets per super-bucket (at most)
#define EXACT_BUCKET_SLOTS 4096  // LDS counting table of the per-bucket kernel (32 KB of keys + counts)

hipError_t launch_exact_insert(const ExactArgs& a, hipStream_t stream);
hipError_t launch_exact_scan(const ExactArgs& a, hipStream_t stream);
// from_list: gather from the scan's compacted list of n_list entries, else from the table
hipError_t launch_exact_gather(const ExactArgs& a, bool from_list, uint64_t n_list, hipStream_t stream);
// Partitioned path (k <= 16): keys, bucket partition, per-bucket count (fills
// hist / list / special like insert + scan).  `count_only` re-runs just the
// per-bucket count (with a.list_min / a.emit_only) on the partition already built.
hipError_t launch_exact_partitioned(const ExactArgs& a, hipStream_t stream);
// Keys per histogram / scatter chunk of the partitioned path for k (8,192 32-bit or 4,096 64-bit keys:
// one chunk staged in 32 KB of LDS; 16,384 gave 2 scatter workgroups per CU, level-2 scatter 37 us).
uint32_t exact_part_chunk(uint32_t k);
hipError_t launch_exact_part_count(const ExactArgs& a, hipStream_t stream);

// Hash of a key for the partition (its top bits pick the bucket) and the per-bucket LDS table (its
// low bits pick the slot): a 32-bit mixer (two u32 multiplies; the 64-bit murmur finaliser costs ~8
// quarter-rate multiplies and the partition hashes every key five times); 64-bit keys fold their
// high half in.  Host and device: the host sorts the forbidden set by bucket with it.
__host__ __device__ inline uint32_t part_hash(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
__host__ __device__ inline uint32_t part_hash(uint64_t x) {
    return part_hash((uint32_t)x ^ part_hash((uint32_t)(x >> 32) + 0x9e3779b9u));
}
template <class K>
__host__ __device__ inline uint32_t bucket_of(K key, uint32_t nb_log2) {
    return part_hash(key) >> (32u - nb_log2);
}

}  // namespace acamd
