// wm_count.h -- launch descriptor shared by the kernel and the C-ABI layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define AC_MAX_SEGS 4    // segments fused into one launch (start + end ends, shards)
#define AC_QUEUE_LINE 32  // u32 per queue counter: one 128-B line each (no false sharing between counters)
#define AC_MAX_PACK 4    // candidates interleaved per 32-bit lane word (P = min(32/k, 4))
// Largest window image (bases, exclusive): the count kernel reads it through buffer descriptors whose
// byte offsets and sizes are 32-bit (2 bits per base: 2^34 bases = 4 GiB of code words).
#define AC_MAX_IMAGE_BASES (1ull << 34)
#ifndef AC_WAVES_PER_BLOCK
#define AC_WAVES_PER_BLOCK 4  // waves per workgroup, all on one candidate group (shared ~Eq table, counts summed in LDS)
#endif
#ifndef AC_WAVES_PER_SIMD
#define AC_WAVES_PER_SIMD 8  // resident count-kernel waves per SIMD, set by the LDS allocation (<= 64 VGPRs)
#endif

// Device error word bits (ac_check, include/approx_counter_amd.h): a window
// that is misaligned or reaches past the image was skipped; the kernel found
// its set-up broken (the ~Eq table not at LDS address 0) and skipped its work.
#define AC_DEVERR_WINDOW 1u
#define AC_DEVERR_SETUP 2u
#define AC_NO_ULEN 0xffffffffu

namespace acamd {

struct SegDev {
    const uint64_t* kmers;
    const uint32_t* codes;
    const uint32_t* nmask;
    const uint64_t* start;
    const uint32_t* length;
    uint32_t* counts;
    uint64_t n_bases;     // image size (bases); windows outside it are skipped
    uint32_t n_kmers;
    uint32_t n_windows;
    uint32_t groups;      // candidate groups of cands_per_wave(P) candidates
    uint32_t chunk;       // windows per work item of the dynamic queues
    uint32_t queue_begin; // index of this segment's first sub-queue (groups x subq of them)
    uint32_t subq;        // sub-queues per candidate group (proportional to n_windows; a multiple of AC_WAVES_PER_BLOCK)
    uint32_t acc_begin;   // this segment's first slot in LaunchArgs::acc (groups x cands_per_wave slots)
    uint32_t ticket_begin;  // this segment's first group ticket in LaunchArgs::tickets
    uint32_t has_n;       // 0: the image holds no N (its N bitmap is not read; every word reads as 0)
    uint32_t ulen;        // AC_NO_ULEN, or every window has this length and window w starts at base
                          // w * ceil32(ulen) (start / length are not read)
};

struct LaunchArgs {
    SegDev seg[AC_MAX_SEGS];
    uint64_t total_waves;
    // Work queues: two banks of `qstride` sub-queue counters, one per
    // AC_QUEUE_LINE-u32 line.  This launch dequeues from bank `bank` (zeroed)
    // and zeroes the first `zero_count` counters of the other bank for the next
    // launch.
    uint32_t* queue;
    uint32_t qstride;
    uint32_t bank;
    uint32_t zero_count;
    uint32_t n_queues;  // sub-queues over all segments (a multiple of AC_WAVES_PER_BLOCK); wave w of
                        // workgroup b serves sub-queue (b % (n_queues / AC_WAVES_PER_BLOCK)) * AC_WAVES_PER_BLOCK + w
    // Count hand-off: workgroups add their sums into `acc` and
    // take a ticket of their candidate group; the group's last workgroup moves
    // the group's sums to the segment's counts (stored, or added when
    // `add_counts`) and zeroes its acc slots and ticket for the next launch, so
    // a launch needs no memset of the counts.
    uint32_t* acc;
    uint32_t* tickets;  // one per AC_QUEUE_LINE u32
    uint32_t* err;      // AC_DEVERR_* bits, or-ed in by the kernel
    uint32_t add_counts;
    uint32_t n_segs;
    uint32_t m;  // k-mer length
    uint32_t P;  // candidates per lane word
};

inline uint32_t pack_factor(uint32_t k) { return (32u / k) < AC_MAX_PACK ? (32u / k) : AC_MAX_PACK; }
inline uint32_t cands_per_wave(uint32_t P) { return 64u * P; }

// Waves of the count kernel for pattern pack P that fit on the device at once.
hipError_t resident_waves(uint32_t P, int cu_count, uint32_t* waves);

#ifdef AC_STAMPS
hipError_t debug_stamps(void* host, size_t bytes);
#endif

hipError_t launch_wm2_count(const LaunchArgs& args, hipStream_t stream);

}  // namespace acamd
