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
// Lane words per wave (P candidates each) for pattern pack P: 2 = two NFAs per lane sharing each
// base's SALU work (LDS table read, M0 set-up) at 4 resident waves per SIMD, 1 = one NFA at 8.
// Two words for P = 2 (k = 11-16): cfg2 kernel 107-108 -> 102-103 us, cfg3 equal; one word for
// P = 1, where two were 0.8 % slower at cfg5 (profiles/r03_dual_ab.log).  P = 3-4 (k <= 10) are
// unmeasured and keep one.  -DAC_WORDS=1 / 2 forces one choice for every P (A/B builds).
// Round 5: the early launch's staged kernel takes two words for P = 1 as well -- with one word (8 resident
// waves, 78 SGPRs per wave) its staging state spilled 140+ SGPRs inside the count loop, with two (4
// waves, 106 SGPRs) 52: cfg5 stage 4.568-4.570 vs 4.669-4.687 ms, same box (profiles/r05_m12), while
// the plain P = 1 kernel stays at one word (4.248 vs 4.362 ms on resident input).
#ifndef AC_P1_STAGED_WORDS
#define AC_P1_STAGED_WORDS 2
#endif
constexpr int words_for(int P, bool staged = false) {
#ifdef AC_WORDS
    return (void)P, (void)staged, AC_WORDS;
#else
    return P == 2 ? 2 : (P == 1 && staged) ? AC_P1_STAGED_WORDS : 1;
#endif
}
// resident count-kernel waves per SIMD, set by the LDS allocation (<= 64 VGPRs with one word)
#ifndef AC_W2_WAVES
#define AC_W2_WAVES 4  // (A/B builds: resident waves per SIMD with two lane words)
#endif
constexpr int waves_per_simd(int W) { return W == 2 ? AC_W2_WAVES : 8; }

// Device error word bits (ac_check, include/approx_counter_amd.h): a window
// that is misaligned or reaches past the image was skipped; the kernel found
// its set-up broken (the ~Eq table not at LDS address 0) and skipped its work.
#define AC_DEVERR_WINDOW 1u
#define AC_DEVERR_SETUP 2u
#define AC_DEVERR_STAGE 4u  // a staged launch timed out waiting for its host inputs (its work was skipped)
#define AC_NO_ULEN 0xffffffffu

// Staged launches ("early launch"): the count kernel is launched
// before the host has packed its inputs and stages them itself.  Per segment,
// one header line of pinned host memory, read by the kernel with ONE 16-byte
// load (words 0-3):
#define AC_HDR_PGEN 0    // progress record, one 8-byte store {PGEN, READY}: valid when PGEN = the launch's generation
#define AC_HDR_READY 1   //   bytes of the segment's region packed and free of N (a prefix: k-mers, then codes)
#define AC_HDR_FLAG 2    // = generation once the segment is complete and INFO holds
#define AC_HDR_INFO 3    //   its final byte count (<= the launch's chunks x AC_STAGE_CHUNK, a multiple of 256)
                         //   | AC_HDR_INFO_HAS_N when it holds an N (its N bitmap sent), or AC_HDR_INFO_ABORT:
                         //   the host gave up on the call (the waves skip the segment)
#define AC_HDR_INFO_HAS_N 0x80000000u
#define AC_HDR_INFO_ABORT 0xffffffffu
#define AC_HDR_LINES AC_MAX_SEGS
#define AC_STAGE_CHUNK 4096u  // bytes one wave copies per claimed chunk (64 lanes x 16 B x 4)
#define AC_STAGE_REPL 32      // replicas of a segment's done counter (pollers spread over lines)
// Device words of a staged launch, one AC_QUEUE_LINE line each, after the
// launch's sub-queue counters in its queue bank (zeroed with them for the next
// launch on that bank; only word 0 of a line is ever used, as the next launch
// zeroes word 0 of each): error bits, then per segment: chunk
// claims, the segment's final header (verdict, bytes, final seen),
// AC_STAGE_REPL replicas of the N-free bytes available so far, AC_STAGE_REPL
// done replicas (every workgroup polls one replica of each: ~1000 waves
// polling one line slowed the chunk copies).
#define AC_STAGE_L_ERR 0
#define AC_STAGE_SEG_LINES (4 + 2 * AC_STAGE_REPL)
#define AC_STAGE_L_SEG(s) (1 + (s) * AC_STAGE_SEG_LINES)
#define AC_STAGE_LINES (1 + AC_MAX_SEGS * AC_STAGE_SEG_LINES)
// 0.5 s of s_memrealtime (100 MHz) WITHOUT PROGRESS: every wait is bounded, and its clock restarts
// whenever the words it waits on advance (a large call may take far longer than this to pack)
#define AC_STAGE_TIMEOUT_TICKS 50000000ull

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
    uint32_t group_begin;  // launch-wide index of this segment's first candidate group (LaunchArgs::grp_err)
    uint32_t has_n;       // 0: the image holds no N (its N bitmap is not read; every word reads as 0)
    uint32_t ulen;        // AC_NO_ULEN, or every window has this length and window w starts at base
                          // w * ceil32(ulen) (start / length are not read)
    uint32_t nrec;        // equal windows with inline N records (nrec.h): the record's bits R, else 0;
                          // has_n then says whether the N bitmap is there (some record overflowed)
    // staged launches: the segment's packed region (k-mers first) is copied from stage_src (the
    // pinned block, device-visible address) to stage_dst (device memory; kmers / codes / ... point
    // into it) in stage_chunks chunks of AC_STAGE_CHUNK bytes once the host flags it
    const uint8_t* stage_src;
    uint8_t* stage_dst;
    uint32_t stage_chunks;
    uint32_t stage_codes_off;  // bytes of the region before the codes (k-mers)
    uint32_t* stage_gen;       // per chunk, one line each: = the launch's generation once copied (early counting)
    // Device packing (staged launches, equal windows of 1..256 bases): the segment's
    // sample is read as Dna5 bytes straight from pinned host memory (ac_host_alloc) by the copier
    // workgroups, which pack each codes chunk themselves (stage_pack_chunk) instead of copying one the
    // host packed.  dp_src = NULL: the host packed the codes into the staging block.
    const uint8_t* dp_src;     // device-visible address the windows' offsets are relative to
    const uint64_t* dp_off;    // device-visible address of the segment's n_windows offsets
    uint32_t dp_src_bytes;     // bytes readable from dp_src (< 2^31); a window outside them is an error
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
    // Count hand-off: each workgroup adds (1 << 32) + its sum into every `acc` slot of
    // its candidate group with one returning 64-bit atomic per slot; the workgroup whose add finds
    // every other workgroup's arrival in the high half is the slot's last, writes the slot's total
    // to the segment's counts (stored, or added when `add_counts`) and zeroes the slot for the next
    // launch, so a launch needs no memset of the counts and no ticket round trip.
    uint64_t* acc;
    uint32_t* err;      // AC_DEVERR_* bits, or-ed in by the kernel
    uint32_t add_counts;
    // Staged launch (nonzero): inputs copied in by the kernel once the host flags each segment in
    // host_hdr (pinned, AC_HDR_LINES lines of AC_QUEUE_LINE u32); counts stored to host memory at
    // system scope, the launch's completion written to host_hdr's result line.  `stage` = this
    // launch's AC_STAGE_LINES device lines.
    uint32_t staged;
    uint32_t gen;
    uint32_t* host_hdr;
    uint32_t* stage;
    uint32_t* err_out;  // staged, counts in device memory (submits): each group ors its error bits in here
    // staged, tagged completion (synchronous calls): counts are u64 host words (generation << 32 | count)
    // and each candidate group stores its error snapshot (generation << 32 | bits) at grp_err[ticket index]
    uint32_t tag;
    uint64_t* grp_err;
    // staged: workgroups 0 .. n-1 stage, every wave of them, every segment in order, then they count
    // like the rest (a workgroup's wave holding a ticket would hold its other waves until its chunk
    // is packed); a staged launch with chunks always has n > 0 (0 is reported as a staging error)
    uint32_t copier_wgs;
    uint32_t n_segs;
    uint32_t eq;  // every live segment has equal windows (ulen), checked on the host to fit its image
    uint32_t m;  // k-mer length
    uint32_t P;  // candidates per lane word
};

inline uint32_t pack_factor(uint32_t k) { return (32u / k) < AC_MAX_PACK ? (32u / k) : AC_MAX_PACK; }
// candidates per wave of the plain (staged = false) or the early launch's staged kernel
inline uint32_t cands_per_wave(uint32_t P, bool staged) { return 64u * P * (uint32_t)words_for((int)P, staged); }

// Waves of the count kernel for pattern pack P that fit on the device at once.
hipError_t resident_waves(uint32_t P, bool staged, int cu_count, uint32_t* waves);

#ifdef AC_STAMPS
hipError_t debug_stamps(void* host, size_t bytes);
#endif

hipError_t launch_wm2_count(const LaunchArgs& args, hipStream_t stream);

}  // namespace acamd
