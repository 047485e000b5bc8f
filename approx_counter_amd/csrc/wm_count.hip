// wm_count.hip -- the approximate-count kernel for MI355X (gfx950).
//
// Replaces the OpenMP/SeqAn search loop of errorCount
// (approx_counter.cpp:550-599): for every (candidate k-mer, sampled window)
// pair it decides, per error level e = 0,1,2, whether the k-mer occurs in the
// window with at most e edits -- the three per-read bitfields tcount[e] of
// approx_counter.cpp:553/563 -- and adds the number of levels hit to the
// candidate's counter (the vectorSum of 590-593).
//
// Algorithm: bit-parallel Wu-Manber NFA for edit distance <= 2 (Wu & Manber
// 1992) in its complemented "shift-or" form (Baeza-Yates & Gonnet 1992), free
// start in the text.  With R_d bit i = "pattern prefix of length i+1 ends at
// the current text position with <= d edits" and D_d = ~R_d:
//   D0' = (D0 >> P) | ~Eq
//   Dd' = ((Dd >> P) | ~Eq) & Dd-1 & (Dd-1 >> P) & (Dd-1' >> P)      d = 1, 2
// The shift brings in zeros, i.e. "R bit set": that is the free start of row
// 0 and the always-set prefix bits of rows 1 and 2, with no mask operation.
// A window hits level d iff the AND of D_d over its positions has the
// pattern's last bit clear; the count adds the three levels.
//
// MI355X mapping:
//  * lane = P candidates, window text wave-uniform.  P = floor(32/k) (<= 4)
//    patterns are INTERLEAVED in one 32-bit register: character i of pattern p
//    sits at bit 31 - (i*P + p), so one logical right shift by P advances every
//    pattern at once and the zero fill reaches every pattern's first character.
//  * W lane words per wave (words_for(P): 2 for P = 2, i.e. k = 11-16, else 1):
//    each lane carries W x P candidates, and the W NFAs share every base's
//    SALU work and text.
//  * ~Eq is a table lookup, as in the textbook algorithm: each WORKGROUP (4
//    waves, all on one candidate group) keeps one W x 5 x 64-word LDS table
//    (per lane word: the lane's ~Eq for A, C, G, T, and all ones for N), built
//    by its wave 0; every wave reads one word per lane, lane word and text base
//    with ds_read_addtid_b32, the address coming from M0 = 256 * character,
//    two SALU ops from the wave-uniform 2-bit text held in an SGPR.  No VALU op
//    per base for ~Eq.
//  * The NFA runs in generated inline-asm blocks (wm_tid_blocks.inc,
//    tools/gen_tid_blocks.py): 8 full-rate VALU ops per base (v_or, v_lshrrev,
//    v_bitop3 -- the forms that issue in 2 cycles per wave64 on gfx950,
//    profiles/r01_ubench_valu.txt) + 1.5 of hit accumulation (AND3 over two
//    bases) = 9.5 VALU ops per base and lane word (P candidates), scheduled
//    skewed (row 0 of base s, row 1 of base s-1, row 2 of base s-2 per step) so
//    a lane word has three independent dependency chains, with the LDS reads
//    three bases ahead.
//  * The table is the workgroup's first LDS object, at address 0, so M0 needs
//    no per-wave add: per base 2 SALU + W LDS + 9.5 W VALU.  The SALU is the
//    CU-shared resource the first table-driven version ran out of (5 SALU per
//    base: no faster than computing ~Eq with 2 VALU ops; profiles/r01_kernel_log.md).
//  * Integer-only VALU work: no MFMA.  Counts are uint32 atomics
//    (order-independent, bit-exact).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nrec.h"
#include "wm_count.h"

namespace acamd {
namespace {

constexpr int WAVES_PER_BLOCK = AC_WAVES_PER_BLOCK;
#ifdef AC_STAMPS
// Diagnostic build only (tools/variants.sh ... -DAC_STAMPS): per-wave
// s_memrealtime stamps (100 MHz) at entry, after the prologue, after the last
// window and at exit; read back with ac_debug_stamps().  No output value is
// computed from them.
}  // namespace
__device__ uint64_t g_stamps[1 << 21];
__device__ uint64_t g_stage_stamps[64];  // per segment s, at [s*8 + i]: 0 final header seen by the poller, 1 its first
                                         // progress record, 2 last chunk in, 3 first record past the k-mers, 4 first
                                         // codes chunk flagged
namespace {
__device__ __forceinline__ void stamp(uint64_t wave, int i) {
    if ((threadIdx.x & 63u) == 0 && wave < (1u << 18)) {
        g_stamps[wave * 8 + i] = __builtin_amdgcn_s_memrealtime();
        if (i == 0) {
            uint32_t hw, xcc;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
            g_stamps[wave * 8 + 4] = hw;
            g_stamps[wave * 8 + 5] = xcc;
        }
    }
}
__device__ __forceinline__ void stamp_val(uint64_t wave, int i, uint64_t v) {
    if ((threadIdx.x & 63u) == 0 && wave < (1u << 18)) g_stamps[wave * 8 + i] = v;
}
__device__ __forceinline__ void stage_stamp(uint32_t si, int i) {
    if ((threadIdx.x & 63u) == 0) g_stage_stamps[si * 8 + i] = __builtin_amdgcn_s_memrealtime();
}
}  // namespace
__device__ uint64_t g_win_stamps[1 << 20];  // per wave w < 2^15: the end of its windows 0..31 at [w * 32 + i]
namespace {
__device__ __forceinline__ void stamp_win(uint64_t wave, uint32_t i) {
    if ((threadIdx.x & 63u) == 0 && wave < (1u << 15) && i < 32u) g_win_stamps[wave * 32 + i] = __builtin_amdgcn_s_memrealtime();
}
#else
__device__ __forceinline__ void stamp_win(uint64_t, uint32_t) {}
__device__ __forceinline__ void stamp(uint64_t, int) {}
__device__ __forceinline__ void stamp_val(uint64_t, int, uint64_t) {}
__device__ __forceinline__ void stage_stamp(uint32_t, int) {}
#endif
constexpr uint32_t SEG = 256;  // window bases fetched per pass (16 code words, 8 N-mask words)

// 32-bit outer unshuffle (Hacker's Delight 7-2): odd bits to the upper half,
// even bits to the lower half, order kept.
__device__ __forceinline__ uint32_t unshuffle32(uint32_t x) {
    uint32_t t;
    t = (x ^ (x >> 1)) & 0x22222222u; x ^= t ^ (t << 1);
    t = (x ^ (x >> 2)) & 0x0c0c0c0cu; x ^= t ^ (t << 2);
    t = (x ^ (x >> 4)) & 0x00f000f0u; x ^= t ^ (t << 4);
    t = (x ^ (x >> 8)) & 0x0000ff00u; x ^= t ^ (t << 8);
    return x;
}

// Lane masks of P k-mers (dna2int layout, approx_counter.cpp:55-62):
// character i of pattern p at bit 31 - (i*P + p); ph holds the high bit of
// each character's 2-bit code, pl the low bit.  No per-character loop for the
// two packs the baseline configurations use (P = 2: k = 11..16, P = 1: k > 16).
template <int P>
__device__ __forceinline__ void build_masks(const uint64_t (&km)[P], uint32_t m, uint32_t& ph, uint32_t& pl) {
    if constexpr (P == 2) {
        // Left-aligned 2-bit codes already interleave a pattern's high and low
        // bits; the second pattern slots in one bit lower.
        const uint32_t a = (uint32_t)km[0] << (32u - 2u * m), b = (uint32_t)km[1] << (32u - 2u * m);
        ph = (a & 0xaaaaaaaau) | ((b & 0xaaaaaaaau) >> 1);
        pl = ((a << 1) & 0xaaaaaaaau) | (b & 0x55555555u);
    } else if constexpr (P == 1) {
        const uint64_t x = km[0] << (64u - 2u * m);
        const uint32_t H = unshuffle32((uint32_t)(x >> 32)), L = unshuffle32((uint32_t)x);
        ph = (H & 0xffff0000u) | (L >> 16);
        pl = (H << 16) | (L & 0xffffu);
    } else {
        ph = 0;
        pl = 0;
#pragma unroll
        for (int p = 0; p < P; ++p)
            for (uint32_t i = 0; i < m; ++i) {
                const uint32_t b = (uint32_t)(km[p] >> (2u * (m - 1u - i))) & 3u;
                ph |= (b >> 1) << (31u - (i * P + p));
                pl |= (b & 1u) << (31u - (i * P + p));
            }
    }
}

#ifdef AC_TID_BLOCKS_INC  // A/B builds (tools/variants.sh) of another generator setting
#include AC_TID_BLOCKS_INC
#else
#include "wm_tid_blocks.inc"
#endif

// Window descriptor (start, length) of window w with scalar loads: the arrays
// do not change during a launch, so the constant address space is legal, and
// both loads are in flight together (as vector loads hipcc waited for the
// start before issuing the length: two round trips per window).
typedef const __attribute__((address_space(4))) uint64_t* cu64p;
typedef const __attribute__((address_space(4))) uint32_t* cu32p;
__device__ __forceinline__ void load_desc(const uint64_t* start, const uint32_t* length, uint32_t w, uint64_t& base,
                                          uint32_t& len) {
#if !defined(AC_VECTOR_DESC)
    base = ((cu64p)start)[w];
    len = ((cu32p)length)[w];
#else
    base = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(start[w] >> 32)) << 32) |
           __builtin_amdgcn_readfirstlane((uint32_t)start[w]);
    len = __builtin_amdgcn_readfirstlane(length[w]);
#endif
}

// The same with vector loads, for staged launches: their descriptors are copied
// in by the kernel itself, so they DO change during the launch, and a scalar
// (constant address space) load could be hoisted above the staging wait or hit
// a scalar-cache line filled before it.
typedef const __attribute__((address_space(1))) uint64_t* gu64p;
typedef const __attribute__((address_space(1))) uint32_t* gu32p;
__device__ __forceinline__ void load_desc_vec(const uint64_t* start, const uint32_t* length, uint32_t w, uint64_t& base,
                                              uint32_t& len) {
    const uint64_t b = ((gu64p)start)[w];
    const uint32_t l = ((gu32p)length)[w];
    base = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
           __builtin_amdgcn_readfirstlane((uint32_t)b);
    len = __builtin_amdgcn_readfirstlane(l);
}

// The workgroup's ~Eq table (shared by its waves): for lane word w, word w*320 + c*64 + lane =
// the lane's ~Eq mask for character c (A C G T, then N = all ones), read per base with
// ds_read_addtid_b32.
template <int W>
struct TidTable {
    uint32_t e[W * 5 * 64];  // lane word w's table at e[w * 320]
};

// A window fetch: bases [pos, pos + 256) -- 16 code words and 8 N-mask words -- through buffer
// descriptors of the segment's two arrays (SGPRs); the byte offset is the window's (an SGPR) plus a
// per-lane constant.  The descriptors' range check (num_records = the array's bytes, voffset
// included) returns 0 for a word past the image, so no clamp: words past the window are never read
// as text (the chunk loop stops at the window length).  The consumer (tid_word) takes lanes 0-15's
// code words and lanes 16-23's N-mask words.
struct Image {
    __amdgpu_buffer_rsrc_t codes, nmask;
};
struct Fetch {
    uint32_t c, n;
};
__device__ __forceinline__ void tid_fetch(Fetch& f, const Image& im, uint64_t pos, uint32_t lane, uint32_t lane_off) {
    // Every lane loads both words -- code word (lane & 15) and N-mask word (lane & 7) of the segment;
    // lanes past 16 / 8 repeat addresses of the same lines, which the load coalesces -- so both results
    // are whole registers.  (Round 4 loaded each half under its own exec mask: hipcc then merged the
    // halves with the previous window's values, copying them back after a wait for both loads
    // -- s_waitcnt vmcnt(0) right after every prefetch inside multi-window items -- and computed the
    // second offset into the first load's destination, another wait.)
    (void)lane;
    f.c = __builtin_amdgcn_raw_buffer_load_b32(im.codes, (uint32_t)(pos >> 2) + (lane_off & 63u), 0, 0);
    f.n = __builtin_amdgcn_raw_buffer_load_b32(im.nmask, (uint32_t)(pos >> 3) + (lane_off >> 8), 0, 0);
}
__device__ __forceinline__ uint32_t tid_word(const Fetch& f, uint32_t lane) { return lane < 16u ? f.c : f.n; }

// start % 32 == 0 && length <= n_bases && start <= n_bases - length, on the
// scalar unit (hipcc compares 64-bit values with VALU ops), written so that no
// sum wraps: a start near 2^64 must not pass.
template <bool RFL>
__device__ __forceinline__ uint32_t window_valid(uint64_t base, uint32_t len, uint64_t nb) {
    // (RFL, the staged kernel: its early-counting gate leaves hipcc holding some of these
    // wave-uniform values in VGPRs; readfirstlane puts them back in SGPRs for the asm)
    const uint32_t nbl = RFL ? __builtin_amdgcn_readfirstlane((uint32_t)nb) : (uint32_t)nb;
    const uint32_t nbh = RFL ? __builtin_amdgcn_readfirstlane((uint32_t)(nb >> 32)) : (uint32_t)(nb >> 32);
    const uint32_t ln = RFL ? __builtin_amdgcn_readfirstlane(len) : len;
    const uint32_t bl = RFL ? __builtin_amdgcn_readfirstlane((uint32_t)base) : (uint32_t)base;
    const uint32_t bh = RFL ? __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32)) : (uint32_t)(base >> 32);
    uint32_t bad, t0, t1;
    asm("s_sub_u32 %[t0], %[nbl], %[len]\n\t"
        "s_subb_u32 %[t1], %[nbh], 0\n\t"  // scc: n_bases < length
        "s_cselect_b32 %[bad], 1, 0\n\t"
        "s_sub_u32 %[t0], %[t0], %[bl]\n\t"
        "s_subb_u32 %[t1], %[t1], %[bh]\n\t"  // scc: n_bases - length < start
        "s_cselect_b32 %[bad], 1, %[bad]\n\t"
        "s_and_b32 %[t0], %[bl], 31\n\t"  // scc: misaligned start
        "s_cselect_b32 %[bad], 1, %[bad]"
        : [bad] "=&s"(bad), [t0] "=&s"(t0), [t1] "=&s"(t1)
        : [nbl] "s"(nbl), [nbh] "s"(nbh), [len] "s"(ln), [bl] "s"(bl), [bh] "s"(bh)
        : "scc");
    return bad ^ 1u;
}

// The workgroup's waves serve one candidate group and share one table, the
// first LDS object, at address 0, so M0 needs no per-base add (the eb0 form of
// tools/gen_tid_blocks.py).
constexpr bool TID_EB0 = true;

// Workgroup LDS: the ~Eq table, then the count vector the waves sum into,
// then the staged launch's verdict for the workgroup's segment.
template <int W>
struct BlockLds {
    TidTable<W> tab;
    uint32_t cnt[W * AC_MAX_PACK * 64];
    uint32_t stage_r;
};

#ifndef AC_COPY_AHEAD
#define AC_COPY_AHEAD 32  // chunks a copier may run ahead of its segment's copied count (0: no limit; 8 / 16 / 32 measured, profiles/r03_m10/ab.log)
#endif
#ifndef AC_STAGE_LOAD_AUX
#define AC_STAGE_LOAD_AUX 2  // cache policy of the staging copy's loads: nt (A/B builds: 17 = sc0 sc1)
#endif

// Staged launch ("early launch"): the kernel is launched before
// the host has packed its inputs.  Wave 0 of every workgroup runs stage_copy
// before the workgroup reads the segment.  It claims tickets of the segment (an
// agent-scope counter): ticket 0 makes it the segment's only host poller,
// ticket c >= 1 the copier of AC_STAGE_CHUNK-byte chunk c - 1 of the region.
// The host packs the region front to back and publishes the packed N-free
// prefix (progress record) as it grows, then the final byte count and N verdict
// (flag).  The poller reads the header with one 16-byte system-scope load per
// poll (~2 us apart: one PCIe round trip) and republishes it in device words:
// the N-free bytes so far, then the final verdict, bytes and a final-seen word.
// A copier waits (polling the device words) until its chunk lies inside the
// N-free prefix -- so chunks cross PCIe while later ones are still being packed
// -- or the final header is out; it copies the chunk from the pinned block to
// device memory with write-through (sc1) stores, waits for them, stores the
// launch's generation into the chunk's flag and adds 1 to every replica of the
// segment's done counter.  Readers either wait for the done counter (the whole
// segment, then its N verdict), or -- equal-window segments -- count a window
// as soon as the chunks its fetches touch are flagged and lie in the N-free
// prefix (stage_gate).  No acquire: the copied lines were not in any L2 at
// launch start and are touched by no one before their flag says so (a fetch
// never reaches past the chunks checked for it, and 128-B lines never straddle
// chunks), so the readers' plain loads fetch them fresh (the hand-off form of
// MI355X_MICROARCH.md's visibility section).  Every wait is bounded
// (AC_STAGE_TIMEOUT_TICKS): a host that never flags makes the waves report
// AC_DEVERR_STAGE and skip, never hang.  (The chunk count covers the region's
// largest layout, N bitmap included, so the last chunk always waits for the
// final header: once the done counter is complete, the verdict words are written.)
struct StageWords {
    uint32_t* claim;
    uint32_t* verdict;  // ~0u: skip; else 1 = has N
    uint32_t* bytes;
    uint32_t* fin;      // 1 once verdict / bytes are written
    uint32_t* avail;    // N-free bytes of the region published so far: AC_STAGE_REPL replicas, one per line
    uint32_t* done;     // chunks copied: AC_STAGE_REPL replicas, one per line
};
__device__ __forceinline__ StageWords stage_words(uint32_t* words) {
    // (one word per line: a launch zeroes only word 0 of each line of the next launch's bank)
    return StageWords{words, words + AC_QUEUE_LINE, words + 2 * AC_QUEUE_LINE, words + 3 * AC_QUEUE_LINE,
                      words + 4 * AC_QUEUE_LINE, words + (4 + AC_STAGE_REPL) * AC_QUEUE_LINE};
}
// per chunk flag: one line each (a chunk's readers poll only its own line)
__device__ __forceinline__ uint32_t* chunk_flag(uint32_t* chunk_gen, uint32_t x) { return chunk_gen + x * AC_QUEUE_LINE; }
__device__ __forceinline__ const uint32_t* chunk_flag(const uint32_t* chunk_gen, uint32_t x) {
    return chunk_gen + x * AC_QUEUE_LINE;
}
__device__ __forceinline__ uint32_t wave_load(const uint32_t* p) {  // lane 0's agent-scope load, wave-uniform
    uint32_t v = 0;
    if ((threadIdx.x & 63u) == 0) v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ void wave_store(uint32_t* p, uint32_t v) {
    if ((threadIdx.x & 63u) == 0) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// A staged wait's bound: AC_STAGE_TIMEOUT_TICKS without progress.  The clock is read lazily -- only on
// a poll that saw no progress (the first such poll starts it), and progress() stops it -- so a wait
// that never stalls, e.g. a chunk copy whose chunk is already packed, reads no clock at all.
struct StageClock {
    uint64_t t0 = 0;
    __device__ __forceinline__ void progress() { t0 = 0; }
    __device__ __forceinline__ bool late() {
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (t0 == 0) {
            t0 = now;
            return false;
        }
        return now - t0 > AC_STAGE_TIMEOUT_TICKS;
    }
};

#ifndef AC_PACK_BLOCKS
#define AC_PACK_BLOCKS 4  // 32-base blocks whose host loads a packing lane keeps in flight at once
#endif
// 4 Dna5 bytes (one per base, ordinal 0-3 = A C G T, anything else N) -> the byte of their four
// 2-bit codes (base i at bits 2i..2i+1) and, in `n`, bit i set iff base i is N.
__device__ __forceinline__ uint32_t dna5_codes4(uint32_t x) {
    uint32_t c = x & 0x03030303u;
    c = (c | (c >> 6)) & 0x000f000fu;  // bases 0-1 at bits 0-3, bases 2-3 at bits 16-19
    return (c | (c >> 12)) & 0xffu;
}
__device__ __forceinline__ uint32_t dna5_n4(uint32_t x) {
    const uint32_t t = x & 0xfcfcfcfcu;                                  // nonzero byte <=> ordinal >= 4
    const uint32_t nz = (((t & 0x7f7f7f7fu) + 0x7f7f7f7fu) | t) & 0x80808080u;  // bit 7 of each such byte
    return (((nz >> 7) * 0x00204081u) >> 21) & 0xfu;                    // bits 7, 15, 23, 31 -> 0..3
}

// Device packing of codes chunk `lo_b` (byte offset in the codes section) of an
// equal-window segment: the windows whose slots overlap the chunk are read as Dna5 bytes from
// pinned host memory (offset of window w at offs[w], relative to src; src_bytes readable), one
// window per lane, and packed exactly as the host packer does (host_pack.cpp pack_dna5_range with
// records): 2-bit codes, padding bases code 0, the window's inline N record (nrec.h) in the top bits
// of its slot's last code word when the segment has records (rec), and its N-bitmap words.  Only
// the code words inside the chunk are stored (a slot that straddles two chunks is packed by both
// owners, each storing its own words), with write-through stores like the copy; the N-bitmap words
// of the chunk's blocks go to the bitmap section (read only by a window whose record overflowed, or
// by every window of a segment without records, and then only once the whole segment is in).
// A window outside src_bytes is stored as zeros and reported (AC_DEVERR_WINDOW).
// Each PCIe round trip costs ~2 us: a lane has its next windows' offsets in flight while it packs,
// and all of a window's loads (AC_PACK_BLOCKS blocks of 32 bases) in flight together.
struct PackOut {
    uint32_t cnt = 0, pos = 0, last_lo = 0, last_hi = 0;
};
struct PackCtx {
    __amdgpu_buffer_rsrc_t rc, rn;
    uint32_t ulen, nblk, SW, cw_lo, cw_hi, cap, pb;
};
typedef uint32_t pk_v2u __attribute__((ext_vector_type(2)));
typedef uint32_t pk_v4u __attribute__((ext_vector_type(4)));
// One 32-base block b of a window from its 9 loaded dwords (the 32 bytes from byte `sh` of the first).
__device__ __forceinline__ void pack_block(const PackCtx& pc, const pk_v4u& d0, const pk_v4u& d1, uint32_t e, uint32_t b,
                                           bool ok, uint32_t sh, uint32_t cw_w, PackOut& o) {
    const uint32_t raw[9] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w, e};
    const uint32_t nv = ok ? min(32u, pc.ulen - 32u * b) : 0u;  // real bases of the block
    uint32_t code0 = 0, code1 = 0, nmw = 0;
#pragma unroll
    for (uint32_t q = 0; q < 8; ++q) {
        uint32_t x = (uint32_t)((((uint64_t)raw[q + 1] << 32) | raw[q]) >> (8u * sh));
        const uint32_t have = nv > 4u * q ? nv - 4u * q : 0u;  // bytes of this dword that are bases
        x = have >= 4u ? x : (have ? x & ((1u << (8u * have)) - 1u) : 0u);
        if (q < 4) code0 |= dna5_codes4(x) << (8u * q);
        else code1 |= dna5_codes4(x) << (8u * (q - 4u));
        nmw |= dna5_n4(x) << (4u * q);
    }
    for (uint32_t m = nmw; m; m &= m - 1u) {  // the record's N positions, in window order
        if (o.cnt < pc.cap) o.pos |= (32u * b + (uint32_t)__builtin_ctz(m)) << nrec_pos_shift(pc.pb, o.cnt);
        ++o.cnt;
    }
    const uint32_t cw = cw_w + 2u * b;
    const bool mine = cw >= pc.cw_lo && cw < pc.cw_hi;  // (a block never straddles a chunk)
    if (b + 1u == pc.nblk) {  // the slot's last block: its second word takes the record
        o.last_lo = code0;
        o.last_hi = code1;
    } else if (mine) {
        __builtin_amdgcn_raw_buffer_store_b64(pk_v2u{code0, code1}, pc.rc, cw * 4u, 0, 16);  // sc1
    }
    if (mine) __builtin_amdgcn_raw_buffer_store_b32(nmw, pc.rn, cw * 2u, 0, 16);
}
__device__ __forceinline__ void pack_finish(const PackCtx& pc, uint32_t rec, uint32_t cw_w, PackOut& o) {
    if (rec && o.cnt) o.last_hi |= o.cnt <= pc.cap ? (o.pos | o.cnt << 29) : (NREC_OVERFLOW << 29);
    const uint32_t cw = cw_w + pc.SW - 2u;
    if (cw >= pc.cw_lo && cw < pc.cw_hi)
        __builtin_amdgcn_raw_buffer_store_b64(pk_v2u{o.last_lo, o.last_hi}, pc.rc, cw * 4u, 0, 16);
}

__device__ __forceinline__ void stage_pack_chunk(const uint8_t* src, const uint64_t* offs, uint32_t src_bytes,
                                                 uint32_t n_windows, uint32_t ulen, uint32_t rec, uint32_t code_bytes,
                                                 uint8_t* codes_dst, uint8_t* nmask_dst, uint32_t lo_b, uint32_t* err) {
    const uint32_t lane = threadIdx.x & 63u;
    PackCtx pc;
    pc.ulen = ulen;
    pc.SW = ((ulen + 31u) & ~31u) / 16u;  // code words per slot (2..16)
    pc.nblk = pc.SW / 2u;                 // 32-base blocks per slot, each holding real bases
    const uint32_t hi_b = min(lo_b + AC_STAGE_CHUNK, code_bytes);
    pc.cw_lo = lo_b / 4u;
    pc.cw_hi = hi_b / 4u;  // the chunk's code words
    pc.cap = nrec_cap(ulen);
    pc.pb = nrec_pos_bits(ulen);
    const uint32_t w0 = pc.cw_lo / pc.SW, w1 = min(n_windows, (pc.cw_hi + pc.SW - 1u) / pc.SW);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, (int)src_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void*)offs, 0, (int)(n_windows * 8u), 0x00020000);
    pc.rc = __builtin_amdgcn_make_buffer_rsrc((void*)codes_dst, 0, (int)code_bytes, 0x00020000);
    pc.rn = __builtin_amdgcn_make_buffer_rsrc((void*)nmask_dst, 0, (int)(code_bytes / 2u), 0x00020000);
    uint32_t bad = 0;
    // The offsets of the lane's first two windows in one round trip (a chunk holds <= 128 slots of
    // >= 128 bases, 2 rounds of 64; shorter slots take more rounds, their offsets loaded per round).
    pk_v2u onext = w0 + lane < w1 ? __builtin_amdgcn_raw_buffer_load_b64(ro, (w0 + lane) * 8u, 0, 0) : pk_v2u{0u, 0u};
    pk_v2u onext2 = w0 + lane + 64u < w1 ? __builtin_amdgcn_raw_buffer_load_b64(ro, (w0 + lane + 64u) * 8u, 0, 0)
                                          : pk_v2u{0u, 0u};
    constexpr uint32_t PB = AC_PACK_BLOCKS;  // blocks per pass: their loads in flight together
    for (uint32_t w = w0 + lane; w < w1; w += 64u) {
        const pk_v2u ov = onext;
        onext = onext2;
        if (w + 128u < w1) onext2 = __builtin_amdgcn_raw_buffer_load_b64(ro, (w + 128u) * 8u, 0, 0);
        const bool ok = ov.y == 0u && ov.x <= src_bytes - ulen;  // (the host checked src_bytes >= ulen)
        bad |= ok ? 0u : 1u;
        const uint32_t off = ok ? ov.x : 0u, a = off & ~3u, sh = off & 3u;  // out of range: read as zeros
        PackOut o;
#pragma unroll 1
        for (uint32_t b0 = 0; b0 < pc.nblk; b0 += PB) {
            pk_v4u d[PB][2];
            uint32_t e[PB];
#pragma unroll
            for (uint32_t i = 0; i < PB; ++i)
                if (b0 + i < pc.nblk) {
                    const uint32_t x = a + 32u * (b0 + i);
                    d[i][0] = __builtin_amdgcn_raw_buffer_load_b128(rs, x, 0, 0);
                    d[i][1] = __builtin_amdgcn_raw_buffer_load_b128(rs, x + 16u, 0, 0);
                    e[i] = __builtin_amdgcn_raw_buffer_load_b32(rs, x + 32u, 0, 0);
                }
#pragma unroll
            for (uint32_t i = 0; i < PB; ++i)
                if (b0 + i < pc.nblk) pack_block(pc, d[i][0], d[i][1], e[i], b0 + i, ok, sh, w * pc.SW, o);
        }
        pack_finish(pc, rec, w * pc.SW, o);
    }
    if (__ballot(bad != 0u) && lane == 0) atomicOr(err, AC_DEVERR_WINDOW);
}

// Claims and serves tickets until none is left; false on timeout.  Chunks below `pre_chunks` (the
// k-mer section, in place in the pinned block before the launch) are copied without waiting.
__device__ __attribute__((noinline)) bool stage_copy(const uint8_t* src, uint8_t* dst, uint32_t chunks,
                                                     uint32_t pre_chunks, uint32_t* hdr, uint32_t* words,
                                                     uint32_t* chunk_gen, uint32_t gen, uint32_t si) {
    const uint32_t lane = threadIdx.x & 63u;
    const StageWords sw = stage_words(words);
    StageClock clk;
    for (;;) {
        uint32_t c = 0;
        if (lane == 0) c = __hip_atomic_fetch_add(sw.claim, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        c = __builtin_amdgcn_readfirstlane(c);
        if (c > chunks) return true;
        clk.progress();  // (each ticket's wait is bounded on its own)
        if (c == 0) {  // the segment's host poller
            // The header's four words in ONE 16-byte system-scope load (one PCIe read): the host
            // stores the progress record as one 8-byte store and the flag after INFO, so a read
            // that returns the flag returns the INFO stored before it.
            typedef uint32_t v4u __attribute__((ext_vector_type(4)));
            static_assert(AC_HDR_PGEN == 0 && AC_HDR_READY == 1 && AC_HDR_FLAG == 2 && AC_HDR_INFO == 3,
                          "header layout");
            const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc((void*)hdr, 0, 16, 0x00020000);
            uint32_t published = 0;
            for (;;) {
                const v4u hv = __builtin_amdgcn_raw_buffer_load_b128(rh, 0, 0, 17);  // sc0 sc1: system scope
                uint32_t ready = __builtin_amdgcn_readfirstlane(hv.x) == gen ? __builtin_amdgcn_readfirstlane(hv.y) : 0u;
                const bool fin = __builtin_amdgcn_readfirstlane(hv.z) == gen;
                uint32_t verdict = 0, bytes = 0;
                if (fin) {
                    const uint32_t info = __builtin_amdgcn_readfirstlane(hv.w);
                    bytes = info & ~AC_HDR_INFO_HAS_N;
                    verdict = (info == AC_HDR_INFO_ABORT || bytes > chunks * AC_STAGE_CHUNK || ready > bytes)
                                  ? ~0u
                                  : (info & AC_HDR_INFO_HAS_N ? 1u : 0u);
                    if (verdict == 0u) ready = bytes;  // no N anywhere: the whole region is N-free
                    // the final words before the prefix they complete: a copier released by the prefix can
                    // finish the segment's last chunk, and a reader that then sees the done count complete
                    // reads the verdict (so it must be there first)
                    wave_store(sw.verdict, verdict);
                    wave_store(sw.bytes, verdict == ~0u ? 0u : bytes);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                if (verdict != ~0u && ready > published && ready <= chunks * AC_STAGE_CHUNK) {
                    if (published == 0) stage_stamp(si, 1);
                    if (published <= pre_chunks * AC_STAGE_CHUNK && ready > pre_chunks * AC_STAGE_CHUNK) stage_stamp(si, 3);
                    if (lane < AC_STAGE_REPL)  // every replica in one wave instruction
                        __hip_atomic_store(sw.avail + lane * AC_QUEUE_LINE, ready, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    published = ready;
                    clk.progress();  // the host is making progress
                }
                if (fin) {
                    stage_stamp(si, 0);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    wave_store(sw.fin, 1u);
                    break;
                }
                if (clk.late()) return false;
                __builtin_amdgcn_s_sleep(8);
            }
            continue;
        }
        // copier of chunk c - 1: wait until it lies inside the N-free prefix or the segment is final
        const uint32_t x = c - 1u, lo = x * AC_STAGE_CHUNK, hi = lo + AC_STAGE_CHUNK;
        uint32_t* my_avail = sw.avail + (x % AC_STAGE_REPL) * AC_QUEUE_LINE;
        uint32_t limit = x < pre_chunks ? hi : 0u;  // bytes of the region known to be valid
        uint32_t seen = 0;  // N-free bytes seen published (the wait's clock restarts when they grow)
        while (limit == 0u) {
            // both words in one wave instruction (lane 0: N-free bytes, lane 1: final seen)
            uint32_t v = 0;
            if (lane < 2u) v = __hip_atomic_load(lane ? sw.fin : my_avail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t av = __builtin_amdgcn_readlane(v, 0);
            if (av >= hi) {
                limit = hi;
                break;
            }
            if (__builtin_amdgcn_readlane(v, 1)) {
                limit = wave_load(sw.verdict) == ~0u ? 0u : wave_load(sw.bytes);
                break;
            }
            if (av > seen) {
                seen = av;
                clk.progress();
            } else if (clk.late()) {
                return false;
            }
            __builtin_amdgcn_s_sleep(8);
        }
#if AC_COPY_AHEAD
        // In chunk order: at most AC_COPY_AHEAD chunks of the segment in flight ahead of the copied
        // count, so the first windows' chunks are not held up behind the whole region's PCIe reads
        // (a segment packed before the poller's first look released all its copiers at once and the
        // first codes chunk landed anywhere in the next 5-18 us: profiles/r03_m9/stamps.log).
        if (x >= AC_COPY_AHEAD) {
            uint32_t* my_done = sw.done + (x % AC_STAGE_REPL) * AC_QUEUE_LINE;
            uint32_t dn = 0, dseen = 0;
            clk.progress();
            while ((dn = wave_load(my_done)) < x - AC_COPY_AHEAD) {
                if (dn > dseen) {  // (the copies ahead of it are moving)
                    dseen = dn;
                    clk.progress();
                } else if (clk.late()) {
                    return false;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
#endif
        if (limit > lo) {
            // range-checked descriptors: bytes past the valid prefix read as 0 and are not stored
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, (int)limit, 0x00020000);
            const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)dst, 0, (int)limit, 0x00020000);
            typedef uint32_t v4u __attribute__((ext_vector_type(4)));
            v4u v[4];
            const uint32_t o = lo + lane * 16u;
#pragma unroll
            // (nontemporal, like the copy kernel's loads of the same pinned block: nothing read these
            // lines before the flag in this launch, so no cache holds them; system-scope loads
            // were split into narrow PCIe reads: 330 KB took ~15 us instead of ~6)
            for (int u = 0; u < 4; ++u) v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, o + u * 1024u, 0, AC_STAGE_LOAD_AUX);
#pragma unroll
            for (int u = 0; u < 4; ++u) __builtin_amdgcn_raw_buffer_store_b128(v[u], rd, o + u * 1024u, 0, 16);  // sc1
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        wave_store(chunk_flag(chunk_gen, x), gen);
        uint32_t prev = 0;
        if (lane < AC_STAGE_REPL)
            prev = __hip_atomic_fetch_add(sw.done + lane * AC_QUEUE_LINE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__builtin_amdgcn_readfirstlane(prev) + 1u == chunks) stage_stamp(si, 2);  // (diagnostic builds) last chunk in
        if (x == pre_chunks) stage_stamp(si, 4);  // (diagnostic builds) first codes chunk in
    }
}

// The copier loop of a device-packed segment: the host published nothing and packs
// nothing -- its Dna5 bytes sit in pinned memory from before the launch -- so ticket 0 publishes the
// segment's final words at once (no header read over PCIe): the verdict (1: the N bitmap is there for
// the windows that need it), the byte count, the whole region as available (with inline N records;
// without them only the k-mers, so readers wait for the whole segment and its bitmap) and `fin`.
// Tickets c >= 1: k-mer chunks are copied from the staging block, codes chunks packed from the Dna5
// bytes (stage_pack_chunk), N-bitmap chunks have no work of their own (their words are stored by the
// codes chunks' owners); then, as in stage_copy, the chunk's flag and the done replicas -- only once
// `fin` is out, so a reader that sees the segment complete reads its verdict.  Inlined into the
// kernel: as a called function its registers came from the budget of the 8-wave kernels (64 VGPRs)
// and it spilled inside the packing loop.
__device__ __forceinline__ bool stage_copy_dp(const SegDev& sg, uint32_t* words, uint32_t gen, uint32_t* err) {
    const uint32_t lane = threadIdx.x & 63u;
    const StageWords sw = stage_words(words);
    const uint32_t chunks = sg.stage_chunks, pre_chunks = sg.stage_codes_off / AC_STAGE_CHUNK;
    const uint32_t code_bytes = (uint32_t)(sg.n_bases >> 2);
    const uint32_t nmask_off = pre_chunks * AC_STAGE_CHUNK + ((code_bytes + 255u) & ~255u);  // (256-B aligned sections)
    StageClock clk;
    bool fin_seen = false;
    for (;;) {
        uint32_t c = 0;
        if (lane == 0) c = __hip_atomic_fetch_add(sw.claim, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        c = __builtin_amdgcn_readfirstlane(c);
        if (c > chunks) return true;
        clk.progress();
        if (c == 0) {
            const uint32_t bytes = chunks * AC_STAGE_CHUNK;  // (the host sized the region: codes + bitmap)
            wave_store(sw.verdict, 1u);
            wave_store(sw.bytes, bytes);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane < AC_STAGE_REPL)
                __hip_atomic_store(sw.avail + lane * AC_QUEUE_LINE, sg.nrec ? bytes : sg.stage_codes_off,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            wave_store(sw.fin, 1u);
            continue;
        }
        const uint32_t x = c - 1u, lo = x * AC_STAGE_CHUNK;
#if AC_COPY_AHEAD
        if (x >= AC_COPY_AHEAD) {  // in chunk order, as stage_copy
            uint32_t* my_done = sw.done + (x % AC_STAGE_REPL) * AC_QUEUE_LINE;
            uint32_t dn = 0, dseen = 0;
            while ((dn = wave_load(my_done)) < x - AC_COPY_AHEAD) {
                if (dn > dseen) {
                    dseen = dn;
                    clk.progress();
                } else if (clk.late()) {
                    return false;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
#endif
        if (x < pre_chunks) {  // k-mers: in the pinned staging block since before the launch
            typedef uint32_t v4u __attribute__((ext_vector_type(4)));
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)sg.stage_src, 0, (int)(pre_chunks * AC_STAGE_CHUNK), 0x00020000);
            const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)sg.stage_dst, 0, (int)(pre_chunks * AC_STAGE_CHUNK), 0x00020000);
            v4u v[4];
            const uint32_t o = lo + lane * 16u;
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, o + u * 1024u, 0, AC_STAGE_LOAD_AUX);
#pragma unroll
            for (int u = 0; u < 4; ++u) __builtin_amdgcn_raw_buffer_store_b128(v[u], rd, o + u * 1024u, 0, 16);  // sc1
        } else if (lo - pre_chunks * AC_STAGE_CHUNK < code_bytes) {
            stage_pack_chunk(sg.dp_src, sg.dp_off, sg.dp_src_bytes, sg.n_windows, sg.ulen, sg.nrec, code_bytes,
                             sg.stage_dst + pre_chunks * AC_STAGE_CHUNK, sg.stage_dst + nmask_off,
                             lo - pre_chunks * AC_STAGE_CHUNK, err);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        while (!fin_seen) {  // (ticket 0's words out before the first chunk counts as done)
            fin_seen = wave_load(sw.fin) != 0u;
            if (!fin_seen) {
                if (clk.late()) return false;
                __builtin_amdgcn_s_sleep(2);
            }
        }
        wave_store(chunk_flag(sg.stage_gen, x), gen);
        if (lane < AC_STAGE_REPL)
            __hip_atomic_fetch_add(sw.done + lane * AC_QUEUE_LINE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Waits for the whole segment (every chunk copied): its N verdict (0 / 1), or ~0u to skip it.
__device__ __attribute__((noinline)) uint32_t stage_wait_all(uint32_t* words, uint32_t chunks, uint32_t replica,
                                                             uint32_t* err) {
    const StageWords sw = stage_words(words);
    StageClock clk;
    uint32_t dn = 0, seen = 0;
    while ((dn = wave_load(sw.done + replica * AC_QUEUE_LINE)) < chunks) {
        if (dn > seen) {  // copies are landing: the wait's clock restarts
            seen = dn;
            clk.progress();
        } else if (clk.late()) {
            if ((threadIdx.x & 63u) == 0) atomicOr(err, AC_DEVERR_STAGE);
            return ~0u;
        }
        __builtin_amdgcn_s_sleep(16);
    }
    // No acquire fence: it would only invalidate this CU's L1, and no CU can hold a line of the
    // region (nothing reads it before the counter says it is complete, and a launch starts with
    // clean caches).  With 8 workgroups per CU the fences cost ~8 us of staging per call (an A/B:
    // profiles/r03_m1/summary.log; -DAC_STAGE_ACQUIRE builds restore it).  Stale-line hazards are
    // what tests/test_gpu_jobs.py::test_early_launch_rotating_inputs_bit_exact rotates data for.
#ifdef AC_STAGE_ACQUIRE
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    return wave_load(sw.verdict);
}

#ifndef AC_GATE_SLEEP
#define AC_GATE_SLEEP 12  // s_sleep units (64 clocks) between a gate's polls
#endif
// Early counting: waits until region bytes [r0, r1) are in device memory (their chunks flagged)
// and inside the N-free prefix, or until the whole segment is in.  Low word: 2 for "count it
// with an all-zero N bitmap" (high word: the byte where the checked chunks' N-free part ends, at
// least r1), the
// segment's verdict (0 / 1) once it is complete, ~0u to skip (timeout: error bit set).
__device__ __forceinline__ uint64_t stage_gate(uint32_t* words, const uint32_t* chunk_gen, uint32_t chunks,
                                                         uint32_t replica, uint32_t gen, uint32_t r0, uint32_t r1,
                                                         uint32_t* err, uint32_t pre = 0u) {
    const uint32_t lane = threadIdx.x & 63u;
    const StageWords sw = stage_words(words);
    StageClock clk;
    const uint32_t x0 = r0 / AC_STAGE_CHUNK, x1 = (r1 - 1u) / AC_STAGE_CHUNK;
    // (more chunks than lanes, or past the launch's chunks: wait for the whole segment)
    const uint32_t nx = (x1 < chunks && x1 - x0 < 62u) ? x1 - x0 + 1u : 0u;
    bool in_prefix = nx && r1 <= pre;  // the N-free prefix covers [r0, r1) (it only grows; `pre`: at launch)
    uint32_t seen = 0;  // done + N-free bytes last seen (the wait's clock restarts when they move)
    for (;;) {
        // one wave instruction: lane 0 the done count, lane 1 the N-free bytes (this workgroup's
        // replicas), lanes 2.. the chunks' flags once the prefix covers them
        const uint32_t* p = lane == 0u ? sw.done + replica * AC_QUEUE_LINE
                          : lane == 1u ? sw.avail + replica * AC_QUEUE_LINE
                                       : (in_prefix && lane - 2u < nx ? chunk_flag(chunk_gen, x0 + (lane - 2u)) : nullptr);
        uint32_t v = 0;
        if (p) v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t dn = __builtin_amdgcn_readlane(v, 0), av = __builtin_amdgcn_readlane(v, 1);
        if (dn >= chunks) return wave_load(sw.verdict);
        const uint64_t miss = __ballot(lane >= 2u && lane - 2u < nx && v != gen);
        if (in_prefix && miss == 0) {
            // the chunks checked, up to where the N-free prefix ends: once the final header is out a
            // flagged chunk may reach past it, and its bytes there can hold N
            const uint32_t lim = av > pre ? av : pre, hi = (x1 + 1u) * AC_STAGE_CHUNK;
            return ((uint64_t)(hi < lim ? hi : lim) << 32) | 2u;
        }
        in_prefix = nx && (r1 <= pre || av >= r1);
        if (dn + av != seen) {
            seen = dn + av;
            clk.progress();
        } else if (clk.late()) {
            if (lane == 0) atomicOr(err, AC_DEVERR_STAGE);
            return ~0u;
        }
        if (!in_prefix) __builtin_amdgcn_s_sleep(AC_GATE_SLEEP);
    }
}

// The NFA blocks over the wave's W lane-word states (two words: the generated
// tid2_* blocks, one base's SALU work and text shared by both words).
#define AC_NFA(nb, s, ...)                                            \
    do {                                                              \
        if constexpr (W == 2)                                         \
            tid2_block##nb<P, TID_EB0>(s[0], s[W - 1], __VA_ARGS__); \
        else                                                          \
            tid_block##nb<P, TID_EB0>(s[0], __VA_ARGS__);            \
    } while (0)
#define AC_NFA_FIRST(s, ...)                                               \
    do {                                                                   \
        if constexpr (W == 2)                                              \
            tid2_block32_first<P, TID_EB0>(s[0], s[W - 1], __VA_ARGS__); \
        else                                                               \
            tid_block32_first<P, TID_EB0>(s[0], __VA_ARGS__);            \
    } while (0)

// The remainder (< 16 bases) of a segment: blocks of 8, 4, 2, 1 bases.
template <int P, int W>
__device__ __forceinline__ void tid_tail(TidNfa* s, uint32_t code, uint32_t nm, uint32_t rem, uint32_t eb) {
    if (rem & 8u) {
        AC_NFA(8, s, code, nm & 0xffu, eb);
        code >>= 16;
        nm >>= 8;
    }
    if (rem & 4u) {
        AC_NFA(4, s, code, nm & 0xfu, eb);
        code >>= 8;
        nm >>= 4;
    }
    if (rem & 2u) {
        AC_NFA(2, s, code, nm & 0x3u, eb);
        code >>= 4;
        nm >>= 2;
    }
    if (rem & 1u) AC_NFA(1, s, code, nm & 0x1u, eb);
}

// STAGED: the early-launch instantiation (staging wait, vector descriptor loads,
// system-scope count stores, tagged completion).  The plain launches get a kernel
// without any of it: in one kernel the extra live values cost SGPR spills inside
// the count loop (+2.5 % VALU, +3.4 % SALU instructions, ~5 % time at cfg2).
// EQ: every live segment holds equal windows back to back (ulen set; the host has checked that they
// fit the image): window places by arithmetic, no descriptor arrays or per-window range checks held
// in registers (the staged kernel spilled SGPRs inside the count loop without this).
template <int P, bool STAGED, bool EQ>
__device__ __forceinline__ void count_body(const LaunchArgs& a, BlockLds<words_for(P, STAGED)>& lds) {
    constexpr int W = words_for(P, STAGED);
    const uint32_t lane = threadIdx.x & 63u;
    // Workgroup b serves one block-queue (all its waves on one candidate
    // group); its waves take the block-queue's AC_WAVES_PER_BLOCK sub-queues.
    const uint32_t wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t wave = (uint64_t)blockIdx.x * WAVES_PER_BLOCK + wib;
    stamp(wave, 0);
    const uint32_t nqb = a.n_queues / WAVES_PER_BLOCK;
    const uint32_t blocks = (uint32_t)(a.total_waves / WAVES_PER_BLOCK);

    // Workgroups are dealt round-robin over the block-queues, so every
    // sub-queue is served by waves of every dispatch age (see the work-queue
    // comment below); q -> (segment, candidate group g, sub-queue j of that group).
    const uint32_t rank = blockIdx.x / nqb;
    // Rank r's workgroups are dealt to the block-queues rotated by shift(r):
    // with a plain b mod nqb deal every workgroup a CU receives belongs to one
    // block-queue, so each candidate group ran on a fixed slice of the chip
    // and inherited its speed (stamps: group median ends 93-101 us, the same
    // order run after run), with no stealing across groups to even it out.
    // Rotated, a CU's workgroups come from all groups and every group runs on
    // every XCD: group median ends 95.1-96.1 us, cfg2 kernel 109.6 -> 103.8 us
    // (profiles/r01_kernel_log.md, round 2).
    auto shift = [&](uint32_t r) { return (r + (r >> 3) * 4u) % nqb; };
    const uint32_t bq = (blockIdx.x % nqb + shift(rank)) % nqb;
    // workgroups dealt to block-queue qb (a complete rank gives each one; the
    // partial last rank the blocks % nqb queues from shift(last) on)
    auto wgs_of = [&](uint32_t qb) {
        return blocks / nqb + ((qb + nqb - shift(blocks / nqb)) % nqb < blocks % nqb ? 1u : 0u);
    };
    const uint32_t q = bq * WAVES_PER_BLOCK + wib;
    int si = 0;
#pragma unroll
    for (int i = 1; i < AC_MAX_SEGS; ++i)
        if (i < (int)a.n_segs && q >= a.seg[i].queue_begin) si = i;
    const SegDev& sg = a.seg[si];
    const uint32_t ql = q - sg.queue_begin;
    // A group's sub-queues are contiguous (g * subq + j), so a workgroup's
    // sub-queues lie in one group.
    const uint32_t g = ql / sg.subq, j = ql % sg.subq;
    // The segment's arrays, pinned in SGPRs for the whole launch: read through the `sg` reference hipcc reloaded them from
    // the kernel arguments in every window, each load waited for on the spot.  The image through buffer
    // descriptors (range-checked fetches, tid_fetch); images are < 2^34 bases (checked on the host), so
    // every byte offset fits 32 bits.
    // (inputs pinned in SGPRs by an asm operand: hipcc must see them wave-uniform, or it wraps every
    // fetch in a waterfall loop)
    // Staged launch: the segment's inputs are not there yet; wave 0 stages them (stage_wait), the
    // workgroup's other waves wait at a barrier, then everyone reads the verdict from LDS.
    uint32_t has_n = sg.has_n;
    bool skip = false;
    // Early counting (staged, equal windows): `partial` while the segment is not known complete;
    // a window is then fetched only once stage_gate has seen the chunks its fetches touch in
    // device memory and inside the N-free prefix ([v_lo, v_hi): chunks already checked), and
    // counted with an all-zero N bitmap.
    bool partial = false;
    uint32_t v_lo = 0, v_hi = 0;
    uint32_t* st_words = nullptr;
    if (STAGED && sg.stage_chunks) {  // (a segment sent ahead of a staged launch has no chunks)
        st_words = a.stage + AC_STAGE_L_SEG(si) * AC_QUEUE_LINE;
        // the k-mer section fills whole chunks and is in the pinned block before the launch
        const uint32_t pre_bytes = sg.stage_codes_off;
        if (blockIdx.x < a.copier_wgs) {
            // Copier workgroup: every wave serves every segment's tickets, starting
            // with segment (workgroup mod segments) -- the host packs a large call's jobs interleaved,
            // so all segments arrive together -- before the workgroup counts like the others.
            for (uint32_t i2 = 0; i2 < a.n_segs; ++i2) {
                const uint32_t s2 = (blockIdx.x + i2) % a.n_segs;
                const SegDev& c2 = a.seg[s2];
                if (!c2.stage_chunks) continue;
#ifndef AC_NO_DEVICE_PACK
                const bool ok = c2.dp_src
                                    ? stage_copy_dp(c2, a.stage + AC_STAGE_L_SEG(s2) * AC_QUEUE_LINE, a.gen, a.err)
                                    : stage_copy(c2.stage_src, c2.stage_dst, c2.stage_chunks,
                                                 c2.stage_codes_off / AC_STAGE_CHUNK, a.host_hdr + s2 * AC_QUEUE_LINE,
                                                 a.stage + AC_STAGE_L_SEG(s2) * AC_QUEUE_LINE, c2.stage_gen, a.gen, s2);
#else  // (A/B builds without the device packer: its code out of the staged kernel, the host never asks for it)
                const bool ok = stage_copy(c2.stage_src, c2.stage_dst, c2.stage_chunks, c2.stage_codes_off / AC_STAGE_CHUNK,
                                           a.host_hdr + s2 * AC_QUEUE_LINE, a.stage + AC_STAGE_L_SEG(s2) * AC_QUEUE_LINE,
                                           c2.stage_gen, a.gen, s2);
#endif
                if (!__builtin_amdgcn_readfirstlane((uint32_t)ok))
                    if (lane == 0) atomicOr(a.err, AC_DEVERR_STAGE);
            }
        }
        if (wib == 0) {
            uint32_t r = ~0u;
            const bool equal = sg.ulen != AC_NO_ULEN && sg.n_kmers;
            // (the copier workgroups stage every chunk: a launch with chunks has them, capi.cpp
            // stage_copiers; round 3's wave-0 tickets in every workgroup were removed in round 5)
            if (!a.copier_wgs) {
                if (lane == 0) atomicOr(a.err, AC_DEVERR_STAGE);
            } else if (equal) {
                // only the k-mers (the ~Eq table) are needed before counting starts
                r = (uint32_t)stage_gate(st_words, sg.stage_gen, sg.stage_chunks, blockIdx.x % AC_STAGE_REPL, a.gen, 0u,
                                         8u * sg.n_kmers, a.err, pre_bytes);
            } else {
                r = stage_wait_all(st_words, sg.stage_chunks, blockIdx.x % AC_STAGE_REPL, a.err);
            }
            if (lane == 0) lds.stage_r = r;
            stamp(wave, 7);  // diagnostic builds (staged): the staging wait is over
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        const uint32_t r = __builtin_amdgcn_readfirstlane(lds.stage_r);
        skip = r == ~0u;
        partial = r == 2u;
        has_n = (skip || partial) ? 0u : r;
    }
    const uint32_t* codes_p = sg.codes;
    const uint32_t* nmask_p = sg.nmask;
    // (an N-free image: a zero-sized N-bitmap descriptor, whose loads all return 0 without a memory access)
    // (a segment with inline N records never fetches bitmap words with its windows: only a window
    // whose record overflowed reads its own, through a descriptor made for it)
    uint32_t code_bytes = (uint32_t)(sg.n_bases >> 2),
             nmask_bytes = (has_n && !sg.nrec) ? (uint32_t)(sg.n_bases >> 3) : 0u;
    asm volatile("" : "+s"(codes_p), "+s"(nmask_p), "+s"(code_bytes), "+s"(nmask_bytes));
    Image im;
    im.codes = __builtin_amdgcn_make_buffer_rsrc((void*)codes_p, 0, (int)code_bytes, 0x00020000);
    im.nmask = __builtin_amdgcn_make_buffer_rsrc((void*)nmask_p, 0, (int)nmask_bytes, 0x00020000);
    const uint64_t* g_start = sg.start;
    const uint32_t* g_length = sg.length;
    uint64_t g_nbases = sg.n_bases;
    // (the claim counters stay addressed from the kernel argument: an opaque
    // pointer would turn the claim into a flat atomic, which also counts in
    // lgkmcnt and so would be waited for by the NFA blocks' LDS waits)
    uint32_t* g_queue = a.queue + ((uint64_t)a.bank * a.qstride + sg.queue_begin + g * sg.subq) * AC_QUEUE_LINE;
    if constexpr (!EQ) asm volatile("" : "+s"(g_start), "+s"(g_length), "+s"(g_nbases));
    // Equal windows packed back to back (the host-buffer stage's image): descriptors by arithmetic.
    uint32_t ulen = sg.ulen;
    asm volatile("" : "+s"(ulen));
    const uint32_t ustride = ulen == AC_NO_ULEN ? 0u : (ulen + 31u) & ~31u;
    // The segment's fields read inside the window loop, pinned: under the staged kernel's SGPR
    // pressure hipcc otherwise reloaded them from the kernel arguments at every item and gate call --
    // scalar loads, which count in lgkmcnt, so the NFA blocks' LDS waits waited for them too (staged
    // kernel on resident input +4.7 % wave-cycles at cfg3, 11x the SMEM instructions,
    // profiles/r05_m22).  Spilled to VGPR lanes instead, a reload is one VALU op.
    uint32_t seg_nw = sg.n_windows, seg_chunk = sg.chunk, seg_qb = sg.queue_begin;
    asm volatile("" : "+s"(seg_nw), "+s"(seg_chunk), "+s"(seg_qb));
    uint32_t st_codes_off = STAGED ? sg.stage_codes_off : 0u, st_nchunks = STAGED ? sg.stage_chunks : 0u;
    uint32_t* st_gen = STAGED ? sg.stage_gen : nullptr;
    if constexpr (STAGED) asm volatile("" : "+s"(st_codes_off), "+s"(st_nchunks), "+s"(st_gen));
    // inline N records (nrec.h): the lane of the fetch holding a window's record word, ~0u: none
    uint32_t rec_lane = sg.nrec ? nrec_word(ulen) : ~0u;
    asm volatile("" : "+s"(rec_lane));
    auto desc = [&](uint32_t ww, uint64_t& base_out, uint32_t& len_out) __attribute__((always_inline)) {
        if (EQ || ulen != AC_NO_ULEN) {
            base_out = (uint64_t)ww * ustride;
            len_out = ulen;
        } else if (STAGED) {
            load_desc_vec(g_start, g_length, ww, base_out, len_out);
        } else {
            load_desc(g_start, g_length, ww, base_out, len_out);
        }
    };
    const uint32_t m = a.m;
    // An occurrence with <= 2 edits spans >= m - 2 bases: none ends in a window's
    // first m - 3 bases, whose hit accumulation the first block skips (12 of them).
    const bool skip_first = m >= 15u;

    // Q = W x P candidates per lane: slot q = w * P + p is pattern p of lane word w
    constexpr int Q = W * P;
    uint32_t cand[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) cand[q] = g * (64u * Q) + (uint32_t)q * 64u + lane;
    uint32_t first = 0;
#pragma unroll
    for (int p = 0; p < P; ++p) first |= 1u << (31 - p);
    // Initial rows (empty text): R1 has character 0 set, R2 characters 0 and 1.
    const uint32_t d1_init = ~first, d2_init = ~(first | (first >> P));
    const TidInit ini = {~0u >> P, d1_init >> P, d2_init >> P, d1_init, d2_init};  // (loop-invariant registers)
    uint32_t cnt[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) cnt[q] = 0;  // (P <= 2: misses, until the loop's end)
    uint32_t n_counted = 0;                   // (wave-uniform) windows whose levels were counted
    const uint32_t eb = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)(&lds.tab.e[0]));
    // The eb0 blocks address the table from LDS 0.  Never expected otherwise;
    // if it were, the waves skip the work (no fault) and report it in the
    // device error word (ac_check) instead of returning short counts silently.
    const bool eb_ok = !TID_EB0 || eb == 0u;
    if (!eb_ok && lane == 0) atomicOr(a.err, AC_DEVERR_SETUP);

    // Counters of the other queue bank are zeroed for the next launch (strided
    // over the waves; nobody dequeues from that bank in this launch).
    for (uint64_t z = wave; z < a.zero_count; z += a.total_waves)
        if (lane == 0)
            __hip_atomic_exchange(&a.queue[((a.bank ^ 1u) * (uint64_t)a.qstride + z) * AC_QUEUE_LINE], 0u,
                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

    // Dynamic work queues.  VALU issue on a SIMD goes to the oldest wave, so
    // with a static split the first waves finish early and the last ones run
    // with few partners (profiles/r01_kernel_log.md).  Instead each candidate
    // group's items (`chunk` windows each) are spread over `subq` sub-queues
    // (strided, see `n_in` below), each a counter on its own
    // 128-B line; a wave's first item is assigned statically, further ones
    // are claimed one at a time (below).  Waves are dealt to sub-queues
    // round-robin, so every sub-queue serves a mix of old and young waves;
    // the sub-queues drain together and the waves finish within about one
    // item of each other.
    // When its sub-queue runs dry a wave steals from the sibling sub-queues of
    // the same candidate group (same lane masks), probing each counter with a
    // plain load before claiming.
    const uint32_t S = sg.subq;
    const uint32_t chunk = seg_chunk;
    const uint32_t n_items = (seg_nw + chunk - 1u) / chunk;
    uint32_t jc = j;  // sub-queue currently served
    auto counter = [&](uint32_t jj) {
        return g_queue + (uint64_t)jj * AC_QUEUE_LINE;
    };
    auto waves_in = [&](uint32_t jj) {  // waves dealt to sub-queue (g, jj): their first items are static
        const uint32_t qq = seg_qb + g * S + jj;
        const uint32_t qb = qq / WAVES_PER_BLOCK;  // one wave of every workgroup dealt to block-queue qb
        return wgs_of(qb);
    };
    // Sub-queue jj holds items jj, jj + S, jj + 2S, ... (strided): the waves'
    // first items are the image's first windows, so a staged launch's waves
    // start on the windows that arrive first and move through the image as it
    // arrives.  Round 3 measured strided against contiguous ranges (sub-queue jj
    // = one slice of the image, so each XCD's L2 fetched a slice): cfg2 kernel
    // 104.8 -> 101.1 us, cfg3 equal, cfg5 -0.5 % (profiles/r03_strided_ab.log);
    // contiguous ranges had been worth 1.5-2 % at cfg5 before two lane words per
    // wave and the rotated workgroup deal.
    auto n_in = [&](uint32_t jj) { return jj < n_items ? (n_items - jj + S - 1u) / S : 0u; };
    // Per-sub-queue constants of the served sub-queue, recomputed only when a
    // steal changes it (their divisions are SALU sequences; with 1-window items
    // they ran once per window).
    uint32_t jc_waves = waves_in(jc), jc_items = n_in(jc);
    auto item_of = [&](uint32_t c) { return c < jc_items ? jc + c * S : n_items; };
    auto dequeue_issue = [&]() -> uint32_t {  // lane 0 holds the result; read with readfirstlane
        uint32_t v = 0;
        if (lane == 0) v = __hip_atomic_fetch_add(counter(jc), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return v;
    };
    // Next item from a sibling sub-queue, or n_items.  One wave-wide probe
    // reads up to 63 sibling counters at once (a sequential probe costs one
    // ~2 µs device-scope round trip per sibling, which used to stretch the
    // launch tail); the wave then claims from the first sibling that still had
    // items.  A failed claim means that sibling is dry for good (counters only
    // grow), so the loop ends after at most S - 1 failed claims, and a wave
    // exits only once every sub-queue of its group has been seen dry.
    auto steal = [&]() -> uint32_t {
        for (;;) {
            uint32_t found = S;
            for (uint32_t b = 1; b < S && found == S; b += 63u) {  // siblings j+b .. j+b+62
                bool have = false;
                if (lane < 63u && b + lane < S) {
                    const uint32_t jj = (j + b + lane) % S;
                    const uint32_t v = __hip_atomic_load(counter(jj), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    have = waves_in(jj) + v < n_in(jj);
                }
                const uint64_t mk = __ballot(have);
                if (mk) found = b + (uint32_t)__builtin_ctzll(mk);
            }
            if (found == S) return n_items;
            const uint32_t jj = (j + found) % S;
            jc = jj;
            jc_waves = waves_in(jj);
            jc_items = n_in(jj);
            const uint32_t c = jc_waves + __builtin_amdgcn_readfirstlane(dequeue_issue());
            if (c < jc_items) return item_of(c);
        }
    };
    uint32_t item = (j < n_items && eb_ok && !skip) ? item_of(rank) : n_items;
    uint32_t pending = 0;
    uint32_t w = item * chunk, item_end = min(seg_nw, w + chunk);

    // Window pipeline: the next window's first segment is fetched while the current one is counted.
    // (written so that no sum wraps: a start near 2^64 must not pass)
    auto valid = [&](uint64_t base, uint32_t len) { return EQ || window_valid<STAGED>(base, len, g_nbases) != 0u; };
    // an empty window reads no word (its start may be the image's end)
    auto fetchable = [&](uint64_t base, uint32_t len) { return len != 0u && valid(base, len); };
    // Staged early counting: before a window's first fetch, make sure every byte its fetches read
    // (256 bases per fetch from `base`, up to the image end) is in; false = skip the segment.
#ifdef AC_STAMPS
    uint64_t gate_ticks = 0, gate_calls = 0;  // (diagnostic: time in the early-counting gate's slow path)
#endif
    uint32_t n_win = 0;  // (diagnostic builds: windows counted, for the per-window stamps)
    // The segment is complete (verdict r: 0 / 1) or skipped (~0u): from here on its own N bitmap,
    // if it has one.
    auto completed = [&](uint32_t r) __attribute__((always_inline)) {
        partial = false;
        if (r == ~0u) return false;
        has_n = r;
        nmask_bytes = (has_n && rec_lane == ~0u) ? (uint32_t)(g_nbases >> 3) : 0u;
        im.nmask = __builtin_amdgcn_make_buffer_rsrc((void*)nmask_p, 0, (int)nmask_bytes, 0x00020000);
        return true;
    };
    auto gate = [&](uint64_t base, uint32_t len) __attribute__((always_inline)) {
        if constexpr (STAGED) {
            if (!partial) return true;
            const uint64_t end = min(base + (((uint64_t)len + 255u) & ~255ull), g_nbases);
            const uint32_t r0 = st_codes_off + (uint32_t)(base >> 2);
            const uint32_t r1 = st_codes_off + (uint32_t)(end >> 2);
            if (r0 >= v_lo && r1 <= v_hi) return true;
            // (a call's results come back in VGPRs: made wave-uniform again, or everything they
            // touch -- the item cursor, window bases -- would turn divergent)
#ifdef AC_STAMPS
            const uint64_t tg = __builtin_amdgcn_s_memrealtime();
#endif
            const uint64_t g = stage_gate(st_words, st_gen, st_nchunks, blockIdx.x % AC_STAGE_REPL, a.gen,
                                          r0, r1, a.err);
#ifdef AC_STAMPS
            gate_ticks += __builtin_amdgcn_s_memrealtime() - tg;
            ++gate_calls;
#endif
            const uint32_t r = __builtin_amdgcn_readfirstlane((uint32_t)g);
            if (r == 2u) {
                v_lo = (r0 / AC_STAGE_CHUNK) * AC_STAGE_CHUNK;
                v_hi = __builtin_amdgcn_readfirstlane((uint32_t)(g >> 32));
                return true;
            }
            return completed(r);
        } else {
            (void)base;
            (void)len;
            return true;
        }
    };
    uint64_t nbase = 0;
    uint32_t nlen = 0;
    Fetch nf = {0u, 0u};
    // this lane's code word (bits 0-5) and N-mask word (bits 8+) of a segment, in bytes
    const uint32_t lane_off = ((lane & 15u) << 2) | ((lane & 7u) << 10);
    auto fetch_next = [&](uint64_t b) __attribute__((always_inline)) { tid_fetch(nf, im, b, lane, lane_off); };
    if (item < n_items) {
        desc(w, nbase, nlen);
        // (staged: after the table barrier -- a wave waiting for its first window must not hold
        // its workgroup's other waves at the barrier)
        if (!STAGED && fetchable(nbase, nlen)) fetch_next(nbase);
    }

    // ~Eq table, built by wave 0 of the workgroup (the waves share the
    // candidates) while the first windows' loads are in flight: ~Eq_c =
    // (ph ^ H_c) | (pl ^ L_c), H_c / L_c = all ones where character c's high /
    // low code bit is set; N matches nothing.  Only wave 0 loads the k-mers
    // (every wave of a group loading them at launch start queued for up to
    // 12 us, tools/stamps.py).  The barrier waits for LDS only, not for the
    // window prefetches.
    if (wib == 0) {
#pragma unroll
        for (int w = 0; w < W; ++w) {
            uint64_t km[P];
#pragma unroll
            for (int p = 0; p < P; ++p) {
                const uint32_t c = cand[w * P + p];
                km[p] = c < sg.n_kmers ? sg.kmers[c] : 0ull;
            }
            uint32_t ph, pl;
            build_masks<P>(km, a.m, ph, pl);
            uint32_t* tw = &lds.tab.e[w * 5 * 64];
#pragma unroll
            for (int c = 0; c < 4; ++c) tw[c * 64 + lane] = ((c & 2) ? ~ph : ph) | ((c & 1) ? ~pl : pl);
            tw[4 * 64 + lane] = ~0u;
        }
#pragma unroll
        for (int q = 0; q < Q; ++q) lds.cnt[q * 64 + lane] = 0u;
    }
    if (!STAGED) stamp(wave, 7);  // diagnostic builds: the wave's own prologue done, before the barrier
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    stamp(wave, 1);
    bool stage_ok = true;
    if (STAGED && item < n_items && fetchable(nbase, nlen)) {
        stage_ok = gate(nbase, nlen);
        if (stage_ok) fetch_next(nbase);
    }
    if (!stage_ok) item = n_items;

    // Per window, the next window's three dependent global accesses (for an
    // item's last window: claim -> descriptor -> first words; otherwise
    // descriptor -> first words) are spread over the gaps between the window's
    // first 32-base blocks, so none of them stalls the wave between windows.
    // The window loop in two copies (staged kernel; GATED a constant in each): while the segment is not known complete (`partial`), a window's fetch first goes
    // through the gate; once it is, the loop without any staging state, so none of it stays live -- in
    // SGPRs or spilled to VGPR lanes -- through the rest of the launch.  The plain kernel runs only the
    // second.
    if constexpr (STAGED) {
#define AC_GATED 1
#include "wm_window_loop.inc"
#undef AC_GATED
    }
#define AC_GATED 0
#include "wm_window_loop.inc"
#undef AC_GATED

    stamp(wave, 2);
    stamp_val(wave, 6, ((uint64_t)si << 32) | ((uint64_t)g << 16) | j);
#ifdef AC_STAMPS
    if (STAGED) {  // (staged diagnostic builds: slots 4 / 5 hold the gate's time and calls, not the HW ids)
        stamp_val(wave, 4, gate_ticks);
        stamp_val(wave, 5, gate_calls);
    }
#endif
    // The workgroup's waves sum their counts in LDS; one wave adds the sums to the group's slots in
    // `acc`, so each slot takes 1/AC_WAVES_PER_BLOCK of the same-address atomics (they serialise at
    // the memory side: ~10 us of launch tail at cfg2 with one atomic per wave; profiles/r01_kernel_log.md).
    // Each add is 64-bit, (1 << 32) + the sum: the returned word says how many workgroups of the group
    // have added before this one, so the last to add -- per slot -- knows the total at once and moves it
    // to the counts.  One device-scope round trip at the launch's end (round 4 had three: the adds, a
    // group ticket taken after them, the slots read back and zeroed).  No fences: the arrival count and
    // the sum change in one atomic.
#pragma unroll
    for (int q = 0; q < Q; ++q)
        if (P <= 2) cnt[q] = 3u * n_counted - cnt[q];
#pragma unroll
    for (int q = 0; q < Q; ++q)
        if (cnt[q]) __hip_atomic_fetch_add(&lds.cnt[q * 64 + lane], cnt[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    // (every wave's error-word atomics are performed before its workgroup's adds: the staged launch's
    // last workgroup of a slot reads the word)
    if (STAGED) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (wib == 0) {
        uint64_t* acc = a.acc + sg.acc_begin + g * (64u * Q);
        // Workgroups serving group g: those dealt to its subq / WPB block-queues.
        const uint32_t qb0 = (sg.queue_begin + g * sg.subq) / WAVES_PER_BLOCK, nq = sg.subq / WAVES_PER_BLOCK;
        uint32_t n_wg = 0;
        for (uint32_t i = 0; i < nq; ++i) n_wg += wgs_of(qb0 + i);
        uint32_t mine[Q];
        uint64_t old[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            mine[q] = lds.cnt[q * 64 + lane];
            old[q] = __hip_atomic_fetch_add(&acc[q * 64 + lane], (1ull << 32) | mine[q], __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            if ((uint32_t)(old[q] >> 32) != n_wg - 1u) continue;  // not the slot's last workgroup
            const uint32_t v = (uint32_t)old[q] + mine[q];
            __hip_atomic_store(&acc[q * 64 + lane], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (cand[q] < sg.n_kmers) {
                if (a.add_counts) {
                    if (v) atomicAdd(&sg.counts[cand[q]], v);
                } else if (STAGED && a.tag) {  // host memory, each count tagged with the launch's generation
                    __hip_atomic_store((uint64_t*)sg.counts + cand[q], ((uint64_t)a.gen << 32) | v, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
                } else {  // (device memory: read after the stream has completed)
                    sg.counts[cand[q]] = v;
                }
            }
            if (STAGED && q == 0 && lane == 0) {
                // The group's error snapshot, by slot (0, lane 0)'s last workgroup: every workgroup's waves
                // performed their error atomics before that workgroup's add to the slot, so the word holds
                // every bit the group set; all groups' snapshots together hold the launch's.  Tagged
                // completion (synchronous calls): the host waits until every count and every group's word
                // carries this launch's generation, so no completion word, no wait for the counts' stores
                // and no launch-wide counter sit on the path to the host.  Submits (counts in device
                // memory): the bits go to the context's word (ac_check).
                const uint32_t e = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (a.tag)
                    __hip_atomic_store(a.grp_err + sg.group_begin + g, ((uint64_t)a.gen << 32) | e, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
                else if (e && a.err_out)
                    atomicOr(a.err_out, e);
            }
        }
    }
    stamp(wave, 3);
}

}  // namespace

template <int P, bool STAGED, bool EQ>
__global__ __launch_bounds__(64 * WAVES_PER_BLOCK, waves_per_simd(words_for(P, STAGED))) void wm2_count_kernel(LaunchArgs a) {
    // The LDS allocation also caps residency at waves_per_simd waves per SIMD
    // (one word: 8, faster than 6 or 10, profiles/r01_kernel_log.md; two words: 4).
    constexpr int W = words_for(P, STAGED);
    constexpr int kBlocksPerCu = 4 * waves_per_simd(W) / WAVES_PER_BLOCK;
    __shared__ BlockLds<W> lds[(160 * 1024 / kBlocksPerCu) / sizeof(BlockLds<W>)];
    count_body<P, STAGED, EQ>(a, lds[0]);
}

namespace {
template <int P, bool STAGED>
hipError_t occupancy(int cu_count, uint32_t* waves) {
    int blocks = 0;
    hipError_t e =
        // (queried on the equal-window kernel, the one the bench's kernel leg, the CLI and the stage launch:
        // the query loads the kernel's code, and that load then is not paid again at its first launch --
        // the instantiations of one word count have the same LDS allocation, so the same residency)
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, wm2_count_kernel<P, STAGED, true>, 64 * WAVES_PER_BLOCK, 0);
    if (e != hipSuccess) return e;
    if (blocks < 1) blocks = 1;
    *waves = (uint32_t)blocks * WAVES_PER_BLOCK * (uint32_t)cu_count;
    return hipSuccess;
}
}  // namespace

#ifdef AC_STAMPS
hipError_t debug_stamps(void* host, size_t bytes) {
    // g_stamps, then g_stage_stamps
    const size_t a = bytes < sizeof(g_stamps) ? bytes : sizeof(g_stamps);
    hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), a, 0, hipMemcpyDeviceToHost);
    if (e != hipSuccess || bytes < sizeof(g_stamps) + sizeof(g_stage_stamps)) return e;
    e = hipMemcpyFromSymbol((char*)host + sizeof(g_stamps), HIP_SYMBOL(g_stage_stamps), sizeof(g_stage_stamps), 0,
                            hipMemcpyDeviceToHost);
    // then the per-window stamps (g_win_stamps), if the buffer holds them
    if (e != hipSuccess || bytes < sizeof(g_stamps) + sizeof(g_stage_stamps) + sizeof(g_win_stamps)) return e;
    return hipMemcpyFromSymbol((char*)host + sizeof(g_stamps) + sizeof(g_stage_stamps), HIP_SYMBOL(g_win_stamps),
                               sizeof(g_win_stamps), 0, hipMemcpyDeviceToHost);
}
#endif

hipError_t resident_waves(uint32_t P, bool staged, int cu_count, uint32_t* waves) {
#define AC_OCC(PP) \
    case PP: return staged ? occupancy<PP, true>(cu_count, waves) : occupancy<PP, false>(cu_count, waves);
    switch (P) {
        AC_OCC(1)
        AC_OCC(2)
        AC_OCC(3)
        AC_OCC(4)
        default: return hipErrorInvalidValue;
    }
#undef AC_OCC
}

hipError_t launch_wm2_count(const LaunchArgs& args, hipStream_t stream) {
    if (args.total_waves == 0) return hipSuccess;
    const uint64_t blocks = (args.total_waves + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK;
    const dim3 grid((uint32_t)blocks), block(64 * WAVES_PER_BLOCK);
#define AC_LAUNCH(PP)                                                                            \
    case PP:                                                                                     \
        if (args.staged && args.eq)                                                              \
            hipLaunchKernelGGL((wm2_count_kernel<PP, true, true>), grid, block, 0, stream, args);   \
        else if (args.staged)                                                                    \
            hipLaunchKernelGGL((wm2_count_kernel<PP, true, false>), grid, block, 0, stream, args);  \
        else if (args.eq)                                                                        \
            hipLaunchKernelGGL((wm2_count_kernel<PP, false, true>), grid, block, 0, stream, args);  \
        else                                                                                     \
            hipLaunchKernelGGL((wm2_count_kernel<PP, false, false>), grid, block, 0, stream, args); \
        break;
    switch (args.P) {
        AC_LAUNCH(1)
        AC_LAUNCH(2)
        AC_LAUNCH(3)
        AC_LAUNCH(4)
        default: return hipErrorInvalidValue;
    }
#undef AC_LAUNCH
    return hipGetLastError();
}

}  // namespace acamd
