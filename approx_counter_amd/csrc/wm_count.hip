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
//  * lane = 2 words x P candidates, window text wave-uniform.  P = floor(32/k) (<= 4)
//    patterns are INTERLEAVED in one 32-bit register: character i of pattern p
//    sits at bit 31 - (i*P + p), so one logical right shift by P advances every
//    pattern at once and the zero fill reaches every pattern's first character.
//    Each lane runs AC_WAVE_WORDS = 2 independent words (two candidate groups)
//    over the same text: two independent dependency chains per wave and one
//    staging / LDS read per base for 2P candidates.
//  * Issue cost drives the instruction choice (tools/ubench_valu.hip,
//    profiles/r01_ubench_valu.txt): on gfx950 v_and/v_or/v_xor/v_add/
//    v_lshrrev_b32 and v_bitop3_b32 issue in 2 cycles per wave64 with VGPR
//    operands; shifts left, v_or3, v_and_or, v_lshl_or and ANY instruction
//    reading an SGPR take 4.  So every 3-input boolean is one v_bitop3_b32 and
//    the text masks reach the VALU as VGPRs: each wave expands its window into
//    per-base masks H = -(bit 1), L = -(bit 0), N in LDS (one lane per 4
//    bases, ~0.1 VALU op per base) and reads them back as wave-uniform
//    broadcast ds_read_b128 (two bases per read).  The next window's code and
//    N-mask words are loaded while the current window is computed.  A base then costs 2 ops of ~Eq
//    ( (ph ^ H) | (pl ^ L) ) + 8 ops of NFA + 1.5 of hit accumulation (v_bitop3
//    AND3 over two bases) = 11.5 full-rate VALU ops for P candidates.
//  * N (any non-ACGT base) never matches: a ballot at staging flags the
//    16-base chunks holding an N; those take a path that ORs the base's N
//    mask (also staged in LDS) into ~Eq at no extra VALU cost.
//  * Integer-only VALU work: no MFMA.  Counts are uint32 atomics
//    (order-independent, bit-exact).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "wm_count.h"

namespace acamd {
namespace {

#ifndef AC_WAVES_PER_BLOCK
#define AC_WAVES_PER_BLOCK 4
#endif
constexpr int WAVES_PER_BLOCK = AC_WAVES_PER_BLOCK;
#ifdef AC_STAMPS
// Diagnostic build only (tools/variants.sh ... -DAC_STAMPS): per-wave
// s_memrealtime stamps (100 MHz) at entry, after the prologue, after the last
// window and at exit; read back with ac_debug_stamps().  No output value is
// computed from them.
}  // namespace
__device__ uint64_t g_stamps[1 << 21];
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
#else
__device__ __forceinline__ void stamp(uint64_t, int) {}
__device__ __forceinline__ void stamp_val(uint64_t, int, uint64_t) {}
#endif
constexpr int W = AC_WAVE_WORDS;
constexpr uint32_t SEG = 256;  // window bases staged in LDS per pass (4 per lane)

// Per-wave LDS staging of one window segment (3 KB).
struct Stage {
    uint4 hl[SEG / 2 + 1];  // (H, L) of bases 2q and 2q+1; one pad pair for the read-ahead past the end
    uint32_t n[SEG];        // N mask of each base (0 or ~0)
};

// v_bitop3_b32 truth tables over (s0, s1, s2) = (0xf0, 0xcc, 0xaa).
constexpr int NEQ = 0xf6;     // a | (b ^ c)      ~Eq from (ph ^ H, pl, L)
constexpr int XOR_OR = 0xbe;  // (a ^ b) | c      ph ^ H with the N mask folded in
constexpr int AND3 = 0x80;    // a & b & c
constexpr int OR_AND = 0xa8;  // (a | b) & c
template <int TT>
__device__ __forceinline__ uint32_t bop3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, TT);
}

struct Nfa {
    uint32_t d0[W], d1[W], d2[W];  // complemented rows
    uint32_t s0[W], s1[W], s2[W];  // rows >> P
    uint32_t a0[W], a1[W], a2[W];  // AND of the rows over the window
};

// One text base (masks H, L, N) for both words: 11 full-rate VALU ops per
// word, 8 of them NFA.  ACC (odd bases): also AND this base's rows and the
// previous base's (still in s.d*) into the hit accumulators (3 more ops per
// word per two bases).
template <int P, bool HAS_N, bool ACC>
__device__ __forceinline__ void step(Nfa& s, const uint32_t (&ph)[W], const uint32_t (&pl)[W], uint32_t H,
                                     uint32_t L, uint32_t N) {
#pragma unroll
    for (int w = 0; w < W; ++w) {
        const uint32_t xh = HAS_N ? bop3<XOR_OR>(ph[w], H, N) : (ph[w] ^ H);
        const uint32_t ne = bop3<NEQ>(xh, pl[w], L);
        const uint32_t d0n = s.s0[w] | ne;
        const uint32_t t0 = d0n >> P;
        const uint32_t d1n = bop3<OR_AND>(s.s1[w], ne, bop3<AND3>(s.s0[w], s.d0[w], t0));
        const uint32_t t1 = d1n >> P;
        const uint32_t d2n = bop3<OR_AND>(s.s2[w], ne, bop3<AND3>(s.s1[w], s.d1[w], t1));
        const uint32_t t2 = d2n >> P;
        if (ACC) {
            s.a0[w] = bop3<AND3>(s.a0[w], s.d0[w], d0n);
            s.a1[w] = bop3<AND3>(s.a1[w], s.d1[w], d1n);
            s.a2[w] = bop3<AND3>(s.a2[w], s.d2[w], d2n);
        }
        s.d0[w] = d0n;
        s.d1[w] = d1n;
        s.d2[w] = d2n;
        s.s0[w] = t0;
        s.s1[w] = t1;
        s.s2[w] = t2;
    }
}

// NB (even) staged bases from pair index q; the next pair is read one pair ahead.
template <int P, int NB, bool HAS_N>
__device__ __forceinline__ void run(Nfa& s, const uint32_t (&ph)[W], const uint32_t (&pl)[W],
                                    const Stage& st, uint32_t q) {
    uint4 cur = st.hl[q];
#pragma unroll
    for (int j = 0; j < NB; j += 2) {
        const uint4 nxt = st.hl[q + j / 2 + 1];  // base + immediate offset (the pad pair absorbs the last read)
        uint32_t n0 = 0, n1 = 0;
        if constexpr (HAS_N) {
            n0 = st.n[2 * (q + j / 2)];
            n1 = st.n[2 * (q + j / 2) + 1];
        }
        step<P, HAS_N, false>(s, ph, pl, cur.x, cur.y, n0);
        step<P, HAS_N, true>(s, ph, pl, cur.z, cur.w, n1);
        cur = nxt;
        // Keep the one-pair-ahead read in this pair's block: without the fence
        // hipcc hoists the whole chunk's reads (32 VGPRs) and occupancy drops.
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <int P, int NB>
__device__ __forceinline__ void run_any(Nfa& s, const uint32_t (&ph)[W], const uint32_t (&pl)[W],
                                        const Stage& st, uint32_t q, bool has_n) {
    if (!has_n) run<P, NB, false>(s, ph, pl, st, q);
    else run<P, NB, true>(s, ph, pl, st, q);
}

// Lane `lane`'s share of staging window bases [sb, sb + SEG): bases sb + 4*lane .. +3.
struct Fetch {
    uint32_t code;  // the code word holding the lane's 4 bases (0 past the window)
    uint32_t nmw;   // the N-mask word holding them
};

__device__ __forceinline__ Fetch fetch(const uint32_t* __restrict__ codes, const uint32_t* __restrict__ nmask,
                                       uint32_t len, uint32_t sb, uint32_t lane) {
    const uint32_t b = sb + 4u * lane;
    Fetch f = {0u, 0u};
    if (b < len) {
        f.code = codes[b >> 4];
        f.nmw = nmask[b >> 5];
    }
    return f;
}

// Writes the lane's 4 bases into the stage; returns the wave's ballot of
// "my 4 bases hold an N" (bit l = bases 4l..4l+3 of the segment).
__device__ __forceinline__ uint64_t stage_write(Stage& st, const Fetch& f, uint32_t lane) {
    const uint32_t sh = 8u * (lane & 3u);  // 2 bits per base, 4 bases per lane, 16 per code word
    const uint32_t c = f.code >> sh;
    auto sx = [](uint32_t v, int bit) { return (uint32_t)(-(int32_t)((v >> bit) & 1u)); };
    st.hl[2 * lane] = make_uint4(sx(c, 1), sx(c, 0), sx(c, 3), sx(c, 2));
    st.hl[2 * lane + 1] = make_uint4(sx(c, 5), sx(c, 4), sx(c, 7), sx(c, 6));
    const uint32_t nb = (f.nmw >> (4u * (lane & 7u))) & 0xfu;
    *reinterpret_cast<uint4*>(&st.n[4 * lane]) = make_uint4(sx(nb, 0), sx(nb, 1), sx(nb, 2), sx(nb, 3));
    return __ballot(nb != 0u);
}

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

#ifdef AC_TID
#include "wm_tid_blocks.inc"

// Per-wave ~Eq table: word c*64 + lane = the lane's ~Eq mask for character c
// (A C G T, then N = all ones), read per base with ds_read_addtid_b32.
struct TidTable {
    uint32_t e[5 * 64];
};

// Lane `lane`'s word of window bases [sb, sb + SEG): lanes 0-15 the 16 code
// words, lanes 16-23 the 8 N-mask words.  One unconditional load per lane with
// the index clamped to the window's last word (always inside the image): a word
// past the window is never read as text (the chunk loop stops at the window
// length), and a branch-free load keeps hipcc from waiting on it before the
// window that uses it.
__device__ __forceinline__ uint32_t tid_fetch(const uint32_t* __restrict__ codes, const uint32_t* __restrict__ nmask,
                                              uint32_t len, uint32_t sb, uint32_t lane) {
    const bool is_code = lane < 16u;
    const uint32_t ci = min((sb >> 4) + lane, (len - 1u) >> 4);
    const uint32_t ni = min((sb >> 5) + ((lane - 16u) & 7u), (len - 1u) >> 5);
    const uint32_t* p = is_code ? codes + ci : nmask + ni;
    return *p;
}

// With one-wave workgroups the wave's table is the block's only LDS object, at
// address 0, and M0 needs no per-base add (tools/gen_tid_blocks.py, eb0).
constexpr bool TID_EB0 = WAVES_PER_BLOCK == 1;

// The remainder (< 16 bases) of a segment: blocks of 8, 4, 2, 1 bases.
template <int P>
__device__ __forceinline__ void tid_tail(TidNfa& s, uint32_t code, uint32_t nm, uint32_t rem, uint32_t eb) {
    if (rem & 8u) {
        tid_block8<P, TID_EB0>(s, code, nm & 0xffu, eb);
        code >>= 16;
        nm >>= 8;
    }
    if (rem & 4u) {
        tid_block4<P, TID_EB0>(s, code, nm & 0xfu, eb);
        code >>= 8;
        nm >>= 4;
    }
    if (rem & 2u) {
        tid_block2<P, TID_EB0>(s, code, nm & 0x3u, eb);
        code >>= 4;
        nm >>= 2;
    }
    if (rem & 1u) tid_block1<P, TID_EB0>(s, code, nm & 0x1u, eb);
}
using StageT = TidTable;
using FetchT = uint32_t;
__device__ __forceinline__ FetchT fetchw(const uint32_t* __restrict__ codes, const uint32_t* __restrict__ nmask,
                                         uint32_t len, uint32_t sb, uint32_t lane) {
    return tid_fetch(codes, nmask, len, sb, lane);
}
#else
using StageT = Stage;
using FetchT = Fetch;
__device__ __forceinline__ FetchT fetchw(const uint32_t* __restrict__ codes, const uint32_t* __restrict__ nmask,
                                         uint32_t len, uint32_t sb, uint32_t lane) {
    return fetch(codes, nmask, len, sb, lane);
}
#endif

template <int P>
__device__ __forceinline__ void count_body(const LaunchArgs& a, StageT& st) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t wave = (uint64_t)blockIdx.x * WAVES_PER_BLOCK + wib;
    if (wave >= a.total_waves) return;
    stamp(wave, 0);

    // Wave -> sub-queue q = wave mod n_queues, so every sub-queue is served by
    // waves of every dispatch age (see the work-queue comment below); q ->
    // (segment, candidate group g, sub-queue j of that group).
    const uint32_t q = (uint32_t)(wave % a.n_queues), rank = (uint32_t)(wave / a.n_queues);
    int si = 0;
#pragma unroll
    for (int i = 1; i < AC_MAX_SEGS; ++i)
        if (i < (int)a.n_segs && q >= a.seg[i].queue_begin) si = i;
    const SegDev& sg = a.seg[si];
    const uint32_t ql = q - sg.queue_begin;
    const uint32_t g = ql % sg.groups, j = ql / sg.groups;
    const uint32_t m = a.m;

    // Lane constants: character i of pattern p of word w at bit 31 - (i*P + p).
    uint32_t ph[W], pl[W], cand[W][P];
    uint32_t first = 0;
#pragma unroll
    for (int p = 0; p < P; ++p) first |= 1u << (31 - p);
#pragma unroll
    for (int w = 0; w < W; ++w) {
        uint64_t km[P];
#pragma unroll
        for (int p = 0; p < P; ++p) {
            cand[w][p] = g * (64u * P * W) + (uint32_t)(w * P + p) * 64u + lane;
            km[p] = cand[w][p] < sg.n_kmers ? sg.kmers[cand[w][p]] : 0ull;
        }
        build_masks<P>(km, m, ph[w], pl[w]);
    }
    // Initial rows (empty text): R1 has character 0 set, R2 characters 0 and 1.
    const uint32_t d1_init = ~first, d2_init = ~(first | (first >> P));
#ifdef AC_TID
    static_assert(W == 1, "the table-driven loop runs one lane word");
#pragma unroll
    for (int c = 0; c < 4; ++c) st.e[c * 64 + lane] = ((c & 2) ? ~ph[0] : ph[0]) | ((c & 1) ? ~pl[0] : pl[0]);
    st.e[4 * 64 + lane] = ~0u;
    const uint32_t eb = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)(&st.e[0]));
    // The eb0 blocks address the table from LDS 0.  Never expected otherwise; if
    // it were, the wave stops (no fault) and the counts come out short, which
    // the parity tests catch.
    if (TID_EB0 && eb != 0u) return;
#endif

    uint32_t cnt[W][P];
#pragma unroll
    for (int w = 0; w < W; ++w)
#pragma unroll
        for (int p = 0; p < P; ++p) cnt[w][p] = 0;

    stamp(wave, 1);

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
    // (item j + c*subq belongs to sub-queue j), each a counter on its own
    // 128-B line; a wave's first item is assigned statically, further ones
    // are claimed one at a time (below).  Waves are dealt to sub-queues
    // round-robin, so every sub-queue serves a mix of old and young waves;
    // the sub-queues drain together and the waves finish within about one
    // item of each other.
    // When its sub-queue runs dry a wave steals from the sibling sub-queues of
    // the same candidate group (same lane masks), probing each counter with a
    // plain load before claiming.
    const uint32_t S = sg.subq;
    const uint32_t chunk = sg.chunk;
    const uint32_t n_items = (sg.n_windows + chunk - 1u) / chunk;
    uint32_t jc = j;  // sub-queue currently served
    auto counter = [&](uint32_t jj) {
        return a.queue + ((uint64_t)a.bank * a.qstride + sg.queue_begin + g + jj * sg.groups) * AC_QUEUE_LINE;
    };
    auto waves_in = [&](uint32_t jj) {  // waves dealt to sub-queue (g, jj): their first items are static
        const uint32_t qq = sg.queue_begin + g + jj * sg.groups;
        return (uint32_t)(a.total_waves / a.n_queues) + (qq < a.total_waves % a.n_queues ? 1u : 0u);
    };
    auto n_in = [&](uint32_t jj) { return jj < n_items ? (n_items - jj + S - 1u) / S : 0u; };  // items of jj
    auto item_of = [&](uint32_t c) { return c < n_in(jc) ? jc + c * S : n_items; };
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
            const uint32_t c = waves_in(jj) + __builtin_amdgcn_readfirstlane(dequeue_issue());
            if (c < n_in(jj)) return jj + c * S;
        }
    };
    uint32_t item = j < n_items ? item_of(rank) : n_items;
    uint32_t pending = 0;
    uint32_t w = item * chunk, item_end = min(sg.n_windows, w + chunk);

    // Window pipeline: the next window's first segment is fetched while the current one is counted.
    auto valid = [&](uint64_t base, uint32_t len) { return !(base & 31u) && base + len <= sg.n_bases; };
    uint64_t nbase = 0;
    uint32_t nlen = 0;
    FetchT nf{};
    if (item < n_items) {
        nbase = sg.start[w];
        nlen = sg.length[w];
        if (valid(nbase, nlen)) nf = fetchw(sg.codes + (nbase >> 4), sg.nmask + (nbase >> 5), nlen, 0, lane);
    }
    while (item < n_items) {
        const uint64_t base = nbase;
        const uint32_t len = nlen;
#ifdef AC_TID
        // Wait for this window's words here, before the next window's fetch is
        // issued: inside the chunk loop hipcc would otherwise wait for both.
        FetchT f0 = nf;
        asm volatile("" : "+v"(f0));
#else
        const FetchT f0 = nf;
#endif
        // Within an item the next window is fetched while this one is counted.
        // During an item's last window the next item is claimed (one returning
        // atomic); it is read after the window, so a wave the arbiter starves
        // never holds more than the item it is working on.
        const uint32_t wn = w + 1;
        if (wn < item_end) {
            nbase = sg.start[wn];
            nlen = sg.length[wn];
            if (valid(nbase, nlen)) nf = fetchw(sg.codes + (nbase >> 4), sg.nmask + (nbase >> 5), nlen, 0, lane);
        } else {
            pending = dequeue_issue();
        }
        if (valid(base, len)) {  // a malformed window is skipped: never read outside the image
        const uint32_t* __restrict__ codes = sg.codes + (base >> 4);
        const uint32_t* __restrict__ nmask = sg.nmask + (base >> 5);
#ifdef AC_TID
        TidNfa s = {~0u, d1_init, d2_init, ~0u >> P, d1_init >> P, d2_init >> P, ~0u, d1_init, d2_init};
        auto segment = [&](uint32_t f, uint32_t sb) {
            const uint32_t nb = min(SEG, len - sb);
            const uint32_t nfull = nb >> 4;
            for (uint32_t ch = 0; ch < nfull; ++ch) {
                const uint32_t code = __builtin_amdgcn_readlane(f, ch);
                const uint32_t nm = (__builtin_amdgcn_readlane(f, 16u + (ch >> 1)) >> ((ch & 1u) * 16u)) & 0xffffu;
                tid_block16<P, TID_EB0>(s, code, nm, eb);
            }
            if (nb & 15u) {
                const uint32_t code = __builtin_amdgcn_readlane(f, nfull);
                const uint32_t nm = (__builtin_amdgcn_readlane(f, 16u + (nfull >> 1)) >> ((nfull & 1u) * 16u)) & 0xffffu;
                tid_tail<P>(s, code, nm, nb & 15u, eb);
            }
        };
        segment(f0, 0u);
        for (uint32_t sb = SEG; sb < len; sb += SEG) {  // windows longer than one segment
            uint32_t f = tid_fetch(codes, nmask, len, sb, lane);
            asm volatile("" : "+v"(f));
            segment(f, sb);
        }
#pragma unroll
        for (int p = 0; p < P; ++p) {
            const uint32_t lb = 31u - ((m - 1u) * P + (uint32_t)p);
            cnt[0][p] += 3u - ((s.a0 >> lb) & 1u) - ((s.a1 >> lb) & 1u) - ((s.a2 >> lb) & 1u);
        }
#else
        Nfa s;
#pragma unroll
        for (int x = 0; x < W; ++x) {
            s.d0[x] = ~0u;
            s.d1[x] = d1_init;
            s.d2[x] = d2_init;
            s.s0[x] = ~0u >> P;
            s.s1[x] = d1_init >> P;
            s.s2[x] = d2_init >> P;
            s.a0[x] = ~0u;
            s.a1[x] = d1_init;
            s.a2[x] = d2_init;  // for k <= 2 the empty alignment already reaches the last character
        }
        for (uint32_t sb = 0; sb < len; sb += SEG) {
            const Fetch f = sb == 0 ? f0 : fetch(codes, nmask, len, sb, lane);
            const uint64_t any_n = stage_write(st, f, lane);
            const uint32_t nb = min(SEG, len - sb);
            const uint32_t nfull = nb >> 4;
            for (uint32_t ch = 0; ch < nfull; ++ch)
                run_any<P, 16>(s, ph, pl, st, ch * 8u, ((any_n >> (4u * ch)) & 0xfu) != 0u);
            const uint32_t rem = nb & 15u;
            if (rem) {
                uint32_t o = nfull * 16u;  // base offset in the segment
                const uint32_t fl = (uint32_t)(any_n >> (o >> 2)) & 0xfu;  // 4-base groups o/4 .. o/4+3
                uint32_t gi = 0;                                        // group index within fl
                if (rem & 8u) {
                    run_any<P, 8>(s, ph, pl, st, o / 2, (fl & 3u) != 0u);
                    o += 8u;
                    gi += 2u;
                }
                if (rem & 4u) {
                    run_any<P, 4>(s, ph, pl, st, o / 2, ((fl >> gi) & 1u) != 0u);
                    o += 4u;
                    gi += 1u;
                }
                if (rem & 2u) {
                    run_any<P, 2>(s, ph, pl, st, o / 2, ((fl >> gi) & 1u) != 0u);
                    o += 2u;
                }
                if (rem & 1u) {
                    const uint4 mm = st.hl[o / 2];
                    step<P, true, false>(s, ph, pl, mm.x, mm.y, st.n[o]);
#pragma unroll
                    for (int x = 0; x < W; ++x) {
                        s.a0[x] &= s.d0[x];
                        s.a1[x] &= s.d1[x];
                        s.a2[x] &= s.d2[x];
                    }
                }
            }
        }
#pragma unroll
        for (int x = 0; x < W; ++x) {
#pragma unroll
            for (int p = 0; p < P; ++p) {
                const uint32_t lb = 31u - ((m - 1u) * P + (uint32_t)p);
                cnt[x][p] += 3u - ((s.a0[x] >> lb) & 1u) - ((s.a1[x] >> lb) & 1u) - ((s.a2[x] >> lb) & 1u);
            }
        }
#endif
        }  // valid window
        // advance the cursor; at an item boundary move to the prefetched item and request another
        if (++w >= item_end) {
            item = item_of(waves_in(jc) + __builtin_amdgcn_readfirstlane(pending));
            if (item >= n_items && S > 1) item = steal();
            if (item < n_items) {
                w = item * chunk;
                item_end = min(sg.n_windows, w + chunk);
                nbase = sg.start[w];
                nlen = sg.length[w];
                if (valid(nbase, nlen)) nf = fetchw(sg.codes + (nbase >> 4), sg.nmask + (nbase >> 5), nlen, 0, lane);
            }
        }
    }

    stamp(wave, 2);
    stamp_val(wave, 6, ((uint64_t)si << 32) | ((uint64_t)g << 16) | j);
#pragma unroll
    for (int x = 0; x < W; ++x)
#pragma unroll
        for (int p = 0; p < P; ++p)
#ifdef AC_TIMING_NO_ATOMICS  // timing-only build: results discarded (kept live by an impossible store)
            if (cand[x][p] < sg.n_kmers && cnt[x][p] == 0xdeadbeefu) sg.counts[cand[x][p]] = 1u;
#else
            if (cand[x][p] < sg.n_kmers && cnt[x][p]) atomicAdd(&sg.counts[cand[x][p]], cnt[x][p]);
#endif
    stamp(wave, 3);
}

}  // namespace

template <int P>
__global__ __launch_bounds__(64 * WAVES_PER_BLOCK, AC_MIN_WAVES_PER_SIMD) void wm2_count_kernel(LaunchArgs a) {
    // The LDS allocation also caps residency at AC_BLOCKS_PER_CU blocks (6 waves
    // per SIMD): measured faster than 8 (fewer waves starved by the oldest-first
    // VALU arbitration; profiles/r01_kernel_log.md).
    __shared__ StageT stage[(160 * 1024 / AC_BLOCKS_PER_CU) / sizeof(StageT)];
    count_body<P>(a, stage[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)]);
}

namespace {
template <int P>
hipError_t occupancy(int cu_count, uint32_t* waves) {
    int blocks = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, wm2_count_kernel<P>, 64 * WAVES_PER_BLOCK, 0);
    if (e != hipSuccess) return e;
    if (blocks < 1) blocks = 1;
    *waves = (uint32_t)blocks * WAVES_PER_BLOCK * (uint32_t)cu_count;
    return hipSuccess;
}
}  // namespace

#ifdef AC_STAMPS
hipError_t debug_stamps(void* host, size_t bytes) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), bytes < sizeof(g_stamps) ? bytes : sizeof(g_stamps), 0,
                               hipMemcpyDeviceToHost);
}
#endif

hipError_t resident_waves(uint32_t P, int cu_count, uint32_t* waves) {
    switch (P) {
        case 1: return occupancy<1>(cu_count, waves);
        case 2: return occupancy<2>(cu_count, waves);
        case 3: return occupancy<3>(cu_count, waves);
        case 4: return occupancy<4>(cu_count, waves);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_wm2_count(const LaunchArgs& args, hipStream_t stream) {
    if (args.total_waves == 0) return hipSuccess;
    const uint64_t blocks = (args.total_waves + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK;
    const dim3 grid((uint32_t)blocks), block(64 * WAVES_PER_BLOCK);
    switch (args.P) {
        case 1: hipLaunchKernelGGL(wm2_count_kernel<1>, grid, block, 0, stream, args); break;
        case 2: hipLaunchKernelGGL(wm2_count_kernel<2>, grid, block, 0, stream, args); break;
        case 3: hipLaunchKernelGGL(wm2_count_kernel<3>, grid, block, 0, stream, args); break;
        case 4: hipLaunchKernelGGL(wm2_count_kernel<4>, grid, block, 0, stream, args); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace acamd
