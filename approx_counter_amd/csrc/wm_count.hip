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
//  * Issue cost drives the instruction choice (tools/ubench_valu.hip,
//    profiles/r01_ubench_valu.txt): on gfx950 v_and/v_or/v_xor/v_add/
//    v_lshrrev_b32 and v_bitop3_b32 issue in 2 cycles per wave64 with VGPR
//    operands; shifts left, v_or3, v_and_or, v_lshl_or and ANY instruction
//    reading an SGPR take 4.  So every 3-input boolean is one v_bitop3_b32 and
//    the text masks reach the VALU as VGPRs: each wave expands its window into
//    per-base masks H = -(bit 1), L = -(bit 0) in LDS (one lane per base pair,
//    ~0.1 VALU op per base) and reads them back as wave-uniform broadcast
//    ds_read_b128 (two bases per read).  A base then costs 2 ops of ~Eq
//    ( (ph ^ H) | (pl ^ L) ) + 8 ops of NFA + 1.5 of hit accumulation (v_bitop3
//    AND3 over two bases) = 11.5 full-rate VALU ops for P candidates.
//  * N (any non-ACGT base) never matches: chunks of 16 bases holding an N take
//    a branch that ORs the N mask into ~Eq (one extra, SGPR-reading op).
//  * Integer-only VALU work: no MFMA.  Counts are uint32 atomics
//    (order-independent, bit-exact).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "wm_count.h"

namespace acamd {
namespace {

constexpr int WAVES_PER_BLOCK = 4;
constexpr uint32_t SEG_BASES = 128;  // window bases staged in LDS per pass (one pair per lane)

// v_bitop3 truth tables over (s0, s1, s2) = (0xf0, 0xcc, 0xaa).
//   0xf6 = a | (b ^ c)      ~Eq from (ph ^ H, pl, L)
//   0xbe = (a ^ b) | c      ph ^ H with the N mask folded in
//   0x80 = a & b & c
//   0xa8 = (a | b) & c
// One text base as ONE asm statement: hipcc pads nothing inside it, and plain
// VALU -> VALU dependencies need no software wait states on gfx950.
#define AC_NEQ "v_xor_b32 %[xh], %[H], %[ph]\n\tv_bitop3_b32 %[ne], %[xh], %[pl], %[L] bitop3:0xf6\n\t"
#define AC_NEQ_N                                                                    \
    "v_bitop3_b32 %[xh], %[ph], %[H], %[N] bitop3:0xbe\n\t"                          \
    "v_bitop3_b32 %[ne], %[xh], %[pl], %[L] bitop3:0xf6\n\t"
#define AC_NFA                                                                  \
    "v_or_b32 %[d0n], %[s0], %[ne]\n\t"                                              \
    "v_lshrrev_b32 %[t0], %[sh], %[d0n]\n\t"                                        \
    "v_bitop3_b32 %[g], %[s0], %[d0], %[t0] bitop3:0x80\n\t"                         \
    "v_bitop3_b32 %[d1n], %[s1], %[ne], %[g] bitop3:0xa8\n\t"                        \
    "v_lshrrev_b32 %[t1], %[sh], %[d1n]\n\t"                                        \
    "v_bitop3_b32 %[g], %[s1], %[d1], %[t1] bitop3:0x80\n\t"                         \
    "v_bitop3_b32 %[d2n], %[s2], %[ne], %[g] bitop3:0xa8\n\t"                        \
    "v_lshrrev_b32 %[t2], %[sh], %[d2n]\n\t"
#define AC_ACC                                                                      \
    "v_bitop3_b32 %[a0], %[a0], %[d0], %[d0n] bitop3:0x80\n\t"                       \
    "v_bitop3_b32 %[a1], %[a1], %[d1], %[d1n] bitop3:0x80\n\t"                       \
    "v_bitop3_b32 %[a2], %[a2], %[d2], %[d2n] bitop3:0x80\n\t"
#define AC_OUT                                                                                  \
    [d0n] "=&v"(d0n), [d1n] "=&v"(d1n), [d2n] "=&v"(d2n), [t0] "=&v"(t0), [t1] "=&v"(t1),        \
        [t2] "=&v"(t2), [xh] "=&v"(xh), [ne] "=&v"(ne), [g] "=&v"(g)
#define AC_IN                                                                                   \
    [d0] "v"(s.d0), [d1] "v"(s.d1), [d2] "v"(s.d2), [s0] "v"(s.s0), [s1] "v"(s.s1),              \
        [s2] "v"(s.s2), [ph] "v"(ph), [pl] "v"(pl), [H] "v"(H), [L] "v"(L), [sh] "i"(P)
#define AC_ACC_OUT [a0] "+v"(s.a0), [a1] "+v"(s.a1), [a2] "+v"(s.a2)

struct Nfa {
    uint32_t d0, d1, d2;  // complemented rows
    uint32_t s0, s1, s2;  // rows >> P
    uint32_t a0, a1, a2;  // AND of the rows over the window
};

// Sign-extended single bit: 0 or 0xffffffff (one s_bfe_i32 on a uniform word).
__device__ __forceinline__ uint32_t sbit(uint32_t w, int bit) {
    return (uint32_t)(((int32_t)(w << (31 - bit))) >> 31);
}

// One text base with masks (H, L).  ACC (odd bases): also AND this base's rows
// and the previous base's (still in s.d*) into the hit accumulators.  HAS_N:
// `nm` bit j marks an N.
template <int P, bool HAS_N, bool ACC>
__device__ __forceinline__ void nfa_base(Nfa& s, uint32_t ph, uint32_t pl, uint32_t H, uint32_t L,
                                         uint32_t nm, int j) {
    uint32_t d0n, d1n, d2n, t0, t1, t2, xh, ne, g;
    if constexpr (!HAS_N && !ACC) {
        asm(AC_NEQ AC_NFA : AC_OUT : AC_IN);
    } else if constexpr (!HAS_N && ACC) {
        asm(AC_NEQ AC_NFA AC_ACC : AC_OUT, AC_ACC_OUT : AC_IN);
    } else if constexpr (HAS_N && !ACC) {
        const uint32_t N = sbit(nm, j);
        asm(AC_NEQ_N AC_NFA : AC_OUT : AC_IN, [N] "s"(N));
    } else {
        const uint32_t N = sbit(nm, j);
        asm(AC_NEQ_N AC_NFA AC_ACC : AC_OUT, AC_ACC_OUT : AC_IN, [N] "s"(N));
    }
    s.d0 = d0n;
    s.d1 = d1n;
    s.d2 = d2n;
    s.s0 = t0;
    s.s1 = t1;
    s.s2 = t2;
}

// NB (even) bases starting at pair index q of the staged masks; `nm` bit j is
// the N flag of base j of this group.
template <int P, int NB, bool HAS_N>
__device__ __forceinline__ void run(Nfa& s, uint32_t ph, uint32_t pl, const uint4* __restrict__ hl,
                                    uint32_t q, uint32_t nm) {
#pragma unroll
    for (int j = 0; j < NB; j += 2) {
        const uint4 m = hl[q + j / 2];
        nfa_base<P, HAS_N, false>(s, ph, pl, m.x, m.y, nm, j);
        nfa_base<P, HAS_N, true>(s, ph, pl, m.z, m.w, nm, j + 1);
    }
}

template <int P, int NB>
__device__ __forceinline__ void run_any(Nfa& s, uint32_t ph, uint32_t pl, const uint4* __restrict__ hl,
                                        uint32_t q, uint32_t nm) {
    if (nm == 0u) run<P, NB, false>(s, ph, pl, hl, q, nm);
    else run<P, NB, true>(s, ph, pl, hl, q, nm);
}

// N flags of bases [b, b + 16) of a window (b a multiple of 16) from the mask image.
__device__ __forceinline__ uint32_t nflags16(const uint32_t* __restrict__ nmask, uint32_t b) {
    return (nmask[b >> 5] >> (b & 16u)) & 0xffffu;
}

template <int P>
__device__ __forceinline__ void count_kernel_body(const LaunchArgs& a, uint4* __restrict__ stage) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t wave = (uint64_t)blockIdx.x * WAVES_PER_BLOCK + wib;
    if (wave >= a.total_waves) return;
    uint4* __restrict__ hl = stage + wib * (SEG_BASES / 2);

    // Segment lookup (wave-uniform, <= AC_MAX_SEGS entries).
    int si = 0;
#pragma unroll
    for (int i = 1; i < AC_MAX_SEGS; ++i)
        if (i < (int)a.n_segs && wave >= a.seg[i].wave_begin) si = i;
    const SegDev& sg = a.seg[si];
    const uint64_t local = wave - sg.wave_begin;
    const uint32_t g = (uint32_t)(local % sg.groups);
    const uint32_t wb = (uint32_t)(local / sg.groups);
    const uint32_t m = a.m;

    // Lane constants: character i of pattern p at bit 31 - (i*P + p).
    uint32_t ph = 0, pl = 0, first = 0, last_bit[P];
    uint32_t cand[P];
#pragma unroll
    for (int p = 0; p < P; ++p) {
        cand[p] = g * 64u * P + (uint32_t)p * 64u + lane;
        last_bit[p] = 31u - ((m - 1u) * P + (uint32_t)p);
        first |= 1u << (31 - p);
        if (cand[p] < sg.n_kmers) {
            const uint64_t km = sg.kmers[cand[p]];
            for (uint32_t i = 0; i < m; ++i) {
                const uint32_t b = (uint32_t)(km >> (2u * (m - 1u - i))) & 3u;
                ph |= (b >> 1) << (31u - (i * P + p));
                pl |= (b & 1u) << (31u - (i * P + p));
            }
        }
    }
    // Initial rows (empty text): R1 has character 0 set, R2 characters 0 and 1.
    const uint32_t d1_init = ~first, d2_init = ~(first | (first >> P));

    uint32_t cnt[P];
#pragma unroll
    for (int p = 0; p < P; ++p) cnt[p] = 0;

    const uint32_t w_begin = wb * sg.wpw;
    const uint32_t w_end = min(sg.n_windows, w_begin + sg.wpw);
    for (uint32_t w = w_begin; w < w_end; ++w) {
        const uint64_t base = sg.start[w];
        const uint32_t len = sg.length[w];
        if ((base & 31u) || base + len > sg.n_bases) continue;  // malformed window: never read outside the image
        const uint32_t* __restrict__ codes = sg.codes + (base >> 4);
        const uint32_t* __restrict__ nmask = sg.nmask + (base >> 5);
        Nfa s;
        s.d0 = ~0u;
        s.d1 = d1_init;
        s.d2 = d2_init;
        s.s0 = ~0u >> P;
        s.s1 = d1_init >> P;
        s.s2 = d2_init >> P;
        s.a0 = ~0u;
        s.a1 = d1_init;
        s.a2 = d2_init;  // for k <= 2 the empty alignment already reaches the last character
        for (uint32_t sb = 0; sb < len; sb += SEG_BASES) {
            // Stage bases [sb, sb + 128) as (H, L) mask pairs: lane l expands bases sb+2l, sb+2l+1.
            {
                const uint32_t b = sb + 2u * lane;
                const uint32_t code = b < len ? codes[b >> 4] : 0u;
                const int sh = (int)(2u * (b & 15u));
                uint4 v;
                v.x = sbit(code, sh + 1);
                v.y = sbit(code, sh);
                v.z = sbit(code, sh + 3);
                v.w = sbit(code, sh + 2);
                hl[lane] = v;
            }
            const uint32_t nb = min(SEG_BASES, len - sb);
            const uint32_t nfull = nb >> 4;
            for (uint32_t ch = 0; ch < nfull; ++ch)
                run_any<P, 16>(s, ph, pl, hl, ch * 8u, nflags16(nmask, sb + ch * 16u));
            const uint32_t rem = nb & 15u;
            if (rem) {
                uint32_t q = nfull * 8u;
                uint32_t nm = nflags16(nmask, sb + nfull * 16u);
                if (rem & 8u) {
                    run_any<P, 8>(s, ph, pl, hl, q, nm);
                    q += 4u;
                    nm >>= 8;
                }
                if (rem & 4u) {
                    run_any<P, 4>(s, ph, pl, hl, q, nm);
                    q += 2u;
                    nm >>= 4;
                }
                if (rem & 2u) {
                    run_any<P, 2>(s, ph, pl, hl, q, nm);
                    q += 1u;
                    nm >>= 2;
                }
                if (rem & 1u) {
                    const uint4 mm = hl[q];
                    nfa_base<P, true, false>(s, ph, pl, mm.x, mm.y, nm, 0);
                    s.a0 &= s.d0;
                    s.a1 &= s.d1;
                    s.a2 &= s.d2;
                }
            }
        }
#pragma unroll
        for (int p = 0; p < P; ++p)
            cnt[p] += 3u - ((s.a0 >> last_bit[p]) & 1u) - ((s.a1 >> last_bit[p]) & 1u) -
                      ((s.a2 >> last_bit[p]) & 1u);
    }

#pragma unroll
    for (int p = 0; p < P; ++p)
        if (cand[p] < sg.n_kmers && cnt[p]) atomicAdd(&sg.counts[cand[p]], cnt[p]);
}

}  // namespace

template <int P>
__global__ __launch_bounds__(64 * WAVES_PER_BLOCK) void wm2_count_kernel(LaunchArgs a) {
    __shared__ uint4 stage[WAVES_PER_BLOCK * (SEG_BASES / 2)];
    count_kernel_body<P>(a, stage);
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
