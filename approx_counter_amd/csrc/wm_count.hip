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
// 1992, "Fast text searching allowing errors"), free start in the text.
// Bit i of row R_d = "pattern prefix of length i+1 ends at the current text
// position with <= d edits":
//   R0' = ((R0 << 1) | 1) & Eq
//   Rd' = ((Rd << 1) & Eq) | Rd-1 | (Rd-1 << 1) | (Rd-1' << 1) | low_d
// (low_d = bits 0..d-1, always set).  The top bit (i = k-1) ORed over the
// window is [d_min <= d]; the count adds the three levels.
//
// MI355X mapping:
//  * lane = candidate(s), window text wave-uniform.  The 2-bit text and the
//    N mask are read with scalar loads; each base becomes sign-extended SGPR
//    masks H, L so Eq = ~(ph ^ H) & ~(pl ^ L) is two VALU ops with no per-lane
//    table lookup.
//  * P = floor(32/k) (<= 4) candidates are packed side by side in one 32-bit
//    register.  Bits shifted out of pattern p land in pattern p+1's always-set
//    low bits (row 0: the "| 1"; rows 1, 2: low_d), so they are absorbed.
//  * Issue cost drives the instruction choice.  On gfx950 v_add_u32, v_and,
//    v_or, v_xor and v_bitop3_b32 issue in 2 cycles per wave64 while shifts,
//    v_lshl_or, v_or3 and v_and_or take 4 (tools/ubench_valu.hip,
//    profiles/r01_ubench_valu.txt).  So every shift is x + x and every 3-input
//    boolean is one v_bitop3_b32; each row's shifted value (t_d = R_d' << 1) is
//    computed once and reused as (R_d << 1) at the next base.  A base costs
//    9 ops of NFA + 2 of Eq + 1.5 of hit accumulation (v_bitop3 OR3 over two
//    bases) = 12.5 full-rate ops for P candidates.
//  * Integer-only VALU work: no MFMA, no LDS.  Counts are uint32 atomics
//    (order-independent, bit-exact).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "wm_count.h"

namespace acamd {
namespace {

// One text base of the NFA as ONE asm statement (no hipcc boundary pads inside;
// plain VALU -> VALU dependencies need no software wait states on gfx950):
//   xh  = ph ^ H ; eq = ~xh & ~(pl ^ L) [& ~N]            Eq of this base
//   x0  = s0 | one ; r0' = x0 & eq ; t0 = r0' + r0'        row 0, t0 = r0' << 1
//   h   = x0 | r0 | t0 ; r1' = (s1 & eq) | h ; t1 = r1' + r1'
//   h   = s1 | r1 | t1 ; r2' = (s2 & eq) | h ; t2 = r2' + r2'
// v_bitop3 tables over (s0, s1, s2) = (0xf0, 0xcc, 0xaa): 0x09 = ~a & ~(b ^ c),
// 0xfe = a | b | c, 0xea = (a & b) | c.  With ACC, the hit accumulators take
// the OR of this base's rows and the previous base's (q0..q2): 0xfe again.
#define AC_STEP_EQ "v_xor_b32 %[xh], %[H], %[ph]\n\tv_bitop3_b32 %[eq], %[xh], %[pl], %[L] bitop3:0x09\n\t"
#define AC_STEP_N "v_and_b32 %[eq], %[nN], %[eq]\n\t"
#define AC_STEP_NFA                                                         \
    "v_or_b32 %[x0], %[one], %[s0]\n\t"                                     \
    "v_and_b32 %[r0n], %[x0], %[eq]\n\t"                                    \
    "v_add_u32 %[t0], %[r0n], %[r0n]\n\t"                                   \
    "v_bitop3_b32 %[h], %[x0], %[r0], %[t0] bitop3:0xfe\n\t"                \
    "v_bitop3_b32 %[r1n], %[s1], %[eq], %[h] bitop3:0xea\n\t"               \
    "v_add_u32 %[t1], %[r1n], %[r1n]\n\t"                                   \
    "v_bitop3_b32 %[h], %[s1], %[r1], %[t1] bitop3:0xfe\n\t"                \
    "v_bitop3_b32 %[r2n], %[s2], %[eq], %[h] bitop3:0xea\n\t"               \
    "v_add_u32 %[t2], %[r2n], %[r2n]\n\t"
#define AC_STEP_ACC                                                         \
    "v_bitop3_b32 %[a0], %[a0], %[r0], %[r0n] bitop3:0xfe\n\t"              \
    "v_bitop3_b32 %[a1], %[a1], %[r1], %[r1n] bitop3:0xfe\n\t"              \
    "v_bitop3_b32 %[a2], %[a2], %[r2], %[r2n] bitop3:0xfe\n\t"
#define AC_STEP_OUT                                                                              \
    [r0n] "=&v"(r0n), [r1n] "=&v"(r1n), [r2n] "=&v"(r2n), [t0] "=&v"(t0), [t1] "=&v"(t1),         \
        [t2] "=&v"(t2), [xh] "=&v"(xh), [eq] "=&v"(eq), [x0] "=&v"(x0), [h] "=&v"(h)
#define AC_STEP_IN                                                                               \
    [r0] "v"(s.r0), [r1] "v"(s.r1), [r2] "v"(s.r2), [s0] "v"(s.s0), [s1] "v"(s.s1), [s2] "v"(s.s2), \
        [ph] "v"(c.ph), [pl] "v"(c.pl), [H] "s"(H), [L] "s"(L), [one] "s"(c.one)

struct Nfa {
    uint32_t r0, r1, r2;  // rows
    uint32_t s0, s1, s2;  // rows << 1
    uint32_t a0, a1, a2;  // OR of the rows over the window
};

struct Lane {
    uint32_t ph, pl;  // high / low bit of every pattern base (lane constants)
    uint32_t one;     // bit 0 of every pattern (wave-uniform)
};

// Sign-extended single bit: 0 or 0xffffffff (one s_bfe_i32 on a uniform word).
__device__ __forceinline__ uint32_t sbit(uint32_t w, int bit) {
    return (uint32_t)(((int32_t)(w << (31 - bit))) >> 31);
}

// One base j of a code word.  ACC: also OR this base's rows and the previous
// base's (still in s.r*) into the hit accumulators (called on odd bases).
template <bool HAS_N, bool ACC>
__device__ __forceinline__ void nfa_base(Nfa& s, const Lane& c, uint32_t code, uint32_t nm, int j) {
    const uint32_t H = sbit(code, 2 * j + 1), L = sbit(code, 2 * j);
    uint32_t r0n, r1n, r2n, t0, t1, t2, xh, eq, x0, h;
    if constexpr (!HAS_N && !ACC) {
        asm(AC_STEP_EQ AC_STEP_NFA : AC_STEP_OUT : AC_STEP_IN);
    } else if constexpr (!HAS_N && ACC) {
        asm(AC_STEP_EQ AC_STEP_NFA AC_STEP_ACC
            : AC_STEP_OUT, [a0] "+v"(s.a0), [a1] "+v"(s.a1), [a2] "+v"(s.a2) : AC_STEP_IN);
    } else if constexpr (HAS_N && !ACC) {
        const uint32_t nN = ~sbit(nm, j);
        asm(AC_STEP_EQ AC_STEP_N AC_STEP_NFA : AC_STEP_OUT : AC_STEP_IN, [nN] "s"(nN));
    } else {
        const uint32_t nN = ~sbit(nm, j);
        asm(AC_STEP_EQ AC_STEP_N AC_STEP_NFA AC_STEP_ACC
            : AC_STEP_OUT, [a0] "+v"(s.a0), [a1] "+v"(s.a1), [a2] "+v"(s.a2) : AC_STEP_IN, [nN] "s"(nN));
    }
    s.r0 = r0n;
    s.r1 = r1n;
    s.r2 = r2n;
    s.s0 = t0;
    s.s1 = t1;
    s.s2 = t2;
}

// NB bases (even) from the low bits of one code word: 12.5 VALU per base.
template <int NB, bool HAS_N>
__device__ __forceinline__ void chunk(Nfa& s, const Lane& c, uint32_t code, uint32_t nm) {
#pragma unroll
    for (int j = 0; j < NB; j += 2) {
        nfa_base<HAS_N, false>(s, c, code, nm, j);
        nfa_base<HAS_N, true>(s, c, code, nm, j + 1);
    }
}

template <int NB>
__device__ __forceinline__ void chunk_any(Nfa& s, const Lane& c, uint32_t code, uint32_t nm) {
    if (nm == 0u) chunk<NB, false>(s, c, code, nm);
    else chunk<NB, true>(s, c, code, nm);
}

__device__ __forceinline__ void one_base(Nfa& s, const Lane& c, uint32_t code, uint32_t nm) {
    nfa_base<true, false>(s, c, code, nm, 0);
    s.a0 |= s.r0;
    s.a1 |= s.r1;
    s.a2 |= s.r2;
}

}  // namespace

__global__ __launch_bounds__(256) void wm2_count_kernel(LaunchArgs a) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t wave =
        (uint64_t)blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wave >= a.total_waves) return;

    // Segment lookup (wave-uniform, <= AC_MAX_SEGS entries).
    int si = 0;
#pragma unroll
    for (int i = 1; i < AC_MAX_SEGS; ++i)
        if (i < (int)a.n_segs && wave >= a.seg[i].wave_begin) si = i;
    const SegDev& sg = a.seg[si];
    const uint64_t local = wave - sg.wave_begin;
    const uint32_t g = (uint32_t)(local % sg.groups);
    const uint32_t wb = (uint32_t)(local / sg.groups);

    const uint32_t m = a.m, P = a.P;

    // Lane constants: P patterns of m bits side by side, pattern base i at bit p*m+i.
    Lane c;
    c.ph = 0;
    c.pl = 0;
    uint32_t one = 0;
    uint32_t cand[AC_MAX_PACK];
#pragma unroll
    for (int p = 0; p < AC_MAX_PACK; ++p) {
        cand[p] = g * 64u * P + (uint32_t)p * 64u + lane;
        if ((uint32_t)p < P) {
            one |= 1u << (p * m);
            if (cand[p] < sg.n_kmers) {
                const uint64_t km = sg.kmers[cand[p]];
                for (uint32_t i = 0; i < m; ++i) {
                    const uint32_t b = (uint32_t)(km >> (2u * (m - 1u - i))) & 3u;
                    c.ph |= (b >> 1) << (p * m + i);
                    c.pl |= (b & 1u) << (p * m + i);
                }
            }
        }
    }
    c.one = __builtin_amdgcn_readfirstlane(one);
    const uint32_t low2 = c.one | (c.one << 1);
    const uint32_t tops = c.one << (m - 1);
    const uint32_t sh = m - 1;

    uint32_t cnt[AC_MAX_PACK] = {0, 0, 0, 0};

    const uint32_t w_begin = wb * sg.wpw;
    const uint32_t w_end = min(sg.n_windows, w_begin + sg.wpw);
    for (uint32_t w = w_begin; w < w_end; ++w) {
        const uint64_t base = sg.start[w];
        const uint32_t len = sg.length[w];
        if ((base & 31u) || base + len > sg.n_bases) continue;  // malformed window: never read outside the image
        const uint32_t* __restrict__ codes = sg.codes + (base >> 4);
        const uint32_t* __restrict__ nmask = sg.nmask + (base >> 5);
        // Initial rows: prefixes of length <= d match the empty text with d deletions.
        Nfa s;
        s.r0 = 0u;
        s.r1 = c.one;
        s.r2 = low2;
        s.s0 = 0u;
        s.s1 = c.one << 1;
        s.s2 = low2 << 1;
        s.a0 = 0u;
        s.a1 = c.one;
        s.a2 = low2;  // for m <= 2 the empty alignment already reaches the top bit
        const uint32_t nfull = len >> 4;
        for (uint32_t ch = 0; ch < nfull; ++ch) {
            const uint32_t code = codes[ch];
            const uint32_t nm = (nmask[ch >> 1] >> ((ch & 1u) << 4)) & 0xffffu;
            chunk_any<16>(s, c, code, nm);
        }
        const uint32_t rem = len & 15u;
        if (rem) {
            uint32_t code = codes[nfull];
            uint32_t nm = (nmask[nfull >> 1] >> ((nfull & 1u) << 4)) & 0xffffu;
            if (rem & 8u) {
                chunk_any<8>(s, c, code, nm);
                code >>= 16;
                nm >>= 8;
            }
            if (rem & 4u) {
                chunk_any<4>(s, c, code, nm);
                code >>= 8;
                nm >>= 4;
            }
            if (rem & 2u) {
                chunk_any<2>(s, c, code, nm);
                code >>= 4;
                nm >>= 2;
            }
            if (rem & 1u) one_base(s, c, code, nm);
        }
        const uint32_t t = ((s.a0 & tops) >> sh) + ((s.a1 & tops) >> sh) + ((s.a2 & tops) >> sh);
#pragma unroll
        for (int p = 0; p < AC_MAX_PACK; ++p)
            if ((uint32_t)p < P) cnt[p] += (t >> (p * m)) & 3u;
    }

#pragma unroll
    for (int p = 0; p < AC_MAX_PACK; ++p)
        if ((uint32_t)p < P && cand[p] < sg.n_kmers && cnt[p]) atomicAdd(&sg.counts[cand[p]], cnt[p]);
}

hipError_t launch_wm2_count(const LaunchArgs& args, hipStream_t stream) {
    if (args.total_waves == 0) return hipSuccess;
    const uint32_t waves_per_block = 4;
    const uint64_t blocks = (args.total_waves + waves_per_block - 1) / waves_per_block;
    hipLaunchKernelGGL(wm2_count_kernel, dim3((uint32_t)blocks), dim3(64 * waves_per_block), 0,
                       stream, args);
    return hipGetLastError();
}

}  // namespace acamd
