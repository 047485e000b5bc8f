// wm_count.hip -- the approximate-count kernel for MI355X (gfx950).
//
// Replaces the OpenMP/SeqAn search loop of errorCount
// (approx_counter.cpp:550-599): for every (candidate k-mer, sampled window)
// pair it decides, per error level e = 0,1,2, whether the k-mer occurs in the
// window with at most e edits -- exactly the three per-read bitfields
// tcount[e] of approx_counter.cpp:553/563 -- and adds the number of levels hit
// to the candidate's counter (the vectorSum of 590-593).
//
// Algorithm: bit-parallel Wu-Manber NFA for edit distance <= 2 (Wu & Manber
// 1992, "Fast text searching allowing errors"), free start in the text:
//   R0' = ((R0<<1)|1) & Eq
//   Rd' = ((Rd<<1)|1) & Eq  |  Rd-1  |  ((Rd-1 | Rd-1') << 1) | 1      (d = 1, 2)
// bit i of Rd = "k-mer prefix of length i+1 ends here with <= d edits".
// The top bit (i = k-1) ORed over the window is [d_min <= d].
//
// MI355X mapping:
//  * lane = candidate(s), window text wave-uniform: the 2-bit text is read
//    with scalar loads and each base becomes two sign-extended SGPR masks
//    (H, L), so Eq = ~(Ph^H) & ~(Pl^L) costs two VALU ops (v_xor + v_bitop3)
//    and no per-lane table lookup.
//  * P = floor(32/k) (capped at 4) candidates are packed side by side in one
//    32-bit register: every carry-in position of a pattern is forced to 1 by
//    the "|1" of the recurrence, so bits shifted out of pattern p into
//    pattern p+1 are absorbed.  R1 keeps bit 0 and R2 bits 0-1 implicit
//    (they are always 1), which removes the explicit "|1" from their
//    recurrences: 12 VALU per text base for P candidates, plus 1.5 for the
//    hit accumulators (v_or3 over two bases).
//  * Integer-only VALU work: no MFMA, no LDS on the hot loop.  Counts are
//    uint32 atomics (order-independent, bit-exact).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "wm_count.h"

namespace acamd {

// v_lshl_or_b32 d, x, 1, y  =  (x << 1) | y.  Kept as one instruction: left to
// itself hipcc reassociates the ORs into v_or3 and loses the fused shift.
__device__ __forceinline__ uint32_t shl1_or(uint32_t x, uint32_t y) {
    uint32_t r;
    asm("v_lshl_or_b32 %0, %1, 1, %2" : "=v"(r) : "v"(x), "v"(y));
    return r;
}

struct NfaState {
    uint32_t r0, r1, r2;  // NFA rows for <= 0, <= 1, <= 2 edits
    uint32_t a0, a1, a2;  // OR of the rows over the window so far
};

struct LaneConsts {
    uint32_t ph, pl;            // high / low bit of every pattern base
    uint32_t one, b01, b012;    // carry-in masks: bit 0 / bits 0-1 / bits 0-2 of each pattern
};

__device__ __forceinline__ void nfa_step(NfaState& s, uint32_t eq, const LaneConsts& c) {
    const uint32_t x0 = shl1_or(s.r0, c.one);
    const uint32_t r0n = x0 & eq;
    const uint32_t x1 = shl1_or(s.r1, c.b01);
    const uint32_t u0 = s.r0 | r0n;
    const uint32_t v1 = shl1_or(u0, s.r0);
    const uint32_t r1n = (x1 & eq) | v1;
    const uint32_t x2 = shl1_or(s.r2, c.b012);
    const uint32_t u1 = s.r1 | r1n;
    const uint32_t v2 = shl1_or(u1, s.r1);
    const uint32_t r2n = (x2 & eq) | v2;
    s.r0 = r0n;
    s.r1 = r1n;
    s.r2 = r2n;
    s.a0 |= r0n;
    s.a1 |= r1n;
    s.a2 |= r2n;
}

// Sign-extended single bit: 0 or 0xffffffff (one s_bfe_i32 on a uniform word).
__device__ __forceinline__ uint32_t sbit(uint32_t w, int bit) {
    return (uint32_t)(((int32_t)(w << (31 - bit))) >> 31);
}

__device__ __forceinline__ uint32_t eq_mask(const LaneConsts& c, uint32_t code, int j) {
    const uint32_t H = sbit(code, 2 * j + 1);
    const uint32_t L = sbit(code, 2 * j);
    return ~(c.ph ^ H) & ~(c.pl ^ L);
}

// 16 bases of one code word, none of them N.
__device__ __forceinline__ void chunk16(NfaState& s, const LaneConsts& c, uint32_t code) {
#pragma unroll
    for (int j = 0; j < 16; ++j) nfa_step(s, eq_mask(c, code, j), c);
}

// 16 bases of one code word, some of them N (nm bit j set -> Eq = 0).
__device__ __forceinline__ void chunk16_n(NfaState& s, const LaneConsts& c, uint32_t code,
                                          uint32_t nm) {
#pragma unroll
    for (int j = 0; j < 16; ++j) nfa_step(s, eq_mask(c, code, j) & ~sbit(nm, j), c);
}

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
    LaneConsts c;
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
    c.one = one;
    c.b01 = one | (one << 1);
    c.b012 = c.b01 | (one << 2);
    const uint32_t tops = one << (m - 1);

    uint32_t cnt[AC_MAX_PACK] = {0, 0, 0, 0};

    const uint32_t w_begin = wb * sg.wpw;
    const uint32_t w_end = min(sg.n_windows, w_begin + sg.wpw);
    for (uint32_t w = w_begin; w < w_end; ++w) {
        const uint64_t base = sg.start[w];
        const uint32_t len = sg.length[w];
        if ((base & 31u) || base + len > sg.n_bases) continue;  // malformed window: never read outside the image
        const uint32_t* __restrict__ codes = sg.codes + (base >> 4);
        const uint32_t* __restrict__ nmask = sg.nmask + (base >> 5);
        NfaState s = {0u, 0u, 0u, 0u, 0u, 0u};
        const uint32_t nfull = len >> 4;
        for (uint32_t ch = 0; ch < nfull; ++ch) {
            const uint32_t code = codes[ch];
            const uint32_t nm = (nmask[ch >> 1] >> ((ch & 1u) << 4)) & 0xffffu;
            if (nm == 0u) chunk16(s, c, code);
            else chunk16_n(s, c, code, nm);
        }
        const uint32_t rem = len & 15u;
        if (rem) {
            const uint32_t code = codes[nfull];
            const uint32_t nm = (nmask[nfull >> 1] >> ((nfull & 1u) << 4)) & 0xffffu;
            for (uint32_t j = 0; j < rem; ++j) {
                const uint32_t H = 0u - ((code >> (2 * j + 1)) & 1u);
                const uint32_t L = 0u - ((code >> (2 * j)) & 1u);
                const uint32_t nok = ((nm >> j) & 1u) - 1u;
                nfa_step(s, ~(c.ph ^ H) & ~(c.pl ^ L) & nok, c);
            }
        }
        if (m <= 2) s.a2 |= tops;  // R2's top bit is one of its implicit bits
        const uint32_t sh = m - 1;
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
