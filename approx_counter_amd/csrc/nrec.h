// nrec.h -- inline N records of equal-window images, shared by the
// host packer (host_pack.cpp) and the count kernel (wm_count.hip).
//
// Equal windows of L bases sit at S = ceil32(L)-base strides, so every window
// slot ends in S - L padding bases that are never read as text.  When a job's
// windows leave room, the packer writes the positions of the window's N bases
// into the top R bits of the slot's last code word:
//   bits 31-29        the number of N bases c (0 = none), or NREC_OVERFLOW when
//                     there are more than fit (then the window's N-bitmap words
//                     are needed, and the image's N bitmap is sent);
//   below them        c positions of PB bits each (base index inside the
//                     window), position i at bits [29 - PB(i+1), 29 - PB i).
// (count at a fixed place: the kernel reads it with one constant shift per window)
// So a window carries everything needed to count it: the count kernel builds the
// window's N-mask words from the record, and the N bitmap (1 bit per base, half
// the size of the codes) stays on the host unless some window overflowed --
// which lets the early launch count windows as they arrive instead of waiting for
// the bitmap at the end of the region.  Plain constexpr (host and device).
#pragma once
#include <stdint.h>

namespace acamd {

constexpr uint32_t NREC_OVERFLOW = 7u;

// R: record bits for windows of `len` bases (0 = no record: no room, or a window
// longer than one 256-base fetch).
constexpr uint32_t nrec_bits(uint32_t len) {
    const uint32_t S = (len + 31u) & ~31u, pad = S - len;
    const uint32_t R = 2u * (pad < 16u ? pad : 16u), pb = S <= 128u ? 7u : 8u;
    return (len == 0u || len > 256u || R < 3u + pb) ? 0u : R;
}
// PB: bits per position
constexpr uint32_t nrec_pos_bits(uint32_t len) { return ((len + 31u) & ~31u) <= 128u ? 7u : 8u; }
// positions a record holds (<= 4)
constexpr uint32_t nrec_cap(uint32_t len) {
    const uint32_t R = nrec_bits(len), c = R ? (R - 3u) / nrec_pos_bits(len) : 0u;
    return c < 4u ? c : 4u;
}
// shift of position i inside the record word
constexpr uint32_t nrec_pos_shift(uint32_t pb, uint32_t i) { return 29u - pb * (i + 1u); }
// index of the slot's code word holding the record (16 bases per word)
constexpr uint32_t nrec_word(uint32_t len) { return ((len + 31u) & ~31u) / 16u - 1u; }

static_assert(nrec_bits(100) == 32 && nrec_cap(100) == 4 && nrec_cap(101) == 4, "cfg2 windows: 4 positions");
static_assert(nrec_bits(150) == 20 && nrec_cap(150) == 2 && nrec_cap(151) == 1, "cfg5 windows");
static_assert(nrec_bits(128) == 0 && nrec_bits(125) == 0 && nrec_bits(300) == 0, "no room");

}  // namespace acamd
