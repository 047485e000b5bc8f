// exact_count.hip -- exact k-mer count of the sampled windows on MI355X.
//
// Replaces count_kmers (approx_counter.cpp:487-519) and the heavy part of the
// candidate selection get_most_frequent / get_solid_kmers (396-405, 372-388):
// SURVEY.md §8(f) rank 1.  Works on the same packed window image as the
// approximate count (2-bit codes + N mask, include/approx_counter_amd.h), so a
// sample is uploaded once for both stages.
//
//  1. insert: every k-mer position of every window with no N in it becomes a
//     key (dna2int layout) counted in an open-addressing hash table in HBM.
//     Each workgroup first aggregates its batch of windows in an LDS table
//     (adapter k-mers occur in most windows, so hot keys are summed locally),
//     then flushes the aggregated (key, count) pairs with global atomics:
//     for k <= 16 into 8-byte slots where one CAS both claims and counts a new
//     key, otherwise into 16-byte slots (CAS on the key + add on the count).
//  2. scan: every occupied slot passes the low-complexity filter (the float
//     DUST score of approx_counter.cpp:247-267, computed exactly as the
//     reference does) and the forbidden set (binary search); kept entries feed
//     a count histogram, and those seen at least twice (EXACT_LIST_MIN) are
//     compacted into a list -- most distinct k-mers of a read sample occur once.
//  3. gather: entries with count >= a threshold chosen on the host from the
//     histogram (the largest count that still yields `limit` entries, or
//     the solid threshold) are compacted from that list (from the table only
//     when the threshold is 1); the host ranks the short result with
//     CompareCount (approx_counter.cpp:275-305).
// HBM-bound integer work (random atomics + streaming scans), no MFMA.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "exact_count.h"

#include <algorithm>

namespace acamd {
namespace {

constexpr int EXACT_THREADS = 256;
#ifndef EXACT_LDS_SLOTS
#define EXACT_LDS_SLOTS 4096
#endif
constexpr uint32_t LDS_SLOTS = EXACT_LDS_SLOTS;  // per-workgroup aggregation table
constexpr uint32_t LDS_PROBES = 32;         // beyond this a key goes straight to the global table
constexpr uint64_t EMPTY = ~0ull;           // never a k-mer value except the all-T 32-mer (kept apart)

__device__ __forceinline__ uint64_t mix64(uint64_t x) {  // murmur3 finaliser
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

// 64-bit value of bases [b, b + k) of the image with base b in the LOW bits.
__device__ __forceinline__ uint64_t gather_bits(const uint32_t* __restrict__ words, uint64_t b, uint32_t bits_per,
                                                uint32_t nbits, uint64_t n_words) {
    const uint64_t bit = b * bits_per;
    const uint64_t w0 = bit >> 5;
    const uint32_t off = (uint32_t)(bit & 31u);
    const uint64_t last = (bit + nbits - 1u) >> 5;  // last word holding a wanted bit
    uint64_t v = words[w0];
    if (w0 + 1 <= last && w0 + 1 < n_words) v |= (uint64_t)words[w0 + 1] << 32;
    v >>= off;
    if (off && w0 + 2 <= last && w0 + 2 < n_words) v |= (uint64_t)words[w0 + 2] << (64u - off);
    return v;
}

// Little-endian 2-bit bases -> dna2int (first base in the most significant used bits).
__device__ __forceinline__ uint64_t to_dna2int(uint64_t le, uint32_t k) {
    uint64_t r = __builtin_bitreverse64(le);
    r = ((r >> 1) & 0x5555555555555555ull) | ((r & 0x5555555555555555ull) << 1);  // restore bit order in each base
    return r >> (64u - 2u * k);
}

// Wide layout: one CAS claims or finds the slot, one add on the same 16-byte
// slot counts.  Compact layout (k <= 16): the CAS that claims a new slot also
// stores its count, so a key seen once costs one atomic; a repeated key adds
// to the low half of its 64-bit word (counts stay below 2^32).
__device__ __forceinline__ void global_insert(const ExactArgs& a, uint64_t key, uint32_t c) {
    if (a.compact) {
        const uint32_t stored = (uint32_t)key + 1u;
        if (!stored) {  // the all-T 16-mer
            atomicAdd(&a.special[0], c);
            return;
        }
        const unsigned long long tag = (unsigned long long)stored << 32;
        uint64_t h = mix64(key) & a.mask;
        for (;;) {
            unsigned long long* sl = &a.ctable[h];
            const unsigned long long cur = atomicCAS(sl, 0ull, tag | c);
            if (cur == 0ull) return;
            if ((uint32_t)(cur >> 32) == stored) {
                atomicAdd(sl, (unsigned long long)c);
                return;
            }
            h = (h + 1u) & a.mask;
        }
    }
    if (key == EMPTY) {  // the all-T 32-mer
        atomicAdd(&a.special[0], c);
        return;
    }
    const unsigned long long stored = (unsigned long long)key + 1ull;
    uint64_t h = mix64(key) & a.mask;
    for (;;) {
        ExactSlot* sl = &a.table[h];
        const unsigned long long cur = atomicCAS((unsigned long long*)&sl->key, 0ull, stored);
        if (cur == 0ull || cur == stored) {
            atomicAdd(&sl->cnt, c);
            return;
        }
        h = (h + 1u) & a.mask;
    }
}

__global__ __launch_bounds__(EXACT_THREADS) void exact_insert_kernel(ExactArgs a) {
    __shared__ unsigned long long lkeys[LDS_SLOTS];
    __shared__ uint32_t lcnt[LDS_SLOTS];
    __shared__ uint32_t wpos[EXACT_WINDOWS_PER_BLOCK + 1];  // prefix sums of k-mer positions per window
    __shared__ uint32_t n_had;
    const uint32_t t = threadIdx.x;
    for (uint32_t s = t; s < LDS_SLOTS; s += EXACT_THREADS) {
        lkeys[s] = EMPTY;
        lcnt[s] = 0;
    }
    const uint32_t w0 = blockIdx.x * EXACT_WINDOWS_PER_BLOCK;
    const uint32_t nw = min((uint32_t)EXACT_WINDOWS_PER_BLOCK, a.n_windows - w0);
    if (t == 0) {
        uint32_t acc = 0;
        for (uint32_t i = 0; i < nw; ++i) {
            wpos[i] = acc;
            const uint64_t st = a.start[w0 + i];
            const uint32_t len = a.length[w0 + i];
            // malformed windows hold no k-mers; the host hears of them (ExactArgs::err)
            const bool ok = !(st & 31u) && len <= a.n_bases && st <= a.n_bases - len;
            if (!ok) atomicOr(a.err, AC_DEVERR_WINDOW);
            acc += (ok && len >= a.k) ? len - a.k + 1u : 0u;
        }
        wpos[nw] = acc;
        n_had = 0;
    }
    __syncthreads();
    const uint32_t total = wpos[nw];
    const uint64_t kmask = (1ull << a.k) - 1ull;  // N flags of the k bases (k <= 32)
    uint32_t had = 0;
    for (uint32_t p = t; p < total; p += EXACT_THREADS) {
        uint32_t i = 0;
        while (wpos[i + 1] <= p) ++i;  // <= EXACT_WINDOWS_PER_BLOCK steps
        const uint64_t b = a.start[w0 + i] + (p - wpos[i]);
        const uint64_t nbits = gather_bits(a.nmask, b, 1u, a.k, a.n_bases >> 5) & kmask;
        if (nbits) {  // count_kmers skips k-mers holding an N (approx_counter.cpp:498, 513-517)
            ++had;
            continue;
        }
        const uint64_t key = to_dna2int(gather_bits(a.codes, b, 2u, 2u * a.k, a.n_bases >> 4), a.k);
        if (key == EMPTY) {
            atomicAdd(&a.special[0], 1u);
            continue;
        }
        uint32_t h = (uint32_t)mix64(key) & (LDS_SLOTS - 1u);
        bool done = false;
        for (uint32_t probe = 0; probe < LDS_PROBES; ++probe) {
            unsigned long long cur = lkeys[h];
            if (cur == EMPTY) {
                cur = atomicCAS(&lkeys[h], (unsigned long long)EMPTY, (unsigned long long)key);
                if (cur == EMPTY) cur = key;
            }
            if (cur == key) {
                atomicAdd(&lcnt[h], 1u);
                done = true;
                break;
            }
            h = (h + 1u) & (LDS_SLOTS - 1u);
        }
        if (!done) global_insert(a, key, 1u);
    }
    if (had) atomicAdd(&n_had, had);
    __syncthreads();
#ifndef EXACT_TIMING_NO_GLOBAL  // timing-only builds: measure the LDS phase alone
    for (uint32_t s = t; s < LDS_SLOTS; s += EXACT_THREADS)
        if (lkeys[s] != EMPTY) global_insert(a, lkeys[s], lcnt[s]);
#endif
    if (t == 0 && n_had) atomicAdd(a.had_n, (unsigned long long)n_had);
}

// getComplexity (approx_counter.cpp:247-267) for k <= 32: the dimer counts, their sum of v * (v - 1)
// (0 * (0 - 1) wraps to 0 in the reference: a zero count adds 0), then one float division exactly as
// the reference.  Counts of up to 31 dimers need more than a nibble, so places 0-14 and 15-29 are
// counted in two nibble histograms (one v_lshl_add_u64 each, as complexity16), spread to bytes and
// added, place 30 added to its byte; below k = 32 the places past the k-mer read zero bases -- one
// (top base, A) dimer and 31 - k (A, A) dimers -- and are subtracted; then sum v^2 - (k - 1) by four
// v_dot4_u32_u8.
__device__ __forceinline__ float complexity(uint64_t kmer, uint32_t k) {
    uint64_t h1 = 0, h2 = 0;
#pragma unroll
    for (uint32_t i = 0; i < 15u; ++i) {
        h1 += 1ull << (4u * ((uint32_t)(kmer >> (2u * i)) & 15u));
        h2 += 1ull << (4u * ((uint32_t)(kmer >> (2u * (i + 15u))) & 15u));
    }
    const uint64_t m = 0x0F0F0F0F0F0F0F0Full;
    uint64_t lo = (h1 & m) + (h2 & m), hi = ((h1 >> 4) & m) + ((h2 >> 4) & m);  // bytes: even / odd dimers
    const uint32_t d30 = (uint32_t)(kmer >> 60) & 15u;  // place 30: bases 30 and 31
    (d30 & 1u ? hi : lo) += 1ull << (8u * (d30 >> 1));
    if (k < 32u) {
        const uint32_t top = (uint32_t)(kmer >> (2u * (k - 1u))) & 15u;  // (top base, A): 0-3
        (top & 1u ? hi : lo) -= 1ull << (8u * (top >> 1));
        lo -= (uint64_t)(31u - k);  // (A, A): dimer 0, byte 0 of the even bytes
    }
    uint32_t sq = __builtin_amdgcn_udot4((uint32_t)lo, (uint32_t)lo, 0u, false);
    sq = __builtin_amdgcn_udot4((uint32_t)(lo >> 32), (uint32_t)(lo >> 32), sq, false);
    sq = __builtin_amdgcn_udot4((uint32_t)hi, (uint32_t)hi, sq, false);
    sq = __builtin_amdgcn_udot4((uint32_t)(hi >> 32), (uint32_t)(hi >> 32), sq, false);
    const uint32_t sum = sq - (k >= 1u ? k - 1u : 0u);
    return (float)sum / (float)(2 * ((int)k - 2));
}

// The same score for k <= 16: at most 15 dimers, so each of the 16 dimer
// counts fits a 4-bit field of one 64-bit register (one shift + add per dimer).
// The sum of v * (v - 1) over the 16 counts is sum v^2 - sum v, and sum v = k - 1 (the dimers):
// the nibbles spread to bytes, sum v^2 is four v_dot4_u32_u8 (was 16 extract / multiply / add
// steps; the score runs once per distinct k-mer in the count kernel).  Counts v = 0 add 0 either way,
// as 0 * (0 - 1) does in the reference.
// All 15 dimer places are counted unconditionally (one v_bfe + one v_lshl_add_u64 each; a guard on k
// made every step a pair of selects): below k = 16 the places k - 1 .. 14 read the zero bases above the
// k-mer -- one (top base, A) dimer and 15 - k (A, A) dimers, taken off again (no nibble exceeds 15).
__device__ __forceinline__ float complexity16(uint32_t kmer, uint32_t k) {
    uint64_t c = 0;
#pragma unroll
    for (uint32_t i = 0; i < 15u; ++i) c += 1ull << (4u * ((kmer >> (2u * i)) & 15u));
    if (k < 16u) c -= (1ull << (4u * ((kmer >> (2u * (k - 1u))) & 15u))) + (uint64_t)(15u - k);
    const uint64_t lo = c & 0x0F0F0F0F0F0F0F0Full, hi = (c >> 4) & 0x0F0F0F0F0F0F0F0Full;
    uint32_t sq = __builtin_amdgcn_udot4((uint32_t)lo, (uint32_t)lo, 0u, false);
    sq = __builtin_amdgcn_udot4((uint32_t)(lo >> 32), (uint32_t)(lo >> 32), sq, false);
    sq = __builtin_amdgcn_udot4((uint32_t)hi, (uint32_t)hi, sq, false);
    sq = __builtin_amdgcn_udot4((uint32_t)(hi >> 32), (uint32_t)(hi >> 32), sq, false);
    const uint32_t sum = sq - (k >= 1u ? k - 1u : 0u);
    return (float)sum / (float)(2 * ((int)k - 2));
}

// The forbidden k-mers of one bucket (the host's per-bucket ranges, ExactArgs::fb_start): a binary
// search over the bucket's few entries, none at all for the many buckets without one.
__device__ __forceinline__ bool forbidden_in(const uint64_t* fb, uint32_t lo, uint32_t hi, uint64_t key) {
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        const uint64_t v = fb[mid];
        if (v == key) return true;
        if (v < key) lo = mid + 1;
        else hi = mid;
    }
    return false;
}

__device__ __forceinline__ bool is_forbidden(const ExactArgs& a, uint64_t key) {
    uint32_t lo = 0, hi = a.n_forbidden;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        const uint64_t v = a.forbidden[mid];
        if (v == key) return true;
        if (v < key) lo = mid + 1;
        else hi = mid;
    }
    return false;
}

// Slot layouts.  load(): one load of slot s, unconditional (clamped address)
// so a thread's loads issue back to back; for s >= slots the value is ignored
// by kept_count.  decode(): count of a loaded slot (0 = empty) and its k-mer.
// special: the all-T k-mer whose stored key wraps to 0, counted in special[0].
template <bool Compact>
struct Layout;
template <>
struct Layout<false> {
    using V = uint4;
    static constexpr uint32_t UNROLL = 4;  // four 16-byte loads in flight per thread
    static constexpr uint64_t special = ~0ull;
    __device__ static V load(const ExactArgs& a, uint64_t s) {
        return *reinterpret_cast<const uint4*>(&a.table[s < a.slots ? s : a.slots - 1u]);
    }
    __device__ static uint32_t decode(V v, uint64_t& key) {
        const uint64_t stored = ((uint64_t)v.y << 32) | v.x;
        if (!stored) return 0;
        key = stored - 1ull;
        return v.z;
    }
};
template <>
struct Layout<true> {
    using V = unsigned long long;
    static constexpr uint32_t UNROLL = 8;  // eight 8-byte loads in flight per thread
    static constexpr uint64_t special = 0xffffffffull;
    __device__ static V load(const ExactArgs& a, uint64_t s) { return a.ctable[s < a.slots ? s : a.slots - 1u]; }
    __device__ static uint32_t decode(V v, uint64_t& key) {
        const uint32_t stored = (uint32_t)(v >> 32);
        if (!stored) return 0;
        key = stored - 1u;
        return (uint32_t)v;
    }
};

// Kept (not low-complexity, not forbidden) entry count of a loaded slot, 0 if
// none; slot index a.slots is the all-T k-mer kept apart from the table.
template <bool Compact>
__device__ __forceinline__ uint32_t kept_count(const ExactArgs& a, uint64_t s, typename Layout<Compact>::V v,
                                               uint64_t& key) {
    uint32_t c;
    if (s == a.slots) {
        key = Layout<Compact>::special;
        c = a.special[0];
    } else {
        c = Layout<Compact>::decode(v, key);
    }
    if (!c) return 0;
    if (complexity(key, a.k) >= a.lc_threshold) return 0;  // haveLowComplexity (214-234)
    if (is_forbidden(a, key)) return 0;                    // isForbiddenKmer (330-332)
    return c;
}

// Block-level compaction: lanes append (key, count) to an LDS buffer; the
// buffer goes to the global list with one atomic per flush, so the list
// counter sees a few hundred atomics per launch instead of one per wave.
constexpr uint32_t APPEND_BUF = 2048;

struct BlockAppender {
    uint64_t* keys;
    uint32_t* cnts;
    unsigned long long* n;
    uint64_t cap;
    uint64_t* lk;  // LDS
    uint32_t* lc;  // LDS
    uint32_t* ln;  // LDS
    unsigned long long* lbase;

    __device__ void push(bool want, uint64_t key, uint32_t c) {
        if (want) {
            const uint32_t i = atomicAdd(ln, 1u);
            lk[i] = key;
            lc[i] = c;
        }
    }
    // Call from every thread of the block; flushes when `force` or when the
    // next round of pushes (at most `max_push` entries) might not fit.
    __device__ void sync_flush(bool force, uint32_t max_push = EXACT_THREADS) {
        __syncthreads();
        const uint32_t m = *ln;
        if (!m || (!force && m + max_push <= APPEND_BUF)) return;  // block-uniform
        if (threadIdx.x == 0) *lbase = atomicAdd(n, (unsigned long long)m);
        __syncthreads();
        const uint64_t b = *lbase;
        for (uint32_t i = threadIdx.x; i < m; i += blockDim.x)
            if (b + i < cap) {
                keys[b + i] = lk[i];
                cnts[b + i] = lc[i];
            }
        __syncthreads();
        if (threadIdx.x == 0) *ln = 0;
        __syncthreads();
    }
};

#define DECLARE_APPENDER(name, K, C, N, CAP)                                              \
    __shared__ uint64_t name##_k[APPEND_BUF];                                             \
    __shared__ uint32_t name##_c[APPEND_BUF];                                             \
    __shared__ uint32_t name##_n;                                                         \
    __shared__ unsigned long long name##_b;                                               \
    if (threadIdx.x == 0) name##_n = 0;                                                   \
    __syncthreads();                                                                      \
    BlockAppender name{K, C, N, CAP, name##_k, name##_c, &name##_n, &name##_b};

// The scan packs each trip's occupied slots densely per wave in LDS before
// scoring them: most slots are empty (the table is sized for the image, load
// <= 2/3, usually far less), and the DUST score of a lane-per-slot pass ran on
// nearly every wave for a fifth of its lanes (VALU-bound, 283 us at 10^5
// windows).  Per trip a block stages and pushes at most
// EXACT_THREADS * UNROLL entries; the appender flushes before that could overflow.
constexpr uint32_t SCAN_WAVES = EXACT_THREADS / 64;

template <bool Compact>
__global__ __launch_bounds__(EXACT_THREADS) void exact_scan_kernel(ExactArgs a) {
    using L = Layout<Compact>;
    constexpr uint32_t SCAN_UNROLL = 4;
    constexpr uint32_t STAGE = 64 * SCAN_UNROLL;
    static_assert(EXACT_THREADS * SCAN_UNROLL <= APPEND_BUF, "a trip must fit the appender");
    __shared__ uint32_t hist[EXACT_HIST_BINS];
    __shared__ uint64_t st_key[SCAN_WAVES][STAGE];
    __shared__ uint32_t st_cnt[SCAN_WAVES][STAGE];
    DECLARE_APPENDER(app, a.list_keys, a.list_cnts, a.n_list, a.list_cap)
    for (uint32_t i = threadIdx.x; i < EXACT_HIST_BINS; i += EXACT_THREADS) hist[i] = 0;
    __syncthreads();
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint64_t n = a.slots + 1;
    const uint64_t step = (uint64_t)EXACT_THREADS * SCAN_UNROLL;
    const uint64_t stride = (uint64_t)gridDim.x * step;
    uint32_t ones = 0;  // kept entries seen once (the bulk): one LDS add per wave at the end
    for (uint64_t s0 = (uint64_t)blockIdx.x * step; s0 < n; s0 += stride) {  // block-uniform trips
        typename L::V v[SCAN_UNROLL];
#pragma unroll
        for (uint32_t j = 0; j < SCAN_UNROLL; ++j) v[j] = L::load(a, s0 + j * EXACT_THREADS + threadIdx.x);
        uint32_t m = 0;  // entries staged by this wave (wave-uniform)
#pragma unroll
        for (uint32_t j = 0; j < SCAN_UNROLL; ++j) {
            const uint64_t s = s0 + j * EXACT_THREADS + threadIdx.x;
            uint64_t key = 0;
            uint32_t c = 0;
            if (s == a.slots) {
                key = L::special;
                c = a.special[0];
            } else if (s < a.slots) {
                c = L::decode(v[j], key);
            }
            const uint64_t occ = __ballot(c != 0u);
            if (c) {
                const uint32_t i = m + __builtin_amdgcn_mbcnt_hi((uint32_t)(occ >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)occ, 0u));
                st_key[wv][i] = key;
                st_cnt[wv][i] = c;
            }
            m += (uint32_t)__popcll(occ);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (uint32_t i0 = 0; i0 < m; i0 += 64u) {  // wave-uniform
            const uint32_t i = i0 + lane;
            uint64_t key = 0;
            uint32_t c = 0;
            if (i < m) {
                key = st_key[wv][i];
                c = st_cnt[wv][i];
                if (complexity(key, a.k) >= a.lc_threshold) c = 0;  // haveLowComplexity (214-234)
                else if (is_forbidden(a, key)) c = 0;              // isForbiddenKmer (330-332)
            }
            if (c == 1u) ++ones;
            else if (c) atomicAdd(&hist[min(c, (uint32_t)EXACT_HIST_BINS - 1u)], 1u);
            app.push(c >= EXACT_LIST_MIN, key, c);
        }
        app.sync_flush(false, EXACT_THREADS * SCAN_UNROLL);
    }
    app.sync_flush(true);
    for (int off = 32; off; off >>= 1) ones += __shfl_xor(ones, off);
    if (__lane_id() == 0 && ones) atomicAdd(&hist[1], ones);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < EXACT_HIST_BINS; i += EXACT_THREADS)
        if (hist[i]) atomicAdd(&a.hist[i], hist[i]);
}

// Entries with count >= threshold from the whole table (threshold below EXACT_LIST_MIN).
template <bool Compact>
__global__ __launch_bounds__(EXACT_THREADS) void exact_gather_table_kernel(ExactArgs a) {
    DECLARE_APPENDER(app, a.out_keys, a.out_cnts, a.n_out, a.out_cap)
    const uint64_t n = a.slots + 1;
    const uint64_t stride = (uint64_t)gridDim.x * EXACT_THREADS;
    for (uint64_t s0 = (uint64_t)blockIdx.x * EXACT_THREADS; s0 < n; s0 += stride) {
        const uint64_t s = s0 + threadIdx.x;
        uint64_t key = 0;
        const uint32_t c = s < n ? kept_count<Compact>(a, s, Layout<Compact>::load(a, s), key) : 0u;
        app.push(c && c >= a.threshold, key, c);
        app.sync_flush(false);
    }
    app.sync_flush(true);
}

// Entries with count >= threshold from the scan's list (already filtered).
__global__ __launch_bounds__(EXACT_THREADS) void exact_gather_list_kernel(ExactArgs a, uint64_t n) {
    DECLARE_APPENDER(app, a.out_keys, a.out_cnts, a.n_out, a.out_cap)
    const uint64_t stride = (uint64_t)gridDim.x * EXACT_THREADS;
    for (uint64_t s0 = (uint64_t)blockIdx.x * EXACT_THREADS; s0 < n; s0 += stride) {
        const uint64_t s = s0 + threadIdx.x;
        const uint32_t c = s < n ? a.list_cnts[s] : 0u;
        app.push(c >= a.threshold, s < n ? a.list_keys[s] : 0ull, c);
        app.sync_flush(false);
    }
    app.sync_flush(true);
}

// ---------------------------------------------------------------------------
// Partitioned path (every k: 32-bit keys for k <= 16, 64-bit keys above).  The
// hash-table insert above is bound by its random read-modify-write atomics in
// HBM (~7.5M at 10^5 windows, ~380 us of a 540 us insert;
// profiles/r02_exact_log.md).  Here every step streams:
//   keys     each window block writes its k-mer keys densely (one reservation
//            per 1,024 positions), no aggregation
//   hist     per chunk of keys, the count of keys per bucket (bucket = high
//            bits of the key's hash)
//   colscan  chunk offsets inside each bucket, bucket starts
//   scatter  keys to their bucket's range (LDS cursors per bucket)
//   count    one workgroup per bucket counts its keys in an LDS table and
//            runs the low-complexity / forbidden filters, the histogram and
//            the list of the scan kernel above
// Keys are only grouped, never ordered, so nothing has to be stable.  Up to
// 2^16 buckets of ~2,048 keys (134M k-mer positions: cfg4's 10^6 windows per
// read end fit); larger samples take the hash table.

constexpr uint32_t MAX_NB_LOG2 = 16;
#ifndef AC_COUNT_PROBES
#define AC_COUNT_PROBES 64
#endif
constexpr uint32_t COUNT_PROBES = AC_COUNT_PROBES;

// Keys per histogram / scatter chunk: the scatter stages a chunk in LDS (32 KB).
template <class K>
struct PartKey {
    static constexpr uint32_t CHUNK = (uint32_t)(32768 / sizeof(K));
};

// (part_hash and bucket_of: exact_count.h, shared with the host, which sorts the forbidden set by bucket)

// Exclusive prefix of a block's values (thread t of NT holds x); returns the total.
template <uint32_t NT = EXACT_THREADS>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t& excl, uint32_t* wsum) {
    const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
    uint32_t incl = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d, 64);
        if ((int)lane >= d) incl += y;
    }
    if (lane == 63u) wsum[wv] = incl;
    __syncthreads();
    uint32_t before = 0, total = 0;
#pragma unroll
    for (uint32_t w = 0; w < NT / 64; ++w) {
        before += w < wv ? wsum[w] : 0u;
        total += wsum[w];
    }
    __syncthreads();  // wsum may be reused
    excl = before + incl - x;
    return total;
}

// In-place exclusive prefix of v[0, n) in LDS (n up to a few thousand: each
// thread scans a contiguous run); returns the total.  The caller has a barrier
// between the writes of v and this call; the scanned v is visible on return.
__device__ __forceinline__ uint32_t block_scan_lds(uint32_t* v, uint32_t n, uint32_t* wsum) {
    const uint32_t t = threadIdx.x;
    const uint32_t per = (n + EXACT_THREADS - 1) / EXACT_THREADS;
    const uint32_t r0 = min(n, t * per), r1 = min(n, r0 + per);
    uint32_t local = 0;
    for (uint32_t i = r0; i < r1; ++i) local += v[i];
    uint32_t run;
    const uint32_t total = block_excl_scan(local, run, wsum);
    for (uint32_t i = r0; i < r1; ++i) {
        const uint32_t x = v[i];
        v[i] = run;
        run += x;
    }
    __syncthreads();
    return total;
}

// LDS bin counter add for the active lanes of a wave, returning each lane's
// rank among the adds to its bin.  The lanes sharing the first active lane's
// bin take one add of their number: a chunk of an adapter-heavy bucket is
// mostly one key, and 64 same-address LDS atomics serialise.  Used by the
// level-2 histogram (16 -> 14 us); in hist1 and the scatters the extra
// ballot / bpermute cost more than the merging saved (9 -> 11, 23 -> 29,
// 37 -> 49 us; profiles/r02_exact_log.md).
__device__ __forceinline__ uint32_t wave_bin_add(uint32_t* cnt, uint32_t b) {
    const uint32_t b0 = __builtin_amdgcn_readfirstlane(b);
    const uint64_t same = __ballot(b == b0);
    const uint32_t pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(same >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)same, 0u));
    uint32_t old = 0;
    if (b != b0 || pre == 0) old = atomicAdd(&cnt[b], b == b0 ? (uint32_t)__popcll(same) : 1u);
    const uint32_t base = __shfl(old, __ffsll((unsigned long long)same) - 1, 64);
    return b == b0 ? base + pre : old;
}

// Keys of every k-mer position, written densely.  A thread takes SEG_POS
// consecutive positions of one window: it gathers the first key's 2k bits and
// N flags once and rolls the rest (one 2-bit code and one N flag per step),
// instead of gathering every position's words anew.
constexpr uint32_t SEG_POS = 16;
// Threads and windows per keys workgroup: ~100-bp windows make 6 segments each,
// so 42 windows per 256 threads fill them once (16 windows left 62 % of the
// threads idle).  Every round takes its output range with one atomic on the
// shared key counter, and those atomics serialise: at 256 threads the kernel
// took 574 us at cfg4, 300 with block-private ranges (r05_m55); 1,024 threads
// (a quarter of the atomics) 209 us, 512 307 (r05_m56).  64-bit keys stay at
// 512: their LDS stage is twice as large (64 KB).
template <class K>
struct KeysShape {
    static constexpr uint32_t THREADS = sizeof(K) == 4 ? 1024u : 512u;
    static constexpr uint32_t WINDOWS = 42u * THREADS / 256u;
};

template <class K>
__global__ __launch_bounds__(KeysShape<K>::THREADS) void part_keys_kernel(ExactArgs a) {
    constexpr uint32_t KEYS_THREADS = KeysShape<K>::THREADS, KEYS_WINDOWS = KeysShape<K>::WINDOWS;
    __shared__ uint32_t wseg[KEYS_WINDOWS + 1];  // prefix sums of segments per window
    __shared__ uint32_t wsum[KEYS_THREADS / 64];
    __shared__ unsigned long long base_sh;
    __shared__ uint32_t n_had, tot_sh;
    // A round's keys, staged at their block-local offsets, then stored with consecutive lanes on
    // consecutive keys: stored straight from the threads' 16-position runs, each store instruction
    // wrote 64 keys 64 B apart (603 us at cfg4 for 340 MB of keys, profiles/r05_m45).
    __shared__ K stage[KEYS_THREADS * SEG_POS];
    K* keys_out = (K*)a.keys;
    const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
    const uint32_t w0 = blockIdx.x * KEYS_WINDOWS;
    const uint32_t nw = min(KEYS_WINDOWS, a.n_windows - w0);
    {  // segments per window: thread i < nw takes window w0 + i, a block scan makes wseg
        uint32_t nseg = 0;
        if (t < nw) {
            const uint64_t st = a.start[w0 + t];
            const uint32_t len = a.length[w0 + t];
            const bool ok = !(st & 31u) && len <= a.n_bases && st <= a.n_bases - len;
            if (!ok) atomicOr(a.err, AC_DEVERR_WINDOW);
            const uint32_t npos = (ok && len >= a.k) ? len - a.k + 1u : 0u;
            nseg = (npos + SEG_POS - 1u) / SEG_POS;
        }
        uint32_t excl;
        const uint32_t tot = block_excl_scan<KEYS_THREADS>(nseg, excl, wsum);
        if (t < nw) wseg[t] = excl;
        if (t == 0) {
            wseg[nw] = tot;
            n_had = 0;
        }
    }
    __syncthreads();
    const uint32_t total = wseg[nw];
    const uint32_t k = a.k;
    const uint64_t kmask = (1ull << k) - 1ull;
    const K keymask = 2u * k >= 8u * sizeof(K) ? (K)~(K)0 : (K)(((K)1 << (2u * k)) - 1u);
    uint32_t had = 0;
    for (uint32_t s0 = 0; s0 < total; s0 += KEYS_THREADS) {  // block-uniform rounds
        const uint32_t sg = s0 + t;
        K key[SEG_POS];
        uint32_t valid = 0, c = 0;
        if (sg < total) {
            uint32_t i = 0, r = nw;  // the window holding segment sg: the last i with wseg[i] <= sg
            while (r - i > 1) {
                const uint32_t m = (i + r) >> 1;
                if (wseg[m] <= sg) i = m; else r = m;
            }
            const uint64_t wst = a.start[w0 + i];
            const uint32_t npos = a.length[w0 + i] - k + 1u;
            const uint32_t p0 = (sg - wseg[i]) * SEG_POS;
            const uint32_t np = min(SEG_POS, npos - p0);
            const uint64_t b = wst + p0;
            // the first position: gathered; N flags of bases b .. b + k + np - 2 (<= 47 bits)
            K cur = (K)to_dna2int(gather_bits(a.codes, b, 2u, 2u * k, a.n_bases >> 4), k);
            const uint64_t nbits = gather_bits(a.nmask, b, 1u, k + np - 1u, a.n_bases >> 5);
            // codes of bases b + k .. b + k + np - 2 for the rolling steps (<= 15 bases: 30 bits)
            const uint64_t nxt = np > 1u ? gather_bits(a.codes, b + k, 2u, 2u * (np - 1u), a.n_bases >> 4) : 0ull;
#pragma unroll
            for (uint32_t j = 0; j < SEG_POS; ++j) {
                if (j < np) {
                    if (j) cur = (K)(((K)(cur << 2) | (K)((nxt >> (2u * (j - 1u))) & 3u)) & keymask);
                    if ((nbits >> j) & kmask) {
                        ++had;  // count_kmers skips k-mers holding an N (approx_counter.cpp:498, 513-517)
                    } else {
                        key[j] = cur;
                        valid |= 1u << j;
                        ++c;
                    }
                }
            }
        }
        uint32_t incl = c;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(incl, d, 64);
            if ((int)lane >= d) incl += y;
        }
        if (lane == 63u) wsum[wv] = incl;
        __syncthreads();
        if (t == 0) {
            uint32_t tot = 0;
            for (uint32_t w = 0; w < KEYS_THREADS / 64; ++w) {
                const uint32_t x = wsum[w];
                wsum[w] = tot;
                tot += x;
            }
            tot_sh = tot;
            base_sh = tot ? atomicAdd(a.n_keys, (unsigned long long)tot) : 0ull;
        }
        __syncthreads();
        uint32_t off = wsum[wv] + incl - c;  // block-local
#pragma unroll
        for (uint32_t j = 0; j < SEG_POS; ++j)
            if (valid & (1u << j)) stage[off++] = key[j];
        __syncthreads();
        const uint64_t base = base_sh;
        const uint32_t tot = tot_sh;
        for (uint32_t i = t; i < tot; i += KEYS_THREADS)
            if (base + i < a.key_cap) keys_out[base + i] = stage[i];
        __syncthreads();  // wsum / base_sh / stage are reused by the next round
    }
    if (had) atomicAdd(&n_had, had);
    __syncthreads();
    if (t == 0 && n_had) atomicAdd(a.had_n, (unsigned long long)n_had);
}

// Two-level partition of the dense keys into the NB = 2^nb_log2 buckets (a
// bucket = the top nb_log2 bits of the key's hash).  One pass into 8,192
// buckets leaves ~2 keys per bucket in a chunk: the per-chunk histogram is as
// large as the keys and the scatter is one isolated 4-byte write per key
// (hist + scans + scatter 166 us at 10^5 windows; profiles/r02_exact_log.md).
// Level 1 moves the keys into S = 2^s_log2 super-buckets (the top s_log2 bits),
// level 2 splits each super-bucket into its SUB = NB / S buckets.  Both levels
// work on chunks of keys, so a super-bucket swollen by one adapter k-mer is
// still split over many workgroups.

template <class K>
__device__ __forceinline__ uint32_t super_of(K key, uint32_t s_log2) {
    return part_hash(key) >> (32u - s_log2);
}

// f(key) for the keys src[lo, hi), the workgroup's threads striding; PART_BATCH
// loads per thread are issued before their keys are used.
constexpr uint32_t PART_BATCH = 8;
template <class K, class F>
__device__ __forceinline__ void for_keys(const K* src, uint64_t lo, uint64_t hi, F f) {
    const uint32_t t = threadIdx.x;
    for (uint64_t i0 = lo; i0 < hi; i0 += EXACT_THREADS * PART_BATCH) {
        K v[PART_BATCH];
#pragma unroll
        for (uint32_t r = 0; r < PART_BATCH; ++r) {
            const uint64_t i = i0 + r * EXACT_THREADS + t;
            v[r] = i < hi ? src[i] : (K)0;
        }
#pragma unroll
        for (uint32_t r = 0; r < PART_BATCH; ++r)
            if (i0 + r * EXACT_THREADS + t < hi) f(v[r]);
    }
}

// Keys the partition holds: every position key, capped at the buffers' size.
__device__ __forceinline__ uint32_t part_n(const ExactArgs& a) {
    return (uint32_t)min((unsigned long long)a.key_cap, *a.n_keys);
}

// Level 1, per chunk: h1[chunk][s] = its keys in super-bucket s.
template <class K>
__global__ __launch_bounds__(EXACT_THREADS) void part_hist1_kernel(ExactArgs a) {
    constexpr uint32_t CHUNK = PartKey<K>::CHUNK;
    __shared__ uint32_t h[EXACT_MAX_SUPER];
    const uint32_t S = 1u << a.s_log2, t = threadIdx.x;
    for (uint32_t i = t; i < S; i += EXACT_THREADS) h[i] = 0;
    __syncthreads();
    const uint32_t n = part_n(a);
    const uint64_t lo = (uint64_t)blockIdx.x * CHUNK, hi = min((uint64_t)n, lo + CHUNK);
    for_keys((const K*)a.keys, lo, hi, [&](K key) { atomicAdd(&h[super_of(key, a.s_log2)], 1u); });
    __syncthreads();
    for (uint32_t i = t; i < S; i += EXACT_THREADS) a.h1[(uint64_t)blockIdx.x * S + i] = h[i];
}

// Level 1 column scan: h1[.][s] -> each chunk's offset inside super-bucket s,
// stot[s] = the super-bucket's size.  A workgroup takes 32 super-buckets x one
// slab of EXACT_SCAN_SLAB rows, so each row it reads is one 128-B line read by
// one workgroup (one workgroup per column read every line 32 times: 487 us of a
// 3.7 ms cfg4 exact count, profiles/r03_final/exact_cfg4_hash0.md).  Step 1: the
// slabs' column sums.
constexpr uint32_t SCAN_G = EXACT_THREADS / 32;              // row groups per workgroup
constexpr uint32_t SCAN_RPG = EXACT_SCAN_SLAB / SCAN_G;      // rows per row group
__global__ __launch_bounds__(EXACT_THREADS) void part_scan1a_kernel(ExactArgs a) {
    __shared__ uint32_t part[SCAN_G][32];
    const uint32_t S = 1u << a.s_log2, t = threadIdx.x, c = t & 31u, g = t >> 5;
    const uint32_t s = blockIdx.x * 32u + c, slab = blockIdx.y;
    const uint32_t r0 = slab * EXACT_SCAN_SLAB + g * SCAN_RPG;
    uint32_t sum = 0;
#pragma unroll 8
    for (uint32_t i = 0; i < SCAN_RPG; ++i)
        if (r0 + i < a.n_chunks) sum += a.h1[(uint64_t)(r0 + i) * S + s];
    part[g][c] = sum;
    __syncthreads();
    if (g == 0) {
        uint32_t tot = 0;
        for (uint32_t q = 0; q < SCAN_G; ++q) tot += part[q][c];
        a.slab[(uint64_t)slab * S + s] = tot;
    }
}

// Step 2: each slab's base (the earlier slabs' sums), then the exclusive scan of its rows.
__global__ __launch_bounds__(EXACT_THREADS) void part_scan1b_kernel(ExactArgs a) {
    __shared__ uint32_t part[SCAN_G][32];
    const uint32_t S = 1u << a.s_log2, t = threadIdx.x, c = t & 31u, g = t >> 5;
    const uint32_t s = blockIdx.x * 32u + c, slab = blockIdx.y;
    uint32_t b = 0;
    for (uint32_t q = g; q < slab; q += SCAN_G) b += a.slab[(uint64_t)q * S + s];
    part[g][c] = b;
    __syncthreads();
    uint32_t base = 0;
    for (uint32_t q = 0; q < SCAN_G; ++q) base += part[q][c];
    const uint32_t r0 = slab * EXACT_SCAN_SLAB + g * SCAN_RPG;
    uint32_t v[SCAN_RPG];
    uint32_t local = 0;
#pragma unroll
    for (uint32_t i = 0; i < SCAN_RPG; ++i) {
        v[i] = r0 + i < a.n_chunks ? a.h1[(uint64_t)(r0 + i) * S + s] : 0u;
        local += v[i];
    }
    __syncthreads();  // (part is reused)
    part[g][c] = local;
    __syncthreads();
    uint32_t run = base;
    for (uint32_t q = 0; q < g; ++q) run += part[q][c];
#pragma unroll
    for (uint32_t i = 0; i < SCAN_RPG; ++i) {
        if (r0 + i < a.n_chunks) a.h1[(uint64_t)(r0 + i) * S + s] = run;
        run += v[i];
    }
    if (slab + 1u == gridDim.y && g == SCAN_G - 1u) a.stot[s] = run;
}

// Every workgroup of the later steps rebuilds, from stot, the super-buckets'
// starts (sstart[0..S]) and the first level-2 chunk of each (cbeg[0..S]).
__device__ __forceinline__ void super_layout(const ExactArgs& a, uint32_t chunk, uint32_t* sstart, uint32_t* cbeg,
                                             uint32_t* wsum) {
    const uint32_t S = 1u << a.s_log2, t = threadIdx.x;
    for (uint32_t i = t; i < S; i += EXACT_THREADS) {
        const uint32_t v = a.stot[i];
        sstart[i] = v;
        cbeg[i] = (v + chunk - 1u) / chunk;
    }
    __syncthreads();
    const uint32_t tv = block_scan_lds(sstart, S, wsum);
    const uint32_t tc = block_scan_lds(cbeg, S, wsum);
    if (t == 0) {
        sstart[S] = tv;
        cbeg[S] = tc;
    }
    __syncthreads();
}

// Scatter of one chunk (n <= CHUNK keys src[lo, lo + n)) into bins: the keys
// are first grouped by bin in LDS (`stage`), then written out in that order, so
// each bin's keys leave as one contiguous run at gcur[bin] (the chunk's global
// start in that bin) instead of as isolated stores.  `cnt` (nbins entries,
// zeroed by the caller) and `stage` are LDS.
template <class K, class Bin>
__device__ __forceinline__ void staged_scatter(const K* __restrict__ src, uint64_t lo, uint32_t n, K* __restrict__ dst,
                                               uint32_t nbins, uint32_t* cnt, const uint32_t* gcur, K* stage,
                                               uint32_t* wsum, Bin bin) {
    constexpr uint32_t PER = PartKey<K>::CHUNK / EXACT_THREADS;
    const uint32_t t = threadIdx.x;
    K key[PER];
    uint32_t rank[PER];
#pragma unroll
    for (uint32_t r = 0; r < PER; ++r) {
        const uint32_t i = r * EXACT_THREADS + t;
        key[r] = i < n ? src[lo + i] : (K)0;
    }
#pragma unroll
    for (uint32_t r = 0; r < PER; ++r)
        if (r * EXACT_THREADS + t < n) rank[r] = atomicAdd(&cnt[bin(key[r])], 1u);
    __syncthreads();
    block_scan_lds(cnt, nbins, wsum);
#pragma unroll
    for (uint32_t r = 0; r < PER; ++r)
        if (r * EXACT_THREADS + t < n) stage[cnt[bin(key[r])] + rank[r]] = key[r];
    __syncthreads();
    for (uint32_t i = t; i < n; i += EXACT_THREADS) {
        const K k = stage[i];
        const uint32_t b = bin(k);
        dst[gcur[b] + (i - cnt[b])] = k;
    }
}

// Level 1 scatter: each chunk's keys to its ranges of the super-buckets (LDS cursors).
template <class K>
__global__ __launch_bounds__(EXACT_THREADS) void part_scatter1_kernel(ExactArgs a) {
    constexpr uint32_t CHUNK = PartKey<K>::CHUNK;
    __shared__ uint32_t sstart[EXACT_MAX_SUPER + 1], cbeg[EXACT_MAX_SUPER + 1], wsum[EXACT_THREADS / 64];
    __shared__ uint32_t cur[EXACT_MAX_SUPER], cnt[EXACT_MAX_SUPER];
    __shared__ K stage[CHUNK];
    const uint32_t S = 1u << a.s_log2, t = threadIdx.x;
    super_layout(a, CHUNK, sstart, cbeg, wsum);
    for (uint32_t i = t; i < S; i += EXACT_THREADS) {
        cur[i] = sstart[i] + a.h1[(uint64_t)blockIdx.x * S + i];
        cnt[i] = 0;
    }
    __syncthreads();
    const uint32_t n = part_n(a);
    const uint64_t lo = (uint64_t)blockIdx.x * CHUNK;
    if (lo >= n) return;
    const uint32_t s_log2 = a.s_log2;
    staged_scatter((const K*)a.keys, lo, (uint32_t)min((uint64_t)CHUNK, n - lo), (K*)a.tmp, S, cnt, cur, stage, wsum,
                   [=](K key) { return super_of(key, s_log2); });
}

// Level-2 chunk i: its super-bucket and key range [lo, hi) in tmp; false past the last chunk.
__device__ __forceinline__ bool chunk2(const ExactArgs& a, uint32_t chunk, const uint32_t* sstart, const uint32_t* cbeg,
                                       uint32_t i, uint32_t& s, uint32_t& lo, uint32_t& hi) {
    const uint32_t S = 1u << a.s_log2;
    if (i >= cbeg[S]) return false;
    uint32_t l = 0, r = S;  // the last s with cbeg[s] <= i (super-buckets without chunks share cbeg)
    while (r - l > 1) {
        const uint32_t m = (l + r) >> 1;
        if (cbeg[m] <= i) l = m; else r = m;
    }
    s = l;
    lo = sstart[s] + (i - cbeg[s]) * chunk;
    hi = min(sstart[s + 1], lo + chunk);
    return true;
}

// Level 2, per chunk of a super-bucket: h2[chunk][j] = its keys in sub-bucket j.
template <class K>
__global__ __launch_bounds__(EXACT_THREADS) void part_hist2_kernel(ExactArgs a) {
    constexpr uint32_t CHUNK = PartKey<K>::CHUNK;
    __shared__ uint32_t sstart[EXACT_MAX_SUPER + 1], cbeg[EXACT_MAX_SUPER + 1], wsum[EXACT_THREADS / 64];
    __shared__ uint32_t h[EXACT_MAX_SUB];
    const uint32_t SUB = 1u << (a.nb_log2 - a.s_log2), t = threadIdx.x;
    super_layout(a, CHUNK, sstart, cbeg, wsum);
    uint32_t s, lo, hi;
    if (!chunk2(a, CHUNK, sstart, cbeg, blockIdx.x, s, lo, hi)) return;
    for (uint32_t j = t; j < SUB; j += EXACT_THREADS) h[j] = 0;
    __syncthreads();
    for_keys((const K*)a.tmp, lo, hi, [&](K key) { wave_bin_add(h, bucket_of(key, a.nb_log2) & (SUB - 1u)); });
    __syncthreads();
    for (uint32_t j = t; j < SUB; j += EXACT_THREADS) a.h2[(uint64_t)blockIdx.x * SUB + j] = h[j];
}

constexpr uint32_t SCAN2_BATCH = 8;  // level-2 scan: chunk rows loaded per batch
// Level 2, per super-bucket (one wave each, lane j = sub-buckets j, j + 64, ..): bucket
// starts bstart[s * SUB + j] (and bstart[NB]), h2 -> each chunk's cursor.
template <class K>
__global__ __launch_bounds__(EXACT_THREADS) void part_scan2_kernel(ExactArgs a) {
    __shared__ uint32_t sstart[EXACT_MAX_SUPER + 1], cbeg[EXACT_MAX_SUPER + 1], wsum[EXACT_THREADS / 64];
    const uint32_t S = 1u << a.s_log2, SUB = 1u << (a.nb_log2 - a.s_log2);
    super_layout(a, PartKey<K>::CHUNK, sstart, cbeg, wsum);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t s = blockIdx.x * (EXACT_THREADS / 64) + (threadIdx.x >> 6);
    if (s >= S) return;
    const uint32_t c0 = cbeg[s], c1 = cbeg[s + 1];
    uint32_t carry = sstart[s];
    for (uint32_t j0 = 0; j0 < SUB; j0 += 64u) {
        const uint32_t j = j0 + lane;
        uint32_t tot = 0;
        if (j < SUB)
            for (uint32_t c = c0; c < c1; c += SCAN2_BATCH) {
                uint32_t x[SCAN2_BATCH];
#pragma unroll
                for (uint32_t u = 0; u < SCAN2_BATCH; ++u) x[u] = c + u < c1 ? a.h2[(uint64_t)(c + u) * SUB + j] : 0u;
#pragma unroll
                for (uint32_t u = 0; u < SCAN2_BATCH; ++u) tot += x[u];
            }
        uint32_t incl = tot;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(incl, d, 64);
            if ((int)lane >= d) incl += y;
        }
        uint32_t run = carry + incl - tot;
        carry += __shfl(incl, 63, 64);
        if (j < SUB) {
            a.bstart[s * SUB + j] = run;
            // (a batch of loads before its stores: one at a time, each load waited for the store before it)
            for (uint32_t c = c0; c < c1; c += SCAN2_BATCH) {
                uint32_t x[SCAN2_BATCH];
#pragma unroll
                for (uint32_t u = 0; u < SCAN2_BATCH; ++u) x[u] = c + u < c1 ? a.h2[(uint64_t)(c + u) * SUB + j] : 0u;
#pragma unroll
                for (uint32_t u = 0; u < SCAN2_BATCH; ++u)
                    if (c + u < c1) {
                        a.h2[(uint64_t)(c + u) * SUB + j] = run;
                        run += x[u];
                    }
            }
        }
    }
    if (s == S - 1u && lane == 0) a.bstart[S * SUB] = sstart[S];
}

// Level 2 scatter: a chunk's keys to their buckets in `parts`.
template <class K>
__global__ __launch_bounds__(EXACT_THREADS) void part_scatter2_kernel(ExactArgs a) {
    constexpr uint32_t CHUNK = PartKey<K>::CHUNK;
    __shared__ uint32_t sstart[EXACT_MAX_SUPER + 1], cbeg[EXACT_MAX_SUPER + 1], wsum[EXACT_THREADS / 64];
    __shared__ uint32_t cur[EXACT_MAX_SUB], cnt[EXACT_MAX_SUB];
    __shared__ K stage[CHUNK];
    const uint32_t SUB = 1u << (a.nb_log2 - a.s_log2), t = threadIdx.x;
    super_layout(a, CHUNK, sstart, cbeg, wsum);
    uint32_t s, lo, hi;
    if (!chunk2(a, CHUNK, sstart, cbeg, blockIdx.x, s, lo, hi)) return;
    for (uint32_t j = t; j < SUB; j += EXACT_THREADS) {
        cur[j] = a.h2[(uint64_t)blockIdx.x * SUB + j];
        cnt[j] = 0;
    }
    __syncthreads();
    const uint32_t nb_log2 = a.nb_log2;
    staged_scatter((const K*)a.tmp, lo, hi - lo, (K*)a.parts, SUB, cnt, cur, stage, wsum,
                   [=](K key) { return bucket_of(key, nb_log2) & (SUB - 1u); });
}

// DUST score of a key (getComplexity, approx_counter.cpp:247-267): the packed
// 4-bit-bin form for 32-bit keys (k <= 16), the general one above.
__device__ __forceinline__ float key_complexity(uint32_t key, uint32_t k) { return complexity16(key, k); }
__device__ __forceinline__ float key_complexity(uint64_t key, uint32_t k) { return complexity(key, k); }

// One workgroup per bucket: count its keys in LDS, then filter, histogram and
// list them like exact_scan_kernel (the all-T k-mer whose key + 1 wraps to 0 --
// the 16-mer of 32-bit keys, the 32-mer of 64-bit keys -- is tallied in
// special[0] and handled by part_special_kernel).  LDS is kept at ~52 KB
// (32-bit keys: three workgroups per CU) / ~68 KB (64-bit keys: two): the
// table, a 32-bin histogram of the counts 1..32 written out per bucket (phist,
// summed by part_hist_reduce_kernel: thousands of buckets adding into the same
// few global bins would serialise), larger counts straight to the global
// histogram, and a small appender.  An adapter k-mer fills most of its bucket
// with one key: a wave first merges the lanes holding its first lane's key, so
// the LDS add on that slot is one per wave instead of one per lane.
#ifndef AC_COUNT_THREADS
#define AC_COUNT_THREADS 512
#endif
// threads per counting workgroup: 512 (24 / 16 waves per CU) against 256 and 1024 measured
// 12 % faster at cfg4 / cfg5, 7 % at cfg3 (profiles/r05_m52): the inserts' dependent LDS
// read -> CAS -> add chains want more waves, the table's size caps the workgroups per CU.
constexpr uint32_t COUNT_THREADS = AC_COUNT_THREADS;
constexpr uint32_t COUNT_APPEND = 2 * COUNT_THREADS;

constexpr uint32_t COUNT_BATCH = 8;  // keys per thread loaded together (one memory latency per batch)

template <class K>
__global__ __launch_bounds__(COUNT_THREADS) void part_count_kernel(ExactArgs a) {
    constexpr uint32_t SLOTS = EXACT_BUCKET_SLOTS;
    __shared__ K tk[SLOTS];  // key + 1; 0 = empty
    __shared__ uint32_t tc[SLOTS];
    __shared__ uint16_t occ[SLOTS];  // the slots claimed, in claim order: only they are scored and cleared
    __shared__ uint32_t n_occ;
    __shared__ uint32_t hist[EXACT_PHIST];  // counts 1 .. EXACT_PHIST
    __shared__ uint64_t app_k[COUNT_APPEND];
    __shared__ uint32_t app_c[COUNT_APPEND];
    __shared__ uint32_t app_n;
    __shared__ unsigned long long app_b;
    __shared__ uint32_t n_allt;
    const K* parts = (const K*)a.parts;
    const uint32_t t = threadIdx.x;
    const uint32_t NB = 1u << a.nb_log2;
    for (uint32_t i = t; i < SLOTS; i += COUNT_THREADS) {
        tk[i] = 0;
        tc[i] = 0;
    }
    if (t == 0) {
        n_allt = 0;
        app_n = 0;
        n_occ = 0;
    }

    BlockAppender app{a.list_keys, a.list_cnts, a.n_list, a.list_cap, app_k, app_c, &app_n, &app_b};
    // Persistent: workgroup g counts buckets g, g + grid, ...; between buckets
    // only the claimed slots are cleared.  The first batch of keys of the next
    // bucket is requested before this bucket is scored, so its load latency
    // hides behind the scoring.
    K nxt[COUNT_BATCH];
    auto load_batch = [&](K* dst, uint32_t i0, uint32_t hi) __attribute__((always_inline)) {
#pragma unroll
        for (uint32_t r = 0; r < COUNT_BATCH; ++r) {
            const uint32_t i = i0 + r * COUNT_THREADS + t;
            dst[r] = i < hi ? parts[i] : (K)0;
        }
    };
    if (blockIdx.x < NB) load_batch(nxt, a.bstart[blockIdx.x], a.bstart[blockIdx.x + 1]);
    for (uint32_t b = blockIdx.x; b < NB; b += gridDim.x) {
        for (uint32_t i = t; i < EXACT_PHIST; i += COUNT_THREADS) hist[i] = 0;
        __syncthreads();
        const uint32_t lo = a.bstart[b], hi = a.bstart[b + 1];
        const uint32_t f0 = a.fb_start ? a.fb_start[b] : 0u, f1 = a.fb_start ? a.fb_start[b + 1] : 0u;
        uint32_t allt = 0;
        for (uint32_t i0 = lo; i0 < hi; i0 += COUNT_THREADS * COUNT_BATCH) {  // block-uniform batches
            K kb[COUNT_BATCH];
            if (i0 == lo) {
#pragma unroll
                for (uint32_t r = 0; r < COUNT_BATCH; ++r) kb[r] = nxt[r];
            } else {
                load_batch(kb, i0, hi);
            }
#pragma unroll
            for (uint32_t r = 0; r < COUNT_BATCH; ++r) {
                const uint32_t i = i0 + r * COUNT_THREADS + t;
                const bool have = i < hi;
                const K key = kb[r], stored = (K)(key + 1u);
                // lanes holding the wave's first key: one add of their number
                const uint32_t lo32 = __builtin_amdgcn_readfirstlane((uint32_t)key);
                K k0 = (K)lo32;
                if constexpr (sizeof(K) == 8)
                    k0 |= (K)__builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)key >> 32)) << 32;
                const uint64_t same = __ballot(have && key == k0);
                uint32_t add = 1u;
                bool go = have;
                if (have && key == k0) {
                    go = __lane_id() == (uint32_t)__builtin_ctzll(same);
                    add = (uint32_t)__popcll(same);
                }
                if (go && !stored) {
                    allt += add;
                    go = false;
                }
                if (go) {
                    uint32_t h = part_hash(key) & (SLOTS - 1u);
                    uint32_t probe = 0;
                    for (; probe < COUNT_PROBES; ++probe) {
                        K cur = tk[h];
                        if (cur == 0u) {
                            cur = atomicCAS(&tk[h], (K)0, stored);
                            if (cur == 0u) {  // claimed: list the slot for scoring and clearing
                                cur = stored;
                                occ[atomicAdd(&n_occ, 1u)] = (uint16_t)h;
                            }
                        }
                        if (cur == stored) {
                            atomicAdd(&tc[h], add);
                            break;
                        }
                        h = (h + 1u) & (SLOTS - 1u);
                    }
                    if (probe == COUNT_PROBES) atomicOr(a.overflow, 1u);  // the host falls back to the hash table
                }
            }
        }
        if (allt) atomicAdd(&n_allt, allt);
        if (b + gridDim.x < NB) load_batch(nxt, a.bstart[b + gridDim.x], a.bstart[b + gridDim.x + 1]);
        __syncthreads();
        uint32_t ones = 0;
        const uint32_t m = n_occ;
        for (uint32_t s0 = 0; s0 < m; s0 += COUNT_THREADS) {  // block-uniform trips over the claimed slots
            uint32_t c = 0;
            uint64_t key = 0;
            if (s0 + t < m) {
                const uint32_t s = occ[s0 + t];
                const K kk = (K)(tk[s] - 1u);
                key = (uint64_t)kk;
                c = tc[s];
                tk[s] = 0;  // cleared for the next bucket
                tc[s] = 0;
                if (key_complexity(kk, a.k) >= a.lc_threshold) c = 0;  // haveLowComplexity (214-234)
                else if (f1 > f0 && forbidden_in(a.fb_bucketed, f0, f1, key)) c = 0;  // isForbiddenKmer (330-332)
            }
            if (!a.emit_only && c) {
                if (c == 1u) ++ones;
                else if (c <= EXACT_PHIST) atomicAdd(&hist[c - 1u], 1u);
                else atomicAdd(&a.hist[min(c, (uint32_t)EXACT_HIST_BINS - 1u)], 1u);
            }
            app.push(c && c >= a.list_min, key, c);
            // flush when the next trip's pushes might not fit (block-uniform test after a barrier)
            __syncthreads();
            if (app_n + COUNT_THREADS > COUNT_APPEND) app.sync_flush(true);
        }
        for (int off = 32; off; off >>= 1) ones += __shfl_xor(ones, off);
        if (__lane_id() == 0 && ones) atomicAdd(&hist[0], ones);
        __syncthreads();
        if (!a.emit_only)
            for (uint32_t i = t; i < EXACT_PHIST; i += COUNT_THREADS) a.phist[(uint64_t)b * EXACT_PHIST + i] = hist[i];
        if (t == 0) n_occ = 0;
        // (the next bucket's first barrier orders these against its inserts)
    }
    app.sync_flush(true);
    if (t == 0 && n_allt && !a.emit_only) atomicAdd(&a.special[0], n_allt);
}

// hist[c] += sum over buckets of phist[bucket][c - 1], c = 1..EXACT_PHIST.  A
// workgroup reads whole rows (HRED_ROWS buckets = 1 KB per pass, coalesced),
// every HRED_PASSES-th slab of them; thread t keeps bin t % EXACT_PHIST, the
// rows are summed in LDS and each bin adds once per workgroup.  (One
// workgroup per bin, reading 4 B of every 128, took 98 us at cfg4: r05_m53.)
constexpr uint32_t HRED_ROWS = EXACT_THREADS / EXACT_PHIST;
constexpr uint32_t HRED_PASSES = 16;
static_assert(EXACT_THREADS % EXACT_PHIST == 0, "a pass covers whole rows");

__global__ __launch_bounds__(EXACT_THREADS) void part_hist_reduce_kernel(ExactArgs a) {
    __shared__ uint32_t red[EXACT_THREADS];
    const uint32_t t = threadIdx.x;
    const uint64_t n = (uint64_t)EXACT_PHIST << a.nb_log2;
    const uint64_t step = (uint64_t)gridDim.x * EXACT_THREADS;  // a multiple of EXACT_PHIST: the bin stays t's
    uint32_t sum = 0;
#pragma unroll 4
    for (uint64_t i = (uint64_t)blockIdx.x * EXACT_THREADS + t; i < n; i += step) sum += a.phist[i];
    red[t] = sum;
    __syncthreads();
    if (t < EXACT_PHIST) {
        uint32_t tot = 0;
        for (uint32_t r = 0; r < HRED_ROWS; ++r) tot += red[r * EXACT_PHIST + t];
        if (tot) atomicAdd(&a.hist[t + 1u], tot);
    }
}

// The all-T k-mer whose key + 1 wraps (counted apart in special[0]): filters,
// histogram, list.  key = all ones of the key width.
__global__ void part_special_kernel(ExactArgs a, uint64_t key) {
    const uint32_t c = a.special[0];
    if (!c) return;
    if (complexity(key, a.k) >= a.lc_threshold || is_forbidden(a, key)) return;
    if (!a.emit_only) atomicAdd(&a.hist[min(c, (uint32_t)EXACT_HIST_BINS - 1u)], 1u);
    if (c >= a.list_min) {
        const unsigned long long i = atomicAdd(a.n_list, 1ull);
        if (i < a.list_cap) {
            a.list_keys[i] = key;
            a.list_cnts[i] = c;
        }
    }
}

template <class K>
hipError_t part_count(const ExactArgs& a, hipStream_t stream) {
    // persistent workgroups: three per CU for 32-bit keys (LDS ~52 KB each), two for 64-bit (~68 KB)
    const uint32_t per_cu = sizeof(K) == 4 ? 3u : 2u;
    const uint32_t grid = std::min<uint32_t>(1u << a.nb_log2, 256u * per_cu);
    hipLaunchKernelGGL(part_count_kernel<K>, dim3(grid), dim3(COUNT_THREADS), 0, stream, a);
    if (!a.emit_only)
        hipLaunchKernelGGL(part_hist_reduce_kernel,
                           dim3(std::max<uint32_t>(1u, (1u << a.nb_log2) / (HRED_ROWS * HRED_PASSES))),
                           dim3(EXACT_THREADS), 0, stream, a);
    hipLaunchKernelGGL(part_special_kernel, dim3(1), dim3(1), 0, stream, a, (uint64_t)(K)~(K)0);
    return hipGetLastError();
}

template <class K>
hipError_t partitioned(const ExactArgs& a, hipStream_t stream) {
    constexpr uint32_t CHUNK = PartKey<K>::CHUNK;
    if (a.nb_log2 < 6 || a.nb_log2 > MAX_NB_LOG2) return hipErrorInvalidValue;
    const uint32_t NB = 1u << a.nb_log2;
    const uint32_t S = 1u << a.s_log2;
    if (a.s_log2 > a.nb_log2 || S > EXACT_MAX_SUPER || S < 32 || (NB >> a.s_log2) > EXACT_MAX_SUB || !a.n_chunks ||
        (uint64_t)a.n_chunks * CHUNK < a.key_cap || a.n_chunks2 < a.n_chunks + S)
        return hipErrorInvalidValue;
    const uint32_t wblocks = (a.n_windows + KeysShape<K>::WINDOWS - 1) / KeysShape<K>::WINDOWS;
    if (wblocks) hipLaunchKernelGGL(part_keys_kernel<K>, dim3(wblocks), dim3(KeysShape<K>::THREADS), 0, stream, a);
    hipLaunchKernelGGL(part_hist1_kernel<K>, dim3(a.n_chunks), dim3(EXACT_THREADS), 0, stream, a);
    const uint32_t slabs = (a.n_chunks + EXACT_SCAN_SLAB - 1) / EXACT_SCAN_SLAB;
    hipLaunchKernelGGL(part_scan1a_kernel, dim3(S / 32, slabs), dim3(EXACT_THREADS), 0, stream, a);
    hipLaunchKernelGGL(part_scan1b_kernel, dim3(S / 32, slabs), dim3(EXACT_THREADS), 0, stream, a);
    hipLaunchKernelGGL(part_scatter1_kernel<K>, dim3(a.n_chunks), dim3(EXACT_THREADS), 0, stream, a);
    hipLaunchKernelGGL(part_hist2_kernel<K>, dim3(a.n_chunks2), dim3(EXACT_THREADS), 0, stream, a);
    hipLaunchKernelGGL(part_scan2_kernel<K>, dim3((S + EXACT_THREADS / 64 - 1) / (EXACT_THREADS / 64)),
                       dim3(EXACT_THREADS), 0, stream, a);
    hipLaunchKernelGGL(part_scatter2_kernel<K>, dim3(a.n_chunks2), dim3(EXACT_THREADS), 0, stream, a);
    if (hipError_t e = hipGetLastError()) return e;
    return part_count<K>(a, stream);
}

}  // namespace

uint32_t exact_part_chunk(uint32_t k) { return k <= EXACT_COMPACT_MAX_K ? PartKey<uint32_t>::CHUNK : PartKey<uint64_t>::CHUNK; }

hipError_t launch_exact_part_count(const ExactArgs& a, hipStream_t stream) {
    return a.k <= EXACT_COMPACT_MAX_K ? part_count<uint32_t>(a, stream) : part_count<uint64_t>(a, stream);
}

hipError_t launch_exact_partitioned(const ExactArgs& a, hipStream_t stream) {
    return a.k <= EXACT_COMPACT_MAX_K ? partitioned<uint32_t>(a, stream) : partitioned<uint64_t>(a, stream);
}

hipError_t launch_exact_insert(const ExactArgs& a, hipStream_t stream) {
    const uint32_t blocks = (a.n_windows + EXACT_WINDOWS_PER_BLOCK - 1) / EXACT_WINDOWS_PER_BLOCK;
    if (!blocks) return hipSuccess;
    hipLaunchKernelGGL(exact_insert_kernel, dim3(blocks), dim3(EXACT_THREADS), 0, stream, a);
    return hipGetLastError();
}

static uint32_t scan_blocks(const ExactArgs& a, uint32_t per_thread) {
    const uint64_t n = a.slots + 1;
    const uint64_t per_block = (uint64_t)EXACT_THREADS * per_thread;
    return (uint32_t)std::min<uint64_t>(4096, (n + per_block - 1) / per_block);
}

hipError_t launch_exact_scan(const ExactArgs& a, hipStream_t stream) {
    if (a.compact)
        hipLaunchKernelGGL(exact_scan_kernel<true>, dim3(scan_blocks(a, Layout<true>::UNROLL)), dim3(EXACT_THREADS),
                           0, stream, a);
    else
        hipLaunchKernelGGL(exact_scan_kernel<false>, dim3(scan_blocks(a, Layout<false>::UNROLL)),
                           dim3(EXACT_THREADS), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_exact_gather(const ExactArgs& a, bool from_list, uint64_t n_list, hipStream_t stream) {
    if (from_list) {
        if (!n_list) return hipSuccess;
        const uint32_t blocks = (uint32_t)std::min<uint64_t>(4096, (n_list + EXACT_THREADS - 1) / EXACT_THREADS);
        hipLaunchKernelGGL(exact_gather_list_kernel, dim3(blocks), dim3(EXACT_THREADS), 0, stream, a, n_list);
    } else if (a.compact) {
        hipLaunchKernelGGL(exact_gather_table_kernel<true>, dim3(scan_blocks(a, 1)), dim3(EXACT_THREADS), 0, stream,
                           a);
    } else {
        hipLaunchKernelGGL(exact_gather_table_kernel<false>, dim3(scan_blocks(a, 1)), dim3(EXACT_THREADS), 0, stream,
                           a);
    }
    return hipGetLastError();
}

}  // namespace acamd
