/*
 * ac_oracle.h -- CPU restatement of the approximate-count stage of
 * qbonenfant/approx_counter (`errorCount`, approx_counter.cpp:531-601).
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is part of the product:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / CPU baseline.
 *
 * PARITY UNPINNED: the reference has no tests, no fixtures and cannot be
 * built here (SeqAn 2.4.0+ headers are absent).  The counting
 * contract is model M1:
 *     count(kmer) = sum over windows w of max(0, 3 - d(kmer, w))
 * with d the semi-global Levenshtein distance of the whole k-mer against the
 * best substring of w (empty substring included), text 'N' (code 4) never
 * matching.  Three independent restatements are provided:
 *   - oracle_count_dp      : plain O(k*L) dynamic programming (Sellers 1980);
 *   - oracle_count_myers   : Myers (1999) bit-vector, OpenMP over candidates
 *                            like the reference's omp for (567) -- this is the
 *                            timed CPU baseline ("port");
 *   - oracle_count_scheme  : a literal simulation of SeqAn 2.4's
 *                            find<0,2>(..., EditDistance()) optimal search
 *                            schemes (approx_counter.cpp:586) over explicit
 *                            occurrence sets, reporting per error level into
 *                            three per-window bitfields exactly like the
 *                            delegate at approx_counter.cpp:556-565 and the
 *                            sum at 590-593.  `strict` switches on the
 *                            SeqAn3-style end-indel pruning (residual risk).
 */
#ifndef AC_ORACLE_H
#define AC_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* Windows are given as Dna5 ordinal bytes (A0 C1 G2 T3 N4), window i being
 * bases[offset[i] .. offset[i]+length[i]).  K-mers use the reference's
 * dna2int layout (approx_counter.cpp:55-62): first base in the most
 * significant used bits, 2 bits per base. */

/* d(kmer, window) capped at `cap`, by DP. */
int oracle_distance_dp(uint64_t kmer, uint32_t k, const uint8_t* text,
                       uint32_t n, int cap);

int oracle_count_dp(uint32_t k, const uint64_t* kmers, uint32_t n_kmers,
                    const uint8_t* bases, const uint64_t* offset,
                    const uint32_t* length, uint32_t n_windows,
                    uint64_t* counts);

int oracle_count_myers(uint32_t k, const uint64_t* kmers, uint32_t n_kmers,
                       const uint8_t* bases, const uint64_t* offset,
                       const uint32_t* length, uint32_t n_windows,
                       uint64_t* counts, int n_threads);

/* levels (optional, may be NULL): n_kmers*n_windows bytes, bit e set when the
 * search reported a hit with e errors in that window (tcount[e][read]). */
int oracle_count_scheme(uint32_t k, const uint64_t* kmers, uint32_t n_kmers,
                        const uint8_t* bases, const uint64_t* offset,
                        const uint32_t* length, uint32_t n_windows,
                        uint64_t* counts, uint8_t* levels, int strict);

#ifdef __cplusplus
}
#endif
#endif
