/*
 * approx_counter_host.h -- C ABI of the host stages of the drop-in CLI
 * (libac_host.so).  These are the reference's CPU stages around the hot path
 * (approx_counter.cpp:183-405, 487-519), exported so tests can check them
 * against the oracle's restatement; the CLI (bin/adaptFinder) links the same
 * code.  Not part of the GPU boundary (include/approx_counter_amd.h).
 */
#ifndef APPROX_COUNTER_HOST_H
#define APPROX_COUNTER_HOST_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* getComplexity (approx_counter.cpp:247-267) */
float ach_complexity(uint64_t kmer, uint32_t k);
/* adjust_threshold (approx_counter.cpp:183-186) */
float ach_adjust_threshold(float c_old, uint32_t k_old, uint32_t k_new);

/*
 * count_kmers (approx_counter.cpp:487-519) over Dna5 windows
 * (bases[off[i] .. off[i]+len[i]), ordinals 0..3 ACGT, >= 4 N).  Writes up to
 * `cap` distinct (kmer, count) pairs in ascending k-mer order; *n_out is the
 * number of distinct k-mers (may exceed cap), *had_n the k-mers skipped for
 * holding an N.  Returns 0, or 1 on a bad argument.
 */
int ach_count_kmers(const uint8_t* bases, const uint64_t* off, const uint32_t* len, uint32_t n, uint32_t k,
                    float threshold, const uint64_t* forbidden, uint32_t n_forbidden, uint64_t* out_kmers,
                    uint64_t* out_counts, uint64_t cap, uint64_t* n_out, uint64_t* had_n);

/*
 * get_most_frequent (approx_counter.cpp:396-405) / get_solid_kmers (372-388):
 * ranks (kmers[i], counts[i]) by CompareCount and writes the first
 * min(limit, kept) into out_kmers/out_counts; solid > 0 keeps only counts >=
 * solid.  Returns the number written.
 */
uint64_t ach_rank(const uint64_t* kmers, const uint64_t* counts, uint64_t n, uint64_t limit, uint64_t solid,
                  uint32_t k, uint64_t* out_kmers, uint64_t* out_counts);

#ifdef __cplusplus
}
#endif
#endif
