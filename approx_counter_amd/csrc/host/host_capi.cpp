// host_capi.cpp -- C ABI over the host stages (include/approx_counter_host.h).
#include "approx_counter_host.h"

#include <algorithm>

#include "host_stages.h"

using namespace achost;

extern "C" {

float ach_complexity(uint64_t kmer, uint32_t k) { return get_complexity(kmer, k); }

float ach_adjust_threshold(float c_old, uint32_t k_old, uint32_t k_new) {
    return adjust_threshold(c_old, k_old, k_new);
}

int ach_count_kmers(const uint8_t* bases, const uint64_t* off, const uint32_t* len, uint32_t n, uint32_t k,
                    float threshold, const uint64_t* forbidden, uint32_t n_forbidden, uint64_t* out_kmers,
                    uint64_t* out_counts, uint64_t cap, uint64_t* n_out, uint64_t* had_n) {
    if (k < 2 || k > 32 || (n && (!bases || !off || !len)) || (cap && (!out_kmers || !out_counts))) return 1;
    SeqSet s;
    for (uint32_t i = 0; i < n; ++i) s.add(bases + off[i], len[i]);
    kmer_set fb;
    for (uint32_t i = 0; i < n_forbidden; ++i) fb.insert(forbidden[i]);
    uint64_t hn = 0;
    const pair_vector r = count_kmers(s, k, threshold, fb, &hn);
    for (uint64_t i = 0; i < std::min<uint64_t>(cap, r.size()); ++i) {
        out_kmers[i] = r[i].first;
        out_counts[i] = r[i].second;
    }
    if (n_out) *n_out = r.size();
    if (had_n) *had_n = hn;
    return 0;
}

uint64_t ach_rank(const uint64_t* kmers, const uint64_t* counts, uint64_t n, uint64_t limit, uint64_t solid,
                  uint32_t k, uint64_t* out_kmers, uint64_t* out_counts) {
    pair_vector v(n);
    for (uint64_t i = 0; i < n; ++i) v[i] = {kmers[i], counts[i]};
    const pair_vector r = solid ? get_solid_kmers(std::move(v), solid, k) : get_most_frequent(std::move(v), limit, k);
    const uint64_t m = std::min<uint64_t>(r.size(), limit);
    for (uint64_t i = 0; i < m; ++i) {
        out_kmers[i] = r[i].first;
        out_counts[i] = r[i].second;
    }
    return m;
}

}  // extern "C"
