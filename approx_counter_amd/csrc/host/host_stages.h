// host_stages.h -- host-side stages of the approximate counter (C++17, no SeqAn).
//
// These are the reference's CPU stages around the approximate-count hot path,
// restated for the drop-in CLI (adaptFinder) because SeqAn is not available
// (SURVEY.md §2, §8(c)).  Each function names the reference code it follows;
// all of them are product code (the oracle lives under oracle/).
#pragma once
#include <cstdint>
#include <random>
#include <set>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace achost {

using kmer_count = std::pair<uint64_t, uint64_t>;  // int_pair, approx_counter.cpp:35
using pair_vector = std::vector<kmer_count>;       // approx_counter.cpp:36
using kmer_set = std::set<uint64_t>;               // kmer_set_t, approx_counter.cpp:44
using arg_map = std::unordered_map<std::string, std::string>;  // approx_counter.cpp:42

// A set of Dna5 sequences: ordinal bytes (A0 C1 G2 T3, anything else 4) back to back.
struct SeqSet {
    std::vector<uint8_t> bases;
    std::vector<uint64_t> offset;  // sequence i = bases[offset[i], offset[i] + length[i])
    std::vector<uint32_t> length;
    size_t size() const { return length.size(); }
    const uint8_t* seq(size_t i) const { return bases.data() + offset[i]; }
    void add(const uint8_t* s, uint32_t n);
    void clear();
};

// SeqAn Dna5 ordinal of a character (A/a 0, C/c 1, G/g 2, T/t/U/u 3, else 4).
uint8_t dna5(char c);

// readRecords(ids, seqs, SeqFileIn) (approx_counter.cpp:819-825): FASTA or
// FASTQ chosen by the first record marker ('>' or '@').  Throws
// std::runtime_error when the file cannot be opened or is not FASTA/FASTQ.
void read_records(const std::string& path, std::vector<std::string>& ids, SeqSet& seqs);

// dna2int / int2dna (approx_counter.cpp:55-78): 2 bits per base, first base in
// the most significant used bits.
uint64_t dna2int(const uint8_t* s, uint32_t k);
std::string int2dna(uint64_t value, uint32_t k);

// adjust_threshold (approx_counter.cpp:183-186).
float adjust_threshold(float c_old, uint32_t k_old, uint32_t k_new);

// getComplexity / haveLowComplexity (approx_counter.cpp:214-267): DUST-like
// dimer score in IEEE single precision.
float get_complexity(uint64_t kmer, uint32_t k);
inline bool have_low_complexity(uint64_t kmer, uint32_t k, float threshold) {
    return get_complexity(kmer, k) >= threshold;
}

// CompareCount (approx_counter.cpp:275-305): count desc, complexity asc, value desc.
struct CompareCount {
    explicit CompareCount(uint32_t k) : k(k) {}
    bool operator()(const kmer_count& a, const kmer_count& b) const;
    uint32_t k;
};

// A window image in the C ABI's layout (ac_windows, include/approx_counter_amd.h):
// 2-bit codes + N bitmap, every window starting at a multiple of 32 bases.
struct PackedImage {
    std::vector<uint32_t> codes, nmask, length;
    std::vector<uint64_t> start;
    uint64_t n_bases = 32;
    size_t size() const { return length.size(); }
};

// ac_pack_windows over sequences [lo, hi) of a SeqSet.
PackedImage pack_sample(const SeqSet& s, size_t lo, size_t hi);

// The reads of a FASTA/FASTQ file kept as their sampling windows only
// (the reader packs on the fly, so no 1 B/base copy of
// the whole file is held).  For every record: its length; for every record
// sample_sequences could pick (length >= 2 cut), its first `cut` bases and its
// last cut + 1 bases, packed at 32-base-aligned offsets.
struct WindowStore {
    uint64_t cut = 0;
    uint64_t prefix_bases = 0, suffix_bases = 32;  // round-ups to 32 of cut and cut + 1
    uint64_t n_slots = 0;
    std::vector<uint32_t> length;        // every record, file order
    std::vector<uint32_t> slot;          // record -> stored window pair, ~0u if never sampled
    std::vector<uint32_t> codes, nmask;  // window pairs: prefix then suffix
    size_t size() const { return length.size(); }
};
// `threads` (0 = up to 16 hardware threads) parse large regular files in
// chunks; the result is identical to the sequential parse, which is used
// whenever the chunk boundaries cannot be confirmed.
void read_windows(const std::string& path, uint64_t cut, WindowStore& out, unsigned threads = 0);

// sample_sequences + pack_sample over a WindowStore built with the same cut:
// the same shuffle draws and picks, written straight into a window image
// (identical to pack_sample(sample_sequences(...)) word for word).
PackedImage sample_windows(const WindowStore& ws, uint64_t nb_sample, bool bot, std::mt19937& rng);

// sampleSequences (approx_counter.cpp:415-476): walks a shuffled permutation
// of the reads and keeps, for up to nb_sample reads of length >= 2*cut, the
// first `cut` bases (start) or the last cut+1 bases (end, `bot`).
SeqSet sample_sequences(const SeqSet& seqs, uint64_t nb_sample, uint64_t cut, bool bot, std::mt19937& rng);

// count_kmers (approx_counter.cpp:487-519): exact counts of the k-mers of the
// sample holding no N, passing the low-complexity filter and not forbidden.
// Returns the distinct k-mers with their counts (ascending k-mer order) and
// the number of k-mers skipped for holding an N.
pair_vector count_kmers(const SeqSet& sample, uint32_t k, float threshold, const kmer_set& forbidden,
                        uint64_t* had_n);

// get_most_frequent (approx_counter.cpp:396-405): the first `limit` entries
// in CompareCount order.
pair_vector get_most_frequent(pair_vector counts, uint64_t limit, uint32_t k);

// get_solid_kmers (approx_counter.cpp:372-388): entries with count >= solid.
// The reference sorts them by count only with an unstable std::sort, leaving
// tie order unspecified; CompareCount order is used here so output is
// deterministic.
pair_vector get_solid_kmers(pair_vector counts, uint64_t solid, uint32_t k);

// exportCounter (approx_counter.cpp:158-174): "KMER\tCOUNT\n" per entry.
bool export_counter(const pair_vector& v, uint32_t k, const std::string& path);

// parse_config (approx_counter.cpp:103-135).
arg_map parse_config(const std::string& path, bool* opened);

// parse_kmer_list (approx_counter.cpp:340-364): only pure-ACGT lines; an empty
// line encodes k-mer value 0.  Returns false if the file cannot be opened.
bool parse_kmer_list(const std::string& path, kmer_set& out);

}  // namespace achost
