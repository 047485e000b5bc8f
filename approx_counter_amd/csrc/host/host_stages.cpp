// host_stages.cpp -- see host_stages.h.  Product code for the CLI's CPU stages.
#include "host_stages.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <numeric>
#include <stdexcept>
#include <thread>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

namespace achost {

void SeqSet::add(const uint8_t* s, uint32_t n) {
    offset.push_back(bases.size());
    length.push_back(n);
    bases.insert(bases.end(), s, s + n);
}

void SeqSet::clear() {
    bases.clear();
    offset.clear();
    length.clear();
}

uint8_t dna5(char c) {
    switch (c) {
        case 'A': case 'a': return 0;
        case 'C': case 'c': return 1;
        case 'G': case 'g': return 2;
        case 'T': case 't': case 'U': case 'u': return 3;
        default: return 4;
    }
}

namespace {

// Streaming line reader that copes with '\r\n' and a missing final newline.
struct LineReader {
    std::FILE* f;
    std::vector<char> buf = std::vector<char>(1 << 20);
    size_t pos = 0, end = 0;
    bool eof = false;
    bool get(std::string& line) {
        line.clear();
        for (;;) {
            if (pos == end) {
                if (eof) return !line.empty();
                end = std::fread(buf.data(), 1, buf.size(), f);
                pos = 0;
                if (end == 0) {
                    eof = true;
                    return !line.empty();
                }
            }
            const char* s = buf.data() + pos;
            const char* nl = static_cast<const char*>(std::memchr(s, '\n', end - pos));
            if (nl) {
                line.append(s, nl - s);
                pos += (nl - s) + 1;
                if (!line.empty() && line.back() == '\r') line.pop_back();
                return true;
            }
            line.append(s, end - pos);
            pos = end;
        }
    }
};

// dna5() as a table; 0xff marks the blanks SeqAn skips inside sequence lines.
struct Dna5Table {
    uint8_t v[256];
    Dna5Table() {
        for (int c = 0; c < 256; ++c) v[c] = dna5((char)c);
        v[(unsigned char)' '] = v[(unsigned char)'\t'] = v[(unsigned char)'\r'] = 0xff;
    }
};
const Dna5Table DNA5_TABLE;

void append_bases(std::vector<uint8_t>& out, const std::string& line) {
    const size_t n0 = out.size();
    out.resize(n0 + line.size());
    uint8_t* o = out.data() + n0;
    for (char c : line) {
        const uint8_t v = DNA5_TABLE.v[(unsigned char)c];
        *o = v;
        o += v != 0xff;
    }
    out.resize((size_t)(o - out.data()));
}

}  // namespace

namespace {

constexpr uint64_t NO_STOP = ~0ull;

// Line source over a memory range [base + begin, base + end) (an mmap'd file):
// the same lines as LineReader, plus the file offset of the last line read.
struct MemLines {
    const char* base;
    const char* p;
    const char* end;
    uint64_t start = 0;  // offset of the last line returned
    bool get(std::string& line) {
        if (p >= end) return false;
        start = (uint64_t)(p - base);
        const char* nl = static_cast<const char*>(std::memchr(p, '\n', (size_t)(end - p)));
        const char* e = nl ? nl : end;
        line.assign(p, (size_t)(e - p));
        if (!line.empty() && line.back() == '\r') line.pop_back();
        p = nl ? nl + 1 : end;
        return true;
    }
    uint64_t last_start() const { return start; }
};

struct FileLines {  // non-mappable inputs (pipes): offsets are not tracked
    LineReader r;
    bool get(std::string& line) { return r.get(line); }
    uint64_t last_start() const { return 0; }
};

// Record loop of readRecords from `line`, a record-start line just read: FASTA
// ('>') or FASTQ ('@'); calls emit(id, dna5 bases, n) per record in order.
// Stops before the first record whose start line lies at offset >= stop and
// returns that offset (NO_STOP at the end of the input).
template <typename Lines, typename Emit>
uint64_t parse_records(Lines& r, std::string& line, Emit&& emit, uint64_t stop, const std::string& path) {
    std::vector<uint8_t> cur;
    if (line[0] == '>') {
        std::string id = line.substr(1);
        for (;;) {
            const bool more = r.get(line);
            if (!more || (!line.empty() && line[0] == '>')) {
                emit(id, cur.data(), cur.size());
                cur.clear();
                if (!more) return NO_STOP;
                if (r.last_start() >= stop) return r.last_start();
                id = line.substr(1);
                continue;
            }
            append_bases(cur, line);
        }
    }
    if (line[0] != '@') throw std::runtime_error("Unknown sequence file format (expected FASTA or FASTQ): " + path);
    for (;;) {
        if (line.empty()) {
            if (!r.get(line)) return NO_STOP;
            continue;
        }
        if (r.last_start() >= stop) return r.last_start();
        if (line[0] != '@') throw std::runtime_error("Malformed FASTQ record in " + path);
        const std::string id = line.substr(1);
        cur.clear();
        // sequence lines until the '+' separator
        bool ok = false;
        while (r.get(line)) {
            if (!line.empty() && line[0] == '+') {
                ok = true;
                break;
            }
            append_bases(cur, line);
        }
        if (!ok) throw std::runtime_error("Truncated FASTQ record in " + path);
        // quality lines: as many characters as the sequence holds
        size_t q = 0;
        while (q < cur.size() && r.get(line)) q += line.size();
        emit(id, cur.data(), cur.size());
        if (!r.get(line)) return NO_STOP;
    }
}

// First record-start line of a source: leading empty lines skipped.  False for an empty input.
template <typename Lines>
bool first_record_line(Lines& r, std::string& line) {
    bool have = false;
    while ((have = r.get(line)) && line.empty()) {
    }
    return have;
}

// Read-only mapping of a regular file (empty or unmappable: data == nullptr).
struct Mapped {
    const char* data = nullptr;
    size_t size = 0;
    int fd = -1;
    explicit Mapped(const std::string& path) {
        fd = ::open(path.c_str(), O_RDONLY);
        if (fd < 0) return;
        struct stat st;
        if (::fstat(fd, &st) != 0 || !S_ISREG(st.st_mode) || st.st_size == 0) return;
        void* m = ::mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
        if (m == MAP_FAILED) return;
        data = static_cast<const char*>(m);
        size = (size_t)st.st_size;
    }
    ~Mapped() {
        if (data) ::munmap(const_cast<char*>(data), size);
        if (fd >= 0) ::close(fd);
    }
    Mapped(const Mapped&) = delete;
    Mapped& operator=(const Mapped&) = delete;
};

// Sequential parse with buffered reads (faster than faulting in a mapping
// page by page on one thread; also reads pipes).
template <typename Emit>
void for_each_record(const std::string& path, Emit&& emit) {
    std::string line;
    std::FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) throw std::runtime_error("Could not open input file: " + path);
    FileLines r{LineReader{f}};
    try {
        if (first_record_line(r, line)) parse_records(r, line, emit, NO_STOP, path);
    } catch (...) {
        std::fclose(f);
        throw;
    }
    std::fclose(f);
}

// Offset of the first plausible record start at or after `from`: a line
// starting with '>' (FASTA) or, for FASTQ, a line starting with '@' whose
// next-but-one line starts with '+' and whose sequence and quality lines have
// equal lengths.  A wrong guess (a quality line starting with '@') is caught
// by the boundary check of read_windows.  Returns size if there is none.
size_t next_record_start(const char* d, size_t size, size_t from, char marker) {
    size_t p = from;
    if (p > 0) {  // move to the start of the next line
        const char* nl = static_cast<const char*>(std::memchr(d + p - 1, '\n', size - (p - 1)));
        if (!nl) return size;
        p = (size_t)(nl + 1 - d);
    }
    while (p < size) {
        if (d[p] == marker) {
            if (marker == '>') return p;
            MemLines r{d, d + p, d + size};
            std::string l0, l1, l2, l3;
            if (r.get(l0) && r.get(l1) && r.get(l2) && r.get(l3) && !l2.empty() && l2[0] == '+' &&
                l1.size() == l3.size())
                return p;
        }
        const char* nl = static_cast<const char*>(std::memchr(d + p, '\n', size - p));
        if (!nl) return size;
        p = (size_t)(nl + 1 - d);
    }
    return size;
}

}  // namespace

void read_records(const std::string& path, std::vector<std::string>& ids, SeqSet& seqs) {
    for_each_record(path, [&](const std::string& id, const uint8_t* b, size_t n) {
        ids.push_back(id);
        seqs.add(b, (uint32_t)n);
    });
}

namespace {

uint64_t round32(uint64_t n) { return (n + 31) / 32 * 32; }

// Packs n Dna5 bases at image base `pos` (a multiple of 32) of codes/nmask,
// which hold zeros there (ac_pack_windows's layout).
void pack_into(uint32_t* codes, uint32_t* nmask, uint64_t pos, const uint8_t* src, uint64_t n) {
    for (uint64_t j = 0; j < n; ++j) {
        const uint64_t b = pos + j;
        const uint8_t v = src[j];
        if (v < 4) codes[b >> 4] |= (uint32_t)v << (2 * (b & 15));
        else nmask[b >> 5] |= 1u << (b & 31);
    }
}

}  // namespace

namespace {

// Keeps a record's length and, if sample_sequences could pick it, its packed windows.
struct WindowPacker {
    WindowStore& ws;
    void operator()(const std::string&, const uint8_t* b, size_t n) {
        const uint64_t cut = ws.cut, pair = ws.prefix_bases + ws.suffix_bases;
        ws.length.push_back((uint32_t)n);
        if (n < 2 * cut) {  // never sampled (sample_sequences)
            ws.slot.push_back(~0u);
            return;
        }
        const uint64_t j = ws.n_slots++;
        ws.slot.push_back((uint32_t)j);
        ws.codes.resize((j + 1) * pair / 16, 0u);
        ws.nmask.resize((j + 1) * pair / 32, 0u);
        pack_into(ws.codes.data(), ws.nmask.data(), j * pair, b, cut);
        if (n >= cut + 1)
            pack_into(ws.codes.data(), ws.nmask.data(), j * pair + ws.prefix_bases, b + (n - 1 - cut), cut + 1);
    }
};

WindowStore empty_store(uint64_t cut) {
    WindowStore ws;
    ws.cut = cut;
    ws.prefix_bases = round32(cut);
    ws.suffix_bases = round32(cut + 1);
    return ws;
}

// Chunked parse of a mapped file: chunk t starts at a plausible record start
// A_t and stops before the first record starting at or after A_{t+1}.  The
// result is taken only if every chunk stopped exactly at the next chunk's start
// (then, by induction from the file start, every A_t is a true record boundary
// of the sequential parse and the fragments are its pieces); false otherwise.
bool read_windows_chunked(const Mapped& m, const std::string& path, uint64_t cut, unsigned threads,
                          WindowStore& ws) {
    const char* d = m.data;
    MemLines head{d, d, d + m.size};
    std::string line;
    if (!first_record_line(head, line) || (line[0] != '>' && line[0] != '@')) return false;
    const char marker = line[0];
    std::vector<size_t> at{(size_t)head.last_start()};
    for (unsigned t = 1; t < threads; ++t) {
        const size_t a = next_record_start(d, m.size, std::max(m.size / threads * t, at.back() + 1), marker);
        if (a >= m.size) break;
        at.push_back(a);
    }
    const size_t n = at.size();
    std::vector<WindowStore> part(n, empty_store(cut));
    std::vector<uint64_t> stopped(n, NO_STOP);
    std::vector<char> ok(n, 1);
    std::vector<std::thread> pool;
    for (size_t t = 0; t < n; ++t)
        pool.emplace_back([&, t] {
            try {
                MemLines r{d, d + at[t], d + m.size};
                std::string l;
                if (!r.get(l)) return;
                WindowPacker pk{part[t]};
                stopped[t] = parse_records(r, l, pk, t + 1 < n ? (uint64_t)at[t + 1] : NO_STOP, path);
            } catch (...) {
                ok[t] = 0;
            }
        });
    for (auto& th : pool) th.join();
    for (size_t t = 0; t < n; ++t)
        if (!ok[t] || stopped[t] != (t + 1 < n ? (uint64_t)at[t + 1] : NO_STOP)) return false;
    ws = empty_store(cut);
    size_t recs = 0, words = 0, masks = 0;
    for (const auto& f : part) {
        recs += f.size();
        words += f.codes.size();
        masks += f.nmask.size();
    }
    ws.length.reserve(recs);
    ws.slot.reserve(recs);
    ws.codes.reserve(words);
    ws.nmask.reserve(masks);
    for (const auto& f : part) {
        ws.length.insert(ws.length.end(), f.length.begin(), f.length.end());
        for (uint32_t sl : f.slot) ws.slot.push_back(sl == ~0u ? ~0u : sl + (uint32_t)ws.n_slots);
        ws.codes.insert(ws.codes.end(), f.codes.begin(), f.codes.end());
        ws.nmask.insert(ws.nmask.end(), f.nmask.begin(), f.nmask.end());
        ws.n_slots += f.n_slots;
    }
    return true;
}

}  // namespace

void read_windows(const std::string& path, uint64_t cut, WindowStore& ws, unsigned threads) {
    if (threads == 0) {
        const char* env = std::getenv("AC_READ_THREADS");  // override, e.g. 1 for the sequential reader
        threads = env ? (unsigned)std::strtoul(env, nullptr, 10)
                      : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    }
    {
        Mapped m(path);
        // below ~8 MB per thread the threads cost more than they save (AC_READ_MIN_CHUNK overrides, for tests)
        const char* mc = std::getenv("AC_READ_MIN_CHUNK");
        const size_t min_chunk = std::max<size_t>(1, mc ? (size_t)std::strtoull(mc, nullptr, 10) : (8u << 20));
        const unsigned t = (unsigned)std::min<size_t>(threads, m.size / min_chunk);
        const bool debug = std::getenv("AC_READ_DEBUG") != nullptr;
        if (m.data && t > 1) {
            if (read_windows_chunked(m, path, cut, t, ws)) {
                if (debug) std::fprintf(stderr, "[reader] chunked parse, %u threads\n", t);
                return;
            }
            if (debug) std::fprintf(stderr, "[reader] chunk boundaries not confirmed: sequential parse\n");
        }
    }
    ws = empty_store(cut);
    for_each_record(path, WindowPacker{ws});
}

PackedImage sample_windows(const WindowStore& ws, uint64_t nb_sample, bool bot, std::mt19937& rng) {
    std::vector<int> vec(ws.size());
    std::iota(vec.begin(), vec.end(), 0);
    std::shuffle(vec.begin(), vec.end(), rng);  // the same draws as sample_sequences
    const uint64_t pair = ws.prefix_bases + ws.suffix_bases;
    const uint64_t wbases = bot ? ws.suffix_bases : ws.prefix_bases;
    const uint64_t off = bot ? ws.prefix_bases : 0;
    const uint32_t wlen = (uint32_t)(bot ? ws.cut + 1 : ws.cut);
    std::vector<uint32_t> picked;
    for (size_t i = 0; picked.size() < nb_sample && i < vec.size(); ++i) {
        const size_t id = (size_t)vec[i];
        if (ws.slot[id] != ~0u && (!bot || ws.length[id] >= ws.cut + 1)) picked.push_back(ws.slot[id]);
    }
    PackedImage p;
    p.n_bases = std::max<uint64_t>(32, wbases * picked.size());
    p.codes.assign(p.n_bases / 16, 0u);
    p.nmask.assign(p.n_bases / 32, 0u);
    p.start.resize(picked.size());
    p.length.assign(picked.size(), wlen);
    for (size_t i = 0; i < picked.size(); ++i) {
        const uint64_t src = (uint64_t)picked[i] * pair + off, dst = (uint64_t)i * wbases;
        p.start[i] = dst;
        std::memcpy(&p.codes[dst / 16], &ws.codes[src / 16], wbases / 16 * sizeof(uint32_t));
        std::memcpy(&p.nmask[dst / 32], &ws.nmask[src / 32], wbases / 32 * sizeof(uint32_t));
    }
    return p;
}

PackedImage pack_sample(const SeqSet& s, size_t lo, size_t hi) {
    PackedImage p;
    uint64_t total = 0;
    for (size_t i = lo; i < hi; ++i) total += round32(s.length[i]);
    p.n_bases = std::max<uint64_t>(32, total);
    p.codes.assign(p.n_bases / 16, 0u);
    p.nmask.assign(p.n_bases / 32, 0u);
    p.start.resize(hi - lo);
    p.length.resize(hi - lo);
    uint64_t pos = 0;
    for (size_t i = lo; i < hi; ++i) {
        p.start[i - lo] = pos;
        p.length[i - lo] = s.length[i];
        pack_into(p.codes.data(), p.nmask.data(), pos, s.seq(i), s.length[i]);
        pos += round32(s.length[i]);
    }
    return p;
}

uint64_t dna2int(const uint8_t* s, uint32_t k) {
    uint64_t v = 0;
    for (uint32_t i = 0; i < k; ++i) v = (v << 2) | s[i];
    return v;
}

std::string int2dna(uint64_t value, uint32_t k) {
    static const char DNA[] = "ACGT";
    std::string s(k, 'A');
    for (uint32_t i = 0; i < k; ++i) {
        s[k - 1 - i] = DNA[value & 3u];
        value >>= 2;
    }
    return s;
}

float adjust_threshold(float c_old, uint32_t k_old, uint32_t k_new) {
    // float(pow(k_new - 1, 2) / pow(k_old - 1, 2)) in double, then a float product.
    const double ratio = ((double)k_new - 2 + 1) * ((double)k_new - 2 + 1) /
                         (((double)k_old - 2 + 1) * ((double)k_old - 2 + 1));
    return c_old * (float)ratio;
}

float get_complexity(uint64_t kmer, uint32_t k) {
    uint64_t counts[16] = {0};
    for (uint32_t i = 0; i + 1 < k; ++i) {
        counts[kmer & 15u]++;
        kmer >>= 2;
    }
    size_t sum = 0;
    for (uint64_t v : counts) sum += v * (v - 1);
    return (float)sum / float(2 * ((int)k - 2));
}

bool CompareCount::operator()(const kmer_count& a, const kmer_count& b) const {
    if (a.second == b.second) {
        const float ac = get_complexity(a.first, k), bc = get_complexity(b.first, k);
        if (ac == bc) return a.first > b.first;
        return ac < bc;
    }
    return a.second > b.second;
}

SeqSet sample_sequences(const SeqSet& seqs, uint64_t nb_sample, uint64_t cut, bool bot, std::mt19937& rng) {
    SeqSet sample;
    std::vector<int> vec(seqs.size());
    std::iota(vec.begin(), vec.end(), 0);
    std::shuffle(vec.begin(), vec.end(), rng);
    uint64_t nb_seq = 0;
    for (size_t i = 0; nb_seq < nb_sample && i < vec.size(); ++i) {
        const size_t id = (size_t)vec[i];
        const uint64_t len = seqs.length[id];
        const uint64_t cur_cut = std::min<uint64_t>(len, cut);
        if (len >= cut * 2 && (!bot || len >= cur_cut + 1)) {  // (an empty read has no end window at cut 0)
            if (bot) {
                const uint64_t from = len - 1 - cur_cut;  // suffix(seq, len - 1 - cut): cut + 1 bases
                sample.add(seqs.seq(id) + from, (uint32_t)(len - from));
            } else {
                sample.add(seqs.seq(id), (uint32_t)cur_cut);
            }
            ++nb_seq;
        }
    }
    return sample;
}

namespace {

// LSD radix sort of 2k-bit keys, 11 bits per pass.
void radix_sort(std::vector<uint64_t>& a, uint32_t bits) {
    std::vector<uint64_t> tmp(a.size());
    constexpr uint32_t R = 11, B = 1u << R;
    std::vector<size_t> cnt(B);
    for (uint32_t sh = 0; sh < bits; sh += R) {
        std::fill(cnt.begin(), cnt.end(), 0);
        for (uint64_t v : a) cnt[(v >> sh) & (B - 1)]++;
        size_t s = 0;
        for (auto& c : cnt) {
            const size_t t = c;
            c = s;
            s += t;
        }
        for (uint64_t v : a) tmp[cnt[(v >> sh) & (B - 1)]++] = v;
        a.swap(tmp);
    }
}

}  // namespace

pair_vector count_kmers(const SeqSet& sample, uint32_t k, float threshold, const kmer_set& forbidden,
                        uint64_t* had_n) {
    std::vector<uint64_t> vals;
    size_t total = 0;
    for (size_t i = 0; i < sample.size(); ++i)
        if (sample.length[i] >= k) total += sample.length[i] - k + 1;
    vals.reserve(total);
    const uint64_t mask = k == 32 ? ~0ull : ((1ull << (2 * k)) - 1);
    uint64_t n_skipped = 0;
    for (size_t i = 0; i < sample.size(); ++i) {
        const uint8_t* s = sample.seq(i);
        const uint32_t len = sample.length[i];
        if (len < k) continue;
        uint64_t v = 0;
        uint32_t run = 0;  // bases since the last N
        for (uint32_t j = 0; j < len; ++j) {
            if (s[j] >= 4) {
                run = 0;
                v = 0;
            } else {
                v = ((v << 2) | s[j]) & mask;
                ++run;
            }
            if (j + 1 >= k) {
                if (run >= k) vals.push_back(v);
                else ++n_skipped;
            }
        }
    }
    if (had_n) *had_n = n_skipped;
    radix_sort(vals, 2 * k);
    pair_vector out;
    for (size_t i = 0; i < vals.size();) {
        size_t j = i + 1;
        while (j < vals.size() && vals[j] == vals[i]) ++j;
        const uint64_t km = vals[i];
        if (!have_low_complexity(km, k, threshold) && forbidden.find(km) == forbidden.end())
            out.emplace_back(km, (uint64_t)(j - i));
        i = j;
    }
    return out;
}

pair_vector get_most_frequent(pair_vector counts, uint64_t limit, uint32_t k) {
    // CompareCount is a strict total order (the k-mer value breaks every tie),
    // so a partial sort gives exactly the first `limit` entries of the full sort.
    struct Keyed {
        uint64_t count, kmer;
        float comp;
    };
    std::vector<Keyed> v(counts.size());
    for (size_t i = 0; i < counts.size(); ++i)
        v[i] = {counts[i].second, counts[i].first, get_complexity(counts[i].first, k)};
    auto less = [](const Keyed& a, const Keyed& b) {
        if (a.count != b.count) return a.count > b.count;
        if (a.comp != b.comp) return a.comp < b.comp;
        return a.kmer > b.kmer;
    };
    const size_t n = std::min<uint64_t>(limit, v.size());
    std::partial_sort(v.begin(), v.begin() + n, v.end(), less);
    pair_vector out(n);
    for (size_t i = 0; i < n; ++i) out[i] = {v[i].kmer, v[i].count};
    return out;
}

pair_vector get_solid_kmers(pair_vector counts, uint64_t solid, uint32_t k) {
    pair_vector kept;
    for (const auto& kv : counts)
        if (kv.second >= solid) kept.push_back(kv);
    return get_most_frequent(std::move(kept), ~0ull, k);
}

bool export_counter(const pair_vector& v, uint32_t k, const std::string& path) {
    std::FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) {
        std::fprintf(stderr, "/!\\ ERROR: COULD NOT OPEN FILE %s\n", path.c_str());
        return false;
    }
    std::string line;
    for (const auto& kv : v) {
        line = int2dna(kv.first, k);
        line += '\t';
        line += std::to_string(kv.second);
        line += '\n';
        std::fwrite(line.data(), 1, line.size(), f);
    }
    std::fclose(f);
    return true;
}

arg_map parse_config(const std::string& path, bool* opened) {
    arg_map params;
    std::ifstream in(path);
    if (opened) *opened = in.is_open();
    if (!in.is_open()) return params;
    std::string line;
    while (std::getline(in, line)) {
        if (!line.empty() && line[0] == '#') continue;
        std::string arg, val;
        bool sep = false;
        for (char c : line) {
            if (c == '=') sep = true;
            else if (c != ' ') (sep ? val : arg) += c;
        }
        params[arg] = val;
    }
    return params;
}

bool parse_kmer_list(const std::string& path, kmer_set& out) {
    std::ifstream in(path);
    if (!in.is_open()) return false;
    std::string line;
    while (std::getline(in, line)) {
        uint64_t v = 0;
        bool ok = true;
        for (char c : line) {
            const uint8_t b = dna5(c);
            if (b >= 4) {
                ok = false;
                break;
            }
            v = (v << 2) | b;
        }
        if (ok) out.insert(v);
    }
    return true;
}

}  // namespace achost
