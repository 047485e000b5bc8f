// host_pack.cpp -- worker pool and Dna5 packer of the host-buffer stage (host_pack.h).
#include "host_pack.h"

#include <immintrin.h>
#include <sched.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>

#include <pthread.h>

namespace acamd {

namespace {

inline void cpu_relax() { _mm_pause(); }

int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

}  // namespace

WorkPool::WorkPool(unsigned n_threads, const std::vector<int>& cpus, bool pin_each) {
    const char* s = std::getenv("AC_HOST_SPIN_US");
    spin_ns_ = (s ? std::atoll(s) : 2000) * 1000;  // 2 ms: consecutive calls find the workers spinning
    cpu_set_t all;
    CPU_ZERO(&all);
    for (int c : cpus) CPU_SET(c, &all);
    for (unsigned i = 1; i < std::max(1u, n_threads); ++i) {
        threads_.emplace_back([this] { worker(); });
        if (cpus.empty()) continue;
        cpu_set_t one;
        CPU_ZERO(&one);
        CPU_SET(cpus[(i - 1) % cpus.size()], &one);
        (void)pthread_setaffinity_np(threads_.back().native_handle(), sizeof(cpu_set_t), pin_each ? &one : &all);
    }
}

WorkPool::~WorkPool() {
    {
        std::lock_guard<std::mutex> lk(m_);
        stop_.store(true);
    }
    cv_.notify_all();
    for (auto& t : threads_) t.join();
}

void WorkPool::drain(uint32_t gen, uint32_t upto, uint32_t max_tasks) {
    const Job& job = jobs_[gen & 1u];
    for (uint32_t ran = 0; ran < max_tasks;) {
        uint64_t s = state_.load(std::memory_order_acquire);
        if ((uint32_t)(s >> 32) != gen) return;  // the job is over (a later one is published)
        const uint32_t i = (uint32_t)s;
        const std::function<void(uint32_t)>* fn = job.fn.load(std::memory_order_relaxed);
        const uint32_t n = job.n.load(std::memory_order_relaxed);
        if (i >= n || i >= upto) return;
        if (!state_.compare_exchange_weak(s, s + 1, std::memory_order_acq_rel, std::memory_order_relaxed)) continue;
        (*fn)(i);
        jobs_[gen & 1u].done.fetch_add(1, std::memory_order_release);
        ++ran;
    }
}

void WorkPool::worker() {
    uint32_t seen = 0;
    for (;;) {
        // Wait for the next job: spin for spin_ns_, then sleep.  pub_ changes
        // under m_, so a sleeper cannot miss it.
        const int64_t t0 = now_ns();
        uint32_t polls = 0;
        while (pub_.load(std::memory_order_acquire) == seen && !stop_.load(std::memory_order_relaxed)) {
            cpu_relax();
            if ((++polls & 255u) == 0 && now_ns() - t0 > spin_ns_) {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return pub_.load(std::memory_order_relaxed) != seen || stop_.load(); });
            }
        }
        if (stop_.load()) return;
        seen = pub_.load(std::memory_order_acquire);
        drain(seen);
    }
}

void WorkPool::run(uint32_t n, const std::function<void(uint32_t)>& fn) {
    begin(n, fn);
    finish();
}

void WorkPool::begin(uint32_t n, const std::function<void(uint32_t)>& fn) {
    // (a plain lock, not a member unique_lock: unique_lock::unlock() releases the mutex before it
    // clears its owns flag, so the next caller's move-assignment could see the flag still set)
    run_m_.lock();
    n_ = n;
    serial_ = threads_.empty() || n <= 1;
    if (serial_) {
        serial_fn_ = &fn;
        serial_next_ = 0;
        return;
    }
    const uint32_t g = ++gen_;
    Job& job = jobs_[g & 1u];  // its previous job (g - 2) finished before run(g - 1) started
    job.fn.store(&fn, std::memory_order_relaxed);
    job.n.store(n, std::memory_order_relaxed);
    job.done.store(0, std::memory_order_relaxed);
    state_.store((uint64_t)g << 32, std::memory_order_release);
    {
        std::lock_guard<std::mutex> l2(m_);
        pub_.store(g, std::memory_order_release);
    }
    cv_.notify_all();
}

void WorkPool::help(uint32_t upto) {
    if (serial_) {
        for (; serial_next_ < std::min(upto, n_); ++serial_next_) (*serial_fn_)(serial_next_);
        return;
    }
    drain(gen_, upto);
}

void WorkPool::help_one() {
    if (serial_) {
        if (serial_next_ < n_) (*serial_fn_)(serial_next_++);
        return;
    }
    drain(gen_, ~0u, 1);
}

void WorkPool::finish() {
    if (serial_) {
        help(n_);
    } else {
        drain(gen_);
        while (jobs_[gen_ & 1u].done.load(std::memory_order_acquire) < n_) cpu_relax();
    }
    run_m_.unlock();
}

namespace {
std::mutex g_plan_m;
HostPlan g_plan;
bool g_plan_set = false;
bool g_pool_made = false;
}  // namespace

bool set_host_plan(const HostPlan& plan) {
    std::lock_guard<std::mutex> lk(g_plan_m);
    if (g_pool_made || g_plan_set) return false;
    g_plan = plan;
    g_plan_set = true;
    return true;
}

HostPlan host_plan() {
    std::lock_guard<std::mutex> lk(g_plan_m);
    return g_plan;
}

std::vector<int> read_cpulist(const char* path) {
    FILE* f = std::fopen(path, "r");
    if (!f) return {};
    char buf[4096];
    const size_t n = std::fread(buf, 1, sizeof buf - 1, f);
    std::fclose(f);
    buf[n] = 0;
    return parse_cpulist(buf);
}

std::vector<int> parse_cpulist(const char* text) {
    std::vector<int> out;
    for (const char* p = text; *p;) {
        char* e;
        const long a = std::strtol(p, &e, 10);
        if (e == p) break;
        long b = a;
        p = e;
        if (*p == '-') {
            b = std::strtol(p + 1, &e, 10);
            p = e;
        }
        for (long c = a; c <= b && c < CPU_SETSIZE; ++c) out.push_back((int)c);
        if (*p == ',') ++p;
        else break;
    }
    std::sort(out.begin(), out.end());
    out.erase(std::unique(out.begin(), out.end()), out.end());
    return out;
}

int sysfs_core_of(int cpu) {
    // the first CPU of its SMT sibling set stands for the physical core
    const std::string path = "/sys/devices/system/cpu/cpu" + std::to_string(cpu) + "/topology/thread_siblings_list";
    const std::vector<int> sib = read_cpulist(path.c_str());
    return sib.empty() ? cpu : sib.front();
}

std::vector<int> plan_host_cpus(const std::vector<std::vector<int>>& rank_lists, int rank,
                                const std::vector<int>& allowed, const std::function<int(int)>& core_of,
                                bool* shared) {
    // This rank's GPU-local CPUs that the process may use (all allowed ones if that leaves none).
    std::vector<int> mine;
    const std::vector<int>& own = rank >= 0 && rank < (int)rank_lists.size() ? rank_lists[rank] : allowed;
    for (int c : own)
        if (std::binary_search(allowed.begin(), allowed.end(), c)) mine.push_back(c);
    if (mine.empty()) mine = allowed;
    // Ranks whose GPUs share this list (same socket / PCIe root, or the same GPU in a rehearsal)
    // split it: this rank's position among them and their number.
    int pos = 0, n = 0;
    for (int r = 0; r < (int)rank_lists.size(); ++r)
        if (rank_lists[r] == own) {
            if (r < rank) ++pos;
            ++n;
        }
    if (n <= 1 || rank < 0 || rank >= (int)rank_lists.size()) {
        n = 1;
        pos = 0;
    }
    // Physical cores in CPU order, each with its SMT siblings; contiguous runs of cores per rank,
    // so two ranks never share a core through its siblings.
    std::vector<std::pair<int, std::vector<int>>> cores;
    for (int c : mine) {
        const int id = core_of ? core_of(c) : c;
        auto it = std::find_if(cores.begin(), cores.end(), [&](const auto& x) { return x.first == id; });
        if (it == cores.end()) cores.push_back({id, {c}});
        else it->second.push_back(c);
    }
    std::sort(cores.begin(), cores.end());
    std::vector<int> out;
    const size_t nc = cores.size();
    if (shared) *shared = nc < (size_t)n;
    if (nc == 0) return out;
    if (nc < (size_t)n) {  // fewer cores than ranks: one core each, shared round-robin
        out = cores[(size_t)pos % nc].second;
        return out;
    }
    const size_t lo = nc * (size_t)pos / (size_t)n, hi = nc * (size_t)(pos + 1) / (size_t)n;
    // first threads of every core, then second threads: the pool's first workers get distinct cores
    for (size_t t = 0;; ++t) {
        bool any = false;
        for (size_t i = lo; i < hi; ++i)
            if (t < cores[i].second.size()) {
                out.push_back(cores[i].second[t]);
                any = true;
            }
        if (!any) break;
    }
    return out;
}

double cgroup_cpu_quota() {
    // cgroup v2 cpu.max: "<quota> <period>" or "max <period>"
    FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r");
    if (!f) return 0.0;
    char q[64] = {0};
    long period = 0;
    const int got = std::fscanf(f, "%63s %ld", q, &period);
    std::fclose(f);
    if (got != 2 || period <= 0 || std::strcmp(q, "max") == 0) return 0.0;
    return std::atof(q) / (double)period;
}

WorkPool& host_pool() {
    static WorkPool pool = [] {
        std::lock_guard<std::mutex> lk(g_plan_m);
        g_pool_made = true;
        unsigned n = 0;
        if (const char* s = std::getenv("AC_HOST_THREADS")) n = (unsigned)std::max(1, std::atoi(s));
        std::vector<int> use;
        cpu_set_t set;
        const bool aff = sched_getaffinity(0, sizeof set, &set) == 0;
        for (int c : g_plan.cpus)
            if (!aff || CPU_ISSET(c, &set)) use.push_back(c);
        if (!n) n = g_plan.participants;
        if (!n) {
            unsigned cpus = std::thread::hardware_concurrency();
            if (aff) cpus = (unsigned)CPU_COUNT(&set);
            n = std::max(1u, std::min(16u, cpus));
        }
        g_plan.participants = n;
        g_plan.cpus = use;
        const char* pin = std::getenv("AC_HOST_PIN");
        if (pin && std::atoi(pin) == 0) use.clear();
        // Each worker may run on any CPU of the set (AC_HOST_PIN=each: one CPU per worker, the round-5
        // default): a worker pinned to one CPU waits out another tenant's time slice on it while holding
        // a claimed task, and the call waits with it -- cfg3, 300 steps: p99 / p50 1.117, max 10.1 ms
        // pinned each vs 1.016, max 3.15 ms on the set, p50 equal (profiles/r06_m6/stall3_*).
        const bool pin_each = pin && std::string(pin) == "each";
        return WorkPool(n, use, pin_each);
    }();
    return pool;
}

namespace {

// 32 Dna5 bases -> two code words (16 bases each, base b at bits 2*(b%16)) and
// one N-mask word (bit b set iff base b > 3).
__attribute__((target("avx2"))) inline void pack32_avx2(const uint8_t* src, uint32_t* code2, uint32_t* nm) {
    const __m256i v = _mm256_loadu_si256((const __m256i*)src);
    const __m256i three = _mm256_set1_epi8(3);
    const uint32_t acgt = (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(_mm256_min_epu8(v, three), v));
    *nm = ~acgt;
    const __m256i c = _mm256_and_si256(v, three);
    // pairs: c0 + 4*c1 (16-bit), then quads: p0 + 16*p1 (32-bit) = one byte of 4 bases
    __m256i t = _mm256_maddubs_epi16(c, _mm256_set1_epi16(0x0401));
    t = _mm256_madd_epi16(t, _mm256_set1_epi32(0x00100001));
    t = _mm256_shuffle_epi8(t, _mm256_setr_epi8(0, 4, 8, 12, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, 0, 4, 8,
                                                12, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1));
    code2[0] = (uint32_t)_mm256_extract_epi32(t, 0);
    code2[1] = (uint32_t)_mm256_extract_epi32(t, 4);
}

inline void pack32_scalar(const uint8_t* src, uint32_t* code2, uint32_t* nm) {
    uint32_t c0 = 0, c1 = 0, n = 0;
    for (int b = 0; b < 16; ++b) {
        c0 |= (uint32_t)(src[b] & 3u) << (2 * b);
        c1 |= (uint32_t)(src[16 + b] & 3u) << (2 * b);
    }
    for (int b = 0; b < 32; ++b) n |= (uint32_t)(src[b] > 3u) << b;
    code2[0] = c0;
    code2[1] = c1;
    *nm = n;
}

// The inline N record of one window (nrec.h), built from its N-mask bits as they are packed:
// add(bits, b) takes the N bits of window bases [b, b + 64); finish(slot) writes the record
// into the top bits of the slot's last code word (padding, zero until then) and returns the
// window's PACK_* flags.  len = 0: no record (PACK_HAS_N only).
struct NRecord {
    uint32_t R, pb, cap, n = 0, pos = 0;
    uint32_t len;
    explicit NRecord(uint32_t l) : R(nrec_bits(l)), pb(nrec_pos_bits(l)), cap(nrec_cap(l)), len(l) {}
    inline void add(uint64_t bits, uint32_t b) {
        for (; bits; bits &= bits - 1) {
            if (n < cap) pos |= (b + (uint32_t)__builtin_ctzll(bits)) << nrec_pos_shift(pb, n);
            ++n;
        }
    }
    inline uint32_t finish(uint32_t* slot) const {
        if (!n) return 0u;
        if (!R) return PACK_HAS_N;
        slot[nrec_word(len)] |= n <= cap ? (pos | n << 29) : NREC_OVERFLOW << 29;
        return PACK_HAS_N | (n > cap ? PACK_OVERFLOW : 0u);
    }
};

// AVX-512BW: 64 bases per step, the tail through a byte-masked load (no
// access past the window, so no over-read of the caller's buffer).  Codes: the
// 2-bit values multiply-added into one byte per 4 bases, vpmovdb narrows 16
// such dwords to the 16 bytes of four code words; N: one compare to a k-mask.
__attribute__((target("avx512f,avx512bw,avx512vl"))) uint32_t pack_range_avx512(
    const uint8_t* bases, const uint64_t* offset, const uint32_t* length, uint32_t w0, uint32_t w1, uint64_t first,
    uint32_t* codes, uint32_t* nmask, uint64_t* start_out, uint32_t* len_out, bool records) {
    const __m512i three = _mm512_set1_epi8(3);
    uint32_t flags = 0;
    const __m512i pair = _mm512_set1_epi16(0x0401);
    const __m512i quad = _mm512_set1_epi32(0x00100001);
    uint64_t pos = first;
    for (uint32_t w = w0; w < w1; ++w) {
        const uint8_t* src = bases + offset[w];
        const uint32_t len = length[w];
        const bool rec = records && nrec_bits(len) != 0u;  // (no room: a plain window)
        if (!rec) {  // (equal windows with records: places by arithmetic, no descriptors needed)
            start_out[w - w0] = pos;
            len_out[w - w0] = len;
        }
        const uint64_t span = image_span(len);
        uint8_t* cw = (uint8_t*)(codes + pos / 16);
        uint8_t* nw = (uint8_t*)(nmask + pos / 32);
        NRecord nr(rec ? len : 0u);
        uint64_t isns[4] = {0, 0, 0, 0};  // (records: the N bits, stored only if the record overflows)
        for (uint32_t b = 0; b < span; b += 64) {
            const uint32_t left = len > b ? len - b : 0u;
            const __mmask64 m = left >= 64 ? ~0ull : ((1ull << left) - 1ull);
            const __m512i v = _mm512_maskz_loadu_epi8(m, src + b);
            const uint64_t isn = _mm512_mask_cmpgt_epu8_mask(m, v, three);
            if (isn) nr.add(isn, b);
            __m512i t = _mm512_maddubs_epi16(_mm512_and_si512(v, three), pair);
            t = _mm512_madd_epi16(t, quad);
            const __m128i c = _mm512_cvtepi32_epi8(t);
            if (span - b >= 64) {
                _mm_storeu_si128((__m128i*)(cw + b / 4), c);
                if (!rec) std::memcpy(nw + b / 8, &isn, 8);
            } else {  // the last 32 bases of the span: half the words (the next window's follow)
                _mm_storel_epi64((__m128i*)(cw + b / 4), c);
                const uint32_t lo = (uint32_t)isn;
                if (!rec) std::memcpy(nw + b / 8, &lo, 4);
            }
            if (rec && b < 256) isns[b / 64] = isn;
        }
        const uint32_t f = nr.finish(codes + pos / 16);
        if (f & PACK_OVERFLOW)  // (a record window spans <= 256 bases: 4 steps)
            for (uint32_t b = 0; b < span; b += 32) {
                const uint32_t word = (uint32_t)(isns[b / 64] >> (b % 64));
                std::memcpy(nw + b / 8, &word, 4);
            }
        flags |= f;
        pos += span;
    }
    return flags;
}

// The stage's common case on AVX-512: equal windows of L bases (a read end: every start window sl
// bases, every end window sl + 1) with inline N records, L <= 256.  One window per iteration with
// every step's masks, shifts and the record's place hoisted out of the loop (they depend on L only),
// the slot's codes kept in registers until the record is in, then stored whole -- with streaming
// stores when the slot is 32-byte aligned (a read end's slots are: the image starts 256-B aligned and
// S = 128 / 256), so the pinned block's lines are not read for ownership first.  NS = 64-base steps
// per slot (S = 32 NS2 bases: NS = ceil(NS2 / 2)).
// (A window of another length -- the caller broke its promise -- goes through the general packer.)
template <int NS>
__attribute__((target("avx512f,avx512bw,avx512vl"))) uint32_t pack_equal_records_avx512(
    const uint8_t* bases, const uint64_t* offset, const uint32_t* length, uint32_t L, uint32_t w0, uint32_t w1,
    uint64_t first, uint32_t* codes, uint32_t* nmask, uint64_t* start_out, uint32_t* len_out) {
    const uint32_t S = (L + 31u) & ~31u;
    const bool half = (S % 64u) != 0u;  // the last step covers 32 bases of the slot
    const __m512i three = _mm512_set1_epi8(3);
    const __m512i pair = _mm512_set1_epi16(0x0401);
    const __m512i quad = _mm512_set1_epi32(0x00100001);
    __mmask64 m[NS];
    for (int b = 0; b < NS; ++b) {
        const uint32_t left = L > 64u * b ? L - 64u * b : 0u;
        m[b] = left >= 64u ? ~0ull : ((1ull << left) - 1ull);
    }
    uint32_t flags = 0;
    uint64_t pos = first;
#ifndef AC_PACK_STREAM
#define AC_PACK_STREAM 1  // (A/B builds: 0 = plain stores)
#endif
    bool stream = AC_PACK_STREAM && ((uintptr_t)(codes + pos / 16) % 32u) == 0u && (S % 128u) == 0u;
    const bool streamed = stream;
    for (uint32_t w = w0; w < w1; ++w, pos += S) {
        if (__builtin_expect(length[w] != L, 0)) {
            flags |= pack_range_avx512(bases, offset, length, w, w + 1, pos, codes, nmask, start_out + (w - w0),
                                       len_out + (w - w0), true);
            pos += image_span(length[w]) - S;
            stream = false;  // (the next slots may not be 32-byte aligned any more)
            continue;
        }
        const uint8_t* src = bases + offset[w];
        __m128i c[NS];
        uint64_t isn[NS];
        uint64_t any = 0;
#pragma GCC unroll 4
        for (int b = 0; b < NS; ++b) {
            const __m512i v = _mm512_maskz_loadu_epi8(m[b], src + 64 * b);
            isn[b] = _mm512_mask_cmpgt_epu8_mask(m[b], v, three);
            any |= isn[b];
            __m512i t = _mm512_maddubs_epi16(_mm512_and_si512(v, three), pair);
            t = _mm512_madd_epi16(t, quad);
            c[b] = _mm512_cvtepi32_epi8(t);
        }
        uint32_t* slot = codes + pos / 16;
        if (__builtin_expect(any != 0, 0)) {  // the record (rare: 0.1 % N per base is ~10 % of windows)
            NRecord nr(L);
            for (int b = 0; b < NS; ++b)
                if (isn[b]) nr.add(isn[b], 64u * b);
            alignas(16) uint32_t words[4 * NS];
            for (int b = 0; b < NS; ++b) _mm_store_si128((__m128i*)(words + 4 * b), c[b]);
            const uint32_t f = nr.finish(words);  // ORs the record into words[rw]
            for (int b = 0; b < NS; ++b) c[b] = _mm_load_si128((const __m128i*)(words + 4 * b));
            if (f & PACK_OVERFLOW) {
                uint8_t* nw = (uint8_t*)(nmask + pos / 32);
                for (uint32_t b = 0; b < S; b += 32) {
                    const uint32_t word = (uint32_t)(isn[b / 64] >> (b % 64));
                    std::memcpy(nw + b / 8, &word, 4);
                }
            }
            flags |= f;
        }
        if (stream) {
#pragma GCC unroll 4
            for (int b = 0; b + 1 < NS; b += 2)
                _mm256_stream_si256((__m256i*)(slot + 4 * b), _mm256_inserti128_si256(_mm256_castsi128_si256(c[b]), c[b + 1], 1));
            if (NS % 2) _mm_stream_si128((__m128i*)(slot + 4 * (NS - 1)), c[NS - 1]);
        } else {
#pragma GCC unroll 4
            for (int b = 0; b + 1 < NS; ++b) _mm_storeu_si128((__m128i*)(slot + 4 * b), c[b]);
            if (half) _mm_storel_epi64((__m128i*)(slot + 4 * (NS - 1)), c[NS - 1]);
            else _mm_storeu_si128((__m128i*)(slot + 4 * (NS - 1)), c[NS - 1]);
        }
    }
    if (streamed) _mm_sfence();  // streamed slots are in memory before the caller publishes them
    return flags;
}

template <bool AVX2>
uint32_t pack_range_impl(const uint8_t* bases, const uint64_t* offset, const uint32_t* length, uint32_t w0,
                         uint32_t w1, uint64_t first, uint32_t* codes, uint32_t* nmask, uint64_t* start_out,
                         uint32_t* len_out, bool records) {
    uint32_t flags = 0;
    uint64_t pos = first;
    alignas(32) uint8_t tail[32];
    uint32_t scratch[8];  // (records: the window's N-mask words, stored only if the record overflows)
    for (uint32_t w = w0; w < w1; ++w) {
        const uint8_t* src = bases + offset[w];
        const uint32_t len = length[w];
        const bool rec = records && nrec_bits(len) != 0u;  // (no room: a plain window)
        if (!rec) {
            start_out[w - w0] = pos;
            len_out[w - w0] = len;
        }
        uint32_t* cw = codes + pos / 16;
        uint32_t* nw = rec ? scratch : nmask + pos / 32;
        const uint32_t full = len / 32;
        for (uint32_t b = 0; b < full; ++b) {
            if (AVX2) pack32_avx2(src + 32 * b, cw + 2 * b, nw + b);
            else pack32_scalar(src + 32 * b, cw + 2 * b, nw + b);
        }
        if (const uint32_t r = len % 32) {  // the last block: padding bases are code 0 (A), not N
            std::memset(tail, 0, sizeof tail);
            std::memcpy(tail, src + 32 * full, r);
            if (AVX2) pack32_avx2(tail, cw + 2 * full, nw + full);
            else pack32_scalar(tail, cw + 2 * full, nw + full);
        }
        NRecord nr(rec ? len : 0u);
        for (uint32_t b = 0; b < (len + 31u) / 32u; ++b)
            if (nw[b]) nr.add(nw[b], 32u * b);
        const uint32_t f = nr.finish(cw);
        if (f & PACK_OVERFLOW) std::memcpy(nmask + pos / 32, scratch, sizeof(uint32_t) * ((len + 31u) / 32u));
        flags |= f;
        pos += image_span(len);
    }
    return flags;
}

// (AC_PACK_ISA=1 / 0: test builds of the AVX2 / scalar packers on an AVX-512 host, tests/test_pack_records.py)
bool have_avx2() {
#if defined(AC_PACK_ISA) && AC_PACK_ISA < 1
    return false;
#else
    static const bool v = __builtin_cpu_supports("avx2");
    return v;
#endif
}

bool have_avx512() {
#if defined(AC_PACK_ISA) && AC_PACK_ISA < 2
    return false;
#else
    static const bool v = __builtin_cpu_supports("avx512bw") && __builtin_cpu_supports("avx512vl");
    return v;
#endif
}

__attribute__((target("avx512f"))) uint64_t span_scan_avx512(const uint32_t* len, uint32_t n, uint32_t f,
                                                              uint32_t* diff) {
    const __m512i c31 = _mm512_set1_epi32(31), fv = _mm512_set1_epi32((int)f);
    __m512i sum_lo = _mm512_setzero_si512(), sum_hi = _mm512_setzero_si512(), d = _mm512_setzero_si512();
    __m512i all = _mm512_setzero_si512();
    uint32_t i = 0;
    for (; i + 16 <= n; i += 16) {
        const __m512i v = _mm512_loadu_si512((const void*)(len + i));
        all = _mm512_or_si512(all, v);
        d = _mm512_or_si512(d, _mm512_xor_si512(v, fv));
        const __m512i blocks = _mm512_srli_epi32(_mm512_add_epi32(v, c31), 5);  // (len + 31) / 32, wraps for len > 2^32 - 32
        sum_lo = _mm512_add_epi64(sum_lo, _mm512_cvtepu32_epi64(_mm512_castsi512_si256(blocks)));
        sum_hi = _mm512_add_epi64(sum_hi, _mm512_cvtepu32_epi64(_mm512_extracti64x4_epi64(blocks, 1)));
    }
    uint64_t b = (uint64_t)_mm512_reduce_add_epi64(_mm512_add_epi64(sum_lo, sum_hi)) * 32u;
    uint32_t dd = (uint32_t)_mm512_reduce_or_epi32(d);
    for (; i < n; ++i) {
        b += image_span(len[i]);
        dd |= len[i] ^ f;
    }
    // (a window of 2^31 bases or more may have wrapped above: recount exactly)
    if ((uint32_t)_mm512_reduce_or_epi32(all) >> 31) {
        b = 0;
        for (uint32_t j = 0; j < n; ++j) b += image_span(len[j]);
    }
    *diff = dd;
    return b;
}

}  // namespace

uint64_t span_scan(const uint32_t* len, uint32_t n, uint32_t* first, uint32_t* diff) {
    const uint32_t f = n ? len[0] : 0u;
    *first = f;
    if (have_avx512()) return span_scan_avx512(len, n, f, diff);
    uint64_t b = 0;
    for (uint32_t w = 0; w < n; ++w) b += image_span(len[w]);
    uint32_t d = 0;  // (a separate OR-reduction: folded into the loop above it did not vectorise)
    for (uint32_t w = 0; w < n; ++w) d |= len[w] ^ f;
    *diff = d;
    return b;
}

uint32_t pack_dna5_range(const uint8_t* bases, const uint64_t* offset, const uint32_t* length, uint32_t w0,
                         uint32_t w1, uint64_t first, uint32_t* codes, uint32_t* nmask, uint64_t* start_out,
                         uint32_t* len_out, bool records) {
    if (have_avx512()) {
        // equal windows with records (the caller's promise: every window of the job has one length)
        const uint32_t L = w1 > w0 ? length[w0] : 0u;
        if (records && nrec_bits(L) != 0u) {
            switch ((((L + 31u) & ~31u) + 63u) / 64u) {
                case 1: return pack_equal_records_avx512<1>(bases, offset, length, L, w0, w1, first, codes, nmask, start_out, len_out);
                case 2: return pack_equal_records_avx512<2>(bases, offset, length, L, w0, w1, first, codes, nmask, start_out, len_out);
                case 3: return pack_equal_records_avx512<3>(bases, offset, length, L, w0, w1, first, codes, nmask, start_out, len_out);
                case 4: return pack_equal_records_avx512<4>(bases, offset, length, L, w0, w1, first, codes, nmask, start_out, len_out);
                default: break;
            }
        }
        return pack_range_avx512(bases, offset, length, w0, w1, first, codes, nmask, start_out, len_out, records);
    }
    if (have_avx2())
        return pack_range_impl<true>(bases, offset, length, w0, w1, first, codes, nmask, start_out, len_out, records);
    return pack_range_impl<false>(bases, offset, length, w0, w1, first, codes, nmask, start_out, len_out, records);
}

}  // namespace acamd
