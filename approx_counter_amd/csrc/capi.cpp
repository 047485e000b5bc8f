// capi.cpp -- C ABI of the MI355X approximate-count stage (include/approx_counter_amd.h).
//
// Replaces errorCount (approx_counter.cpp:531-601): where the reference builds
// a bidirectional FM index over the sample (537-541) and runs SeqAn's
// find<0,2> per candidate under OpenMP (547-599), this layer uploads the
// packed sample once per call and launches one HIP kernel over the
// candidate x window grid.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "approx_counter_amd.h"
#include "exact_count.h"
#include "wm_count.h"

struct ac_ctx {
    int device = 0;
    int cu_count = 256;
    hipStream_t stream = nullptr;
    std::string err;
    // grow-only device buffers for the host-buffer entry point
    void* d_buf[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    size_t d_cap[6] = {0, 0, 0, 0, 0, 0};
    std::vector<uint32_t> h_counts;
    // ac_error_count staging: the inputs packed back to back in pinned host
    // memory, one H2D copy into d_stage, counts copied back into the same
    // pinned block (grow-only)
    void* h_stage = nullptr;
    void* d_stage = nullptr;
    size_t h_stage_cap = 0, d_stage_cap = 0;
    // ac_sample_upload buffers (codes, nmask, start, length) and the exact-count
    // working set (table keys, table counts, small scalars + histogram, forbidden, gather out)
    void* s_buf[4] = {nullptr, nullptr, nullptr, nullptr};
    size_t s_cap[4] = {0, 0, 0, 0};
    void* e_buf[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    size_t e_cap[6] = {0, 0, 0, 0, 0, 0};
    // work-queue counters: two banks of qcap u32; dirty[b] =
    // counters of bank b used by the last launch on it (zeroed by the next launch)
    uint32_t* queue = nullptr;
    uint32_t qcap = 0, bank = 0, dirty[2] = {0, 0};
    // count hand-off scratch: per-group sums and tickets (zero between launches)
    uint32_t* acc = nullptr;
    uint32_t* tickets = nullptr;
    uint32_t acc_cap = 0, ticket_cap = 0;
    // resident waves of the count kernel per pattern pack P (0 = not queried yet)
    uint32_t resident[AC_MAX_PACK + 1] = {0, 0, 0, 0, 0};
    // last launch geometry
    uint64_t last_waves = 0;
    uint32_t last_wpw = 0, last_groups = 0;
    // ac_create_multi: contexts of shards 1..n-1 (this context is shard 0)
    std::vector<ac_ctx*> peers;
};

namespace {

thread_local std::string g_err;

ac_status fail(ac_ctx* ctx, ac_status st, const std::string& msg) {
    if (ctx) ctx->err = msg;
    g_err = msg;
    return st;
}

ac_status hip_fail(ac_ctx* ctx, hipError_t e, const char* what) {
    return fail(ctx, e == hipErrorOutOfMemory ? AC_ERR_NOMEM : AC_ERR_DEVICE,
                std::string(what) + ": " + hipGetErrorString(e));
}

#define AC_HIP(ctx, expr)                                  \
    do {                                                   \
        hipError_t e_ = (expr);                            \
        if (e_ != hipSuccess) return hip_fail(ctx, e_, #expr); \
    } while (0)

ac_status check_k(ac_ctx* ctx, uint32_t k) {
    // approx_counter.cpp:781-783: k must lie in [2, 32].
    if (k < 2 || k > 32) return fail(ctx, AC_ERR_INVALID, "kmer size must be between 2 and 32 (included)");
    return AC_OK;
}

ac_status grow(ac_ctx* ctx, void** buf, size_t* cap, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (*cap >= bytes) return AC_OK;
    if (*buf) (void)hipFree(*buf);
    *buf = nullptr;
    *cap = 0;
    AC_HIP(ctx, hipMalloc(buf, bytes));
    *cap = bytes;
    return AC_OK;
}

ac_status ensure(ac_ctx* ctx, int slot, size_t bytes) { return grow(ctx, &ctx->d_buf[slot], &ctx->d_cap[slot], bytes); }

// Host -> device copy of n host arrays through the context's pinned staging
// block.  Array i lands at offset off(i) = sum of the earlier sizes rounded up
// to 256 B, in the staging block and in the device block `dst` alike.  The
// block is filled and sent in 1 MB pieces, each piece's DMA queued as soon as
// it is filled, so the CPU fills the next piece while the previous one crosses
// PCIe (pageable copies, one per array, each paid the driver's own staging
// overhead; one DMA per array instead of per piece cost 70 us more at cfg2).
// Asynchronous on ctx->stream; the block is reused by the next call, so callers
// synchronise the stream before returning.  `extra` bytes after the arrays are
// reserved (the counts' way back).
size_t staged_bytes(int n, const size_t* sz) {
    size_t total = 0;
    for (int i = 0; i < n; ++i) total += (sz[i] + 255) / 256 * 256;
    return total;
}

ac_status h2d_staged(ac_ctx* ctx, int n, const void* const* src, const size_t* sz, void* dst, size_t extra = 0) {
    const size_t in_bytes = staged_bytes(n, sz), total = in_bytes + extra;
    if (ctx->h_stage_cap < total) {
        if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
        ctx->h_stage = nullptr;
        ctx->h_stage_cap = 0;
        AC_HIP(ctx, hipHostMalloc(&ctx->h_stage, total, hipHostMallocDefault));
        ctx->h_stage_cap = total;
    }
    constexpr size_t CHUNK = size_t(1) << 20;
    char* h = (char*)ctx->h_stage;
    for (size_t c0 = 0; c0 < in_bytes; c0 += CHUNK) {
        const size_t c1 = std::min(in_bytes, c0 + CHUNK);
        size_t off = 0;
        for (int i = 0; i < n; ++i) {
            const size_t lo = std::max(c0, off), hi = std::min(c1, off + sz[i]);
            if (lo < hi) std::memcpy(h + lo, (const char*)src[i] + (lo - off), hi - lo);
            off += (sz[i] + 255) / 256 * 256;
        }
        AC_HIP(ctx, hipMemcpyAsync((char*)dst + c0, h + c0, c1 - c0, hipMemcpyHostToDevice, ctx->stream));
    }
    return AC_OK;
}

// getComplexity (approx_counter.cpp:247-267) and CompareCount (275-305), for the
// final ranking of the exact count's short list.
float complexity(uint64_t kmer, uint32_t k) {
    uint64_t counts[16] = {0};
    for (uint32_t i = 0; i + 1 < k; ++i) {
        counts[kmer & 15u]++;
        kmer >>= 2;
    }
    size_t sum = 0;
    for (uint64_t v : counts) sum += v * (v - 1);
    return (float)sum / float(2 * ((int)k - 2));
}

ac_status check_sample(ac_ctx* ctx, const ac_windows* s) {
    if (!s) return fail(ctx, AC_ERR_INVALID, "sample is NULL");
    if (s->n_bases % 32) return fail(ctx, AC_ERR_INVALID, "sample n_bases must be a multiple of 32");
    if (s->n_windows && (!s->codes || !s->nmask || !s->start || !s->length))
        return fail(ctx, AC_ERR_INVALID, "sample has a NULL array");
    return AC_OK;
}

ac_status launch(ac_ctx* ctx, uint32_t k, const ac_segment* segs, uint32_t n, hipStream_t stream,
                 bool zero) {
    if (ac_status st = check_k(ctx, k)) return st;
    if (n > AC_MAX_SEGS) return fail(ctx, AC_ERR_INVALID, "too many segments in one launch (max 4)");
    if (n && !segs) return fail(ctx, AC_ERR_INVALID, "segments is NULL");
    const uint32_t P = acamd::pack_factor(k);
    const uint32_t cpw = acamd::cands_per_wave(P);
    acamd::LaunchArgs a;
    std::memset(&a, 0, sizeof a);
    a.n_segs = n;
    a.m = k;
    a.P = P;
    uint64_t items = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const ac_segment& s = segs[i];
        if (s.n_kmers && (!s.kmers || !s.counts)) return fail(ctx, AC_ERR_INVALID, "segment kmers/counts is NULL");
        if (s.n_kmers && s.sample.n_windows &&
            (!s.sample.codes || !s.sample.nmask || !s.sample.start || !s.sample.length))
            return fail(ctx, AC_ERR_INVALID, "segment sample has a NULL array");
        if (s.sample.n_bases % 32) return fail(ctx, AC_ERR_INVALID, "sample n_bases must be a multiple of 32");
        const uint32_t groups = (s.n_kmers + cpw - 1) / cpw;
        items += (uint64_t)groups * s.sample.n_windows;
    }
    // Launch plan.  One round of resident waves; work is pulled
    // from dynamic queues: items of `chunk` windows (1 when waves get few
    // windows, so the launch tail is about one window; up to 8 when they get
    // hundreds, for fewer atomics), each candidate group's items spread over
    // sub-queues of about 64 waves.  A segment gets sub-queues in proportion
    // to its windows, so every sub-queue holds about the same work.  Workgroups
    // of AC_WAVES_PER_BLOCK waves are dealt round-robin over blocks of that many
    // consecutive sub-queues (one candidate group each).
    if (!ctx->resident[P]) AC_HIP(ctx, acamd::resident_waves(P, ctx->cu_count, &ctx->resident[P]));
    const uint64_t resident = ctx->resident[P];
    const uint32_t wpw = (uint32_t)std::max<uint64_t>(1, (items + resident - 1) / resident);
#ifdef AC_FORCE_CHUNK  // A/B builds (tools/variants.sh): fixed item size
    const uint32_t chunk = AC_FORCE_CHUNK;
    (void)wpw;
#else
    const uint32_t chunk = std::max<uint32_t>(1, std::min<uint32_t>(8, wpw / 64));
#endif
    uint32_t groups_live = 0, max_nw = 1;
    for (uint32_t i = 0; i < n; ++i)
        if (segs[i].n_kmers && segs[i].sample.n_windows) {
            groups_live += (segs[i].n_kmers + cpw - 1) / cpw;
            max_nw = std::max<uint32_t>(max_nw, segs[i].sample.n_windows);
        }
    const uint64_t s_base = std::max<uint64_t>(1, std::min<uint64_t>(32, resident / (64ull * std::max(1u, groups_live))));
    uint64_t wave = 0;
    uint32_t groups_total = 0, qbegin = 0, acc_slots = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const ac_segment& s = segs[i];
        acamd::SegDev& d = a.seg[i];
        d.kmers = s.kmers;
        d.codes = s.sample.codes;
        d.nmask = s.sample.nmask;
        d.start = s.sample.start;
        d.length = s.sample.length;
        d.n_bases = s.sample.n_bases;
        d.counts = s.counts;
        d.n_kmers = s.n_kmers;
        d.n_windows = s.sample.n_windows;
        d.groups = std::max<uint32_t>(1, (s.n_kmers + cpw - 1) / cpw);
        d.chunk = chunk;
        {  // a multiple of the workgroup size: a workgroup's waves take consecutive sub-queues of one group
            const uint64_t sq = std::max<uint64_t>(1, (s_base * s.sample.n_windows + max_nw / 2) / max_nw);
            d.subq = (uint32_t)((sq + AC_WAVES_PER_BLOCK - 1) / AC_WAVES_PER_BLOCK * AC_WAVES_PER_BLOCK);
        }
        d.queue_begin = qbegin;
        d.acc_begin = acc_slots;
        d.ticket_begin = groups_total;
        if (s.n_kmers && s.sample.n_windows) {
            qbegin += d.groups * d.subq;
            acc_slots += d.groups * cpw;
            groups_total += d.groups;
        } else {
            d.queue_begin = ~0u;  // never selected by the kernel's segment lookup
            // no workgroup writes this segment's counts
            if (zero && s.n_kmers) AC_HIP(ctx, hipMemsetAsync(s.counts, 0, sizeof(uint32_t) * s.n_kmers, stream));
        }
    }
    // The group's last workgroup stores its counts (no memset), unless live
    // segments share count slots (window shards of one candidate set): then
    // zero them once and let every group add.
    bool alias = false;
    for (uint32_t i = 0; i < n && !alias; ++i)
        for (uint32_t j = i + 1; j < n && !alias; ++j) {
            const acamd::SegDev &x = a.seg[i], &y = a.seg[j];
            if (x.queue_begin == ~0u || y.queue_begin == ~0u) continue;
            alias = x.counts < y.counts + y.n_kmers && y.counts < x.counts + x.n_kmers;
        }
#ifdef AC_COUNTS_DIRECT  // A/B variant: memset + direct atomics
    alias = true;
#endif
    a.add_counts = (!zero || alias) ? 1u : 0u;
    if (zero && alias)
        for (uint32_t i = 0; i < n; ++i)
            if (a.seg[i].queue_begin != ~0u)
                AC_HIP(ctx, hipMemsetAsync(a.seg[i].counts, 0, sizeof(uint32_t) * a.seg[i].n_kmers, stream));
    if (acc_slots > ctx->acc_cap) {
        if (ctx->acc) AC_HIP(ctx, hipFree(ctx->acc));
        ctx->acc = nullptr;
        ctx->acc_cap = 0;
        AC_HIP(ctx, hipMalloc(&ctx->acc, sizeof(uint32_t) * acc_slots));
        AC_HIP(ctx, hipMemsetAsync(ctx->acc, 0, sizeof(uint32_t) * acc_slots, stream));
        ctx->acc_cap = acc_slots;
    }
    if (groups_total > ctx->ticket_cap) {
        if (ctx->tickets) AC_HIP(ctx, hipFree(ctx->tickets));
        ctx->tickets = nullptr;
        ctx->ticket_cap = 0;
        const size_t bytes = sizeof(uint32_t) * AC_QUEUE_LINE * (size_t)groups_total;
        AC_HIP(ctx, hipMalloc(&ctx->tickets, bytes));
        AC_HIP(ctx, hipMemsetAsync(ctx->tickets, 0, bytes, stream));
        ctx->ticket_cap = groups_total;
    }
    a.acc = ctx->acc;
    a.tickets = ctx->tickets;
    const uint32_t n_counters = qbegin;
    if (n_counters) wave = std::max<uint64_t>(resident, n_counters);
    if (n_counters > ctx->qcap) {
        if (ctx->queue) AC_HIP(ctx, hipFree(ctx->queue));
        ctx->queue = nullptr;
        ctx->qcap = 0;
        const uint32_t cap = std::max<uint32_t>(n_counters, 1024);
        const size_t bytes = sizeof(uint32_t) * AC_QUEUE_LINE * 2 * (size_t)cap;
        AC_HIP(ctx, hipMalloc(&ctx->queue, bytes));
        AC_HIP(ctx, hipMemsetAsync(ctx->queue, 0, bytes, stream));
        ctx->qcap = cap;
        ctx->bank = 0;
        ctx->dirty[0] = ctx->dirty[1] = 0;
    }
    a.queue = ctx->queue;
    a.qstride = ctx->qcap;
    a.bank = ctx->bank;
    a.zero_count = ctx->dirty[ctx->bank ^ 1u];
    a.n_queues = std::max<uint32_t>(1, n_counters);
    // Live segments' queue_begin values are increasing; the kernel picks the
    // last live segment whose queue_begin <= its sub-queue.
    a.total_waves = wave;
    ctx->last_waves = wave;
    ctx->last_wpw = wpw;
    ctx->last_groups = groups_total;
    AC_HIP(ctx, acamd::launch_wm2_count(a, stream));
    if (wave) {  // the launch dequeued from `bank` and zeroed the other one
        ctx->dirty[ctx->bank] = n_counters;
        ctx->dirty[ctx->bank ^ 1u] = 0;
        ctx->bank ^= 1u;
    }
    return AC_OK;
}

}  // namespace

extern "C" {

int ac_abi_version(void) { return AC_ABI_VERSION; }

int ac_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char* ac_last_error(const ac_ctx* ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

ac_status ac_create(ac_ctx** out, int device) {
    if (!out) return fail(nullptr, AC_ERR_INVALID, "out is NULL");
    *out = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0)
        return fail(nullptr, AC_ERR_DEVICE, "no HIP device available (the approximate count runs on the GPU only)");
    if (device < 0) {
        if (hipGetDevice(&device) != hipSuccess) device = 0;
    }
    if (device >= n) return fail(nullptr, AC_ERR_INVALID, "device ordinal out of range");
    ac_ctx* ctx = new (std::nothrow) ac_ctx();
    if (!ctx) return fail(nullptr, AC_ERR_NOMEM, "cannot allocate context");
    ctx->device = device;
    hipDeviceProp_t prop;
    if ((e = hipSetDevice(device)) != hipSuccess || (e = hipGetDeviceProperties(&prop, device)) != hipSuccess ||
        (e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking)) != hipSuccess) {
        ac_status st = hip_fail(nullptr, e, "device setup");
        delete ctx;
        return st;
    }
    ctx->cu_count = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    *out = ctx;
    return AC_OK;
}

void ac_destroy(ac_ctx* ctx) {
    if (!ctx) return;
    for (ac_ctx* p : ctx->peers) ac_destroy(p);
    (void)hipSetDevice(ctx->device);
    for (void* p : ctx->d_buf)
        if (p) (void)hipFree(p);
    if (ctx->d_stage) (void)hipFree(ctx->d_stage);
    if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
    if (ctx->queue) (void)hipFree(ctx->queue);
    if (ctx->acc) (void)hipFree(ctx->acc);
    if (ctx->tickets) (void)hipFree(ctx->tickets);
    for (void* p : ctx->s_buf)
        if (p) (void)hipFree(p);
    for (void* p : ctx->e_buf)
        if (p) (void)hipFree(p);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

ac_status ac_error_count_device(ac_ctx* ctx, uint32_t k, const ac_segment* segments, uint32_t n_segments,
                                void* hip_stream) {
    if (!ctx) return fail(nullptr, AC_ERR_INVALID, "ctx is NULL");
    AC_HIP(ctx, hipSetDevice(ctx->device));
    return launch(ctx, k, segments, n_segments, (hipStream_t)hip_stream, true);
}

ac_status ac_error_count_device_accumulate(ac_ctx* ctx, uint32_t k, const ac_segment* segments,
                                           uint32_t n_segments, void* hip_stream) {
    if (!ctx) return fail(nullptr, AC_ERR_INVALID, "ctx is NULL");
    AC_HIP(ctx, hipSetDevice(ctx->device));
    return launch(ctx, k, segments, n_segments, (hipStream_t)hip_stream, false);
}

}  // extern "C"

namespace {

ac_status error_count_one(ac_ctx* ctx, uint32_t k, const uint64_t* kmers, uint32_t n_kmers,
                          const ac_windows* sample, uint64_t* counts) {
    if (!ctx) return fail(nullptr, AC_ERR_INVALID, "ctx is NULL");
    if (ac_status st = check_k(ctx, k)) return st;
    if (n_kmers == 0) return AC_OK;
    if (!kmers || !counts || !sample) return fail(ctx, AC_ERR_INVALID, "NULL argument");
    const ac_windows& s = *sample;
    if (s.n_bases % 32) return fail(ctx, AC_ERR_INVALID, "sample n_bases must be a multiple of 32");
    if (s.n_windows && (!s.codes || !s.nmask || !s.start || !s.length))
        return fail(ctx, AC_ERR_INVALID, "sample has a NULL array");
    // Host-side layout check: every window inside the image and 32-aligned.
    for (uint32_t i = 0; i < s.n_windows; ++i) {
        if (s.start[i] % 32 || s.start[i] + s.length[i] > s.n_bases)
            return fail(ctx, AC_ERR_INVALID, "window " + std::to_string(i) + " is misaligned or outside the image");
    }
    AC_HIP(ctx, hipSetDevice(ctx->device));
    // Device block: kmers | codes | nmask | start | length | counts, each
    // 256-B aligned, filled through the pinned staging block (h2d_staged).
    const size_t sz[6] = {sizeof(uint64_t) * n_kmers, sizeof(uint32_t) * (s.n_bases / 16),
                          sizeof(uint32_t) * (s.n_bases / 32), sizeof(uint64_t) * s.n_windows,
                          sizeof(uint32_t) * s.n_windows, sizeof(uint32_t) * n_kmers};
    const void* src[5] = {kmers, s.codes, s.nmask, s.start, s.length};
    size_t off[7];
    off[0] = 0;
    for (int i = 0; i < 6; ++i) off[i + 1] = (off[i] + sz[i] + 255) / 256 * 256;
    if (ac_status rc = grow(ctx, &ctx->d_stage, &ctx->d_stage_cap, off[6])) return rc;
    char* d = (char*)ctx->d_stage;
    // the counts come back into the staging block, after the inputs
    if (ac_status rc = h2d_staged(ctx, 5, src, sz, d, (sz[5] + 255) / 256 * 256)) return rc;
    char* h = (char*)ctx->h_stage;
    hipStream_t st = ctx->stream;
    ac_segment seg;
    seg.kmers = (const uint64_t*)(d + off[0]);
    seg.n_kmers = n_kmers;
    seg.sample.codes = (const uint32_t*)(d + off[1]);
    seg.sample.nmask = (const uint32_t*)(d + off[2]);
    seg.sample.start = (const uint64_t*)(d + off[3]);
    seg.sample.length = (const uint32_t*)(d + off[4]);
    seg.sample.n_windows = s.n_windows;
    seg.sample.n_bases = s.n_bases;
    seg.counts = (uint32_t*)(d + off[5]);
    if (ac_status rc = launch(ctx, k, &seg, 1, st, true)) return rc;
    AC_HIP(ctx, hipMemcpyAsync(h + off[5], d + off[5], sz[5], hipMemcpyDeviceToHost, st));
    AC_HIP(ctx, hipStreamSynchronize(st));
    const uint32_t* hc = (const uint32_t*)(h + off[5]);
    for (uint32_t i = 0; i < n_kmers; ++i) counts[i] = hc[i];
    return AC_OK;
}

}  // namespace

extern "C" {

ac_status ac_error_count(ac_ctx* ctx, uint32_t k, const uint64_t* kmers, uint32_t n_kmers,
                         const ac_windows* sample, uint64_t* counts) {
    if (!ctx || ctx->peers.empty()) return error_count_one(ctx, k, kmers, n_kmers, sample, counts);
    if (ac_status st = check_k(ctx, k)) return st;
    if (n_kmers == 0) return AC_OK;
    if (!kmers || !counts || !sample) return fail(ctx, AC_ERR_INVALID, "NULL argument");
    if (ac_status st = check_sample(ctx, sample)) return st;
    const ac_windows& s = *sample;
    for (uint32_t i = 0; i < s.n_windows; ++i)
        if (s.start[i] % 32 || s.start[i] + s.length[i] > s.n_bases)
            return fail(ctx, AC_ERR_INVALID, "window " + std::to_string(i) + " is misaligned or outside the image");
    // Shards: contiguous window ranges balanced by bases; shard g is a slice of
    // the image (codes/nmask from its first window's start), starts rebased.
    const size_t G = ctx->peers.size() + 1;
    uint64_t total = 0;
    for (uint32_t i = 0; i < s.n_windows; ++i) total += s.length[i];
    std::vector<uint32_t> cut(G + 1, s.n_windows);
    cut[0] = 0;
    {
        uint64_t acc = 0;
        size_t g = 1;
        for (uint32_t i = 0; i < s.n_windows && g < G; ++i) {
            acc += s.length[i];
            while (g < G && acc * G >= total * g) cut[g++] = i + 1;
        }
    }
    std::vector<std::vector<uint64_t>> part(G, std::vector<uint64_t>(n_kmers, 0));
    std::vector<ac_status> rc(G, AC_OK);
    auto run = [&](size_t g) {
        ac_ctx* c = g == 0 ? ctx : ctx->peers[g - 1];
        const uint32_t lo = cut[g], hi = cut[g + 1];
        if (hi == lo) return;
        const uint64_t b0 = s.start[lo];
        uint64_t b1 = b0;
        for (uint32_t i = lo; i < hi; ++i) b1 = std::max<uint64_t>(b1, s.start[i] + s.length[i]);
        b1 = (b1 + 31) / 32 * 32;
        if (b1 == b0) return;  // only empty windows: no occurrences
        std::vector<uint64_t> st(hi - lo);
        for (uint32_t i = lo; i < hi; ++i) st[i - lo] = s.start[i] - b0;
        const ac_windows w{s.codes + b0 / 16, s.nmask + b0 / 32, st.data(), s.length + lo, hi - lo, b1 - b0};
        rc[g] = error_count_one(c, k, kmers, n_kmers, &w, part[g].data());
    };
    std::vector<std::thread> th;
    for (size_t g = 1; g < G; ++g) th.emplace_back(run, g);
    run(0);
    for (auto& t : th) t.join();
    for (size_t g = 0; g < G; ++g)
        if (rc[g] != AC_OK) {
            ac_ctx* c = g == 0 ? ctx : ctx->peers[g - 1];
            return fail(ctx, rc[g], "shard " + std::to_string(g) + ": " + c->err);
        }
    for (uint32_t i = 0; i < n_kmers; ++i) {
        uint64_t v = 0;
        for (size_t g = 0; g < G; ++g) v += part[g][i];
        counts[i] = v;
    }
    return AC_OK;
}

ac_status ac_create_multi(ac_ctx** out, int n_gpus) {
    if (!out) return fail(nullptr, AC_ERR_INVALID, "out is NULL");
    *out = nullptr;
    if (n_gpus < 1) return fail(nullptr, AC_ERR_INVALID, "n_gpus must be >= 1");
    const int n_dev = ac_device_count();
    if (n_dev < 1) return fail(nullptr, AC_ERR_DEVICE, "no HIP device available (the approximate count runs on the GPU only)");
    ac_ctx* root = nullptr;
    if (ac_status st = ac_create(&root, 0)) return st;
    for (int g = 1; g < n_gpus; ++g) {
        ac_ctx* c = nullptr;
        if (ac_status st = ac_create(&c, g % n_dev)) {
            ac_destroy(root);
            return st;
        }
        root->peers.push_back(c);
    }
    *out = root;
    return AC_OK;
}

ac_status ac_count(ac_ctx* ctx, uint32_t k, const uint64_t* kmers, uint32_t n_kmers, const uint32_t* win_bits,
                   const uint32_t* win_nmask, const uint64_t* win_word_offset, const uint16_t* win_len,
                   uint32_t n_windows, uint64_t* counts_out) {
    if (!ctx) return fail(nullptr, AC_ERR_INVALID, "ctx is NULL");
    if (n_windows && (!win_bits || !win_nmask || !win_word_offset || !win_len))
        return fail(ctx, AC_ERR_INVALID, "NULL window array");
    std::vector<uint64_t> start(n_windows);
    std::vector<uint32_t> len(n_windows);
    uint64_t n_bases = 32;
    for (uint32_t i = 0; i < n_windows; ++i) {
        if (win_word_offset[i] % 2)
            return fail(ctx, AC_ERR_INVALID, "window " + std::to_string(i) + " starts at an odd 2-bit word");
        start[i] = win_word_offset[i] * 16;
        len[i] = win_len[i];
        n_bases = std::max<uint64_t>(n_bases, (start[i] + len[i] + 31) / 32 * 32);
    }
    const ac_windows w{win_bits, win_nmask, start.data(), len.data(), n_windows, n_bases};
    return ac_error_count(ctx, k, kmers, n_kmers, &w, counts_out);
}

ac_status ac_sample_upload(ac_ctx* ctx, const ac_windows* host, ac_windows* dev) {
    if (!ctx || !dev) return fail(ctx, AC_ERR_INVALID, "ctx or dev is NULL");
    if (ac_status st = check_sample(ctx, host)) return st;
    // layout check on the host copy: every window inside the image, 32-aligned
    for (uint32_t i = 0; i < host->n_windows; ++i)
        if (host->start[i] % 32 || host->start[i] + host->length[i] > host->n_bases)
            return fail(ctx, AC_ERR_INVALID, "window " + std::to_string(i) + " is misaligned or outside the image");
    AC_HIP(ctx, hipSetDevice(ctx->device));
    const size_t sz[4] = {sizeof(uint32_t) * (host->n_bases / 16), sizeof(uint32_t) * (host->n_bases / 32),
                          sizeof(uint64_t) * host->n_windows, sizeof(uint32_t) * host->n_windows};
    const void* src[4] = {host->codes, host->nmask, host->start, host->length};
    // one device block (s_buf[0]) holding the four arrays at the staging offsets
    if (ac_status st = grow(ctx, &ctx->s_buf[0], &ctx->s_cap[0], staged_bytes(4, sz))) return st;
    if (ac_status st = h2d_staged(ctx, 4, src, sz, ctx->s_buf[0])) return st;
    AC_HIP(ctx, hipStreamSynchronize(ctx->stream));
    const char* blk = (const char*)ctx->s_buf[0];
    size_t off = 0;
    const void* at[4];
    for (int i = 0; i < 4; ++i) {
        at[i] = blk + off;
        off += (sz[i] + 255) / 256 * 256;
    }
    dev->codes = (const uint32_t*)at[0];
    dev->nmask = (const uint32_t*)at[1];
    dev->start = (const uint64_t*)at[2];
    dev->length = (const uint32_t*)at[3];
    dev->n_windows = host->n_windows;
    dev->n_bases = host->n_bases;
    return AC_OK;
}

ac_status ac_exact_count_device(ac_ctx* ctx, uint32_t k, const ac_windows* dev, float lc_threshold,
                                const uint64_t* forbidden, uint32_t n_forbidden, uint64_t limit, uint64_t solid,
                                uint64_t* kmers_out, uint64_t* counts_out, uint64_t capacity, uint64_t* n_out,
                                uint64_t* n_distinct, uint64_t* had_n) {
    if (!ctx) return fail(nullptr, AC_ERR_INVALID, "ctx is NULL");
    if (ac_status st = check_k(ctx, k)) return st;
    if (ac_status st = check_sample(ctx, dev)) return st;
    if (!n_out || (capacity && (!kmers_out || !counts_out)) || (n_forbidden && !forbidden))
        return fail(ctx, AC_ERR_INVALID, "NULL output or forbidden array");
    AC_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    // Table: a power of two >= 1.5 x the image size (an upper bound on k-mer
    // positions): load <= 2/3 even when every position is a new k-mer.
    uint64_t slots = 1024;
    while (slots < dev->n_bases + dev->n_bases / 2) slots <<= 1;
    // Kept entries seen >= EXACT_LIST_MIN (2) times: at most n_bases / 2 (+ the all-T 32-mer).
    const uint64_t list_cap = dev->n_bases / 2 + 2;
    // small block: special[0..1] u32, had_n u64 @16, n_out u64 @24, n_list u64 @32, hist[EXACT_HIST_BINS] u32 @64
    const size_t small_bytes = 64 + sizeof(uint32_t) * EXACT_HIST_BINS;
    std::vector<uint64_t> fb(forbidden, forbidden + n_forbidden);
    std::sort(fb.begin(), fb.end());
    fb.erase(std::unique(fb.begin(), fb.end()), fb.end());
    // k <= 16: compact 8-byte slots (key and count in one word, exact_count.h)
    const bool compact = k <= acamd::EXACT_COMPACT_MAX_K;
    const size_t slot_bytes = compact ? sizeof(unsigned long long) : sizeof(acamd::ExactSlot);
    if (ac_status s2 = grow(ctx, &ctx->e_buf[0], &ctx->e_cap[0], slot_bytes * slots)) return s2;
    if (ac_status s2 = grow(ctx, &ctx->e_buf[1], &ctx->e_cap[1], (sizeof(uint64_t) + sizeof(uint32_t)) * list_cap))
        return s2;
    if (ac_status s2 = grow(ctx, &ctx->e_buf[2], &ctx->e_cap[2], small_bytes)) return s2;
    if (ac_status s2 = grow(ctx, &ctx->e_buf[3], &ctx->e_cap[3], sizeof(uint64_t) * std::max<size_t>(1, fb.size())))
        return s2;
    AC_HIP(ctx, hipMemsetAsync(ctx->e_buf[0], 0, slot_bytes * slots, st));
    AC_HIP(ctx, hipMemsetAsync(ctx->e_buf[2], 0, small_bytes, st));
    if (!fb.empty())
        AC_HIP(ctx, hipMemcpyAsync(ctx->e_buf[3], fb.data(), sizeof(uint64_t) * fb.size(), hipMemcpyHostToDevice, st));
    char* small = (char*)ctx->e_buf[2];
    acamd::ExactArgs a;
    std::memset(&a, 0, sizeof a);
    a.codes = dev->codes;
    a.nmask = dev->nmask;
    a.start = dev->start;
    a.length = dev->length;
    a.n_bases = dev->n_bases;
    a.n_windows = dev->n_windows;
    a.k = k;
    a.table = (acamd::ExactSlot*)ctx->e_buf[0];
    a.ctable = (unsigned long long*)ctx->e_buf[0];
    a.compact = compact ? 1u : 0u;
    a.slots = slots;
    a.mask = slots - 1;
    a.special = (uint32_t*)small;
    a.had_n = (unsigned long long*)(small + 16);
    a.n_out = (unsigned long long*)(small + 24);
    a.n_list = (unsigned long long*)(small + 32);
    a.hist = (uint32_t*)(small + 64);
    a.list_keys = (uint64_t*)ctx->e_buf[1];
    a.list_cnts = (uint32_t*)((char*)ctx->e_buf[1] + sizeof(uint64_t) * list_cap);
    a.list_cap = list_cap;
    a.lc_threshold = lc_threshold;
    a.forbidden = (const uint64_t*)ctx->e_buf[3];
    a.n_forbidden = (uint32_t)fb.size();
    AC_HIP(ctx, acamd::launch_exact_insert(a, st));
    AC_HIP(ctx, acamd::launch_exact_scan(a, st));
    std::vector<char> h_small(small_bytes);
    AC_HIP(ctx, hipMemcpyAsync(h_small.data(), small, small_bytes, hipMemcpyDeviceToHost, st));
    AC_HIP(ctx, hipStreamSynchronize(st));
    const uint32_t* hist = (const uint32_t*)(h_small.data() + 64);
    uint64_t kept = 0;
    for (int i = 0; i < EXACT_HIST_BINS; ++i) kept += hist[i];
    if (n_distinct) *n_distinct = kept;
    if (had_n) *had_n = *(const unsigned long long*)(h_small.data() + 16);
    const uint64_t n_list = *(const unsigned long long*)(h_small.data() + 32);
    if (n_list > list_cap) return fail(ctx, AC_ERR_INTERNAL, "exact count: candidate list overflow");
    // Threshold: solid mode keeps count >= solid; otherwise the largest count c
    // such that at least `limit` kept entries have count >= c (all if fewer).
    uint64_t thr = 1, due = kept;
    if (solid) {
        thr = solid;
        due = 0;
        for (uint64_t c = std::min<uint64_t>(solid, EXACT_HIST_BINS - 1); c < EXACT_HIST_BINS; ++c) due += hist[c];
    } else if (limit < kept) {
        uint64_t acc = 0;
        for (int c = EXACT_HIST_BINS - 1; c >= 1; --c) {
            acc += hist[c];
            if (acc >= limit) {
                thr = (uint64_t)c;
                due = acc;
                break;
            }
        }
    }
    // (a solid threshold past the last bin is applied exactly on the gathered list)
    const uint64_t gather_cap = std::max<uint64_t>(1, due);
    if (ac_status s2 = grow(ctx, &ctx->e_buf[4], &ctx->e_cap[4], sizeof(uint64_t) * gather_cap)) return s2;
    if (ac_status s2 = grow(ctx, &ctx->e_buf[5], &ctx->e_cap[5], sizeof(uint32_t) * gather_cap)) return s2;
    a.threshold = (uint32_t)std::min<uint64_t>(thr, 0xffffffffu);
    a.out_keys = (uint64_t*)ctx->e_buf[4];
    a.out_cnts = (uint32_t*)ctx->e_buf[5];
    a.out_cap = gather_cap;
    AC_HIP(ctx, acamd::launch_exact_gather(a, thr >= EXACT_LIST_MIN, n_list, st));
    unsigned long long got = 0;
    AC_HIP(ctx, hipMemcpyAsync(&got, a.n_out, sizeof got, hipMemcpyDeviceToHost, st));
    AC_HIP(ctx, hipStreamSynchronize(st));
    if (got > gather_cap) return fail(ctx, AC_ERR_INTERNAL, "exact count: gathered more entries than the histogram");
    std::vector<uint64_t> gk(got);
    std::vector<uint32_t> gc(got);
    if (got) {
        AC_HIP(ctx, hipMemcpyAsync(gk.data(), a.out_keys, sizeof(uint64_t) * got, hipMemcpyDeviceToHost, st));
        AC_HIP(ctx, hipMemcpyAsync(gc.data(), a.out_cnts, sizeof(uint32_t) * got, hipMemcpyDeviceToHost, st));
        AC_HIP(ctx, hipStreamSynchronize(st));
    }
    struct Entry {
        uint64_t count, kmer;
        float comp;
    };
    std::vector<Entry> v;
    v.reserve(got);
    for (uint64_t i = 0; i < got; ++i)
        if (!solid || gc[i] >= solid) v.push_back({gc[i], gk[i], complexity(gk[i], k)});
    auto less = [](const Entry& x, const Entry& y) {  // CompareCount: a strict total order
        if (x.count != y.count) return x.count > y.count;
        if (x.comp != y.comp) return x.comp < y.comp;
        return x.kmer > y.kmer;
    };
    const size_t n = solid ? v.size() : std::min<size_t>(v.size(), limit);
    std::partial_sort(v.begin(), v.begin() + n, v.end(), less);
    *n_out = n;
    if (n > capacity) return fail(ctx, AC_ERR_INVALID, "exact count: capacity too small (n_out holds the size needed)");
    for (size_t i = 0; i < n; ++i) {
        kmers_out[i] = v[i].kmer;
        counts_out[i] = v[i].count;
    }
    return AC_OK;
}

ac_status ac_exact_count(ac_ctx* ctx, uint32_t k, const ac_windows* host, float lc_threshold,
                         const uint64_t* forbidden, uint32_t n_forbidden, uint64_t limit, uint64_t solid,
                         uint64_t* kmers_out, uint64_t* counts_out, uint64_t capacity, uint64_t* n_out,
                         uint64_t* n_distinct, uint64_t* had_n) {
    if (!ctx) return fail(nullptr, AC_ERR_INVALID, "ctx is NULL");
    if (ac_status st = check_k(ctx, k)) return st;
    ac_windows dev;
    if (ac_status st = ac_sample_upload(ctx, host, &dev)) return st;
    return ac_exact_count_device(ctx, k, &dev, lc_threshold, forbidden, n_forbidden, limit, solid, kmers_out,
                                 counts_out, capacity, n_out, n_distinct, had_n);
}

ac_status ac_error_count_sample(ac_ctx* ctx, uint32_t k, const uint64_t* kmers, uint32_t n_kmers,
                                const ac_windows* dev, uint64_t* counts) {
    if (!ctx) return fail(nullptr, AC_ERR_INVALID, "ctx is NULL");
    if (ac_status st = check_k(ctx, k)) return st;
    if (n_kmers == 0) return AC_OK;
    if (!kmers || !counts) return fail(ctx, AC_ERR_INVALID, "NULL argument");
    if (ac_status st = check_sample(ctx, dev)) return st;
    AC_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    if (ac_status s2 = ensure(ctx, 0, sizeof(uint64_t) * n_kmers)) return s2;
    if (ac_status s2 = ensure(ctx, 5, sizeof(uint32_t) * n_kmers)) return s2;
    AC_HIP(ctx, hipMemcpyAsync(ctx->d_buf[0], kmers, sizeof(uint64_t) * n_kmers, hipMemcpyHostToDevice, st));
    ac_segment seg;
    seg.kmers = (const uint64_t*)ctx->d_buf[0];
    seg.n_kmers = n_kmers;
    seg.sample = *dev;
    seg.counts = (uint32_t*)ctx->d_buf[5];
    if (ac_status rc = launch(ctx, k, &seg, 1, st, true)) return rc;
    ctx->h_counts.resize(n_kmers);
    AC_HIP(ctx, hipMemcpyAsync(ctx->h_counts.data(), ctx->d_buf[5], sizeof(uint32_t) * n_kmers, hipMemcpyDeviceToHost, st));
    AC_HIP(ctx, hipStreamSynchronize(st));
    for (uint32_t i = 0; i < n_kmers; ++i) counts[i] = ctx->h_counts[i];
    return AC_OK;
}

ac_status ac_last_launch(const ac_ctx* ctx, uint64_t* waves, uint32_t* windows_per_wave, uint32_t* groups) {
    if (!ctx) return fail(nullptr, AC_ERR_INVALID, "ctx is NULL");
    if (waves) *waves = ctx->last_waves;
    if (windows_per_wave) *windows_per_wave = ctx->last_wpw;
    if (groups) *groups = ctx->last_groups;
    return AC_OK;
}

uint64_t ac_image_bases(const uint32_t* seq_len, uint32_t n) {
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; ++i) total += ((uint64_t)seq_len[i] + 31) / 32 * 32;
    return total ? total : 32;
}

ac_status ac_pack_windows(const uint8_t* dna5, const uint64_t* seq_start, const uint32_t* seq_len, uint32_t n,
                          uint32_t* codes, uint32_t* nmask, uint64_t* start, uint32_t* length, uint64_t n_bases) {
    if (n && (!dna5 || !seq_start || !seq_len || !start || !length))
        return fail(nullptr, AC_ERR_INVALID, "NULL argument");
    if (!codes || !nmask) return fail(nullptr, AC_ERR_INVALID, "NULL image");
    if (n_bases % 32 || n_bases < ac_image_bases(seq_len, n))
        return fail(nullptr, AC_ERR_INVALID, "image too small (use ac_image_bases)");
    std::memset(codes, 0, sizeof(uint32_t) * (n_bases / 16));
    std::memset(nmask, 0, sizeof(uint32_t) * (n_bases / 32));
    uint64_t pos = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint8_t* src = dna5 + seq_start[i];
        const uint32_t len = seq_len[i];
        start[i] = pos;
        length[i] = len;
        for (uint32_t j = 0; j < len; ++j) {
            const uint64_t b = pos + j;
            const uint8_t v = src[j];
            if (v < 4) codes[b >> 4] |= (uint32_t)v << (2 * (b & 15));
            else nmask[b >> 5] |= 1u << (b & 31);
        }
        pos += ((uint64_t)len + 31) / 32 * 32;
    }
    return AC_OK;
}

#ifdef AC_STAMPS
// Diagnostic builds only: per-wave timestamps of the last launch (not declared in the public header).
int ac_debug_stamps(void* host, size_t bytes) { return (int)acamd::debug_stamps(host, bytes); }
#endif

}  // extern "C"
