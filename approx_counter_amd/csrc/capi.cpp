// capi.cpp -- C ABI of the MI355X approximate-count stage (include/approx_counter_amd.h).
//
// Replaces errorCount (approx_counter.cpp:531-601): where the reference builds
// a bidirectional FM index over the sample (537-541) and runs SeqAn's
// find<0,2> per candidate under OpenMP (547-599), this layer uploads the
// packed sample once per call and launches one HIP kernel over the
// candidate x window grid.
#include <dlfcn.h>
#include <sched.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // types only: RCCL is resolved at run time (rccl() below)

#include <algorithm>
#include <cctype>
#include <cmath>
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <memory>
#include <mutex>
#include <vector>

#include "approx_counter_amd.h"
#include "approx_counter_amd_testing.h"
#include "exact_count.h"
#include "host_pack.h"
#include "wm_count.h"

static_assert(AC_MAX_JOBS <= AC_MAX_SEGS, "every job of ac_error_count_jobs is one segment of one launch");

// A synchronous jobs call is cut into up to this many parts (window ranges of
// every job), each packed, sent and counted on its own stream, so a part's
// packing and DMA overlap the previous part's kernel.
#define AC_STAGE_MAX_PARTS 4

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
    // what the upload found about each slot's image: equal windows back to back (their length,
    // else AC_NO_ULEN) and no N anywhere, so the count launch can take the EQ kernel and skip the
    // N bitmap; keyed by the device image it describes
    const uint32_t* s_codes[4] = {nullptr, nullptr, nullptr, nullptr};
    const uint64_t* s_start[4] = {nullptr, nullptr, nullptr, nullptr};
    uint32_t s_ulen[4] = {AC_NO_ULEN, AC_NO_ULEN, AC_NO_ULEN, AC_NO_ULEN};
    bool s_no_n[4] = {false, false, false, false};
    uint64_t s_windows[4] = {0, 0, 0, 0}, s_bases[4] = {0, 0, 0, 0};
    // (+ the partitioned path's keys, parts, tmp, h1/h2/stot, bstart, phist: e_buf[6..11]; the forbidden
    // set by bucket and its bucket starts: e_buf[12..13])
    void* e_buf[14] = {};
    size_t e_cap[14] = {};
    // the exact count's readbacks (the small block, the list count, the gathered entries): pinned, so each
    // is one DMA into place instead of a copy through HIP's staging buffer (32 KB + 16 MB, at the first call)
    char* e_pin = nullptr;
    size_t e_pin_cap = 0;
    // Count-kernel scratch, one set per stream a launch may run on at the same
    // time as another: the parts of a synchronous jobs call (0 .. MAX_PARTS-1),
    // the parts of a submit (MAX_PARTS ..), so a synchronous call never shares
    // queues / sums / tickets with a submit still in flight on another stream.
    struct Scratch {
        // work-queue counters: two banks of qcap u32; dirty[b] =
        // counters of bank b used by the last launch on it (zeroed by the next launch)
        uint32_t* queue = nullptr;
        uint32_t qcap = 0, bank = 0, dirty[2] = {0, 0};
        // count hand-off scratch: per-slot arrivals and sums, (workgroups << 32) + sum (zero between launches)
        uint64_t* acc = nullptr;
        uint32_t acc_cap = 0;
        // staged launches: per-chunk "copied" flags (= the launch's generation once in device memory)
        uint32_t* stage_gen = nullptr;
        uint32_t stage_gen_cap = 0;
    } sc[2 * AC_STAGE_MAX_PARTS];
    // streams of parts 1.. of a synchronous jobs call (part 0 runs on `stream`)
    // and of a submit (part 0 runs on the caller's stream), with the events that
    // order a submit's parts around the caller's stream
    hipStream_t part_stream[AC_STAGE_MAX_PARTS] = {};
    hipStream_t sub_stream[AC_STAGE_MAX_PARTS] = {};
    hipEvent_t sub_ev[AC_STAGE_MAX_PARTS] = {};
    hipEvent_t sub_zero_ev = nullptr;
    // resident waves of the count kernel per pattern pack P (0 = not queried yet)
    uint32_t resident[2][AC_MAX_PACK + 1] = {};  // [staged][P]
    // last launch geometry
    uint64_t last_waves = 0;
    uint32_t last_wpw = 0, last_groups = 0;
    // ac_create_multi: contexts of shards 1..n-1 (this context is shard 0)
    std::vector<ac_ctx*> peers;
    // RCCL communicator of a multi-process job (ac_comm_init), or null
    ncclComm_t comm = nullptr;
    // device error word of the asynchronous entry points (ac_check), and a
    // pinned word to read it back through
    uint32_t* d_err = nullptr;
    uint32_t* h_err = nullptr;
    // ac_error_count_jobs staging: two slots used alternately, so a submit
    // packs into one while the previous launch still reads the other.  Each is
    // a pinned host block, a device block (same layout) and an event recorded
    // after the last stream work that reads either.
    struct Slot {
        void* h = nullptr;
        void* d = nullptr;
        void* hd = nullptr;  // device address of the pinned block (staging reads, counts written back)
        size_t h_cap = 0, d_cap = 0;
        hipEvent_t ev = nullptr;
        bool pending = false;
        // the early launch's header (flags, completion): coherent (fine-grained) pinned memory, so
        // the kernel's polls of it reach host memory every time instead of an L2 line
        uint32_t* hdr = nullptr;
        uint32_t* hdr_d = nullptr;
    } slot[3 * AC_STAGE_MAX_PARTS];  // synchronous parts, then two sets of submit parts
    uint32_t next_slot = 0;          // the submit set the next submit uses
    uint32_t gen = 0;                // generation of the last early-launch call (never 0 once used)
    uint32_t early_flip = 0;         // early-launch calls alternate between staging slots 0 and 1
    int exact_path = -1;             // the last exact count's path: 1 partitioned, 0 hash table
    int last_mode = -1;  // ac_stage_mode: 2 the last jobs call was an early launch, 0 the DMA path
    // Warm-up started by ac_create on a thread of its own (ensure_warm joins it before the first count
    // launch): the count kernels' code object is loaded by the occupancy queries, so the first launch
    // -- the CLI's one approximate count per run -- does not pay for it; it overlaps the caller's FASTA
    // parsing and exact count instead.
    std::thread warm;
    uint32_t warm_resident[2][AC_MAX_PACK + 1] = {};
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
inline size_t align256(size_t x) { return (x + 255) / 256 * 256; }

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
    if (s->n_bases % 32 || s->n_bases >= AC_MAX_IMAGE_BASES)
        return fail(ctx, AC_ERR_INVALID, "sample n_bases must be a multiple of 32 below 2^34");
    if (s->n_windows && (!s->codes || !s->nmask || !s->start || !s->length))
        return fail(ctx, AC_ERR_INVALID, "sample has a NULL array");
    return AC_OK;
}

// Every window inside the image and 32-aligned, written so that no sum can
// wrap: a start near 2^64 must not pass as "start + length <= n_bases".
inline bool window_ok(uint64_t start, uint32_t length, uint64_t n_bases) {
    return start % 32 == 0 && length <= n_bases && start <= n_bases - length;
}

// Status for a device error word read back after a launch (wm_count.h).
ac_status device_error(ac_ctx* ctx, uint32_t word) {
    if (word & AC_DEVERR_STAGE)
        return fail(ctx, AC_ERR_INTERNAL, "early launch: the kernel timed out waiting for the host's packed inputs");
    if (word & AC_DEVERR_SETUP)
        return fail(ctx, AC_ERR_INTERNAL, "count kernel set-up fault (~Eq table not at LDS 0): its work was skipped");
    if (word & AC_DEVERR_WINDOW)
        return fail(ctx, AC_ERR_INVALID,
                    "malformed window skipped on the device (misaligned start or past n_bases): counts are short");
    return AC_OK;
}

ac_status check_layout(ac_ctx* ctx, const ac_windows& s) {
    for (uint32_t i = 0; i < s.n_windows; ++i)
        if (!window_ok(s.start[i], s.length[i], s.n_bases))
            return fail(ctx, AC_ERR_INVALID, "window " + std::to_string(i) + " is misaligned or outside the image");
    return AC_OK;
}

// One fused count launch over `n` device segments.  `err` = the device word
// the kernel reports skipped windows in (the context's, for ac_check, when NULL).
// `sc` = the scratch set (one per concurrently running stream); `wave_cap` (0
// = none) limits the launch to that many waves, so another launch's waves can
// be resident beside it.
// `no_n` (optional, per segment): the segment's image is known to hold no N.
// `ulen` (optional, per segment): AC_NO_ULEN, or all windows have this length
// and sit back to back at ceil32(ulen)-base strides (start / length unread).
// `nrec` (optional, per equal-window segment): its windows carry inline N records (nrec.h).
// Staged launch (the early-launch stage): the kernel copies each
// segment's region from src (the pinned block) to dst once the host flags it in
// host_hdr, and reports its completion there.
// Copier workgroups of a large staged launch (AC_COPIER_WGS overrides, for A/B runs): 16 = 2 per XCD,
// 4 CUs' worth of resident slots, 64 waves, enough to keep the AC_COPY_AHEAD window of chunk reads in
// flight over PCIe.
uint32_t stage_copier_wgs() {
    static const uint32_t v = [] {
        const char* e = std::getenv("AC_COPIER_WGS");
        return e ? (uint32_t)std::max(1, std::atoi(e)) : 16u;
    }();
    return v;
}

struct StageLaunch {
    uint32_t gen = 0;
    uint32_t* host_hdr = nullptr;
    const uint8_t* src[AC_MAX_SEGS] = {};
    uint8_t* dst[AC_MAX_SEGS] = {};
    uint32_t chunks[AC_MAX_SEGS] = {};
    uint32_t codes_off[AC_MAX_SEGS] = {};  // bytes of the region before its codes (the k-mers section)
    uint32_t* err_out = nullptr;  // device word the launch's error bits are also or-ed into (submits: ac_check)
    uint32_t tag = 0;              // tagged completion (wm_count.h LaunchArgs::tag)
    uint64_t* grp_err = nullptr;   // its per-group error words (device-visible pinned address)
    uint32_t copiers = 0;          // copier workgroups (wm_count.h LaunchArgs::copier_wgs; 0: nothing to stage)
    // device packing (wm_count.h SegDev::dp_*): the segment's Dna5 bytes and window offsets in
    // pinned host memory, device-visible addresses; dp_src = NULL: the host packed the segment
    const uint8_t* dp_src[AC_MAX_SEGS] = {};
    const uint64_t* dp_off[AC_MAX_SEGS] = {};
    uint32_t dp_bytes[AC_MAX_SEGS] = {};
};

// Who stages a staged launch (wm_count.h LaunchArgs::copier_wgs): a few copier workgroups stage
// every chunk while the others count as chunks land.  Round 3 let every workgroup's wave 0 claim
// tickets instead: fine while a call's chunks are packed within microseconds of the launch, but each
// such wave held its workgroup's other three waves at the table barrier until its chunk was in (the
// p90 workgroup started counting ~30 us into a cfg2 launch, profiles/r04_m1/stamps_staged.log), and a
// large call's chunks arrive over the whole packing time.  Copier workgroups at cfg2: stage p50
// 0.1143-0.1146 vs 0.1189-0.1193 ms (same box, profiles/r04_m7/ab_table.txt); the round-3 scheme was
// removed in round 5.
uint32_t stage_copiers(uint64_t tickets) { return tickets ? stage_copier_wgs() : 0u; }

// Joins ac_create's warm-up thread (once) and takes the resident-wave counts it queried.
void ensure_warm(ac_ctx* ctx) {
    if (!ctx->warm.joinable()) return;
    ctx->warm.join();
    for (int st = 0; st < 2; ++st)
        for (uint32_t P = 1; P <= AC_MAX_PACK; ++P)
            if (!ctx->resident[st][P]) ctx->resident[st][P] = ctx->warm_resident[st][P];
}

ac_status launch(ac_ctx* ctx, uint32_t k, const ac_segment* segs, uint32_t n, hipStream_t stream,
                 bool zero, uint32_t* err = nullptr, int scratch = 0, uint64_t wave_cap = 0,
                 const bool* no_n = nullptr, const uint32_t* ulen = nullptr, const StageLaunch* stage = nullptr,
                 const bool* nrec = nullptr) {
    ensure_warm(ctx);
    ac_ctx::Scratch& sc = ctx->sc[scratch];
    if (ac_status st = check_k(ctx, k)) return st;
    if (n > AC_MAX_SEGS) return fail(ctx, AC_ERR_INVALID, "too many segments in one launch (max 4)");
    if (n && !segs) return fail(ctx, AC_ERR_INVALID, "segments is NULL");
    const uint32_t P = acamd::pack_factor(k);
    const bool staged = stage != nullptr;
    const uint32_t cpw = acamd::cands_per_wave(P, staged);
    acamd::LaunchArgs a;
    std::memset(&a, 0, sizeof a);
    a.n_segs = n;
    a.m = k;
    a.P = P;
    uint64_t items = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const ac_segment& s = segs[i];
        if (s.n_kmers && (!s.kmers || !s.counts)) return fail(ctx, AC_ERR_INVALID, "segment kmers/counts is NULL");
        const bool equal = ulen && ulen[i] != AC_NO_ULEN;  // windows back to back at ceil32(ulen[i])
        if (s.n_kmers && s.sample.n_windows &&
            (!s.sample.codes || !s.sample.nmask || (!equal && (!s.sample.start || !s.sample.length))))
            return fail(ctx, AC_ERR_INVALID, "segment sample has a NULL array");
        if (equal && (uint64_t)s.sample.n_windows * ((ulen[i] + 31ull) & ~31ull) > s.sample.n_bases)
            return fail(ctx, AC_ERR_INVALID, "equal windows reach past n_bases");
        if (s.sample.n_bases % 32 || s.sample.n_bases >= AC_MAX_IMAGE_BASES)
            return fail(ctx, AC_ERR_INVALID, "sample n_bases must be a multiple of 32 below 2^34");
        // The count hand-off adds (1 << 32) + sum into 64-bit slots (wm_count.hip): a candidate's sum,
        // at most 3 per window, must stay below 2^32 or its carry would count as an arrival and the
        // slot would never see its last workgroup.
        if (s.n_kmers && 3ull * s.sample.n_windows >= (1ull << 32))
            return fail(ctx, AC_ERR_INVALID, "a segment of 2^32 / 3 windows or more: its counts would overflow");
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
    uint32_t& res_p = ctx->resident[staged][P];
    if (!res_p) AC_HIP(ctx, acamd::resident_waves(P, staged, ctx->cu_count, &res_p));
    const uint64_t resident = wave_cap ? std::max<uint64_t>(AC_WAVES_PER_BLOCK, std::min<uint64_t>(wave_cap, res_p) /
                                                                  AC_WAVES_PER_BLOCK * AC_WAVES_PER_BLOCK)
                                       : res_p;
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
#ifndef AC_SUBQ_WAVES
#define AC_SUBQ_WAVES 64  // waves per sub-queue (16 / 32 / 128 measured equal or slower, profiles/r05_m36)
#endif
    const uint64_t s_base = std::max<uint64_t>(
        1, std::min<uint64_t>(32, resident / ((uint64_t)AC_SUBQ_WAVES * std::max(1u, groups_live))));
    uint64_t wave = 0;
    uint32_t groups_total = 0, qbegin = 0, acc_slots = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const ac_segment& s = segs[i];
        acamd::SegDev& d = a.seg[i];
        d.kmers = s.kmers;
        d.codes = s.sample.codes;
        d.nmask = s.sample.nmask;
        d.has_n = (no_n && no_n[i]) ? 0u : 1u;
        d.ulen = ulen ? ulen[i] : AC_NO_ULEN;
        d.nrec = (nrec && nrec[i] && d.ulen != AC_NO_ULEN) ? acamd::nrec_bits(d.ulen) : 0u;
        d.start = s.sample.start;
        d.length = s.sample.length;
        d.n_bases = s.sample.n_bases;
        d.counts = s.counts;
        if (stage) {
            d.stage_src = stage->src[i];
            d.stage_dst = stage->dst[i];
            d.stage_chunks = stage->chunks[i];
            d.stage_codes_off = stage->codes_off[i];
            d.dp_src = stage->dp_src[i];
            d.dp_off = stage->dp_off[i];
            d.dp_src_bytes = stage->dp_bytes[i];
        }
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
        d.group_begin = groups_total;
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
    a.add_counts = (!zero || alias) ? 1u : 0u;
    if (zero && alias)
        for (uint32_t i = 0; i < n; ++i)
            if (a.seg[i].queue_begin != ~0u)
                AC_HIP(ctx, hipMemsetAsync(a.seg[i].counts, 0, sizeof(uint32_t) * a.seg[i].n_kmers, stream));
    if (acc_slots > sc.acc_cap) {
        if (sc.acc) AC_HIP(ctx, hipFree(sc.acc));
        sc.acc = nullptr;
        sc.acc_cap = 0;
        AC_HIP(ctx, hipMalloc(&sc.acc, sizeof(uint64_t) * acc_slots));
        AC_HIP(ctx, hipMemsetAsync(sc.acc, 0, sizeof(uint64_t) * acc_slots, stream));
        sc.acc_cap = acc_slots;
    }
    a.acc = sc.acc;
    a.err = err ? err : ctx->d_err;
    const uint32_t n_counters = qbegin;
    if (n_counters) wave = std::max<uint64_t>(resident, n_counters);
    // a staged launch's device words follow its sub-queue counters in the bank (zeroed with them)
    const uint32_t used = n_counters + (stage ? AC_STAGE_LINES : 0u);
    if (used > sc.qcap) {
        if (sc.queue) AC_HIP(ctx, hipFree(sc.queue));
        sc.queue = nullptr;
        sc.qcap = 0;
        const uint32_t cap = std::max<uint32_t>(used, 1024);
        const size_t bytes = sizeof(uint32_t) * AC_QUEUE_LINE * 2 * (size_t)cap;
        AC_HIP(ctx, hipMalloc(&sc.queue, bytes));
        AC_HIP(ctx, hipMemsetAsync(sc.queue, 0, bytes, stream));
        sc.qcap = cap;
        sc.bank = 0;
        sc.dirty[0] = sc.dirty[1] = 0;
    }
    a.queue = sc.queue;
    a.qstride = sc.qcap;
    a.bank = sc.bank;
    a.zero_count = sc.dirty[sc.bank ^ 1u];
    a.n_queues = std::max<uint32_t>(1, n_counters);
    if (stage) {
        uint32_t total_chunks = 0;
        for (uint32_t i = 0; i < n; ++i) total_chunks += stage->chunks[i];
        if (total_chunks > sc.stage_gen_cap) {  // (zeroed once: generations are never 0)
            if (sc.stage_gen) AC_HIP(ctx, hipFree(sc.stage_gen));
            sc.stage_gen = nullptr;
            sc.stage_gen_cap = 0;
            const uint32_t cap = std::max<uint32_t>(total_chunks, 1024);
            const size_t bytes = sizeof(uint32_t) * AC_QUEUE_LINE * (size_t)cap;  // one line per chunk flag
            AC_HIP(ctx, hipMalloc(&sc.stage_gen, bytes));
            AC_HIP(ctx, hipMemsetAsync(sc.stage_gen, 0, bytes, stream));
            sc.stage_gen_cap = cap;
        }
        uint32_t off = 0;
        for (uint32_t i = 0; i < n; ++i) {
            a.seg[i].stage_gen = sc.stage_gen + (size_t)off * AC_QUEUE_LINE;
            off += stage->chunks[i];
        }
        a.staged = 1;
        a.gen = stage->gen;
        a.host_hdr = stage->host_hdr;
        a.stage = sc.queue + ((uint64_t)sc.bank * sc.qcap + n_counters) * AC_QUEUE_LINE;
        a.err = a.stage + AC_STAGE_L_ERR * AC_QUEUE_LINE;
        a.err_out = stage->err_out;
        a.tag = stage->tag;
        a.grp_err = stage->grp_err;
        const uint64_t blocks = (wave + AC_WAVES_PER_BLOCK - 1) / AC_WAVES_PER_BLOCK;
        a.copier_wgs = (uint32_t)std::min<uint64_t>(blocks, stage->copiers);
    }
    // the equal-window instantiation when every live segment has equal windows (their fit in the
    // image checked above)
    a.eq = 1u;
    for (uint32_t i = 0; i < n; ++i)
        if (a.seg[i].queue_begin != ~0u && a.seg[i].ulen == AC_NO_ULEN) a.eq = 0u;
    // Live segments' queue_begin values are increasing; the kernel picks the
    // last live segment whose queue_begin <= its sub-queue.
    a.total_waves = wave;
    ctx->last_waves = wave;
    ctx->last_wpw = wpw;
    ctx->last_groups = groups_total;
    AC_HIP(ctx, acamd::launch_wm2_count(a, stream));
    if (wave) {  // the launch dequeued from `bank` and zeroed the other one
        sc.dirty[sc.bank] = used;
        sc.dirty[sc.bank ^ 1u] = 0;
        sc.bank ^= 1u;
    }
    return AC_OK;
}

}  // namespace

// RCCL for the multi-process path (ac_comm_*): resolved at run time with dlopen, so the
// library itself does not depend on it; an RCCL already in the process (torch's) is reused.
namespace {
struct Rccl {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    std::string err;  // empty when usable
};
const Rccl& rccl() {
    static const Rccl r = [] {
        Rccl x;
        void* h = nullptr;
        for (const char* name : {"librccl.so.1", "librccl.so"})
            if (!h) h = dlopen(name, RTLD_NOW | RTLD_NOLOAD);
        for (const char* name : {"librccl.so.1", "librccl.so"})
            if (!h) h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            const char* e = dlerror();
            x.err = std::string("RCCL (librccl.so) could not be loaded: ") + (e ? e : "?");
            return x;
        }
        x.get_unique_id = (decltype(x.get_unique_id))dlsym(h, "ncclGetUniqueId");
        x.comm_init_rank = (decltype(x.comm_init_rank))dlsym(h, "ncclCommInitRank");
        x.all_reduce = (decltype(x.all_reduce))dlsym(h, "ncclAllReduce");
        x.comm_destroy = (decltype(x.comm_destroy))dlsym(h, "ncclCommDestroy");
        x.error_string = (decltype(x.error_string))dlsym(h, "ncclGetErrorString");
        if (!x.get_unique_id || !x.comm_init_rank || !x.all_reduce || !x.comm_destroy || !x.error_string)
            x.err = "RCCL is missing one of ncclGetUniqueId / ncclCommInitRank / ncclAllReduce / ncclCommDestroy";
        return x;
    }();
    return r;
}
}  // namespace

namespace {

// CPUs local to a device's PCIe root (sysfs local_cpulist), empty if unknown.
std::vector<int> device_local_cpus(int device) {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof bus, device) != hipSuccess) return {};
    for (char* c = bus; *c; ++c) *c = (char)std::tolower((unsigned char)*c);
    const std::string path = std::string("/sys/bus/pci/devices/") + bus + "/local_cpulist";
    return acamd::read_cpulist(path.c_str());
}

std::vector<int> allowed_cpus() {
    std::vector<int> out;
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) != 0) return out;
    for (int c = 0; c < CPU_SETSIZE; ++c)
        if (CPU_ISSET(c, &set)) out.push_back(c);
    return out;
}

int env_int(const char* name, int dflt) {
    const char* e = std::getenv(name);
    return e && *e ? std::atoi(e) : dflt;
}

// The host pool's CPUs, once per process, before its first use: it packs into
// memory this GPU reads, so it runs on the CPUs local to the GPU's PCIe root.
// One process per GPU (torchrun: LOCAL_RANK / LOCAL_WORLD_SIZE, local rank r
// on device r mod the visible devices): the local ranks whose GPUs share a
// CPU list split it into disjoint runs of physical cores, and each rank's pool
// takes at most its share of the cgroup CPU quota minus headroom (below; 16
// participants at most), so 8 ranks on one node never pin their workers onto the
// same CPUs nor spin more threads than the quota runs.  (The reference sizes its one OpenMP team
// with omp_set_num_threads(nb_thread), approx_counter.cpp:547.)
void plan_host_pool(int device, int n_dev) {
    if (acamd::host_plan().participants) return;  // set already (ac_set_host_cpus or an earlier context)
    int lws = env_int("LOCAL_WORLD_SIZE", 1), lr = env_int("LOCAL_RANK", 0);
    if (lws < 1 || lr < 0 || lr >= lws) lws = 1, lr = 0;
    std::vector<std::vector<int>> lists((size_t)lws);
    for (int r = 0; r < lws; ++r) lists[(size_t)r] = r == lr ? device_local_cpus(device) : device_local_cpus(r % n_dev);
    const std::vector<int> allowed = allowed_cpus();
    bool shared = false;
    acamd::HostPlan plan;
    plan.cpus = acamd::plan_host_cpus(lists, lr, allowed, acamd::sysfs_core_of, &shared);
    size_t n = plan.cpus.empty() ? allowed.size() : plan.cpus.size();
    // Headroom under the quota: a pool of all of it (16 participants spinning on a 16-CPU quota, with
    // Python's and the HIP runtime's threads beside them) was throttled in 91 of 100 CFS periods of a
    // 10-s cfg2 run (191 ms throttled, 59 of its 60 steps over 2x p50 inside throttled periods; 14
    // participants: none, p50 equal; profiles/r06_m3/stall_*.log): 2 CPUs of headroom above a share
    // of 4, 1 below.
    const double quota = acamd::cgroup_cpu_quota();
    if (quota > 0.0) {
        const double share = quota / lws;
        n = std::min<size_t>(n, (size_t)std::max(1.0, std::floor(share) - (share > 4.0 ? 2.0 : 1.0)));
    }
    plan.participants = shared ? 1u : (unsigned)std::max<size_t>(1, std::min<size_t>(16, n));
    (void)acamd::set_host_plan(plan);
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
    plan_host_pool(device, n);
    if ((e = hipMalloc(&ctx->d_err, sizeof(uint32_t))) != hipSuccess ||
        (e = hipMemset(ctx->d_err, 0, sizeof(uint32_t))) != hipSuccess ||
        (e = hipHostMalloc(&ctx->h_err, sizeof(uint32_t), hipHostMallocDefault)) != hipSuccess) {
        ac_status st = hip_fail(nullptr, e, "device setup");
        ac_destroy(ctx);
        return st;
    }
    // (a query that fails leaves its count 0: launch() queries again and reports the error there)
    // The warm-up also allocates the first scratch set at the sizes a few-candidate-group launch needs
    // (it grows on demand later), so that launch does not wait for allocations either.
    ctx->warm = std::thread([ctx] {
        if (hipSetDevice(ctx->device) != hipSuccess) return;
        for (uint32_t P = 1; P <= AC_MAX_PACK; ++P)
            for (int st = 0; st < 2; ++st)
                (void)acamd::resident_waves(P, st != 0, ctx->cu_count, &ctx->warm_resident[st][P]);
        ac_ctx::Scratch& sc = ctx->sc[0];
        auto zeroed = [](void** p, size_t bytes) {
            if (hipMalloc(p, bytes) != hipSuccess) return false;
            if (hipMemset(*p, 0, bytes) == hipSuccess) return true;
            (void)hipFree(*p);
            *p = nullptr;
            return false;
        };
        constexpr uint32_t QCAP = 2048, ACC = 64 * 256, CHUNKS = 1024;
        if (zeroed((void**)&sc.queue, sizeof(uint32_t) * AC_QUEUE_LINE * 2 * QCAP)) sc.qcap = QCAP;
        if (zeroed((void**)&sc.acc, sizeof(uint64_t) * ACC)) sc.acc_cap = ACC;
        if (zeroed((void**)&sc.stage_gen, sizeof(uint32_t) * AC_QUEUE_LINE * CHUNKS)) sc.stage_gen_cap = CHUNKS;
    });
    *out = ctx;
    return AC_OK;
}

void ac_destroy(ac_ctx* ctx) {
    if (!ctx) return;
    if (ctx->warm.joinable()) ctx->warm.join();
    for (ac_ctx* p : ctx->peers) ac_destroy(p);
    (void)hipSetDevice(ctx->device);
    if (ctx->comm) (void)rccl().comm_destroy(ctx->comm);
    for (void* p : ctx->d_buf)
        if (p) (void)hipFree(p);
    if (ctx->d_stage) (void)hipFree(ctx->d_stage);
    if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
    for (auto& sc : ctx->sc) {
        if (sc.queue) (void)hipFree(sc.queue);
        if (sc.acc) (void)hipFree(sc.acc);
        if (sc.stage_gen) (void)hipFree(sc.stage_gen);
    }
    for (hipStream_t ps : ctx->part_stream)
        if (ps) (void)hipStreamDestroy(ps);
    for (hipStream_t ps : ctx->sub_stream)
        if (ps) (void)hipStreamDestroy(ps);
    for (hipEvent_t ev : ctx->sub_ev)
        if (ev) (void)hipEventDestroy(ev);
    if (ctx->sub_zero_ev) (void)hipEventDestroy(ctx->sub_zero_ev);
    for (void* p : ctx->s_buf)
        if (p) (void)hipFree(p);
    for (void* p : ctx->e_buf)
        if (p) (void)hipFree(p);
    if (ctx->e_pin) (void)hipHostFree(ctx->e_pin);
    if (ctx->d_err) (void)hipFree(ctx->d_err);
    if (ctx->h_err) (void)hipHostFree(ctx->h_err);
    for (auto& sl : ctx->slot) {
        if (sl.ev) (void)hipEventSynchronize(sl.ev);
        if (sl.hdr) (void)hipHostFree(sl.hdr);
        if (sl.h) (void)hipHostFree(sl.h);
        if (sl.d) (void)hipFree(sl.d);
        if (sl.ev) (void)hipEventDestroy(sl.ev);
    }
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

ac_status ac_error_count_device(ac_ctx* ctx, uint32_t k, const ac_segment* segments, uint32_t n_segments,
                                const uint32_t* window_len, uint32_t flags, void* hip_stream) {
    if (!ctx) return fail(nullptr, AC_ERR_INVALID, "ctx is NULL");
    if (flags & ~AC_DEVICE_ACCUMULATE) return fail(ctx, AC_ERR_INVALID, "unknown flags");
    if (n_segments > AC_MAX_SEGS) return fail(ctx, AC_ERR_INVALID, "too many segments in one launch (max 4)");
    uint32_t ul[AC_MAX_SEGS];
    if (window_len)
        for (uint32_t i = 0; i < n_segments; ++i) {
            if (window_len[i] == AC_NO_ULEN) return fail(ctx, AC_ERR_INVALID, "window_len out of range");
            ul[i] = window_len[i];
        }
    AC_HIP(ctx, hipSetDevice(ctx->device));
    return launch(ctx, k, segments, n_segments, (hipStream_t)hip_stream, !(flags & AC_DEVICE_ACCUMULATE), nullptr, 0,
                  0, nullptr, window_len ? ul : nullptr);
}

}  // extern "C"

namespace {

// errorCount (approx_counter.cpp:531-601) for up to AC_MAX_JOBS host images on
// one device, ONE fused launch: every job's k-mers and image go up through the
// pinned staging block (h2d_staged), the counts and the device error word come
// back in one copy.  jobs[j].sample holds host pointers.
ac_status count_images_one(ac_ctx* ctx, uint32_t k, const ac_sample_job* jobs, uint32_t n) {
    if (!ctx) return fail(nullptr, AC_ERR_INVALID, "ctx is NULL");
    if (ac_status st = check_k(ctx, k)) return st;
    if (n > AC_MAX_JOBS) return fail(ctx, AC_ERR_INVALID, "too many jobs in one call (max 4)");
    uint64_t total_k = 0;
    for (uint32_t j = 0; j < n; ++j) {
        const ac_sample_job& b = jobs[j];
        if (b.n_kmers && (!b.kmers || !b.counts)) return fail(ctx, AC_ERR_INVALID, "NULL argument");
        if (ac_status st = check_sample(ctx, &b.sample)) return st;
        if (ac_status st = check_layout(ctx, b.sample)) return st;
        total_k += b.n_kmers;
    }
    if (total_k == 0) return AC_OK;
    AC_HIP(ctx, hipSetDevice(ctx->device));
    // Device block: per job kmers | codes | nmask | start | length, then err | counts of every
    // job, each 256-B aligned (the staging offsets; the error word goes up as a zero).
    static const uint32_t zero_word = 0;
    std::vector<const void*> src;
    std::vector<size_t> sz;
    for (uint32_t j = 0; j < n; ++j) {
        const ac_windows& w = jobs[j].sample;
        src.insert(src.end(), {jobs[j].kmers, w.codes, w.nmask, w.start, w.length});
        sz.insert(sz.end(), {sizeof(uint64_t) * jobs[j].n_kmers, sizeof(uint32_t) * (w.n_bases / 16),
                             sizeof(uint32_t) * (w.n_bases / 32), sizeof(uint64_t) * w.n_windows,
                             sizeof(uint32_t) * w.n_windows});
    }
    src.push_back(&zero_word);
    sz.push_back(sizeof(uint32_t));
    const size_t in_bytes = staged_bytes((int)sz.size(), sz.data());
    size_t back = 0;
    for (uint32_t j = 0; j < n; ++j) back += align256(sizeof(uint32_t) * jobs[j].n_kmers);
    if (ac_status rc = grow(ctx, &ctx->d_stage, &ctx->d_stage_cap, in_bytes + back)) return rc;
    char* d = (char*)ctx->d_stage;
    if (ac_status rc = h2d_staged(ctx, (int)sz.size(), src.data(), sz.data(), d, back)) return rc;
    char* h = (char*)ctx->h_stage;
    const size_t off_err = in_bytes - align256(sizeof(uint32_t));
    ac_segment seg[AC_MAX_JOBS];
    size_t off = 0, coff = in_bytes;
    size_t c_off[AC_MAX_JOBS];
    for (uint32_t j = 0; j < n; ++j) {
        const ac_windows& w = jobs[j].sample;
        size_t o[5];
        for (int i = 0; i < 5; ++i) {
            o[i] = off;
            off += align256(sz[5 * j + i]);
        }
        seg[j].kmers = (const uint64_t*)(d + o[0]);
        seg[j].n_kmers = jobs[j].n_kmers;
        seg[j].sample = ac_windows{(const uint32_t*)(d + o[1]), (const uint32_t*)(d + o[2]), (const uint64_t*)(d + o[3]),
                                   (const uint32_t*)(d + o[4]), w.n_windows, w.n_bases};
        seg[j].counts = (uint32_t*)(d + coff);
        c_off[j] = coff;
        coff += align256(sizeof(uint32_t) * jobs[j].n_kmers);
    }
    hipStream_t st = ctx->stream;
    if (ac_status rc = launch(ctx, k, seg, n, st, true, (uint32_t*)(d + off_err))) return rc;
    AC_HIP(ctx, hipMemcpyAsync(h + off_err, d + off_err, coff - off_err, hipMemcpyDeviceToHost, st));
    AC_HIP(ctx, hipStreamSynchronize(st));
    if (ac_status rc = device_error(ctx, *(const uint32_t*)(h + off_err))) return rc;
    for (uint32_t j = 0; j < n; ++j) {
        const uint32_t* hc = (const uint32_t*)(h + c_off[j]);
        for (uint32_t i = 0; i < jobs[j].n_kmers; ++i) jobs[j].counts[i] = hc[i];
    }
    return AC_OK;
}

// The same over an ac_create_multi context: every job's windows cut into one
// contiguous shard per device (balanced by bases), each device counting its
// shards of all jobs in one fused launch, the shard counts summed on the host.
ac_status count_images(ac_ctx* ctx, uint32_t k, const ac_sample_job* jobs, uint32_t n) {
    if (!ctx || ctx->peers.empty()) return count_images_one(ctx, k, jobs, n);
    if (ac_status st = check_k(ctx, k)) return st;
    if (n > AC_MAX_JOBS) return fail(ctx, AC_ERR_INVALID, "too many jobs in one call (max 4)");
    for (uint32_t j = 0; j < n; ++j) {
        if (jobs[j].n_kmers && (!jobs[j].kmers || !jobs[j].counts)) return fail(ctx, AC_ERR_INVALID, "NULL argument");
        if (ac_status st = check_sample(ctx, &jobs[j].sample)) return st;
        if (ac_status st = check_layout(ctx, jobs[j].sample)) return st;
    }
    const size_t G = ctx->peers.size() + 1;
    // shard g of job j: windows [cut[j][g], cut[j][g + 1]), a slice of the image from its
    // lowest start to its highest end (windows may come in any order and overlap;
    // window_ok guarantees start + length <= n_bases, so nothing here wraps)
    std::vector<std::vector<uint32_t>> cut(n);
    for (uint32_t j = 0; j < n; ++j) {
        const ac_windows& s = jobs[j].sample;
        uint64_t total = 0;
        for (uint32_t i = 0; i < s.n_windows; ++i) total += s.length[i];
        cut[j].assign(G + 1, s.n_windows);
        cut[j][0] = 0;
        uint64_t acc = 0;
        size_t g = 1;
        for (uint32_t i = 0; i < s.n_windows && g < G; ++i) {
            acc += s.length[i];
            while (g < G && acc * G >= total * g) cut[j][g++] = i + 1;
        }
    }
    std::vector<std::vector<std::vector<uint64_t>>> part(G, std::vector<std::vector<uint64_t>>(n));
    std::vector<ac_status> rc(G, AC_OK);
    auto run = [&](size_t g) {
        ac_ctx* c = g == 0 ? ctx : ctx->peers[g - 1];
        ac_sample_job sj[AC_MAX_JOBS];
        std::vector<std::vector<uint64_t>> st(n);
        uint32_t m = 0;
        for (uint32_t j = 0; j < n; ++j) {
            const ac_windows& s = jobs[j].sample;
            const uint32_t lo = cut[j][g], hi = cut[j][g + 1];
            part[g][j].assign(jobs[j].n_kmers, 0);
            if (hi == lo || !jobs[j].n_kmers) continue;
            uint64_t b0 = s.start[lo], b1 = 0;
            for (uint32_t i = lo; i < hi; ++i) {
                b0 = std::min<uint64_t>(b0, s.start[i]);
                b1 = std::max<uint64_t>(b1, s.start[i] + s.length[i]);
            }
            b1 = std::max<uint64_t>(b0 + 32, (b1 + 31) / 32 * 32);  // empty windows still count (k = 2: d = 2)
            if (b1 > s.n_bases) b1 = s.n_bases;  // b0 + 32 <= n_bases: b0 is a 32-aligned start < n_bases or 0
            st[j].resize(hi - lo);
            for (uint32_t i = lo; i < hi; ++i) st[j][i - lo] = s.start[i] - b0;
            sj[m++] = ac_sample_job{jobs[j].kmers, jobs[j].n_kmers,
                                    ac_windows{s.codes + b0 / 16, s.nmask + b0 / 32, st[j].data(), s.length + lo, hi - lo,
                                               b1 - b0},
                                    part[g][j].data()};
        }
        if (m) rc[g] = count_images_one(c, k, sj, m);
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
    for (uint32_t j = 0; j < n; ++j)
        for (uint32_t i = 0; i < jobs[j].n_kmers; ++i) {
            uint64_t v = 0;
            for (size_t g = 0; g < G; ++g) v += part[g][j][i];
            jobs[j].counts[i] = v;
        }
    return AC_OK;
}

}  // namespace

extern "C" {

ac_status ac_error_count(ac_ctx* ctx, uint32_t k, const uint64_t* kmers, uint32_t n_kmers,
                         const ac_windows* sample, uint64_t* counts) {
    if (!ctx) return fail(nullptr, AC_ERR_INVALID, "ctx is NULL");
    if (ac_status st = check_k(ctx, k)) return st;
    if (n_kmers == 0) return AC_OK;
    if (!kmers || !counts || !sample) return fail(ctx, AC_ERR_INVALID, "NULL argument");
    const ac_sample_job job{kmers, n_kmers, *sample, counts};
    return count_images(ctx, k, &job, 1);
}

ac_status ac_error_count_images(ac_ctx* ctx, uint32_t k, const ac_sample_job* jobs, uint32_t n_jobs) {
    if (n_jobs && !jobs) return fail(ctx, AC_ERR_INVALID, "jobs is NULL");
    return count_images(ctx, k, jobs, n_jobs);
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

ac_status ac_sample_upload_slot(ac_ctx* ctx, int slot, const ac_windows* host, ac_windows* dev) {
    if (!ctx || !dev) return fail(ctx, AC_ERR_INVALID, "ctx or dev is NULL");
    if (slot < 0 || slot >= AC_MAX_JOBS) return fail(ctx, AC_ERR_INVALID, "upload slot outside [0, AC_MAX_JOBS)");
    if (ac_status st = check_sample(ctx, host)) return st;
    if (ac_status st = check_layout(ctx, *host)) return st;  // on the host copy
    AC_HIP(ctx, hipSetDevice(ctx->device));
    // the slot's notes describe its image only once the upload below has completed (a
    // failure part way must not leave notes that a later count matches to a freed or partial buffer)
    ctx->s_codes[slot] = nullptr;
    ctx->s_start[slot] = nullptr;
    ctx->s_ulen[slot] = AC_NO_ULEN;
    ctx->s_no_n[slot] = false;
    const size_t sz[4] = {sizeof(uint32_t) * (host->n_bases / 16), sizeof(uint32_t) * (host->n_bases / 32),
                          sizeof(uint64_t) * host->n_windows, sizeof(uint32_t) * host->n_windows};
    const void* src[4] = {host->codes, host->nmask, host->start, host->length};
    // one device block (s_buf[slot]) holding the four arrays at the staging offsets
    if (ac_status st = grow(ctx, &ctx->s_buf[slot], &ctx->s_cap[slot], staged_bytes(4, sz))) return st;
    if (ac_status st = h2d_staged(ctx, 4, src, sz, ctx->s_buf[slot])) return st;
    AC_HIP(ctx, hipStreamSynchronize(ctx->stream));
    const char* blk = (const char*)ctx->s_buf[slot];
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
    // equal windows back to back at ceil32(length) strides (the CLI's samples: every start window
    // sl bases, every end window sl + 1), and an N-free image
    uint32_t ulen = host->n_windows ? host->length[0] : AC_NO_ULEN;
    const uint64_t stride = ((uint64_t)ulen + 31u) & ~31ull;
    for (uint32_t i = 0; i < host->n_windows && ulen != AC_NO_ULEN; ++i)
        if (host->length[i] != ulen || host->start[i] != (uint64_t)i * stride) ulen = AC_NO_ULEN;
    uint32_t any_n = 0;
    for (uint64_t i = 0; i < host->n_bases / 32; ++i) any_n |= host->nmask[i];
    ctx->s_codes[slot] = dev->codes;
    ctx->s_start[slot] = dev->start;
    ctx->s_ulen[slot] = ulen;
    ctx->s_no_n[slot] = any_n == 0u;
    ctx->s_windows[slot] = host->n_windows;
    ctx->s_bases[slot] = host->n_bases;
    return AC_OK;
}

ac_status ac_sample_upload(ac_ctx* ctx, const ac_windows* host, ac_windows* dev) {
    return ac_sample_upload_slot(ctx, 0, host, dev);
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
    // The partitioned path (exact_count.hip: dense keys -- 32-bit for k <= 16, 64-bit above --,
    // bucket partition, per-bucket LDS count; no global table); a sample too large for it, or
    // a bucket that outgrows its LDS table, takes the hash-table path.  AC_EXACT_HASH=1 forces
    // the hash table (A/B; tests/test_gpu_exact.py runs both).
    const bool compact = k <= acamd::EXACT_COMPACT_MAX_K;
    static const bool force_hash = std::getenv("AC_EXACT_HASH") != nullptr;
    bool partitioned = !force_hash;
    const size_t key_bytes = compact ? sizeof(uint32_t) : sizeof(uint64_t);
    // k-mer positions <= image bases: the capacity of the dense key arrays,
    // and of the list when every kept entry must be listed (threshold 1).
    const uint64_t key_cap = std::max<uint64_t>(32, dev->n_bases);
    // Up to 2^16 buckets of <= ~2,048 keys (the per-bucket LDS table holds 4,096; 1,024 super-buckets
    // of 64 buckets, one LDS cursor each in the scatters): 134M positions, cfg4's 10^6 windows per
    // read end included; larger samples take the hash table.
    if (key_cap > (uint64_t(1) << (16 + 11))) partitioned = false;
    // Distinct kept k-mers <= image positions (a k-mer is fixed by its image position, whichever
    // overlapping windows cover it), so this list never overflows; n_bases / 2 (entries seen at
    // least twice, disjoint windows) did for duplicated windows.
    const uint64_t list_cap = key_cap + 2;
    // small block: special[0..1] u32, had_n u64 @16, n_out u64 @24, n_list u64 @32, err u32 @40,
    // overflow u32 @44, n_keys u64 @48, hist[EXACT_HIST_BINS] u32 @64
    const size_t small_bytes = 64 + sizeof(uint32_t) * EXACT_HIST_BINS;
    std::vector<uint64_t> fb(forbidden, forbidden + n_forbidden);
    std::vector<uint64_t> fbb;  // (the partitioned path: fb by bucket, and the bucket starts; host copies
    std::vector<uint32_t> fst;  // live until the call's syncs)
    std::sort(fb.begin(), fb.end());
    fb.erase(std::unique(fb.begin(), fb.end()), fb.end());
    if (ac_status s2 = grow(ctx, &ctx->e_buf[1], &ctx->e_cap[1], (sizeof(uint64_t) + sizeof(uint32_t)) * list_cap))
        return s2;
    if (ac_status s2 = grow(ctx, &ctx->e_buf[2], &ctx->e_cap[2], small_bytes)) return s2;
    if (ac_status s2 = grow(ctx, &ctx->e_buf[3], &ctx->e_cap[3], sizeof(uint64_t) * std::max<size_t>(1, fb.size())))
        return s2;
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
    a.compact = compact ? 1u : 0u;
    a.special = (uint32_t*)small;
    a.had_n = (unsigned long long*)(small + 16);
    a.n_out = (unsigned long long*)(small + 24);
    a.n_list = (unsigned long long*)(small + 32);
    a.err = (uint32_t*)(small + 40);
    a.overflow = (uint32_t*)(small + 44);
    a.n_keys = (unsigned long long*)(small + 48);
    a.hist = (uint32_t*)(small + 64);
    a.list_keys = (uint64_t*)ctx->e_buf[1];
    a.list_cnts = (uint32_t*)((char*)ctx->e_buf[1] + sizeof(uint64_t) * list_cap);
    a.list_cap = list_cap;
    a.lc_threshold = lc_threshold;
    a.forbidden = (const uint64_t*)ctx->e_buf[3];
    a.n_forbidden = (uint32_t)fb.size();
    a.list_min = EXACT_LIST_MIN;
    // readbacks into the context's pinned block: [0, 32 KB) the small block and the list / gather counts,
    // then the gathered entries when they fit (else pageable vectors)
    constexpr size_t PIN_HEAD = 32768, PIN_MAX = size_t(16) << 20;
    static_assert(64 + sizeof(uint32_t) * EXACT_HIST_BINS + 16 <= PIN_HEAD, "small block fits the pinned head");
    if (!ctx->e_pin) {  // (allocated once at its full size: no pinned block freed or moved while a call runs)
        AC_HIP(ctx, hipHostMalloc((void**)&ctx->e_pin, PIN_HEAD + PIN_MAX, hipHostMallocDefault));
        ctx->e_pin_cap = PIN_HEAD + PIN_MAX;
    }
    char* h_small = ctx->e_pin;
    if (partitioned) {
        // buckets: about 1,024-2,048 keys each (the LDS table holds 4,096)
#ifndef AC_BUCKET_KEYS
#define AC_BUCKET_KEYS 2048  // (A/B builds: the bucket size target)
#endif
        uint32_t nb_log2 = 6;
        while (nb_log2 < 16 && (key_cap >> nb_log2) > AC_BUCKET_KEYS) ++nb_log2;
        a.nb_log2 = nb_log2;
        a.key_cap = key_cap;
        // super-buckets of <= 2^AC_SUB_LOG2 (128) buckets, at least 128 of them when there are that many buckets
        a.s_log2 = std::max(std::min(nb_log2, 7u), nb_log2 > AC_SUB_LOG2 ? nb_log2 - (uint32_t)AC_SUB_LOG2 : 0u);
        const uint32_t chunk = acamd::exact_part_chunk(k);
        a.n_chunks = (uint32_t)((key_cap + chunk - 1) / chunk);
        a.n_chunks2 = a.n_chunks + (1u << a.s_log2);
        const size_t NB = size_t(1) << nb_log2, S = size_t(1) << a.s_log2;
        const size_t h1 = S * a.n_chunks, h2 = (NB / S) * a.n_chunks2;
        if (ac_status s2 = grow(ctx, &ctx->e_buf[6], &ctx->e_cap[6], key_bytes * key_cap)) return s2;
        if (ac_status s2 = grow(ctx, &ctx->e_buf[7], &ctx->e_cap[7], key_bytes * key_cap)) return s2;
        if (ac_status s2 = grow(ctx, &ctx->e_buf[8], &ctx->e_cap[8], key_bytes * key_cap)) return s2;
        const size_t slabs = (a.n_chunks + EXACT_SCAN_SLAB - 1) / EXACT_SCAN_SLAB;
        if (ac_status s2 = grow(ctx, &ctx->e_buf[9], &ctx->e_cap[9], sizeof(uint32_t) * (h1 + h2 + S + slabs * S)))
            return s2;
        if (ac_status s2 = grow(ctx, &ctx->e_buf[10], &ctx->e_cap[10], sizeof(uint32_t) * (NB + 1))) return s2;
        if (ac_status s2 = grow(ctx, &ctx->e_buf[11], &ctx->e_cap[11], sizeof(uint32_t) * NB * EXACT_PHIST)) return s2;
        a.phist = (uint32_t*)ctx->e_buf[11];
        a.keys = ctx->e_buf[6];
        a.parts = ctx->e_buf[7];
        a.tmp = ctx->e_buf[8];
        a.h1 = (uint32_t*)ctx->e_buf[9];
        a.h2 = a.h1 + h1;
        a.stot = a.h2 + h2;
        a.slab = a.stot + S;
        a.bstart = (uint32_t*)ctx->e_buf[10];
        if (!fb.empty()) {  // the forbidden set by bucket: the count kernel searches only its bucket's entries
            std::vector<std::pair<uint32_t, uint64_t>> byb(fb.size());
            for (size_t i = 0; i < fb.size(); ++i)
                byb[i] = {compact ? acamd::bucket_of((uint32_t)fb[i], nb_log2) : acamd::bucket_of(fb[i], nb_log2), fb[i]};
            std::sort(byb.begin(), byb.end());
            fbb.assign(fb.size(), 0);
            fst.assign(NB + 1, 0);
            for (size_t i = 0; i < byb.size(); ++i) {
                fbb[i] = byb[i].second;
                ++fst[byb[i].first + 1];
            }
            for (size_t b = 0; b < NB; ++b) fst[b + 1] += fst[b];
            if (ac_status s2 = grow(ctx, &ctx->e_buf[12], &ctx->e_cap[12], sizeof(uint64_t) * fbb.size())) return s2;
            if (ac_status s2 = grow(ctx, &ctx->e_buf[13], &ctx->e_cap[13], sizeof(uint32_t) * (NB + 1))) return s2;
            AC_HIP(ctx, hipMemcpyAsync(ctx->e_buf[12], fbb.data(), sizeof(uint64_t) * fbb.size(), hipMemcpyHostToDevice, st));
            AC_HIP(ctx, hipMemcpyAsync(ctx->e_buf[13], fst.data(), sizeof(uint32_t) * (NB + 1), hipMemcpyHostToDevice, st));
            a.fb_bucketed = (const uint64_t*)ctx->e_buf[12];
            a.fb_start = (const uint32_t*)ctx->e_buf[13];
        }
        AC_HIP(ctx, hipMemsetAsync(small, 0, small_bytes, st));
        AC_HIP(ctx, acamd::launch_exact_partitioned(a, st));
        AC_HIP(ctx, hipMemcpyAsync(h_small, small, small_bytes, hipMemcpyDeviceToHost, st));
        AC_HIP(ctx, hipStreamSynchronize(st));
        if (*(const uint32_t*)(h_small + 44)) partitioned = false;  // a bucket overflowed its LDS table
        // Overlapping windows (allowed by ac_windows) hold more k-mer positions than the image
        // has bases: the dense key arrays dropped the excess, so count on the hash table instead
        // (its distinct keys are still bounded by the image's positions).
        if (*(const unsigned long long*)(h_small + 48) > key_cap) partitioned = false;
    }
    if (!partitioned) {
        // Table: a power of two >= 1.5 x the image size (an upper bound on k-mer
        // positions): load <= 2/3 even when every position is a new k-mer.  (1.25 x,
        // 2^24 slots at 10^5 windows: insert 530 -> 644 us from the longer probe
        // chains, scan 139 -> 104 us; profiles/r02_exact_log.md.)
        uint64_t slots = 1024;
        while (slots < dev->n_bases + dev->n_bases / 2) slots <<= 1;
        const size_t slot_bytes = compact ? sizeof(unsigned long long) : sizeof(acamd::ExactSlot);
        if (ac_status s2 = grow(ctx, &ctx->e_buf[0], &ctx->e_cap[0], slot_bytes * slots)) return s2;
        a.table = (acamd::ExactSlot*)ctx->e_buf[0];
        a.ctable = (unsigned long long*)ctx->e_buf[0];
        a.slots = slots;
        a.mask = slots - 1;
        AC_HIP(ctx, hipMemsetAsync(ctx->e_buf[0], 0, slot_bytes * slots, st));
        AC_HIP(ctx, hipMemsetAsync(small, 0, small_bytes, st));
        AC_HIP(ctx, acamd::launch_exact_insert(a, st));
        AC_HIP(ctx, acamd::launch_exact_scan(a, st));
        AC_HIP(ctx, hipMemcpyAsync(h_small, small, small_bytes, hipMemcpyDeviceToHost, st));
        AC_HIP(ctx, hipStreamSynchronize(st));
    }
    if (ac_status rc = device_error(ctx, *(const uint32_t*)(h_small + 40))) return rc;
    ctx->exact_path = partitioned ? 1 : 0;
    const uint32_t* hist = (const uint32_t*)(h_small + 64);
    uint64_t kept = 0;
    for (int i = 0; i < EXACT_HIST_BINS; ++i) kept += hist[i];
    if (n_distinct) *n_distinct = kept;
    if (had_n) *had_n = *(const unsigned long long*)(h_small + 16);
    uint64_t n_list = *(const unsigned long long*)(h_small + 32);
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
    bool from_list = thr >= EXACT_LIST_MIN;
    if (!from_list && partitioned) {
        // threshold 1: list every kept entry (the count kernel again, listing only)
        a.list_min = 1;
        a.emit_only = 1;
        AC_HIP(ctx, hipMemsetAsync(a.n_list, 0, sizeof(unsigned long long), st));
        AC_HIP(ctx, acamd::launch_exact_part_count(a, st));
        unsigned long long* nl = (unsigned long long*)(ctx->e_pin + PIN_HEAD - 16);
        AC_HIP(ctx, hipMemcpyAsync(nl, a.n_list, sizeof *nl, hipMemcpyDeviceToHost, st));
        AC_HIP(ctx, hipStreamSynchronize(st));
        n_list = *nl;
        if (n_list > list_cap) return fail(ctx, AC_ERR_INTERNAL, "exact count: candidate list overflow");
        from_list = true;
    }
    // (a solid threshold past the last bin is applied exactly on the gathered list)
    const uint64_t gather_cap = std::max<uint64_t>(1, due);
    if (ac_status s2 = grow(ctx, &ctx->e_buf[4], &ctx->e_cap[4], sizeof(uint64_t) * gather_cap)) return s2;
    if (ac_status s2 = grow(ctx, &ctx->e_buf[5], &ctx->e_cap[5], sizeof(uint32_t) * gather_cap)) return s2;
    a.threshold = (uint32_t)std::min<uint64_t>(thr, 0xffffffffu);
    a.out_keys = (uint64_t*)ctx->e_buf[4];
    a.out_cnts = (uint32_t*)ctx->e_buf[5];
    a.out_cap = gather_cap;
    AC_HIP(ctx, acamd::launch_exact_gather(a, from_list, n_list, st));
    // The gathered count is at most gather_cap (the histogram's due entries): with room in the pinned
    // block, the count and gather_cap entries come back in one synchronised batch of DMAs (the extra
    // entries, if any, are ignored); otherwise the count first, then exactly that many entries.
    unsigned long long* got_p = (unsigned long long*)(ctx->e_pin + PIN_HEAD - 8);
    const size_t entry_bytes = (sizeof(uint64_t) + sizeof(uint32_t)) * gather_cap;
    const bool pin_entries = entry_bytes <= PIN_MAX;
    uint64_t* gk_p = (uint64_t*)(ctx->e_pin + PIN_HEAD);
    uint32_t* gc_p = (uint32_t*)(ctx->e_pin + PIN_HEAD + sizeof(uint64_t) * gather_cap);
    std::vector<uint64_t> gk;
    std::vector<uint32_t> gc;
    AC_HIP(ctx, hipMemcpyAsync(got_p, a.n_out, sizeof *got_p, hipMemcpyDeviceToHost, st));
    if (pin_entries) {
        AC_HIP(ctx, hipMemcpyAsync(gk_p, a.out_keys, sizeof(uint64_t) * gather_cap, hipMemcpyDeviceToHost, st));
        AC_HIP(ctx, hipMemcpyAsync(gc_p, a.out_cnts, sizeof(uint32_t) * gather_cap, hipMemcpyDeviceToHost, st));
    }
    AC_HIP(ctx, hipStreamSynchronize(st));
    const unsigned long long got = *got_p;
    if (got > gather_cap) return fail(ctx, AC_ERR_INTERNAL, "exact count: gathered more entries than the histogram");
    if (!pin_entries && got) {
        gk.resize(got);
        gc.resize(got);
        AC_HIP(ctx, hipMemcpyAsync(gk.data(), a.out_keys, sizeof(uint64_t) * got, hipMemcpyDeviceToHost, st));
        AC_HIP(ctx, hipMemcpyAsync(gc.data(), a.out_cnts, sizeof(uint32_t) * got, hipMemcpyDeviceToHost, st));
        AC_HIP(ctx, hipStreamSynchronize(st));
        gk_p = gk.data();
        gc_p = gc.data();
    }
    // CompareCount (275-305): count descending, DUST score ascending, k-mer descending.  For k > 2 the
    // score is a non-negative float, so its bits order like it and the whole order is one 128-bit key
    // ((~count, score bits), ~k-mer) compared as two integers; the first n by nth_element, then sorted
    // (partial_sort with the three-field comparator was most of a cfg3 call's host time).  k = 2 (a
    // score of 0 / 0) keeps the comparator, whose NaN ties are the reference's.
    const size_t n_all = solid ? (size_t)std::count_if(gc_p, gc_p + got, [&](uint32_t c) { return c >= solid; })
                               : (size_t)got;
    const size_t n = solid ? n_all : std::min<size_t>(n_all, limit);
    *n_out = n;
    if (n > capacity) return fail(ctx, AC_ERR_INVALID, "exact count: capacity too small (n_out holds the size needed)");
    if (k > 2) {
        struct Key {
            uint64_t hi, lo;
        };
        std::vector<Key> w;
        w.reserve(n_all);
        for (uint64_t i = 0; i < got; ++i)
            if (!solid || gc_p[i] >= solid) {
                const float c = complexity(gk_p[i], k);
                uint32_t cb;
                std::memcpy(&cb, &c, sizeof cb);
                w.push_back({((uint64_t)(0xffffffffu - gc_p[i]) << 32) | cb, ~gk_p[i]});
            }
        auto kl = [](const Key& x, const Key& y) { return x.hi < y.hi || (x.hi == y.hi && x.lo < y.lo); };
        if (n < w.size()) std::nth_element(w.begin(), w.begin() + n, w.end(), kl);
        std::sort(w.begin(), w.begin() + n, kl);
        for (size_t i = 0; i < n; ++i) {
            kmers_out[i] = ~w[i].lo;
            counts_out[i] = 0xffffffffu - (uint32_t)(w[i].hi >> 32);
        }
        return AC_OK;
    }
    struct Entry {
        uint64_t count, kmer;
        float comp;
    };
    std::vector<Entry> v;
    v.reserve(n_all);
    for (uint64_t i = 0; i < got; ++i)
        if (!solid || gc_p[i] >= solid) v.push_back({gc_p[i], gk_p[i], complexity(gk_p[i], k)});
    auto less = [](const Entry& x, const Entry& y) {
        if (x.count != y.count) return x.count > y.count;
        if (x.comp != y.comp) return x.comp < y.comp;
        return x.kmer > y.kmer;
    };
    std::partial_sort(v.begin(), v.begin() + n, v.end(), less);
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

ac_status ac_error_count_samples(ac_ctx* ctx, uint32_t k, const ac_sample_job* jobs, uint32_t n_jobs) {
    if (!ctx) return fail(nullptr, AC_ERR_INVALID, "ctx is NULL");
    if (ac_status st = check_k(ctx, k)) return st;
    if (n_jobs > AC_MAX_JOBS) return fail(ctx, AC_ERR_INVALID, "too many jobs in one call (max 4)");
    if (n_jobs && !jobs) return fail(ctx, AC_ERR_INVALID, "jobs is NULL");
    uint64_t total = 0;
    for (uint32_t j = 0; j < n_jobs; ++j) {
        if (jobs[j].n_kmers && (!jobs[j].kmers || !jobs[j].counts)) return fail(ctx, AC_ERR_INVALID, "NULL argument");
        if (ac_status st = check_sample(ctx, &jobs[j].sample)) return st;
        total += jobs[j].n_kmers;
    }
    if (total == 0) return AC_OK;
    AC_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    // every job's k-mers in one upload (d_buf[0]); uint32 counts in d_buf[5], one D2H
    std::vector<uint64_t> km;
    km.reserve(total);
    for (uint32_t j = 0; j < n_jobs; ++j) km.insert(km.end(), jobs[j].kmers, jobs[j].kmers + jobs[j].n_kmers);
    if (ac_status s2 = ensure(ctx, 0, sizeof(uint64_t) * total)) return s2;
    if (ac_status s2 = ensure(ctx, 5, sizeof(uint32_t) * total)) return s2;
    AC_HIP(ctx, hipMemcpyAsync(ctx->d_buf[0], km.data(), sizeof(uint64_t) * total, hipMemcpyHostToDevice, st));
    ac_segment seg[AC_MAX_JOBS];
    uint64_t base = 0;
    for (uint32_t j = 0; j < n_jobs; ++j) {
        seg[j].kmers = (const uint64_t*)ctx->d_buf[0] + base;
        seg[j].n_kmers = jobs[j].n_kmers;
        seg[j].sample = jobs[j].sample;
        seg[j].counts = (uint32_t*)ctx->d_buf[5] + base;
        base += jobs[j].n_kmers;
    }
    // images this context uploaded: their equal-window / N-free findings (others: the general form)
    uint32_t ulen[AC_MAX_JOBS];
    bool no_n[AC_MAX_JOBS];
    for (uint32_t j = 0; j < n_jobs; ++j) {
        ulen[j] = AC_NO_ULEN;
        no_n[j] = false;
        for (int sl = 0; sl < AC_MAX_JOBS; ++sl)
            if (ctx->s_codes[sl] && ctx->s_codes[sl] == jobs[j].sample.codes &&
                jobs[j].sample.nmask == (const uint32_t*)((const char*)ctx->s_codes[sl] +
                                                          (sizeof(uint32_t) * (ctx->s_bases[sl] / 16) + 255) / 256 * 256) &&
                jobs[j].sample.n_windows == ctx->s_windows[sl] && jobs[j].sample.n_bases == ctx->s_bases[sl] &&
                jobs[j].sample.start == ctx->s_start[sl] &&
                (const char*)jobs[j].sample.length >= (const char*)ctx->s_buf[sl] &&
                (const char*)jobs[j].sample.length < (const char*)ctx->s_buf[sl] + ctx->s_cap[sl]) {
                ulen[j] = ctx->s_ulen[sl];
                no_n[j] = ctx->s_no_n[sl];
            }
        // (the launch's own check: equal windows must fit the image)
        if (ulen[j] != AC_NO_ULEN &&
            (uint64_t)jobs[j].sample.n_windows * (((uint64_t)ulen[j] + 31u) & ~31ull) > jobs[j].sample.n_bases)
            ulen[j] = AC_NO_ULEN;
    }
    if (ac_status rc = launch(ctx, k, seg, n_jobs, st, true, nullptr, 0, 0, no_n, ulen)) return rc;
    ctx->h_counts.resize(total);
    AC_HIP(ctx, hipMemcpyAsync(ctx->h_counts.data(), ctx->d_buf[5], sizeof(uint32_t) * total, hipMemcpyDeviceToHost, st));
    if (ac_status rc = ac_check(ctx, st)) return rc;  // synchronises the stream
    base = 0;
    for (uint32_t j = 0; j < n_jobs; ++j)
        for (uint32_t i = 0; i < jobs[j].n_kmers; ++i) jobs[j].counts[i] = ctx->h_counts[base++];
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
    // The same packer as the jobs stage (host_pack.cpp); it writes every
    // 32-base block the windows occupy, the rest of the image is zeroed here.
    uint64_t used = 0;
    for (uint32_t i = 0; i < n; ++i) used += acamd::image_span(seq_len[i]);
    acamd::pack_dna5_range(dna5, seq_start, seq_len, 0, n, 0, codes, nmask, start, length);
    std::memset(codes + used / 16, 0, sizeof(uint32_t) * ((n_bases - used) / 16));
    std::memset(nmask + used / 32, 0, sizeof(uint32_t) * ((n_bases - used) / 32));
    return AC_OK;
}

ac_status ac_check(ac_ctx* ctx, void* hip_stream) {
    if (!ctx) return fail(nullptr, AC_ERR_INVALID, "ctx is NULL");
    AC_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t st = (hipStream_t)hip_stream;
    AC_HIP(ctx, hipMemcpyAsync(ctx->h_err, ctx->d_err, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    AC_HIP(ctx, hipStreamSynchronize(st));
    const uint32_t word = *ctx->h_err;
    if (!word) return AC_OK;
    AC_HIP(ctx, hipMemsetAsync(ctx->d_err, 0, sizeof(uint32_t), st));
    AC_HIP(ctx, hipStreamSynchronize(st));
    return device_error(ctx, word);
}

int ac_comm_id_bytes(void) { return (int)sizeof(ncclUniqueId); }

ac_status ac_comm_unique_id(ac_ctx* ctx, void* id_out) {
    if (!ctx || !id_out) return fail(ctx, AC_ERR_INVALID, "ctx or id_out is NULL");
    const Rccl& r = rccl();
    if (!r.err.empty()) return fail(ctx, AC_ERR_DEVICE, r.err);
    AC_HIP(ctx, hipSetDevice(ctx->device));
    ncclUniqueId id;
    const ncclResult_t e = r.get_unique_id(&id);
    if (e != ncclSuccess) return fail(ctx, AC_ERR_DEVICE, std::string("ncclGetUniqueId: ") + r.error_string(e));
    std::memcpy(id_out, &id, sizeof id);
    return AC_OK;
}

ac_status ac_comm_init(ac_ctx* ctx, int n_ranks, int rank, const void* id) {
    if (!ctx || !id) return fail(ctx, AC_ERR_INVALID, "ctx or id is NULL");
    if (n_ranks < 1 || rank < 0 || rank >= n_ranks) return fail(ctx, AC_ERR_INVALID, "rank outside [0, n_ranks)");
    if (!ctx->peers.empty()) return fail(ctx, AC_ERR_INVALID, "ac_comm_init needs a single-device context");
    if (ctx->comm) return fail(ctx, AC_ERR_INVALID, "the context already has a communicator");
    const Rccl& r = rccl();
    if (!r.err.empty()) return fail(ctx, AC_ERR_DEVICE, r.err);
    AC_HIP(ctx, hipSetDevice(ctx->device));
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    ncclComm_t c = nullptr;
    const ncclResult_t e = r.comm_init_rank(&c, n_ranks, u, rank);
    if (e != ncclSuccess) return fail(ctx, AC_ERR_DEVICE, std::string("ncclCommInitRank: ") + r.error_string(e));
    ctx->comm = c;
    return AC_OK;
}

ac_status ac_allreduce_counts(ac_ctx* ctx, uint32_t* d_counts, uint64_t n, void* hip_stream) {
    if (!ctx) return fail(ctx, AC_ERR_INVALID, "ctx is NULL");
    if (!ctx->comm) return fail(ctx, AC_ERR_INVALID, "no communicator: call ac_comm_init first");
    if (n == 0) return AC_OK;
    if (!d_counts) return fail(ctx, AC_ERR_INVALID, "d_counts is NULL");
    AC_HIP(ctx, hipSetDevice(ctx->device));
    const Rccl& r = rccl();
    const ncclResult_t e = r.all_reduce(d_counts, d_counts, (size_t)n, ncclUint32, ncclSum, ctx->comm,
                                        (hipStream_t)hip_stream);
    if (e != ncclSuccess) return fail(ctx, AC_ERR_DEVICE, std::string("ncclAllReduce: ") + r.error_string(e));
    return AC_OK;
}

ac_status ac_set_host_cpus(const int* cpus, int n_cpus, int participants) {
    if (n_cpus < 0 || (n_cpus && !cpus) || participants < 0) return fail(nullptr, AC_ERR_INVALID, "bad CPU list");
    acamd::HostPlan plan;
    plan.cpus.assign(cpus, cpus + n_cpus);
    std::sort(plan.cpus.begin(), plan.cpus.end());
    plan.participants = participants ? (unsigned)participants : (unsigned)std::max(1, std::min(16, n_cpus ? n_cpus : 16));
    if (!acamd::set_host_plan(plan))
        return fail(nullptr, AC_ERR_INVALID, "the host pool's CPUs are already fixed (set before the first ac_create)");
    return AC_OK;
}

int ac_host_pool_cpus(int* participants, int* cpus, int cap) {
    const acamd::HostPlan p = acamd::host_plan();
    if (participants) *participants = (int)p.participants;
    for (int i = 0; i < cap && i < (int)p.cpus.size(); ++i) cpus[i] = p.cpus[(size_t)i];
    return (int)p.cpus.size();
}

int ac_plan_host_cpus(const char* const* rank_cpulists, int n_ranks, int rank, const char* allowed_cpulist,
                      const int* core_of, int n_core_of, int* out, int cap) {
    if (n_ranks < 1 || rank < 0 || rank >= n_ranks || !rank_cpulists || !allowed_cpulist) return -1;
    std::vector<std::vector<int>> lists((size_t)n_ranks);
    for (int r = 0; r < n_ranks; ++r) lists[(size_t)r] = acamd::parse_cpulist(rank_cpulists[r] ? rank_cpulists[r] : "");
    std::function<int(int)> core;
    if (core_of) core = [=](int c) { return c >= 0 && c < n_core_of ? core_of[c] : c; };
    const std::vector<int> v = acamd::plan_host_cpus(lists, rank, acamd::parse_cpulist(allowed_cpulist), core);
    for (int i = 0; i < cap && i < (int)v.size(); ++i) out[i] = v[(size_t)i];
    return (int)v.size();
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Pinned host blocks (ac_host_alloc): a sample whose Dna5 bytes and window offsets lie
// in them is read by the count kernel itself (device packing), so a jobs call does no per-window host
// work beyond the length scan.  Process-wide: one registry for every context and device.
namespace {
struct HostBlock {
    char* h = nullptr;
    size_t n = 0;
    char* d = nullptr;  // device-visible address of h
};
std::mutex g_blocks_m;
std::vector<HostBlock> g_blocks;

// The block holding [p, p + bytes) (bytes >= 1), if any.
bool find_block(const void* p, size_t bytes, HostBlock* out) {
    const char* c = (const char*)p;
    std::lock_guard<std::mutex> lk(g_blocks_m);
    for (const HostBlock& b : g_blocks)
        if (c >= b.h && c < b.h + b.n && bytes <= (size_t)(b.h + b.n - c)) {
            *out = b;
            return true;
        }
    return false;
}
}  // namespace

extern "C" {
ac_status ac_host_alloc(size_t bytes, void** out) {
    if (!out) return fail(nullptr, AC_ERR_INVALID, "out is NULL");
    *out = nullptr;
    HostBlock b;
    b.n = bytes ? bytes : 16;
    hipError_t e = hipHostMalloc((void**)&b.h, b.n, hipHostMallocDefault);
    if (e != hipSuccess) return hip_fail(nullptr, e, "hipHostMalloc");
    e = hipHostGetDevicePointer((void**)&b.d, b.h, 0);
    if (e != hipSuccess) {
        (void)hipHostFree(b.h);
        return hip_fail(nullptr, e, "hipHostGetDevicePointer");
    }
    {
        std::lock_guard<std::mutex> lk(g_blocks_m);
        g_blocks.push_back(b);
    }
    *out = b.h;
    return AC_OK;
}

ac_status ac_host_free(void* p) {
    if (!p) return AC_OK;
    HostBlock b;
    {
        std::lock_guard<std::mutex> lk(g_blocks_m);
        auto it = std::find_if(g_blocks.begin(), g_blocks.end(), [&](const HostBlock& x) { return x.h == p; });
        if (it == g_blocks.end()) return fail(nullptr, AC_ERR_INVALID, "ac_host_free: not a block of ac_host_alloc");
        b = *it;
        g_blocks.erase(it);
    }
    const hipError_t e = hipHostFree(b.h);
    return e == hipSuccess ? AC_OK : hip_fail(nullptr, e, "hipHostFree");
}
}  // extern "C"

// ---------------------------------------------------------------------------
// ac_error_count_jobs: the whole errorCount stage from Dna5 host buffers.
namespace {

// Device packing of jobs whose samples lie in ac_host_alloc blocks: 2 = auto (default),
// 1 = every eligible job (AC_DEVICE_PACK=1), 0 = never (AC_DEVICE_PACK=0: the host pool packs).
int device_pack_mode() {
#ifdef AC_NO_DEVICE_PACK
    return 0;  // (A/B builds: the kernel has no device packer)
#endif
    static const int v = [] {
        const char* e = std::getenv("AC_DEVICE_PACK");
        return (e && *e) ? (std::atoi(e) ? 1 : 0) : 2;
    }();
    return v;
}
// Auto: the kernel packs a call of at least this many windows.  Below it the host pool, which packs a
// cfg2 call in a few microseconds, is ahead: cfg2 stage 0.1145-0.1149 ms host-packed against
// 0.1262-0.1292 device-packed (the image crosses PCIe as 1 B/base instead of 0.25, 2 MB per call;
// profiles/r06_m4/abdev_*), and still with an 8-rank node's 1-participant pool: 0.1150 / 0.1158
// against 0.1270 / 0.1302 (profiles/r06_m10/rank8_*; round 6 first device-packed every call of a pool
// of <= 2 participants, which cost a cfg2 rank at N = 8 those 12 us).  At cfg3-cfg5 the two are within
// 1-3 % and the device-packed steps have no host-side tail (profiles/r06_m3/stall*, abbig_*).
uint64_t device_pack_min_windows() {
    static const uint64_t v = (uint64_t)std::max(0, env_int("AC_DEVICE_PACK_MIN_WINDOWS", 1 << 16));
    return v;
}

// AC_STAGE_TRACE=1: per-phase host timings of the jobs stage, summed over the
// calls and printed to stderr at exit (a measurement aid; no effect otherwise).
struct StageTrace {
    bool on = std::getenv("AC_STAGE_TRACE") != nullptr;
    double sum[8] = {};
    double cur[8] = {};
    uint64_t calls = 0;
    std::vector<std::vector<double>> per_call;  // AC_STAGE_TRACE=2: every call's phases
    void end_call() {
        if (std::getenv("AC_STAGE_TRACE")[0] == '2') per_call.emplace_back(cur, cur + 8);
        for (double& x : cur) x = 0.0;
    }
    void skip_warmup() {  // the first calls allocate: leave them out of the means
        if (calls == 5) {
            for (double& x : sum) x = 0.0;
        }
    }
    ~StageTrace() {
        if (!on || !calls) return;
        static const char* names[8] = {"span", "layout", "pack", "h2d_enq", "launch_enq", "d2h_enq", "sync", "widen"};
        const double n = calls > 5 ? double(calls - 5) : double(calls);
        const char* lr = std::getenv("LOCAL_RANK");
        std::fprintf(stderr, "[ac stage trace] local rank %s, %llu calls (first 5 left out), mean us:", lr ? lr : "-",
                     (unsigned long long)calls);
        for (int i = 0; i < 8; ++i) std::fprintf(stderr, " %s %.1f", names[i], sum[i] / n);
        std::fprintf(stderr, "\n");
        for (size_t c = 0; c < per_call.size(); ++c) {
            std::fprintf(stderr, "[ac stage call %zu]", c);
            for (int i = 0; i < 8; ++i) std::fprintf(stderr, " %s %.1f", names[i], per_call[c][i]);
            std::fprintf(stderr, "\n");
        }
    }
};
StageTrace g_trace;
inline double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Where one device's part of a jobs call lives in its staging slot (the same
// offsets in the pinned host block and the device block).  Inputs first
// (sent by one DMA), then the device error word and the uint32 counts (the
// way back: one DMA from off_err to the end).
struct JobPlan {
    uint32_t n = 0;
    uint32_t lo[AC_MAX_JOBS] = {}, hi[AC_MAX_JOBS] = {};  // window range of each job on this device
    uint64_t n_bases[AC_MAX_JOBS] = {};
    size_t off_kmers[AC_MAX_JOBS] = {}, off_codes[AC_MAX_JOBS] = {}, off_nmask[AC_MAX_JOBS] = {};
    size_t off_start[AC_MAX_JOBS] = {}, off_len[AC_MAX_JOBS] = {}, off_counts[AC_MAX_JOBS] = {};
    size_t off_err = 0, total = 0;
    bool early = false;  // the early-launch stage (the kernel stages its own inputs, host-polled completion)
    // early launch with host counts (synchronous calls): tagged completion -- u64 counts (generation << 32 |
    // count) and one tagged error word per candidate group at off_gerr (n_gerr of them)
    bool tag = false;
    size_t off_gerr = 0;
    uint32_t n_gerr = 0;
    uint32_t gen = 0;    // its generation (the header flags and the tagged counts carry it)
    int slot = 0;     // staging slot (set by the caller: a synchronous part q uses slot q, a submit part its set's)
    int scratch = 0;  // count-kernel scratch set (ac_ctx::sc)
    // early launch: what the launch is made of
    uint32_t ulen[AC_MAX_JOBS] = {}, chunks[AC_MAX_JOBS] = {}, codes_off[AC_MAX_JOBS] = {};
    bool nrec[AC_MAX_JOBS] = {};
    uint32_t pre = 0, copiers = 0;
    // device packing: job j's Dna5 bytes / offsets read by the kernel from pinned memory
    bool dp[AC_MAX_JOBS] = {};
    bool dp_any = false;
};

// Calls whose pack and DMA take hundreds of
// microseconds or more are cut into parts (equal bases, one stream each), so
// part q + 1 is packed and sent while part q counts: two parts from 2^17
// windows, four from 2^19.  Same box, interleaved (profiles/r02_stage_parts_ab2.log):
// cfg4 (2M windows) step p50 10.26-10.31 ms in four parts, 10.42-10.49 in three,
// 11.27 in two (13.3 in one, r02_stage_parts_ab.log); cfg3 (200k windows)
// 3.27-3.29 ms in two vs 3.24-3.40 one-part with round 2's (since removed) zero-copy / DMA chooser
// and 3.42 one-part DMA.  Eight parts from 2^20 windows: cfg4 9.77-9.86 vs 9.79-9.96 ms in four
// (profiles/r03_m14/parts_ab.log, round 3), not kept.
constexpr uint64_t STAGE_PARTS2_MIN_WINDOWS = 1ull << 17, STAGE_PARTS4_MIN_WINDOWS = 1ull << 19;
int stage_parts(uint64_t total_w) {
    return total_w >= STAGE_PARTS4_MIN_WINDOWS ? 4 : total_w >= STAGE_PARTS2_MIN_WINDOWS ? 2 : 1;
}
// DMA-mode transfer of a one-part call: a copy kernel on the compute queue reads the pinned
// block once over PCIe and writes the device block, so the count kernel follows it on the
// same queue, rather than hipMemcpyAsync (the copy engine, whose completion -> kernel start
// costs ~9 us at cfg2); job by job, so job j's inputs travel while job j + 1 is packed; equal
// windows counted with arithmetic descriptors.  Each won its A/B (profiles/r02_stage_pipe_blit_ab.log:
// sync 114-118 vs 130-132 us; r02_stage_ulen_ab.log), and the switches are gone.
// Shape (A/B builds: tools/variants.sh).  64-thread workgroups with 4 loads in flight per
// thread measured faster on one box -- cfg2 stage p50 0.146-0.147 ms vs 0.150-0.159 for
// 256 x 2 (profiles/r02_blit_shape_ab.log) -- but no GPU box was free to run the test
// suite on it before round 2 ended, so the tested 256 x 2 stays the default.
#ifndef AC_BLIT_THREADS
#define AC_BLIT_THREADS 256
#endif
#ifndef AC_BLIT_UNROLL
#define AC_BLIT_UNROLL 2
#endif
constexpr uint32_t BLIT_THREADS = AC_BLIT_THREADS, BLIT_UNROLL = AC_BLIT_UNROLL;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(BLIT_THREADS) stage_blit_kernel(const u32x4* __restrict__ src,
                                                                  u32x4* __restrict__ dst, uint32_t n16) {
    const uint32_t i0 = blockIdx.x * (BLIT_THREADS * BLIT_UNROLL) + threadIdx.x;
    u32x4 v[BLIT_UNROLL];
#pragma unroll
    for (uint32_t u = 0; u < BLIT_UNROLL; ++u)
        if (i0 + u * BLIT_THREADS < n16) v[u] = __builtin_nontemporal_load(src + i0 + u * BLIT_THREADS);
#pragma unroll
    for (uint32_t u = 0; u < BLIT_UNROLL; ++u)
        if (i0 + u * BLIT_THREADS < n16) dst[i0 + u * BLIT_THREADS] = v[u];
}
// bytes: a multiple of 16 (the stage's offsets are 256-aligned)
hipError_t stage_blit_launch(const void* src_dev, void* dst, size_t bytes, hipStream_t stream) {
    const size_t n16 = bytes / 16;
    if (n16 == 0) return hipSuccess;
    if (n16 >= (1ull << 32)) return hipErrorInvalidValue;
    const uint32_t per = BLIT_THREADS * BLIT_UNROLL;
    const uint32_t blocks = (uint32_t)((n16 + per - 1) / per);
    stage_blit_kernel<<<blocks, BLIT_THREADS, 0, stream>>>((const u32x4*)src_dev, (u32x4*)dst, (uint32_t)n16);
    return hipGetLastError();
}

// The early-launch stage for calls on one device, synchronous calls and submits alike (default:
// AC_STAGE_EARLY=1).  0 = the pack -> copy kernel / copy engine -> launch order of round 2; 2 = the
// first job sent ahead of the launch by the copy kernel, the others staged by the count kernel.
// Same box, interleaved (profiles/r03_m2/summary.log): cfg2 step 0.141-0.143 vs 0.148-0.149 ms.
int stage_early() {
    static const int v = [] {
        const char* e = std::getenv("AC_STAGE_EARLY");
        return e ? std::max(0, std::min(2, std::atoi(e))) : 1;
    }();
    return v;
}

// Test-only hooks (ac_testing_stage_hooks, include/approx_counter_amd_testing.h; never set by the
// product): AC_TESTING_UNFLAG_LAST leaves a call's last job unflagged, so the kernel's bounded wait
// runs out (the synchronous call then retries through the DMA path); AC_TESTING_ALL_AHEAD sends every
// job ahead of the staged launch (the staged kernel on resident input, a diagnostic of its own cost).
std::atomic<uint32_t> g_test_hooks{0};

// Some job has candidates and windows (a launch with work, so tagged counts to wait for).
bool live_work(const ac_job* jobs, uint32_t n_jobs) {
    for (uint32_t j = 0; j < n_jobs; ++j)
        if (jobs[j].n_kmers && jobs[j].sample.n_windows) return true;
    return false;
}

// Spin until every count of the live jobs and every group error word of a tagged early launch
// carries the launch's generation (high half); hipStreamQuery every 1024 spins catches a launch that
// failed or finished without writing them.
ac_status wait_tagged(ac_ctx* ctx, const ac_job* jobs, uint32_t n_jobs, const JobPlan& p, const char* h,
                      hipStream_t stream) {
    uint32_t spins = 0;
    auto await = [&](const uint64_t* w) -> ac_status {
        while ((uint32_t)(__atomic_load_n(w, __ATOMIC_ACQUIRE) >> 32) != p.gen) {
            __builtin_ia32_pause();
            if ((++spins & 1023u) == 0u) {
                const hipError_t q = hipStreamQuery(stream);
                if (q == hipErrorNotReady) continue;
                if (q != hipSuccess) return hip_fail(ctx, q, "early launch");
                if ((uint32_t)(__atomic_load_n(w, __ATOMIC_ACQUIRE) >> 32) == p.gen) break;
                return fail(ctx, AC_ERR_INTERNAL, "early launch finished without writing its counts");
            }
        }
        return AC_OK;
    };
    // the group error words first (one per candidate group: each arrives with its group's counts)
    const uint64_t* ge = (const uint64_t*)(h + p.off_gerr);
    for (uint32_t i = 0; i < p.n_gerr; ++i)
        if (ac_status st = await(ge + i)) return st;
    for (uint32_t j = 0; j < n_jobs && j < p.n; ++j) {
        if (!jobs[j].n_kmers || p.hi[j] <= p.lo[j]) continue;
        const uint64_t* hc = (const uint64_t*)(h + p.off_counts[j]);
        for (uint32_t i = 0; i < jobs[j].n_kmers; ++i)
            if (ac_status st = await(hc + i)) return st;
    }
    return AC_OK;
}

ac_status check_jobs(ac_ctx* ctx, uint32_t k, const ac_job* jobs, uint32_t n_jobs) {
    if (!ctx) return fail(nullptr, AC_ERR_INVALID, "ctx is NULL");
    if (ac_status st = check_k(ctx, k)) return st;
    if (n_jobs > AC_MAX_JOBS) return fail(ctx, AC_ERR_INVALID, "too many jobs in one call (max 4)");
    if (n_jobs && !jobs) return fail(ctx, AC_ERR_INVALID, "jobs is NULL");
    for (uint32_t j = 0; j < n_jobs; ++j) {
        const ac_job& b = jobs[j];
        if (b.n_kmers && !b.kmers) return fail(ctx, AC_ERR_INVALID, "job kmers is NULL");
        if (b.sample.n_windows && (!b.sample.bases || !b.sample.offset || !b.sample.length))
            return fail(ctx, AC_ERR_INVALID, "job sample has a NULL array");
    }
    return AC_OK;
}

// Packs the jobs' window ranges p.lo/p.hi into a staging slot of ctx (the
// host worker pool writes the 2-bit codes, N bitmap and window descriptors
// straight into pinned memory), moves each job's region into device memory
// (p.early: the count kernel copies it itself once the host flags the job;
// otherwise the copy kernel on `stream`, or the copy engine for multi-part
// calls) and launches the fused count kernel, whose counts go to d_counts
// (job j at d_counts + sum of the earlier n_kmers) or, when NULL, to the
// slot's pinned counts area.  Records the slot's event after the launch.
// Staging slots: a synchronous call's part q uses slot q (a one-part early
// launch alternates between slots 0 and 1); submits alternate between two
// sets of slots of their own.
ac_status stage_and_launch(ac_ctx* ctx, uint32_t k, const ac_job* jobs, JobPlan& p, hipStream_t stream,
                           uint32_t* d_counts, int part = 0, uint32_t wave_div = 0, bool zero = true) {
    using acamd::image_span;
    acamd::WorkPool& pool = acamd::host_pool();
    // Tasks: contiguous window ranges, about 4 per pool thread.
    struct Task {
        uint32_t job, w0, w1;
        uint64_t bases;  // image bases the range occupies, then its first image base
        uint64_t span;   // image bases the range occupies
        uint32_t first_len, len_diff;  // the range's first window length; OR of (length ^ first_len)
    };
    uint64_t total_w = 0;
    for (uint32_t j = 0; j < p.n; ++j)
        if (jobs[j].n_kmers) total_w += p.hi[j] - p.lo[j];
    // (tasks of 128 windows, or the first tasks of every job packed first, were slower: the claims
    // contend on the pool's one state line, profiles/r03_m8/ab.log).  The early launch publishes
    // progress a finished task at a time, so its tasks stay at most 2,048 windows (~20 us of one
    // thread's packing): a large call's first windows then reach the GPU within tens of microseconds
    // rather than after a 1/(4 x participants) share of the whole call.
    // (Packing a small call with part of the pool -- the others sleeping through it -- was slower:
    // cfg2 stage p50 0.129-0.138 vs 0.120-0.122 ms, with multi-ms stalls from waking the sleepers at
    // every call; profiles/r04_m6/ab_table.txt.)
    // Tasks of at least 1,280 windows: with the round-4 packer (~2.3 ns per 100-base window) a
    // 313-window task is shorter than the pool's contended claim, so a cfg2 end took ~15 us to pack
    // on 16 threads; 1,280 gave cfg2 stage p50 0.1189-0.1193 vs 0.1223-0.1243 ms at 256, 640 and 2,560
    // in between (same box, profiles/r04_m7/ab_table.txt).  AC_TASK_WINDOWS overrides (A/B runs).
    static const uint64_t min_task = (uint64_t)std::max(1, env_int("AC_TASK_WINDOWS", 1280));
    const uint64_t per = std::max<uint64_t>(
        min_task, std::min<uint64_t>(p.early ? std::max<uint64_t>(2048, min_task) : 65536, total_w / (4ull * pool.size()) + 1));
    std::vector<Task> tasks;
    for (uint32_t j = 0; j < p.n; ++j) {
        if (!jobs[j].n_kmers) continue;  // nothing to count: its windows are not needed
        for (uint64_t w = p.lo[j]; w < p.hi[j]; w += per)
            tasks.push_back({j, (uint32_t)w, (uint32_t)std::min<uint64_t>(p.hi[j], w + per), 0, 0, 0u, 0u});
    }
    const std::function<void(uint32_t)> span_of = [&](uint32_t t) {
        Task& x = tasks[t];
        x.bases = acamd::span_scan(jobs[x.job].sample.length + x.w0, x.w1 - x.w0, &x.first_len, &x.len_diff);
    };
    double tt = g_trace.on ? now_us() : 0.0;
    auto mark = [&](int i) {
        if (!g_trace.on) return;
        const double t = now_us();
        g_trace.sum[i] += t - tt;
        g_trace.cur[i] += t - tt;
        tt = t;
    };
    if (total_w <= (1u << 18)) {  // a serial pass is cheaper than a pool round trip up to ~256k windows
        for (uint32_t t = 0; t < (uint32_t)tasks.size(); ++t) span_of(t);
    } else {
        // in blocks of consecutive tasks, ~2 per participant: one pool task per packing task (~1,000 at
        // cfg4) spent ~220 us in contended claims for a ~30 us scan (profiles/r04_m1/bench_cfg4.log)
        const uint32_t nt = (uint32_t)tasks.size(), nb = std::min<uint32_t>(nt, 2u * pool.size());
        pool.run(nb, [&](uint32_t b) {
            for (uint32_t t = (uint32_t)((uint64_t)nt * b / nb); t < (uint32_t)((uint64_t)nt * (b + 1) / nb); ++t) span_of(t);
        });
    }
    mark(0);
    // Image of each job: its tasks' ranges back to back; at least one 32-base block.
    uint64_t acc[AC_MAX_JOBS] = {};
    for (Task& x : tasks) {
        const uint64_t b = x.bases;
        x.span = b;
        x.bases = acc[x.job];
        acc[x.job] += b;
    }
    size_t off = 0;
    for (uint32_t j = 0; j < p.n; ++j) {
        const uint32_t nw = jobs[j].n_kmers ? p.hi[j] - p.lo[j] : 0;
        p.n_bases[j] = std::max<uint64_t>(32, acc[j]);
        // the N bitmap, then the window descriptors: a job without N / with equal windows is
        // sent without them (job by job, below)
        p.off_kmers[j] = off;
        // (early launch: the k-mer section fills whole staging chunks, which the kernel copies
        // without waiting for the host -- the k-mers are in place before the launch)
        off = p.early ? off + (sizeof(uint64_t) * jobs[j].n_kmers + AC_STAGE_CHUNK - 1) / AC_STAGE_CHUNK * AC_STAGE_CHUNK
                      : align256(off + sizeof(uint64_t) * jobs[j].n_kmers);
        p.off_codes[j] = off;
        off = align256(off + sizeof(uint32_t) * (p.n_bases[j] / 16));
        p.off_nmask[j] = off;
        off = align256(off + sizeof(uint32_t) * (p.n_bases[j] / 32));
        p.off_start[j] = off;
        off = align256(off + sizeof(uint64_t) * nw);
        p.off_len[j] = off;
        off = align256(off + sizeof(uint32_t) * nw);
    }
    p.off_err = off;
    off = align256(off + sizeof(uint32_t));
    p.tag = p.early && !d_counts;
    for (uint32_t j = 0; j < p.n; ++j) {
        p.off_counts[j] = off;
        off = align256(off + (p.tag ? sizeof(uint64_t) : sizeof(uint32_t)) * jobs[j].n_kmers);
    }
    p.off_gerr = off;
    p.n_gerr = 0;
    if (p.tag) {
        const uint32_t cpw = acamd::cands_per_wave(acamd::pack_factor(k), true);  // (tagged: a staged launch)
        for (uint32_t j = 0; j < p.n; ++j)
            if (jobs[j].n_kmers && p.hi[j] > p.lo[j]) p.n_gerr += (jobs[j].n_kmers + cpw - 1) / cpw;
        off = align256(off + sizeof(uint64_t) * p.n_gerr);
    }
    p.total = off;
    // (the early launch's header and buffer descriptors count a segment's bytes in 31 bits)
    if (p.early && p.total >= (size_t(1) << 31)) p.early = p.tag = false;
    // equal windows (the common case: every start window sl bases, every end window sl + 1)
    uint32_t* ulen = p.ulen;
    // inline N records (nrec.h): equal windows whose slots leave room carry their N positions, so
    // the job's N bitmap is needed (and sent) only if some window overflowed its record
    bool* nrec = p.nrec;
    for (uint32_t j = 0; j < p.n; ++j) {
        bool any = false, equal = true;
        uint32_t l0 = 0;
        for (const Task& x : tasks)
            if (x.job == j) {
                if (!any) l0 = x.first_len;
                any = true;
                equal = equal && x.len_diff == 0u && x.first_len == l0;
            }
        ulen[j] = (any && equal) ? l0 : AC_NO_ULEN;
        nrec[j] = ulen[j] != AC_NO_ULEN && acamd::nrec_bits(ulen[j]) != 0u;
    }
    // Early launch: what the launch is made of -- the first `pre` jobs sent ahead of it (AC_STAGE_EARLY=2:
    // the first; a test hook: all), each job's region and chunks, the copier workgroups.
    size_t region[AC_MAX_JOBS] = {};
    if (p.early) {
        const uint32_t hooks = g_test_hooks.load(std::memory_order_relaxed);
        p.pre = (hooks & AC_TESTING_ALL_AHEAD) ? p.n : (stage_early() == 2 && p.n > 1) ? 1u : 0u;
        for (uint32_t j = 0; j < p.n; ++j) {
            const size_t end = ulen[j] != AC_NO_ULEN ? p.off_start[j] : (j + 1 < p.n ? p.off_kmers[j + 1] : p.off_err);
            region[j] = end - p.off_kmers[j];
            p.chunks[j] = j < p.pre ? 0u : (uint32_t)((region[j] + AC_STAGE_CHUNK - 1) / AC_STAGE_CHUNK);
            p.codes_off[j] = (uint32_t)(p.off_codes[j] - p.off_kmers[j]);
        }
        ensure_warm(ctx);
        const uint32_t P = acamd::pack_factor(k);
        if (!ctx->resident[1][P]) AC_HIP(ctx, acamd::resident_waves(P, true, ctx->cu_count, &ctx->resident[1][P]));
        uint64_t tickets = 0;
        for (uint32_t j = 0; j < p.n; ++j) tickets += p.chunks[j] ? p.chunks[j] + 1u : 0u;
        p.copiers = stage_copiers(tickets);
    }
    // Device packing: a job of equal windows (1..256 bases) whose Dna5 bytes and window
    // offsets lie in ac_host_alloc blocks is packed by the kernel's copier workgroups straight from them;
    // the host packs nothing of it (its region in the staging block stays unwritten).  Not with jobs sent
    // ahead of the launch (p.pre: those are host-packed and copied by the copy kernel).
    const uint8_t* dp_src[AC_MAX_JOBS] = {};
    const uint64_t* dp_off[AC_MAX_JOBS] = {};
    uint32_t dp_bytes[AC_MAX_JOBS] = {};
    p.dp_any = false;
    const int dpm = (g_test_hooks.load(std::memory_order_relaxed) & AC_TESTING_DEVICE_PACK) ? 1 : device_pack_mode();
    if (p.early && p.pre == 0 && (dpm == 1 || (dpm == 2 && total_w >= device_pack_min_windows())))
        for (uint32_t j = 0; j < p.n; ++j) {
            p.dp[j] = false;
            const ac_dna5_windows& w = jobs[j].sample;
            const uint32_t nw = p.hi[j] - p.lo[j];
            if (!jobs[j].n_kmers || !nw || ulen[j] == AC_NO_ULEN || ulen[j] == 0 || ulen[j] > 256 || !p.chunks[j]) continue;
            HostBlock bb, bo;
            if (!find_block(w.bases, 1, &bb) || !find_block(w.offset + p.lo[j], sizeof(uint64_t) * nw, &bo)) continue;
            const size_t extent = (size_t)(bb.h + bb.n - (const char*)w.bases);  // bytes readable from `bases`
            if (extent < ulen[j] || extent >= (size_t(1) << 31)) continue;
            p.dp[j] = p.dp_any = true;
            dp_src[j] = (const uint8_t*)(bb.d + ((const char*)w.bases - bb.h));
            dp_off[j] = (const uint64_t*)(bo.d + ((const char*)(w.offset + p.lo[j]) - bo.h));
            dp_bytes[j] = (uint32_t)extent;
        }
    if (p.dp_any) {  // the host packs only the other jobs' windows
        tasks.erase(std::remove_if(tasks.begin(), tasks.end(), [&](const Task& x) { return p.dp[x.job]; }), tasks.end());
    }
    // The slot: wait until the launch that last read it has finished, grow it.
    ac_ctx::Slot& sl = ctx->slot[p.slot];
    if (sl.pending) {
        AC_HIP(ctx, hipEventSynchronize(sl.ev));
        sl.pending = false;
    }
    if (!sl.ev) AC_HIP(ctx, hipEventCreateWithFlags(&sl.ev, hipEventDisableTiming));
    if (sl.h_cap < p.total) {
        if (sl.h) (void)hipHostFree(sl.h);
        sl.h = nullptr;
        sl.hd = nullptr;
        sl.h_cap = 0;
        const size_t cap = p.total + p.total / 4;
        AC_HIP(ctx, hipHostMalloc(&sl.h, cap, hipHostMallocDefault));
        sl.h_cap = cap;
        AC_HIP(ctx, hipHostGetDevicePointer(&sl.hd, sl.h, 0));
    }
    if (ac_status st = grow(ctx, &sl.d, &sl.d_cap, p.total)) return st;
    char* h = (char*)sl.h;
    for (uint32_t j = 0; j < p.n; ++j) {
        if (jobs[j].n_kmers) std::memcpy(h + p.off_kmers[j], jobs[j].kmers, sizeof(uint64_t) * jobs[j].n_kmers);
        if (acc[j] == 0) {  // no window bases: the one 32-base block is zero
            std::memset(h + p.off_codes[j], 0, 2 * sizeof(uint32_t));
            std::memset(h + p.off_nmask[j], 0, sizeof(uint32_t));
        }
    }
    *(uint32_t*)(h + p.off_err) = 0u;
    // tagged completion: no count or error word may carry this call's generation before the kernel
    // writes it (the slot last held other data)
    if (p.tag) std::memset(h + p.off_counts[0], 0, p.total - p.off_counts[0]);
    // early launch: flags cleared before the launch (the slot's last
    // launch has finished: its event was waited for above)
    const size_t hdr_bytes = sizeof(uint32_t) * AC_QUEUE_LINE * AC_HDR_LINES;
    if (p.early && !sl.hdr) {
        AC_HIP(ctx, hipHostMalloc((void**)&sl.hdr, hdr_bytes, hipHostMallocCoherent | hipHostMallocMapped));
        AC_HIP(ctx, hipHostGetDevicePointer((void**)&sl.hdr_d, sl.hdr, 0));
    }
    uint32_t* hdr = sl.hdr;
    if (p.early) std::memset(hdr, 0, hdr_bytes);
    mark(1);
    // per task: does the job need its N bitmap for these windows (an N, or with records an
    // overflowed record)
    std::vector<uint8_t> task_n(tasks.size(), 0);
    const std::function<void(uint32_t)> pack = [&](uint32_t t) {
        const Task& x = tasks[t];
        const ac_dna5_windows& w = jobs[x.job].sample;
        const uint32_t j = x.job, r = x.w0 - p.lo[j];
        const uint32_t f = acamd::pack_dna5_range(w.bases, w.offset, w.length, x.w0, x.w1, x.bases,
                                                  (uint32_t*)(h + p.off_codes[j]), (uint32_t*)(h + p.off_nmask[j]),
                                                  (uint64_t*)(h + p.off_start[j]) + r,
                                                  (uint32_t*)(h + p.off_len[j]) + r, nrec[j]);
        task_n[t] = (f & (nrec[j] ? acamd::PACK_OVERFLOW : acamd::PACK_HAS_N)) != 0u;
    };
    bool no_n[AC_MAX_JOBS] = {};
    auto job_no_n = [&](uint32_t j) {
        for (size_t t = 0; t < tasks.size(); ++t)
            if (tasks[t].job == j && task_n[t]) return false;
        return true;
    };
    char* d = (char*)sl.d;
    // The kernel writes the error word and the counts straight into the pinned block (hd), so
    // no copy comes back (profiles/r02_stage_dma_back_ab.log).
    char* hd = (char*)sl.hd;
    auto make_segs = [&](ac_segment* segs) {
        uint64_t cbase = 0;
        for (uint32_t j = 0; j < p.n; ++j) {
            ac_segment& g = segs[j];
            const uint32_t nw = jobs[j].n_kmers ? p.hi[j] - p.lo[j] : 0;
            g.kmers = (const uint64_t*)(d + p.off_kmers[j]);
            g.n_kmers = jobs[j].n_kmers;
            g.sample = ac_windows{(const uint32_t*)(d + p.off_codes[j]), (const uint32_t*)(d + p.off_nmask[j]),
                                  (const uint64_t*)(d + p.off_start[j]), (const uint32_t*)(d + p.off_len[j]), nw,
                                  p.n_bases[j]};
            g.counts = d_counts ? d_counts + cbase : (uint32_t*)(hd + p.off_counts[j]);
            cbase += jobs[j].n_kmers;
        }
    };
    if (p.early) {
        // Early launch: the count kernel is launched before the later jobs are
        // packed; the pool packs job by job and the host flags each job in the header as soon
        // as it is complete; the kernel copies a flagged job's region into device memory itself
        // and counts it while the next job is still being packed.  The region of job j: k-mers,
        // codes, then the N bitmap unless the job holds no N, and the window descriptors unless
        // its windows have one length.  The first `pre` jobs (AC_STAGE_EARLY=2: the first) are
        // sent before the launch by the copy kernel instead, stream-ordered ahead of it.
        // (AC_STAGE_EARLY=3, diagnostic: every job sent ahead, so the staged kernel runs on resident
        // input -- its own cost against the plain kernel's)
        const uint32_t hooks = g_test_hooks.load(std::memory_order_relaxed);
        const uint32_t pre = p.pre;
        // (Packing the jobs' tasks interleaved, so both ends arrive together, was slower:
        // 0.144 vs 0.134 ms per cfg2 step -- each end's last chunk waits for its final header,
        // which then came ~27 us into the kernel for both; profiles/r03_stage/r03_early12_step3.log.)
        StageLaunch stg;
        if (++ctx->gen == 0) ++ctx->gen;
        p.gen = stg.gen = ctx->gen;
        stg.host_hdr = sl.hdr_d;
        stg.err_out = d_counts ? ctx->d_err : nullptr;  // a submit reports through ac_check
        stg.tag = p.tag ? 1u : 0u;
        stg.grp_err = p.tag ? (uint64_t*)(hd + p.off_gerr) : nullptr;
        for (uint32_t j = 0; j < p.n; ++j) {
            stg.src[j] = (const uint8_t*)(hd + p.off_kmers[j]);
            stg.dst[j] = (uint8_t*)(d + p.off_kmers[j]);
            stg.chunks[j] = p.chunks[j];
            stg.codes_off[j] = p.codes_off[j];
        }
        stg.copiers = p.copiers;
        for (uint32_t j = 0; j < p.n; ++j) {
            stg.dp_src[j] = dp_src[j];
            stg.dp_off[j] = dp_off[j];
            stg.dp_bytes[j] = dp_bytes[j];
        }
        // A large call (copier workgroups) packs its jobs' tasks interleaved, so every segment's
        // windows arrive from the start and no segment's waves sit idle while the jobs before it are
        // packed (each copier workgroup starts on its own segment, wm_count.hip).  Small calls keep
        // job order (see above).
        if (stg.copiers && p.n > 1 && pre == 0) {
            std::vector<Task> by_job[AC_MAX_JOBS];
            for (const Task& x : tasks) by_job[x.job].push_back(x);
            tasks.clear();
            for (size_t i = 0; tasks.size() < task_n.size(); ++i)
                for (uint32_t j = 0; j < p.n; ++j)
                    if (i < by_job[j].size()) tasks.push_back(by_job[j][i]);
        }
        // (the slot's event is recorded after the publishing loop, not right after the launch: the
        // caller's first progress records went out 1.2 us later with it there)
        bool launched = false;
        auto record_slot = [&]() -> ac_status {
            if (!launched) return AC_OK;
            launched = false;
            AC_HIP(ctx, hipEventRecord(sl.ev, stream));
            sl.pending = true;
            return AC_OK;
        };
        auto go = [&]() -> ac_status {
            ac_segment segs[AC_MAX_JOBS];
            make_segs(segs);
            if (ac_status st = launch(ctx, k, segs, p.n, stream, zero, nullptr, p.scratch, 0, no_n, ulen, &stg, nrec))
                return st;
            mark(4);
            launched = true;
            return AC_OK;
        };
        // Progress records: the packed N-free prefix of each job's region (its k-mers, then the
        // codes of its first tasks up to the first task holding an N), so the kernel moves chunks
        // over PCIe -- and counts their windows -- while the rest of the job is packed.  Tasks are
        // claimed in order but finish out of order; this thread alone publishes (a plain 8-byte
        // store, read whole by the kernel's 16-byte header load): between the tasks it packs
        // itself, it advances over the tasks the workers have finished.  (Publishing from the
        // workers -- CAS on the one header line the GPU polls -- cost ~7 us of packing per call.)
        struct alignas(64) Done {
            std::atomic<uint32_t> v;
        };
        std::unique_ptr<Done[]> t_done(new Done[tasks.size() + 1]);
        for (size_t t = 0; t < tasks.size(); ++t) t_done[t].v.store(0, std::memory_order_relaxed);
        const bool slow_host = (hooks & AC_TESTING_SLOW_HOST) != 0u;  // (test-only hook)
        uint32_t slow_left = slow_host ? 12u : 0u;
        auto publish = [&](uint32_t j, uint64_t ready) {
            __atomic_store_n((uint64_t*)(hdr + j * AC_QUEUE_LINE + AC_HDR_PGEN), (ready << 32) | p.gen, __ATOMIC_RELEASE);
            if (launched && slow_left) {
                --slow_left;
                std::this_thread::sleep_for(std::chrono::milliseconds(60));
            }
        };
        const std::function<void(uint32_t)> pack_counted = [&](uint32_t t) {
            pack(t);
            t_done[t].v.store(1, std::memory_order_release);
        };
        // the k-mers are in place already (copied with the layout)
        for (uint32_t j = 0; j < p.n; ++j) publish(j, p.off_codes[j] - p.off_kmers[j]);
        // the workers start packing job 0 while this thread launches the kernel
        pool.begin((uint32_t)tasks.size(), pack_counted);
        if (pre == 0)
            if (ac_status st = go()) {
                pool.finish();
                return st;
            }
#ifndef AC_PUBLISH_STEP
#define AC_PUBLISH_STEP 16384
#endif
        constexpr uint64_t PUBLISH_STEP = AC_PUBLISH_STEP;  // bytes of new prefix worth a header store
        // per job: its tasks in claim order
        std::vector<uint32_t> jt[AC_MAX_JOBS];
        for (uint32_t t = 0; t < (uint32_t)tasks.size(); ++t) jt[tasks[t].job].push_back(t);
        uint64_t ready[AC_MAX_JOBS], published[AC_MAX_JOBS];
        uint32_t nt[AC_MAX_JOBS];  // jt[j][0, nt[j]) seen finished
        bool n_seen[AC_MAX_JOBS] = {}, flagged[AC_MAX_JOBS] = {};
        for (uint32_t j = 0; j < p.n; ++j) {
            ready[j] = published[j] = p.off_codes[j] - p.off_kmers[j];
            nt[j] = 0;
        }
        uint32_t helped = 0, left_jobs = p.n;
        for (uint32_t j = 0; j < p.n; ++j)
            if (p.dp[j]) {  // the kernel publishes a device-packed job's words itself: nothing to flag
                flagged[j] = true;
                --left_jobs;
            }
        bool first_flag = true;
        // Job j is finished: its final byte count and N verdict, then its flag (or, jobs below
        // `pre`, the copy kernel sends it ahead of the launch; those finish in job order).
        auto finalize = [&](uint32_t j) -> ac_status {
            const bool nn = job_no_n(j);
            const size_t bytes = nn && ulen[j] != AC_NO_ULEN ? p.off_nmask[j] - p.off_kmers[j] : region[j];
            if (j < pre) {  // sent ahead of the launch, which follows it on the stream
                no_n[j] = nn;
                hipError_t e = stage_blit_launch(hd + p.off_kmers[j], d + p.off_kmers[j], bytes, stream);
                ac_status st = e == hipSuccess ? AC_OK : hip_fail(ctx, e, "stage transfer");
                if (st == AC_OK && j + 1 == pre) st = go();
                return st;
            }
            uint32_t* line = hdr + j * AC_QUEUE_LINE;
            // no N: the whole region is N-free (never below a prefix: the codes end inside the
            // bytes sent); with N the published prefix stays where the first N stopped it
            if (nn) publish(j, bytes);
            line[AC_HDR_INFO] = (uint32_t)bytes | (nn ? 0u : AC_HDR_INFO_HAS_N);
            // (test-only hook: the last job left unflagged, tests/test_gpu_jobs.py)
            if (!((hooks & AC_TESTING_UNFLAG_LAST) && j + 1 == p.n))
                __atomic_store_n(&line[AC_HDR_FLAG], p.gen, __ATOMIC_RELEASE);  // the kernel's waves may go
            if (first_flag) mark(3);  // (AC_STAGE_TRACE: launch -> first job flagged, in "h2d_enq")
            first_flag = false;
            return AC_OK;
        };
        // With workers, this thread only publishes: packing a task of its own (~8 us at cfg2's
        // 312-window tasks) held every progress record back until it was done.  It still packs when
        // no worker has finished a task for 20 us (workers asleep or descheduled).
        const bool serial = pool.serial();
        // ... except when packing, not publishing, is the bottleneck: a pool of <= 4 participants (a
        // rank's share of the host) or a large call (the kernel counts faster than a few threads
        // pack), where a task of its own delays the records by one task but adds a packer.
        const bool caller_packs = !serial && (pool.size() <= 4 || total_w >= (1u << 16));
        uint32_t seen_done = 0, idle_polls = 0;
        auto last_seen = std::chrono::steady_clock::now();
        while (left_jobs) {
            bool help_now = false;
            if (!serial && (++idle_polls & 63u) == 0u) {
                uint32_t d = 0;
                for (uint32_t j = 0; j < p.n; ++j) d += nt[j];
                const auto now = std::chrono::steady_clock::now();
                if (d != seen_done) {
                    seen_done = d;
                    last_seen = now;
                } else if (now - last_seen > std::chrono::microseconds(20)) {
                    help_now = true;
                    last_seen = now;
                }
            }
            if (serial && helped < (uint32_t)tasks.size()) pool.help(++helped);  // packs task helped - 1
            else if (help_now || caller_packs) pool.help_one();
            for (uint32_t j = 0; j < p.n; ++j) {
                if (flagged[j] || (j > 0 && j <= pre && !flagged[j - 1])) continue;  // (pre: in job order)
                const uint64_t base_off = p.off_codes[j] - p.off_kmers[j];
                const uint32_t nj = (uint32_t)jt[j].size();
                while (nt[j] < nj && t_done[jt[j][nt[j]]].v.load(std::memory_order_acquire)) {
                    const Task& x = tasks[jt[j][nt[j]]];
                    // (with records the kernel counts any packed window; one that overflowed its
                    // record waits for the job's N bitmap by itself)
                    n_seen[j] = n_seen[j] || (task_n[jt[j][nt[j]]] && !nrec[j]);
                    if (!n_seen[j]) ready[j] = base_off + (x.bases + x.span) / 4;
                    ++nt[j];
                }
                // (the first codes at once, however few: the kernel may be waiting for them)
                if (ready[j] >= published[j] + PUBLISH_STEP || (nt[j] == nj && ready[j] > published[j]) ||
                    (published[j] == base_off && ready[j] > published[j])) {
                    // (test-only slow host: one step per record while its sleeps last)
                    const uint64_t r = slow_left ? std::min(ready[j], published[j] + PUBLISH_STEP) : ready[j];
                    publish(j, r);
                    published[j] = r;
                }
                if (nt[j] == nj && published[j] == ready[j]) {
                    if (ac_status st = finalize(j)) {
                        pool.finish();
                        (void)record_slot();
                        return st;
                    }
                    flagged[j] = true;
                    --left_jobs;
                }
            }
            if (!(serial && helped < (uint32_t)tasks.size()) && left_jobs) __builtin_ia32_pause();
        }
        pool.finish();
        mark(2);
        return record_slot();
    }
    // DMA mode sends the inputs [r0, r1) of the slot (copy engine or blit kernel)
    auto transfer = [&](size_t r0, size_t r1) -> hipError_t {
        if (r1 <= r0) return hipSuccess;
        if (part == 0 && wave_div == 0) return stage_blit_launch(hd + r0, d + r0, r1 - r0, stream);
        return hipMemcpyAsync(d + r0, h + r0, r1 - r0, hipMemcpyHostToDevice, stream);
    };
    if (p.n > 1) {
        // job by job: job j's inputs travel while job j + 1 is packed.  One pool job for all
        // tasks (they are in job order); the caller packs job j's share, waits for its last
        // task, sends it, then helps with job j + 1 while the workers carry on.
        std::atomic<uint32_t> left[AC_MAX_JOBS];
        for (uint32_t j = 0; j < AC_MAX_JOBS; ++j) left[j].store(0, std::memory_order_relaxed);
        for (const Task& x : tasks) left[x.job].fetch_add(1, std::memory_order_relaxed);
        const std::function<void(uint32_t)> pack_counted = [&](uint32_t t) {
            pack(t);
            left[tasks[t].job].fetch_sub(1, std::memory_order_release);
        };
        pool.begin((uint32_t)tasks.size(), pack_counted);
        uint32_t t0 = 0;
        for (uint32_t j = 0; j < p.n; ++j) {
            uint32_t t1 = t0;
            while (t1 < (uint32_t)tasks.size() && tasks[t1].job == j) ++t1;
            pool.help(t1);
            while (left[j].load(std::memory_order_acquire) != 0u) __builtin_ia32_pause();
            no_n[j] = job_no_n(j);
            if (const hipError_t e = transfer(p.off_kmers[j], no_n[j] ? p.off_nmask[j] : p.off_start[j]); e != hipSuccess) {
                pool.finish();
                return hip_fail(ctx, e, "stage transfer");
            }
            if (ulen[j] == AC_NO_ULEN) {
                const hipError_t e = transfer(p.off_start[j], j + 1 < p.n ? p.off_kmers[j + 1] : p.off_err);
                if (e != hipSuccess) {
                    pool.finish();
                    return hip_fail(ctx, e, "stage transfer");
                }
            }
            t0 = t1;
        }
        pool.finish();
        mark(2);
    } else {
        pool.run((uint32_t)tasks.size(), pack);
        for (uint32_t j = 0; j < p.n; ++j) no_n[j] = job_no_n(j);
        mark(2);
        AC_HIP(ctx, transfer(0, p.off_err));
    }
    mark(3);
    ac_segment segs[AC_MAX_JOBS];
    make_segs(segs);
    // the synchronous path reads the error word back with the counts; a
    // submit reports through the context's word (ac_check)
    uint64_t cap = 0;
    if (wave_div > 1) {
        const uint32_t P = acamd::pack_factor(k);
        if (!ctx->resident[0][P]) AC_HIP(ctx, acamd::resident_waves(P, false, ctx->cu_count, &ctx->resident[0][P]));
        cap = ctx->resident[0][P] / wave_div;
    }
    if (ac_status st = launch(ctx, k, segs, p.n, stream, zero, d_counts ? nullptr : (uint32_t*)(hd + p.off_err),
                              p.scratch, cap, no_n, ulen, nullptr, nrec))
        return st;
    mark(4);
    mark(5);
    AC_HIP(ctx, hipEventRecord(sl.ev, stream));
    sl.pending = true;
    return AC_OK;
}

// Shard g of G of job windows [0, n): contiguous, balanced by bases (the rule
// of ac_error_count's multi-device split and approx_counter_amd/shard.py).
// All G + 1 cut points of job windows [0, n) in one pass (shard g = [cut[g], cut[g + 1])).
std::vector<uint32_t> shard_cuts(const uint32_t* length, uint32_t n, size_t G) {
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; ++i) total += length[i];
    std::vector<uint32_t> cut(G + 1, n);
    cut[0] = 0;
    uint64_t acc = 0;
    size_t c = 1;
    for (uint32_t i = 0; i < n && c < G; ++i) {
        acc += length[i];
        while (c < G && acc * G >= total * c) cut[c++] = i + 1;
    }
    return cut;
}

// The two parts of a single-device call: windows [0, cut) and [cut, n), the
// first holding `frac` of the bases.
uint32_t part_cut(const uint32_t* length, uint32_t n, double frac) {
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; ++i) total += length[i];
    const double want = frac * (double)total;
    uint64_t acc = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if ((double)acc >= want) return i;
        acc += length[i];
    }
    return n;
}

// Every job's part boundaries of a single-device call in `parts` parts, once
// (equal shares of the bases).
std::vector<std::vector<uint32_t>> part_cuts(const ac_job* jobs, uint32_t n_jobs, int parts) {
    std::vector<std::vector<uint32_t>> cuts;
    for (uint32_t j = 0; j < n_jobs; ++j) {
        const uint32_t n = jobs[j].sample.n_windows;
        if (parts == 1)
            cuts.push_back({0u, n});
        else if (parts == 2)
            cuts.push_back({0u, part_cut(jobs[j].sample.length, n, 0.5), n});
        else
            cuts.push_back(shard_cuts(jobs[j].sample.length, n, (size_t)parts));
    }
    return cuts;
}

}  // namespace

namespace {

// The synchronous jobs stage (ac_error_count_jobs).  allow_early = false: the DMA path whatever
// AC_STAGE_EARLY says.  *stage_timeout: the early launch gave up waiting for the host's inputs.
ac_status count_jobs_sync(ac_ctx* ctx, uint32_t k, const ac_job* jobs, uint32_t n_jobs, bool allow_early,
                          bool* stage_timeout) {
    *stage_timeout = false;
    // Units of work: on an ac_create_multi context one per device (shard g of
    // every job's windows on context g); on one device up to AC_STAGE_MAX_PARTS
    // parts on their own streams, the first launched with half the resident
    // waves so the second part's waves run beside it as soon as its DMA lands.
    struct Unit {
        ac_ctx* c;
        int part;
        hipStream_t stream;
        uint32_t wave_div;
        JobPlan plan;
    };
    std::vector<Unit> units;
    uint64_t total_w = 0;
    for (uint32_t j = 0; j < n_jobs; ++j) total_w += jobs[j].sample.n_windows;
    if (!ctx->peers.empty()) {
        const size_t G = ctx->peers.size() + 1;
        std::vector<std::vector<uint32_t>> cuts;
        for (uint32_t j = 0; j < n_jobs; ++j) cuts.push_back(shard_cuts(jobs[j].sample.length, jobs[j].sample.n_windows, G));
        for (size_t g = 0; g < G; ++g) {
            Unit u{g == 0 ? ctx : ctx->peers[g - 1], 0, nullptr, 0, JobPlan()};
            u.stream = u.c->stream;
            u.plan.n = n_jobs;
            u.plan.slot = 0;
            u.plan.scratch = 0;
            for (uint32_t j = 0; j < n_jobs; ++j) {
                u.plan.lo[j] = cuts[j][g];
                u.plan.hi[j] = cuts[j][g + 1];
            }
            units.push_back(u);
        }
    } else {
        // The early launch takes every size in one part (large ones through copier workgroups); the
        // copy-engine parts remain for AC_STAGE_EARLY=0.  (A region of 2^31 bytes or more falls back
        // to one DMA part inside stage_and_launch.)
        const bool early = allow_early && stage_early() && live_work(jobs, n_jobs);
        const int parts = (!early && total_w >= 2048) ? stage_parts(total_w) : 1;
        const std::vector<std::vector<uint32_t>> cuts = part_cuts(jobs, n_jobs, parts);
        for (int q = 0; q < parts; ++q) {
            if (q > 0 && !ctx->part_stream[q])
                AC_HIP(ctx, hipStreamCreateWithFlags(&ctx->part_stream[q], hipStreamNonBlocking));
            Unit u{ctx, q, q == 0 ? ctx->stream : ctx->part_stream[q], (parts > 1 && q == 0) ? 2u : 0u, JobPlan()};
            u.plan.n = n_jobs;
            u.plan.slot = q;
            u.plan.scratch = q;
            if (early) {
                // one part: the early-launch stage (alternating slots 0 / 1, so a call never waits for
                // the previous call's launch to retire before it packs)
                u.plan.early = true;
                u.plan.slot = (int)ctx->early_flip;
                ctx->early_flip ^= 1u;
            }
            for (uint32_t j = 0; j < n_jobs; ++j) {
                u.plan.lo[j] = cuts[j][q];
                u.plan.hi[j] = cuts[j][q + 1];
            }
            units.push_back(u);
        }
    }
    // Units are staged one after another on the host pool; a unit's DMA and
    // kernel run while the next one is packed.
    for (size_t g = 0; g < units.size(); ++g) {
        Unit& u = units[g];
        AC_HIP(u.c, hipSetDevice(u.c->device));
        if (ac_status st = stage_and_launch(u.c, k, jobs, u.plan, u.stream, nullptr, u.part, u.wave_div))
            return u.c != ctx ? fail(ctx, st, "shard " + std::to_string(g) + ": " + u.c->err) : st;
    }
    for (uint32_t j = 0; j < n_jobs; ++j)
        for (uint32_t i = 0; i < jobs[j].n_kmers; ++i) jobs[j].counts[i] = 0;
    ac_status first_err = AC_OK;
    double t_sync = g_trace.on ? now_us() : 0.0;
    for (size_t g = 0; g < units.size(); ++g) {
        Unit& u = units[g];
        AC_HIP(u.c, hipSetDevice(u.c->device));
        ac_ctx::Slot& sl = u.c->slot[u.plan.slot];
        const char* h = (const char*)sl.h;
        uint32_t err_word;
        if (u.plan.tag) {
            // every count and every group's error word is tagged with the launch's generation: poll
            // them instead of the stream (the launch's event is waited for when the slot is next used)
            if (ac_status st = wait_tagged(u.c, jobs, n_jobs, u.plan, h, u.stream)) return st;
            err_word = 0;
            const uint64_t* ge = (const uint64_t*)(h + u.plan.off_gerr);
            for (uint32_t i = 0; i < u.plan.n_gerr; ++i) err_word |= (uint32_t)ge[i];
        } else {
            AC_HIP(u.c, hipStreamSynchronize(u.stream));
            sl.pending = false;
            err_word = *(const uint32_t*)(h + u.plan.off_err);
        }
        if (g_trace.on && g + 1 == units.size()) {
            const double t = now_us();
            g_trace.sum[6] += t - t_sync;
            g_trace.cur[6] += t - t_sync;
            t_sync = t;
        }
        if (u.plan.early && (err_word & AC_DEVERR_STAGE)) *stage_timeout = true;
        if (ac_status st = device_error(u.c, err_word)) {
            if (first_err == AC_OK)
                first_err = u.c != ctx ? fail(ctx, st, "shard " + std::to_string(g) + ": " + u.c->err) : st;
            continue;
        }
        for (uint32_t j = 0; j < n_jobs; ++j) {
            if (u.plan.tag) {
                const uint64_t* hc = (const uint64_t*)(h + u.plan.off_counts[j]);
                if (u.plan.hi[j] > u.plan.lo[j])  // (a job without windows here: its counts are 0)
                    for (uint32_t i = 0; i < jobs[j].n_kmers; ++i) jobs[j].counts[i] += (uint32_t)hc[i];
                continue;
            }
            const uint32_t* hc = (const uint32_t*)(h + u.plan.off_counts[j]);
            for (uint32_t i = 0; i < jobs[j].n_kmers; ++i) jobs[j].counts[i] += hc[i];
        }
    }
    if (first_err == AC_OK) units[0].c->last_mode = units[0].plan.dp_any ? 3 : units[0].plan.early ? 2 : 0;
    if (g_trace.on) {
        g_trace.sum[7] += now_us() - t_sync;
        g_trace.cur[7] += now_us() - t_sync;
        ++g_trace.calls;
        g_trace.skip_warmup();
        g_trace.end_call();
    }
    return first_err;
}

}  // namespace

extern "C" {

ac_status ac_error_count_jobs(ac_ctx* ctx, uint32_t k, const ac_job* jobs, uint32_t n_jobs) {
    if (ac_status st = check_jobs(ctx, k, jobs, n_jobs)) return st;
    for (uint32_t j = 0; j < n_jobs; ++j)
        if (jobs[j].n_kmers && !jobs[j].counts) return fail(ctx, AC_ERR_INVALID, "job counts is NULL");
    if (n_jobs == 0) return AC_OK;
    bool stage_timeout = false;
    const ac_status st = count_jobs_sync(ctx, k, jobs, n_jobs, true, &stage_timeout);
    // An early launch whose host inputs stopped arriving for 0.5 s (a stalled host: the kernel's waits
    // restart their clock on every bit of progress) skipped its work and said so: the call is run
    // again through the DMA path, which has no such wait, instead of failing.
    if (st != AC_OK && stage_timeout) {
        std::fprintf(stderr, "[approx_counter_amd] early launch timed out waiting for the host; retrying via DMA\n");
        return count_jobs_sync(ctx, k, jobs, n_jobs, false, &stage_timeout);
    }
    return st;
}

uint32_t ac_testing_stage_hooks(uint32_t flags) { return g_test_hooks.exchange(flags); }


ac_status ac_error_count_jobs_submit(ac_ctx* ctx, uint32_t k, const ac_job* jobs, uint32_t n_jobs,
                                     uint32_t* d_counts, void* hip_stream) {
    if (ac_status st = check_jobs(ctx, k, jobs, n_jobs)) return st;
    if (!ctx->peers.empty())
        return fail(ctx, AC_ERR_INVALID, "ac_error_count_jobs_submit needs a single-device context");
    uint64_t n_counts = 0, total_w = 0;
    for (uint32_t j = 0; j < n_jobs; ++j) {
        n_counts += jobs[j].n_kmers;
        total_w += jobs[j].sample.n_windows;
    }
    if (n_counts && !d_counts) return fail(ctx, AC_ERR_INVALID, "d_counts is NULL");
    if (n_jobs == 0) return AC_OK;
    AC_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t caller = (hipStream_t)hip_stream;
    // Large submits are cut into parts like the synchronous stage (a rank's shard of cfg4 is
    // 2^17-2^18 windows): part q + 1 is packed and sent while part q counts.  The parts add
    // into d_counts, zeroed first on the caller's stream; parts 1.. run on the context's
    // submit streams, ordered after the zeroing and joined back into the caller's stream.
    // Submits alternate between two sets of staging slots, so a submit packs while the
    // previous one's launch may still read its inputs.
    const bool early = stage_early() && live_work(jobs, n_jobs);  // every size in one part (as above)
    const int parts = (!early && total_w >= 2048) ? stage_parts(total_w) : 1;
    const int set = (int)ctx->next_slot;
    ctx->next_slot ^= 1u;
    const std::vector<std::vector<uint32_t>> cuts = part_cuts(jobs, n_jobs, parts);
    if (parts > 1) {
        AC_HIP(ctx, hipMemsetAsync(d_counts, 0, sizeof(uint32_t) * n_counts, caller));
        if (!ctx->sub_zero_ev) AC_HIP(ctx, hipEventCreateWithFlags(&ctx->sub_zero_ev, hipEventDisableTiming));
        AC_HIP(ctx, hipEventRecord(ctx->sub_zero_ev, caller));
    }
    for (int q = 0; q < parts; ++q) {
        hipStream_t st = caller;
        if (q > 0) {
            if (!ctx->sub_stream[q]) AC_HIP(ctx, hipStreamCreateWithFlags(&ctx->sub_stream[q], hipStreamNonBlocking));
            if (!ctx->sub_ev[q]) AC_HIP(ctx, hipEventCreateWithFlags(&ctx->sub_ev[q], hipEventDisableTiming));
            st = ctx->sub_stream[q];
            AC_HIP(ctx, hipStreamWaitEvent(st, ctx->sub_zero_ev, 0));
        }
        JobPlan p;
        p.n = n_jobs;
        for (uint32_t j = 0; j < n_jobs; ++j) {
            p.lo[j] = cuts[j][q];
            p.hi[j] = cuts[j][q + 1];
        }
        p.slot = AC_STAGE_MAX_PARTS * (1 + set) + q;
        p.scratch = AC_STAGE_MAX_PARTS + q;
        // one part: the early launch, counts and errors into device memory (ac_check reads them)
        p.early = early;
        if (ac_status rc = stage_and_launch(ctx, k, jobs, p, st, d_counts, q, (parts > 1 && q == 0) ? 2u : 0u,
                                            parts == 1))
            return rc;
        if (q > 0) AC_HIP(ctx, hipEventRecord(ctx->sub_ev[q], st));
        if (q == 0) ctx->last_mode = p.dp_any ? 3 : p.early ? 2 : 0;
    }
    for (int q = 1; q < parts; ++q) AC_HIP(ctx, hipStreamWaitEvent(caller, ctx->sub_ev[q], 0));
    if (g_trace.on) {
        ++g_trace.calls;
        g_trace.skip_warmup();
        g_trace.end_call();
    }
    return AC_OK;
}

int ac_exact_path(const ac_ctx* ctx) { return ctx ? ctx->exact_path : -1; }

int ac_stage_mode(const ac_ctx* ctx) { return ctx ? ctx->last_mode : -1; }

#ifdef AC_STAMPS
// Diagnostic builds only: per-wave timestamps of the last launch (not declared in the public header).
int ac_debug_stamps(void* host, size_t bytes) { return (int)acamd::debug_stamps(host, bytes); }
#endif

}  // extern "C"
