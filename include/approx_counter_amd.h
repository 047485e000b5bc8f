/*
 * approx_counter_amd.h -- C ABI of the MI355X approximate-count stage.
 *
 * Drop-in boundary for qbonenfant/approx_counter's hot path.  The reference
 * has no plugin/FFI API; its one internal seam on the hot
 * path is
 *
 *     counter errorCount(sequence_set_type& sequences, pair_vector& exact_count,
 *                        uint8_t nb_thread, uint8_t k, uint8_t v);
 *                                              -- approx_counter.cpp:531
 *
 * called once per (run, end) from main (approx_counter.cpp:922).  Every entry
 * point below names the reference code it replaces.  Plain C types only; no
 * exceptions and no exit() cross this boundary: every call returns an
 * ac_status (0 = OK) and the text of the last failure is available from
 * ac_last_error().  The library has no CPU fallback: without a HIP device
 * ac_create() fails with AC_ERR_DEVICE.
 *
 * Counting contract (model M1): for every candidate k-mer,
 *     count = sum over windows w of max(0, 3 - d(kmer, w))
 * where d is the semi-global Levenshtein distance between the whole k-mer and
 * the best substring of w, a non-ACGT base matching nothing.  This equals the
 * reference's  sum_e popcount(tcount[e])  (approx_counter.cpp:553-593) under
 * SeqAn 2.4's find<0,2>(..., EditDistance()) semantics.
 */
#ifndef APPROX_COUNTER_AMD_H
#define APPROX_COUNTER_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AC_ABI_VERSION 8

typedef int32_t ac_status;
#define AC_OK 0
#define AC_ERR_INVALID 1  /* bad argument (k outside [2,32], NULL pointer, layout) */
#define AC_ERR_DEVICE 2   /* no HIP device, or a HIP runtime failure               */
#define AC_ERR_NOMEM 3    /* device or host allocation failed                     */
#define AC_ERR_INTERNAL 4

typedef struct ac_ctx ac_ctx;

/*
 * Packed sample ("window image").  Replaces the StringSet<Dna5String> sample
 * (approx_counter.cpp:38, built by sampleSequences 415-476).
 *   codes : 2 bits per base (A0 C1 G2 T3; any value for N), base b at bits
 *           2*(b%16)..2*(b%16)+1 of codes[b/16]          (n_bases/16 words)
 *   nmask : bit (b%32) of nmask[b/32] set iff base b is not A/C/G/T
 *           (Dna5 ordValue 4, "N")                       (n_bases/32 words)
 *   start : window i occupies bases [start[i], start[i]+length[i]);
 *           start[i] % 32 == 0 (each window begins on a 32-base boundary)
 *   length: window length in bases (sl for a start window, sl+1 for an end
 *           window, approx_counter.cpp:463/466); 0 is allowed
 *   n_bases: size of the image in bases, a multiple of 32 below 2^34
 * All pointers are host pointers for ac_error_count() and device pointers for
 * the *_device entry points.
 */
typedef struct ac_windows {
    const uint32_t* codes;
    const uint32_t* nmask;
    const uint64_t* start;
    const uint32_t* length;
    uint32_t n_windows;
    uint64_t n_bases;
} ac_windows;

/* One approximate-count job = one errorCount call (approx_counter.cpp:922). */
typedef struct ac_segment {
    const uint64_t* kmers; /* dna2int layout (approx_counter.cpp:55-62)     */
    uint32_t n_kmers;
    ac_windows sample;
    uint32_t* counts;      /* n_kmers counters, input order                 */
} ac_segment;

/* Opens a context on HIP device `device` (-1: the current device).  Replaces
 * the index construction + omp_set_num_threads of errorCount (537-547). */
ac_status ac_create(ac_ctx** out, int device);
void ac_destroy(ac_ctx* ctx);
/*
 * A context over `n_gpus` devices of this node (device g mod the visible
 * devices for shard g; SURVEY.md §8(b) "ac_create(ac_ctx**, int n_gpus)").
 * ac_error_count and ac_count on it split the windows into n_gpus contiguous
 * shards balanced by bases, count each shard on its device concurrently and
 * sum the counts on the host (errorCount's OpenMP loop, 547-599, spread over
 * GPUs; integer sums, so bit-identical to one device).  The device-buffer
 * entry points use the first device only.  n_gpus = 1 is ac_create(out, 0).
 */
ac_status ac_create_multi(ac_ctx** out, int n_gpus);

/*
 * SURVEY.md §8(b)'s count entry point, argument for argument: errorCount
 * (531-601) over windows given as a 2-bit image (win_bits, 16 bases per
 * little-endian u32, A0 C1 G2 T3) and an N bitmap (win_nmask, 32 bases per
 * u32); window i starts at 2-bit word win_word_offset[i] (an even word: 32-base
 * aligned, so the same offset indexes the bitmap) and holds win_len[i] bases.
 * counts_out[i] = M1 count of kmers[i].  Synchronous, host buffers.
 */
ac_status ac_count(ac_ctx* ctx, uint32_t k, const uint64_t* kmers, uint32_t n_kmers, const uint32_t* win_bits,
                   const uint32_t* win_nmask, const uint64_t* win_word_offset, const uint16_t* win_len,
                   uint32_t n_windows, uint64_t* counts_out);

/* Number of HIP devices visible to this process (0 without a GPU).  The
 * reference has no counterpart: its errorCount runs on the host's OpenMP
 * threads (approx_counter.cpp:547); the CLI uses this to map -g shards onto
 * devices. */
int ac_device_count(void);
/* Last failure text for ctx (or for the calling thread when ctx is NULL). */
const char* ac_last_error(const ac_ctx* ctx);
int ac_abi_version(void);

/*
 * errorCount (approx_counter.cpp:531-601), host buffers in and out:
 * counts[i] = M1 count of kmers[i] over `sample`.  Copies the inputs to the
 * device, runs the HIP kernel, copies the counts back; synchronous.
 * Replaces: index build (537-541), the omp parallel search loop (550-599),
 * the per-level bitfields and their sum (553, 580-593) and results[kmer]=total
 * (595-596).  Duplicate k-mers are allowed and counted independently.
 */
ac_status ac_error_count(ac_ctx* ctx, uint32_t k, const uint64_t* kmers, uint32_t n_kmers,
                         const ac_windows* sample, uint64_t* counts);

/*
 * Device-resident form (same semantics), asynchronous on `hip_stream`
 * (a hipStream_t; NULL = the default stream).  All segments share k and run
 * in ONE kernel launch (both read ends of one run, 858-953), uint32 counters.
 * The launch itself stores each segment's counts (no memset dispatch): the
 * last workgroup of every candidate group writes the group's sums.  Segments
 * whose count vectors overlap (window shards of one candidate set) are zeroed
 * on the stream first and summed.  The context's scratch (work queues, group
 * sums) is stream-ordered: do not run two launches of one context on
 * different streams at the same time.
 *   window_len  NULL: every window's start / length is read from the segment's sample.  Otherwise
 *               one length per segment for samples whose windows all have it -- the reference's
 *               own sample: every start window holds sl bases and every end window sl + 1
 *               (sampleSequences, approx_counter.cpp:415-476): segment i's window w starts at base
 *               w * ceil32(window_len[i]), n_windows * ceil32(window_len[i]) <= n_bases, and
 *               sample.start / .length are not read (may be NULL) -- the kernel computes each
 *               window's place instead of loading its descriptor, as the host-buffer stage does.
 *   flags       AC_DEVICE_ACCUMULATE: add into `counts` without zeroing them first (window shards
 *               combined on one device); 0: store them.
 * (ABI 8 folded ac_error_count_device_accumulate and ac_error_count_device_equal into this call.)
 */
#define AC_DEVICE_ACCUMULATE 1u
ac_status ac_error_count_device(ac_ctx* ctx, uint32_t k, const ac_segment* segments, uint32_t n_segments,
                                const uint32_t* window_len, uint32_t flags, void* hip_stream);

/*
 * Device copy of a packed sample, owned by the context (valid until the next
 * ac_sample_upload on ctx or ac_destroy).  Lets one upload serve both the
 * exact count and the approximate count of one read end.  The closest
 * reference step is the index build over the sample (approx_counter.cpp:537-541).
 * `dev` receives the device pointers.
 */
ac_status ac_sample_upload(ac_ctx* ctx, const ac_windows* host, ac_windows* dev);

/*
 * count_kmers (approx_counter.cpp:487-519) + get_most_frequent (396-405) or,
 * with solid > 0, get_solid_kmers (372-388), on the GPU over a device sample:
 * exact counts of the k-mers of every window that hold no N, pass the
 * low-complexity filter (float DUST score >= lc_threshold is dropped,
 * 214-234; lc_threshold already adjusted for k, 183-186) and are not in
 * `forbidden` (host array, any order, 330-332).  Writes the kept k-mers in
 * CompareCount order (275-305): the first `limit` of them, or all with count >=
 * solid when solid > 0 (the reference does not truncate solid k-mers).
 * *n_out = number written; if more than `capacity` are due, nothing is written,
 * *n_out = the number needed and AC_ERR_INVALID is returned.  *n_distinct =
 * distinct kept k-mers (the reference's count.size(), 883), *had_n = k-mer
 * positions skipped for holding an N (513-517).  Synchronous.
 */
ac_status ac_exact_count_device(ac_ctx* ctx, uint32_t k, const ac_windows* dev, float lc_threshold,
                                const uint64_t* forbidden, uint32_t n_forbidden, uint64_t limit, uint64_t solid,
                                uint64_t* kmers_out, uint64_t* counts_out, uint64_t capacity, uint64_t* n_out,
                                uint64_t* n_distinct, uint64_t* had_n);

/* Which counting path the last exact count of ctx took (for measurement and
 * tests): 1 = partitioned (dense keys, bucket partition, per-bucket LDS count;
 * every k, samples up to 2^27 k-mer positions), 0 = the global hash table
 * (larger samples, a bucket that outgrew its LDS table, or AC_EXACT_HASH=1),
 * -1 = none yet. */
int ac_exact_path(const ac_ctx* ctx);

/* Same with a host sample (uploads it with ac_sample_upload first). */
ac_status ac_exact_count(ac_ctx* ctx, uint32_t k, const ac_windows* host, float lc_threshold,
                         const uint64_t* forbidden, uint32_t n_forbidden, uint64_t limit, uint64_t solid,
                         uint64_t* kmers_out, uint64_t* counts_out, uint64_t capacity, uint64_t* n_out,
                         uint64_t* n_distinct, uint64_t* had_n);

/*
 * ac_sample_upload into upload slot `slot` (0 .. AC_MAX_JOBS-1; slot 0 is
 * ac_sample_upload's), so both read ends of a run stay on the device at once:
 * each is uploaded once and serves its exact count and the fused approximate
 * count below.  Valid until the next upload into the same slot.
 */
ac_status ac_sample_upload_slot(ac_ctx* ctx, int slot, const ac_windows* host, ac_windows* dev);

/* One errorCount call (approx_counter.cpp:922) over a packed sample: host
 * k-mers, host uint64 counts; `sample` is a device sample (ac_error_count_samples)
 * or a host image (ac_error_count_images). */
typedef struct ac_sample_job {
    const uint64_t* kmers;
    uint32_t n_kmers;
    ac_windows sample;
    uint64_t* counts;
} ac_sample_job;

/*
 * errorCount for up to AC_MAX_JOBS calls sharing k -- both read ends of one run
 * (the loop at approx_counter.cpp:858-953) -- in ONE fused kernel launch over
 * samples already on the device (ac_sample_upload_slot): the CLI's path, where
 * each end's upload first serves its exact count.  Synchronous.
 */
ac_status ac_error_count_samples(ac_ctx* ctx, uint32_t k, const ac_sample_job* jobs, uint32_t n_jobs);

/*
 * The same over host images: on one device one fused launch; on an
 * ac_create_multi context every job's windows are cut into one contiguous shard
 * per device (balanced by bases), each device counts its shards of all jobs in
 * one fused launch, and the shard counts are summed (the CLI's -g N).
 */
ac_status ac_error_count_images(ac_ctx* ctx, uint32_t k, const ac_sample_job* jobs, uint32_t n_jobs);

/*
 * Host packing of Dna5 windows into a window image (no reference counterpart:
 * SeqAn keeps 1 byte per base; this is the boundary's wire format).
 *   dna5     : window bytes, ordValues 0..3 for ACGT, >= 4 for N
 *   seq_start/seq_len: window i = dna5[seq_start[i] .. +seq_len[i])
 * ac_image_bases() returns the image size (bases) needed for these lengths.
 * The caller allocates codes (n_bases/16 words), nmask (n_bases/32 words),
 * start (n windows) and length (n windows).
 */
uint64_t ac_image_bases(const uint32_t* seq_len, uint32_t n);
ac_status ac_pack_windows(const uint8_t* dna5, const uint64_t* seq_start, const uint32_t* seq_len,
                          uint32_t n, uint32_t* codes, uint32_t* nmask, uint64_t* start,
                          uint32_t* length, uint64_t n_bases);

/*
 * The sample exactly as errorCount receives it: a StringSet<Dna5String>
 * (approx_counter.cpp:38, filled by sampleSequences 415-476), one byte per
 * base.  Window i is bases[offset[i] .. offset[i] + length[i]); bases are
 * Dna5 ordinals (0..3 = A C G T, anything else = N; SeqAn's ordValue).
 * Windows may overlap or come in any order.  Precondition (the struct carries
 * no size for `bases`, so the library cannot check it): every
 * offset[i] + length[i] lies within the caller's `bases` buffer.
 */
typedef struct ac_dna5_windows {
    const uint8_t* bases;
    const uint64_t* offset;
    const uint32_t* length;
    uint32_t n_windows;
} ac_dna5_windows;

/*
 * Pinned host memory for the sample (ABI 7; no reference counterpart: the reference's
 * sampleSequences, approx_counter.cpp:415-476, fills an ordinary StringSet<Dna5String>).
 * A job of ac_error_count_jobs / _submit whose windows all have one length of 1..256 bases (a read
 * end: sl or sl + 1) and whose `bases` and `offset` arrays lie inside blocks of ac_host_alloc is
 * packed on the device when the call is large (>= 2^16 windows; AC_DEVICE_PACK_MIN_WINDOWS): the
 * count kernel's copier workgroups read its Dna5 bytes over PCIe and pack them into HBM themselves,
 * so the host does no per-window work for it beyond scanning the lengths (ac_stage_mode then reports
 * 3).  Smaller calls are packed by the host pool, which is faster there, a 1-participant pool
 * included (AC_DEVICE_PACK=1 / 0: always / never).  The bytes readable from `bases` are those up to
 * the end of its block; a window reaching past them is an error (AC_ERR_INVALID, its counts short).
 * Blocks are process-wide (any context, any device).  A submit's device-packed jobs are read by
 * the device until its stream work completes: do not change or free them before that.
 *   ac_host_alloc  a pinned, device-mapped block of `bytes` (AC_ERR_DEVICE without a HIP device)
 *   ac_host_free   releases a block of ac_host_alloc (NULL: no-op; another pointer: AC_ERR_INVALID)
 */
ac_status ac_host_alloc(size_t bytes, void** out);
ac_status ac_host_free(void* p);

/* One errorCount call (approx_counter.cpp:922) over a Dna5 sample. */
typedef struct ac_job {
    const uint64_t* kmers; /* dna2int layout (approx_counter.cpp:55-62)         */
    uint32_t n_kmers;
    ac_dna5_windows sample;
    uint64_t* counts;      /* host, n_kmers; ignored by ac_error_count_jobs_submit */
} ac_job;

/*
 * errorCount (approx_counter.cpp:531-601) for up to AC_MAX_JOBS calls that
 * share k -- both read ends of one run (the loop at 858-953) -- in one
 * synchronous call, host buffers in and out: jobs[j].counts[i] = M1 count of
 * jobs[j].kmers[i] over jobs[j].sample.  The whole stage runs here: the Dna5
 * windows are packed to 2-bit codes + N bitmap by the host worker pool
 * straight into a pinned staging block, moved into device memory job by job
 * (ac_stage_mode: by the count kernel itself -- launched first -- or by a copy
 * ahead of it), counted by ONE fused kernel launch over all jobs (every size
 * since ABI 4; with AC_STAGE_EARLY=0, calls of >= 2^17 windows are cut into 2-4
 * parts, each launched once it is sent), and the kernel writes the counts into
 * the pinned block.  An early launch that times out waiting for the host (0.5 s
 * without progress) is run again through the DMA path.  On an
 * ac_create_multi context every job's windows are split into contiguous shards
 * balanced by bases, one per device, and the shard counts are summed.
 * Replaces the index build (537-541), the OpenMP search loop (547-599) and
 * results[kmer] = total (595-596) of each call.
 */
#define AC_MAX_JOBS 4
ac_status ac_error_count_jobs(ac_ctx* ctx, uint32_t k, const ac_job* jobs, uint32_t n_jobs);

/*
 * (ABI 7 removed ac_idle -- a no-op since ABI 6 removed the armed launches it cancelled -- and
 * ac_error_count_sample, which ac_error_count_samples with one job replaces.)
 */

/*
 * The same stage without the way back, for callers that combine shards with
 * a device collective (one process per GPU, RCCL all-reduce of the count
 * vector): packs and sends the jobs and launches the count
 * kernel on `hip_stream`, which writes uint32 counts to DEVICE memory
 * d_counts (jobs concatenated in order, sum of n_kmers entries).  Returns once
 * the host inputs have been consumed (packed into the context's staging
 * block); the device work is asynchronous on `hip_stream`.  Consecutive
 * submits on one context must use the same stream.  Single-device contexts.
 */
ac_status ac_error_count_jobs_submit(ac_ctx* ctx, uint32_t k, const ac_job* jobs, uint32_t n_jobs,
                                     uint32_t* d_counts, void* hip_stream);

/*
 * Device-side error check.  The count kernels never read outside a window's
 * image: a window that is misaligned or reaches past n_bases is skipped, and
 * the kernel records that in a context-owned device word instead of failing
 * silently.  The host-buffer entry points check the word themselves (they
 * synchronise); after the asynchronous *_device entry points call ac_check:
 * it waits for `hip_stream`, reads and clears the word, and returns
 * AC_ERR_INVALID ("malformed window skipped") or AC_ERR_INTERNAL (kernel
 * set-up fault) if a launch since the last check hit one, AC_OK otherwise.
 */
ac_status ac_check(ac_ctx* ctx, void* hip_stream);

/*
 * Multi-process data parallelism (one process per GPU): window
 * shards are counted independently (ac_error_count_jobs_submit leaves each
 * shard's counts in device memory) and the count vectors are summed by one RCCL
 * all-reduce over xGMI, owned by the context.  There is no reference
 * counterpart (errorCount runs on one host's OpenMP threads, approx_counter.cpp:547).
 *   ac_comm_id_bytes    size of the RCCL unique id (128)
 *   ac_comm_unique_id   a fresh id (rank 0); the caller sends it to every rank
 *   ac_comm_init        join the n_ranks-rank communicator as `rank`
 *                       (single-device contexts; ranks on distinct devices)
 *   ac_allreduce_counts in-place uint32 sum of d_counts[0, n) over the ranks,
 *                       asynchronous on hip_stream
 * RCCL (librccl.so) is loaded at the first of these calls, not at library load.
 */
int ac_comm_id_bytes(void);
ac_status ac_comm_unique_id(ac_ctx* ctx, void* id_out);
ac_status ac_comm_init(ac_ctx* ctx, int n_ranks, int rank, const void* id);
ac_status ac_allreduce_counts(ac_ctx* ctx, uint32_t* d_counts, uint64_t n, void* hip_stream);

/*
 * The host worker pool that packs the Dna5 sample (ac_error_count_jobs*).  The
 * reference sizes its one OpenMP team with omp_set_num_threads(nb_thread)
 * (approx_counter.cpp:547); here the pool is process-wide and planned once, at
 * the first ac_create: the CPUs local to the GPU's PCIe root, split among the
 * local ranks (LOCAL_RANK / LOCAL_WORLD_SIZE, local rank r on device r mod the
 * visible devices) whose GPUs share them -- disjoint runs of physical cores per
 * rank -- with at most min(16, this rank's share of the cgroup CPU quota less
 * 2 CPUs of headroom, 1 for a share of 4 or less) participants (the calling
 * thread included): a pool spinning on the whole quota was throttled by the CFS.
 *   ac_set_host_cpus   the pool's CPUs and participants (0 = min(16, n_cpus))
 *                      instead; only before the first ac_create
 *                      (AC_ERR_INVALID afterwards)
 *   ac_host_pool_cpus  the plan in force: *participants, the CPUs (up to cap
 *                      written into cpus); returns the number of CPUs
 *   ac_plan_host_cpus  the rule itself, for callers that place threads on their
 *                      own: the CPUs of local rank `rank` given every local
 *                      rank's GPU cpulist ("0-63,128-191") and the CPUs the
 *                      process may use; core_of[c] = physical core of CPU c
 *                      (NULL: every CPU its own core).  Returns the count (up
 *                      to cap written), -1 on bad arguments.
 */
ac_status ac_set_host_cpus(const int* cpus, int n_cpus, int participants);
int ac_host_pool_cpus(int* participants, int* cpus, int cap);
int ac_plan_host_cpus(const char* const* rank_cpulists, int n_ranks, int rank, const char* allowed_cpulist,
                      const int* core_of, int n_core_of, int* out, int cap);

/*
 * How the last ac_error_count_jobs / _submit call on ctx moved its packed
 * inputs (no reference counterpart).  ABI note: the values changed in ABI 3 --
 * 1 (zero-copy, round 2) is no longer returned -- and in ABI 4 large calls moved
 * from 0 to 2; callers should compare against 2 / 0 only.
 * 3 = the early launch with at least one job packed on the device (ac_host_alloc samples, ABI 7).
 * 2 = the early launch, for every single-device call
 * (default; AC_STAGE_EARLY=0 turns it off): the count kernel is
 * launched before the host packs, the host flags each job in a pinned header as
 * soon as it is packed, the kernel copies the flagged job into device memory
 * itself and counts it while later jobs are still being packed, and each
 * candidate group's last workgroup stores its counts and error bits, tagged with
 * the call's generation, into pinned memory, which the host polls.  A few copier
 * workgroups of the kernel do the copying (every early-launch call) while the
 * others count.  0 = the DMA path (AC_STAGE_EARLY=0: calls
 * of >= 2^17 windows cut into 2-4 parts, each packed and copied by the copy
 * engine while the previous part counts; a multi-device context; a staging
 * region of 2^31 bytes or more; the retry of a timed-out early launch).  Either
 * way a job is sent without its N bitmap when no window needs it (no N, or, for
 * equal windows, every N inside the window's inline record) and without window
 * descriptors when its windows have one length.  -1 = no
 * call yet.  ac_error_count_jobs_submit takes the early launch too (its counts
 * and errors go to device memory; ac_check reports the errors).
 */
int ac_stage_mode(const ac_ctx* ctx);

/*
 * Launch geometry actually used for the last device launch of ctx (for
 * measurement): waves launched, windows per wave, candidate groups.
 */
ac_status ac_last_launch(const ac_ctx* ctx, uint64_t* waves, uint32_t* windows_per_wave,
                         uint32_t* groups);

#ifdef __cplusplus
}
#endif
#endif /* APPROX_COUNTER_AMD_H */
