// host_pack.h -- host side of the host-buffer entry points: a persistent worker
// pool and the Dna5 -> window-image packer (include/approx_counter_amd.h,
// ac_error_count_jobs).  The reference hands errorCount its sample as a
// StringSet<Dna5String>, one byte per base (approx_counter.cpp:38, 531); the
// GPU reads 2-bit codes + an N bitmap, so the packing is part of the stage.
#pragma once
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "nrec.h"

namespace acamd {

// A fixed set of worker threads that run the tasks [0, n) of one job
// together with the calling thread.  Workers spin for a short while after a
// job (back-to-back calls find them awake: a futex wake costs tens of us,
// the whole cfg2 stage ~150 us) and then sleep on a condition variable.
class WorkPool {
public:
    // total participants, caller included; when cpus is non-empty, worker i is pinned to
    // cpus[(i - 1) % size] (pin_each) or every worker to the whole set
    explicit WorkPool(unsigned n_threads, const std::vector<int>& cpus = {}, bool pin_each = true);
    ~WorkPool();
    WorkPool(const WorkPool&) = delete;
    WorkPool& operator=(const WorkPool&) = delete;

    unsigned size() const { return (unsigned)threads_.size() + 1; }
    // fn(i) for every i in [0, n); returns when all have run.  One run() at a
    // time (serialised by a mutex); fn must not call run() itself.
    void run(uint32_t n, const std::function<void(uint32_t)>& fn);
    // The same in steps, so the caller can act on a prefix of the tasks while
    // the workers go on with the rest: begin() publishes the job (and holds
    // the pool until finish()), help(upto) makes the caller run unclaimed tasks
    // below `upto`, finish() runs what is left and waits for every task.
    void begin(uint32_t n, const std::function<void(uint32_t)>& fn);
    void help(uint32_t upto);
    void help_one();  // runs at most one unclaimed task
    void finish();
    // (between begin() and finish()) the caller runs every task itself: no workers, or one task
    bool serial() const { return serial_; }

private:
    void worker();
    void drain(uint32_t gen, uint32_t upto = ~0u, uint32_t max_tasks = ~0u);

    // A job is published as state_ = gen << 32 | next task; a participant
    // claims task i by a CAS of state_ from (gen, i) to (gen, i + 1), having
    // read the job's fn / n from slot gen & 1 before it: state_ only grows, so
    // a successful CAS proves the slot still held that job.  run() returns once
    // the job's tasks are done, without waiting for workers that never got to
    // it (a descheduled spinning worker used to hold every call up).
    struct Job {
        std::atomic<const std::function<void(uint32_t)>*> fn{nullptr};
        std::atomic<uint32_t> n{0};
        std::atomic<uint32_t> done{0};
    };
    std::vector<std::thread> threads_;
    std::mutex run_m_;  // held from begin() to finish()
    std::mutex m_;
    std::condition_variable cv_;
    std::atomic<uint64_t> state_{0};
    std::atomic<uint32_t> pub_{0};  // last published gen (sleepers wait for it to change, under m_)
    uint32_t gen_ = 0;               // run()'s own counter (under run_m_)
    bool serial_ = false;            // begin() without workers (or <= 1 task): the caller runs the tasks
    uint32_t serial_next_ = 0, n_ = 0;
    const std::function<void(uint32_t)>* serial_fn_ = nullptr;
    Job jobs_[2];
    std::atomic<bool> stop_{false};
    int64_t spin_ns_ = 0;
};

// Where the process-wide pool runs: its participants (caller included) and
// the CPUs its workers are pinned to.  ac_create fills it in once, before the
// pool's first use (capi.cpp: the CPUs local to the GPU's PCIe root, split
// among the local ranks whose GPUs share them, and a participant count within
// the rank's share of the cgroup CPU quota); ac_set_host_cpus overrides it.
struct HostPlan {
    std::vector<int> cpus;
    unsigned participants = 0;  // 0: min(16, CPUs this process may run on)
};
// false once the pool exists or a plan was already set (the first plan wins)
bool set_host_plan(const HostPlan& plan);
HostPlan host_plan();  // the plan in force (after the pool's creation: what it actually used)

// The process-wide pool of the host-buffer entry points.  Size: the
// AC_HOST_THREADS environment variable, else the plan's participants, else
// min(16, CPUs this process may run on); AC_HOST_THREADS=1 packs on the
// calling thread alone.  Workers are pinned to the plan's CPUs (minus those
// the process may not use), each to the whole set: AC_HOST_PIN=0 disables,
// AC_HOST_PIN=each pins worker i to one CPU of it instead.
WorkPool& host_pool();
// CPUs of a sysfs cpulist file / text ("0-63,128-191"), sorted; empty if unreadable.
std::vector<int> read_cpulist(const char* path);
std::vector<int> parse_cpulist(const char* text);
// The physical core of a CPU (its first SMT sibling, from sysfs).
int sysfs_core_of(int cpu);
// The pool CPUs of local rank `rank`: rank_lists[r] = the GPU-local CPU list of
// local rank r.  Ranks with identical lists split them (contiguous runs of
// physical cores, never one core's siblings across two ranks), intersected
// with `allowed` (sorted); ordered first SMT threads first.  core_of maps a CPU
// to its core (NULL: every CPU its own core).  *shared = fewer cores than ranks
// (this rank's core is another rank's too).
std::vector<int> plan_host_cpus(const std::vector<std::vector<int>>& rank_lists, int rank,
                                const std::vector<int>& allowed, const std::function<int(int)>& core_of,
                                bool* shared = nullptr);
// cgroup v2 CPU quota in CPUs (cpu.max), 0 when unlimited or unknown.
double cgroup_cpu_quota();

// Image bases a window of `len` bases occupies (windows start on 32-base
// boundaries, include/approx_counter_amd.h).
inline uint64_t image_span(uint32_t len) { return ((uint64_t)len + 31u) / 32u * 32u; }

// Image bases of windows len[0, n) (sum of image_span), the first length and the OR of
// (length ^ first) -- zero iff every window has one length.  AVX-512 when the CPU has it.
uint64_t span_scan(const uint32_t* len, uint32_t n, uint32_t* first, uint32_t* diff);

// Packs windows [w0, w1) of a Dna5 window set into a window image whose window
// w0 starts at image base `first`: writes the 2-bit codes and the N bitmap of
// every 32-base block the windows occupy (padding bases as code 0, not N), and
// the image start / length of each window into start_out[w - w0] /
// len_out[w - w0].  `codes` / `nmask` are the image's word arrays (indexed by
// absolute image base).  Dna5 ordinals: 0..3 = A C G T, anything else = N.
// `records`: the windows are equal (one length) and each gets its inline N
// record (nrec.h; the caller has checked that their length leaves room); their
// start / length are not written, and their N-bitmap words only for a window
// whose record overflowed (the kernel reads no others).  Returns the
// PACK_* bits of the range: PACK_HAS_N = some window holds an N, PACK_OVERFLOW =
// some window's N bases did not fit its record (its N-bitmap words are needed).
constexpr uint32_t PACK_HAS_N = 1u, PACK_OVERFLOW = 2u;
uint32_t pack_dna5_range(const uint8_t* bases, const uint64_t* offset, const uint32_t* length, uint32_t w0,
                         uint32_t w1, uint64_t first, uint32_t* codes, uint32_t* nmask, uint64_t* start_out,
                         uint32_t* len_out, bool records = false);

}  // namespace acamd
