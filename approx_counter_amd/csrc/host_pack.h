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

namespace acamd {

// A fixed set of worker threads that run the tasks [0, n) of one job
// together with the calling thread.  Workers spin for a short while after a
// job (back-to-back calls find them awake: a futex wake costs tens of us,
// the whole cfg2 stage ~150 us) and then sleep on a condition variable.
class WorkPool {
public:
    // total participants, caller included; worker i is pinned to cpus[i % size] when cpus is non-empty
    explicit WorkPool(unsigned n_threads, const std::vector<int>& cpus = {});
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
    void finish();

private:
    void worker();
    void drain(uint32_t gen, uint32_t upto = ~0u);

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
    std::mutex run_m_;
    std::mutex m_;
    std::condition_variable cv_;
    std::atomic<uint64_t> state_{0};
    std::atomic<uint32_t> pub_{0};  // last published gen (sleepers wait for it to change, under m_)
    uint32_t gen_ = 0;               // run()'s own counter (under run_m_)
    std::unique_lock<std::mutex> held_;  // run_m_ between begin() and finish()
    bool serial_ = false;            // begin() without workers (or <= 1 task): the caller runs the tasks
    uint32_t serial_next_ = 0, n_ = 0;
    const std::function<void(uint32_t)>* serial_fn_ = nullptr;
    Job jobs_[2];
    std::atomic<bool> stop_{false};
    int64_t spin_ns_ = 0;
};

// The process-wide pool of the host-buffer entry points.  Size: the
// AC_HOST_THREADS environment variable, else min(16, CPUs this process may
// run on); AC_HOST_THREADS=1 packs on the calling thread alone.  Its workers
// are pinned to the CPUs given to set_host_cpus() before the pool's first use
// (the CPUs local to the GPU's PCIe root: the packed block they write is read
// by that GPU), minus those the process may not use; AC_HOST_PIN=0 disables.
WorkPool& host_pool();
void set_host_cpus(const std::vector<int>& cpus);
// CPUs of a sysfs cpulist ("0-63,128-191"); empty if unreadable.
std::vector<int> read_cpulist(const char* path);

// Image bases a window of `len` bases occupies (windows start on 32-base
// boundaries, include/approx_counter_amd.h).
inline uint64_t image_span(uint32_t len) { return ((uint64_t)len + 31u) / 32u * 32u; }

// Packs windows [w0, w1) of a Dna5 window set into a window image whose window
// w0 starts at image base `first`: writes the 2-bit codes and the N bitmap of
// every 32-base block the windows occupy (padding bases as code 0, not N), and
// the image start / length of each window into start_out[w - w0] /
// len_out[w - w0].  `codes` / `nmask` are the image's word arrays (indexed by
// absolute image base).  Dna5 ordinals: 0..3 = A C G T, anything else = N.
void pack_dna5_range(const uint8_t* bases, const uint64_t* offset, const uint32_t* length, uint32_t w0, uint32_t w1,
                     uint64_t first, uint32_t* codes, uint32_t* nmask, uint64_t* start_out, uint32_t* len_out);

}  // namespace acamd
