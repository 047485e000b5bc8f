#!/usr/bin/env python3
"""Benchmark of the approximate-count stage (errorCount, approx_counter.cpp:531-601).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2|cfg3|cfg4|cfg5]
                    [--scaling weak|strong]

A step is one pass of the stage BASELINE.md defines over one batch: both read
ends of one run (start + end windows, approx_counter.cpp:858), each against its
own top-`lim` candidates, from HOST buffers to HOST counts -- the sample as a
StringSet<Dna5String> (one byte per base, what errorCount receives; built once,
outside the timed steps, in pinned memory from ac_host_alloc, `--sample pinned`),
ONE fused kernel launch over both ends issued first in the call, the windows
packed to 2-bit codes (N positions inline) either by the library's host pool
(cfg2-sized calls) or by the count kernel's own copier workgroups straight from
the pinned Dna5 bytes (calls of >= 2^16 windows, or a rank's small host share:
DESIGN.md 4d), pulled into HBM while the other workgroups count, (N > 1: one
RCCL all-reduce of the count vector), counts back.  That is `value`.  Default workload = BASELINE.json
configs[1] (k=16, sn=10,000, sl=100, lim=500), on seeded synthetic reads
(SURVEY.md §8(d)).

Multi-GPU (one process per GPU, torchrun): `--scaling weak` (default except
cfg4) gives every rank its own sn reads against the same candidates;
`--scaling strong` (cfg4's default, BASELINE "sn=1M sharded over 8 GPUs") builds
ONE sample and gives rank r its contiguous shard (balanced by bases,
approx_counter_amd/shard.py).  Either way each step ends with one RCCL
all-reduce (sum) of the per-candidate count vector and its copy to the host.

Also reported (never as `value`): `kernel_ms` / `kernel_kmer_bp_per_s`, the
count kernel alone on device-resident inputs (HIP events around every 5th
launch, on the launch stream), the basis of `roofline`; `pipelined`, the same
host-buffer steps issued back to back with ac_error_count_jobs_submit (a step's
packing overlaps the previous step's kernel: runs of -mr are independent).

Roofline: the count kernel is bound by integer VALU issue, not
HBM and not MFMA.  `roofline.frac` = algorithmic lane-ops / kernel time / peak,
with 9.5 lane-ops per text base per lane word of P = floor(32/k) candidates
(the Wu-Manber NFA's 8 + 1.5 of hit accumulation; ~Eq a table lookup);
`frac_survey_basis` is the same time on SURVEY.md §8(d)'s 20 ops per kmer*bp;
`sq_insts_valu` is the measured wave-instruction count of a committed PMC pass
(profiles/*_pmc_traffic.json), next to the 9.5/P model.  `peak` = 256 CU x 4
SIMD x 32 lanes x 2.4 GHz.  `traffic` = HBM bytes per launch from the same PMC
files (FETCH_SIZE doubled per the gfx950 correction), or null.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "approx-count kmer×base pairs/sec (k=16, lim=500, 10k×100bp ends)"
VALU_PEAK_OPS = 256 * 4 * 32 * 2.4e9       # int32 lane-ops/s (2-cycle wave64 issue per SIMD-32)
HBM_PEAK = 8.0e12                           # B/s (MI355X_MICROARCH.md, spec)
OPS_PER_BASE_WORD = 9.5                     # 8 NFA + 1.5 hit accumulation (~Eq: LDS table)
SURVEY_OPS_PER_UNIT = 20.0                  # one Myers column, 20 int32 ops per kmer*bp
SAMPLE_BYTES_PER_BASE = 0.375               # 2-bit code + 1-bit N mask, read once
DATA_NOTE = ("synthetic (seeded reads, SURVEY.md 8(d)); host Dna5 buffers in, host counts out; "
             "bit-exact vs model M1 (oracle/), parity with SeqAn unpinned (SURVEY.md 0)")

CONFIGS = {  # BASELINE.json configs
    "cfg2": dict(k=16, sn=10_000, sl=100, lim=500, scaling="weak"),
    "cfg3": dict(k=16, sn=100_000, sl=100, lim=2000, scaling="weak"),
    "cfg4": dict(k=16, sn=1_000_000, sl=100, lim=500, scaling="strong"),
    "cfg5": dict(k=22, sn=100_000, sl=150, lim=1000, scaling="weak"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="cfg2", choices=sorted(CONFIGS))
    ap.add_argument("--scaling", choices=("weak", "strong"),
                    help="N > 1: weak = every rank its own sn reads; strong = one sample sharded over the ranks")
    ap.add_argument("--k", type=int)
    ap.add_argument("--sn", type=int)
    ap.add_argument("--sl", type=int)
    ap.add_argument("--lim", type=int)
    ap.add_argument("--read-len", type=int, default=400)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="total duration of the bounded CPU-baseline samples")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-leg", action="store_true",
                    help="skip the device-resident kernel timing (and with it the roofline)")
    ap.add_argument("--no-pipelined", action="store_true", help="skip the informational pipelined leg")
    ap.add_argument("--no-exact", action="store_true", help="skip the exact-count block (SURVEY.md 8(f) rank 1)")
    ap.add_argument("--verify", action="store_true", help="check the stage's counts against the oracle (slow)")
    ap.add_argument("--shard", metavar="R/N",
                    help="rehearsal on one GPU: time rank R's shard of an N-rank strong-scaling run alone "
                         "(the projection basis for N GPUs; never the default line)")
    ap.add_argument("--step-form", choices=("auto", "submit"), default="auto",
                    help="submit: at N = 1 run the N > 1 step form (ac_error_count_jobs_submit, the library's RCCL "
                         "all-reduce on a one-rank communicator, counts copied back, stream synchronised) -- a "
                         "rehearsal of the multi-GPU step's own costs, never the default line")
    ap.add_argument("--sample", choices=("pinned", "heap"), default="pinned",
                    help="where the Dna5 sample lives: pinned = ac_host_alloc memory, packed on the device by the "
                         "count kernel's copier workgroups (DESIGN.md 4d); heap = ordinary memory, packed by the host "
                         "pool (4c)")
    ap.add_argument("--kernel-launches", type=int, default=100,
                    help="launches of the kernel-only leg (at least --steps); it runs before the stage, so the "
                         "device is at its sustained clock when the stage's warmup starts (DESIGN.md 4c)")
    ap.add_argument("--event-every", type=int, default=5,
                    help="bracket every N-th kernel-leg launch with HIP events (each event is a queue "
                         "packet of its own: ~3 us between launches when every launch is bracketed)")
    a = ap.parse_args()
    for key, v in CONFIGS[a.config].items():
        if getattr(a, key) is None:
            setattr(a, key, v)
    a.read_len = max(a.read_len, 2 * a.sl)
    return a


def _ranges(cpus):
    """'0-15,128-143' for a CPU list."""
    out, run = [], []
    for c in sorted(cpus):
        if run and c == run[-1] + 1:
            run.append(c)
        else:
            if run:
                out.append(f"{run[0]}-{run[-1]}" if len(run) > 1 else str(run[0]))
            run = [c]
    if run:
        out.append(f"{run[0]}-{run[-1]}" if len(run) > 1 else str(run[0]))
    return ",".join(out) or "unpinned"


def cpu_share():
    """(CPUs this process may run on = nproc, CPU quota of its cgroup or None)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    return n, quota


def cgroup_cpu_stat():
    """cgroup v2 cpu.stat (nr_periods, nr_throttled, throttled_usec, usage_usec ...) as ints, {} if unreadable."""
    out = {}
    try:
        for ln in open("/sys/fs/cgroup/cpu.stat"):
            key, v = ln.split()
            out[key] = int(v)
    except (OSError, ValueError):
        pass
    return out


def cpu_baseline(wl, k, seconds):
    """The oracle's OpenMP Myers restatement (kind "port": the reference's SeqAn
    FM-index path cannot be built here) on this host's cores: the
    threads the host sustains (the cgroup CPU quota when below nproc: the headline),
    all `nproc` CPUs, and one thread on a bounded subset of the candidates."""
    import oracle

    nproc, quota = cpu_share()
    ends = ("start", "end")
    bases = {e: sum(int(w.size) for w in wl[e]["windows"]) for e in ends}

    def run(threads, frac):
        sub = {e: wl[e]["kmers"][: max(1, int(round(wl[e]["kmers"].size * frac)))] for e in ends}
        t = time.perf_counter()
        for e in ends:
            oracle.count_myers(k, sub[e], wl[e]["windows"], threads)
        return sum(sub[e].size * bases[e] for e in ends), time.perf_counter() - t

    def leg(threads, frac_cands, budget):
        # a probe on a few candidates sizes the sample: the full workload repeated when one
        # pass fits the budget, else the largest candidate fraction that does (cfg3-cfg5)
        u0, t0 = run(threads, min(frac_cands, 0.02))
        rate0 = u0 / max(t0, 1e-6)
        full = sum(wl[e]["kmers"].size * bases[e] for e in ends) * frac_cands
        frac = frac_cands if full / rate0 <= budget else max(0.002, frac_cands * budget / (full / rate0))
        units, dt1 = run(threads, frac)
        reps = max(1, int(budget / max(dt1, 1e-6)))
        t = time.perf_counter()
        for _ in range(reps):
            run(threads, frac)
        dt = time.perf_counter() - t
        return units * reps / dt, units, reps, dt

    # Headline: as many threads as the host can actually run -- the cgroup CPU quota when it is
    # below nproc (oversubscribing a 16-CPU quota with 256 OpenMP threads measured 2.4x slower);
    # the nproc figure stays on the line beside it.
    q = max(1, int(quota)) if quota and int(quota) < nproc else nproc
    v, units, reps, dt = leg(q, 1.0, seconds * 0.5)
    out = {"value": v, "unit": "kmer*bp/s", "cores": q, "kind": "port",
           "sample": f"both ends, {units:.4g} kmer*bp per pass (all windows; all candidates when a pass fits "
                     f"the budget, else a prefix of them) x {reps} = {dt:.1f} s on {q} OpenMP threads "
                     f"({'the cgroup CPU quota' if q < nproc else 'nproc'}; nproc {nproc}, quota "
                     f"{quota if quota else 'none'}); oracle/ac_oracle.c Myers bit-vector, OpenMP over candidates "
                     f"(restated CPU path: SeqAn is absent, SURVEY.md 8(c))"}
    if q < nproc:
        vn, units, reps, dt = leg(nproc, 1.0, seconds * 0.25)
        out["nproc_threads"] = {"value": vn, "threads": nproc,
                                "sample": f"{units:.4g} kmer*bp x {reps} = {dt:.1f} s on {nproc} threads (nproc, "
                                          f"oversubscribing the {q}-CPU quota)"}
    v1, units, reps, dt = leg(1, 0.05, seconds * 0.25)
    out["one_thread"] = {"value": v1, "threads": 1,
                         "sample": f"a prefix (<= 5%) of the candidates of both ends over all windows ({units:.4g} kmer*bp) x {reps} "
                                   f"= {dt:.1f} s"}
    return out


EXACT_CONFIGS = {  # the exact count (count_kmers + get_most_frequent) at BASELINE's sample sizes, start windows
    "cfg3": dict(n=100_000, L=100, k=16, lim=2000),
    "cfg4": dict(n=1_000_000, L=100, k=16, lim=500),
    "cfg5": dict(n=100_000, L=150, k=22, lim=1000),
}


def exact_block(dev_index: int, calls: int = 10):
    """Row f1: ac_exact_count_device -- count_kmers (approx_counter.cpp:487-519) with
    the low-complexity / N / forbidden filters and get_most_frequent's top-lim (396-405) -- on a sample
    resident in HBM, at cfg3 / cfg4 / cfg5's sizes, against the HBM roofline of its partitioned passes
    (DESIGN.md 4b): the image read once (0.375 B/base), then per k-mer position a B-byte key (4 B for
    k <= 16, 8 B above) written by the keys pass and moved through 7 more streaming touches (level-1
    histogram read, scatter read + write, level-2 histogram read, scatter read + write, count read).
    `pmc` = the committed rocprof FETCH_SIZE (x2, MI355X_MICROARCH.md's gfx950 correction) and WRITE_SIZE
    per call, summed over the call's kernels (profiles/*_exact_pmc.json), when present."""
    import ctypes

    import approx_counter_amd as ac
    from approx_counter_amd import _lib
    from approx_counter_amd.counter import _ptr
    from tools.synth import make_windows_fast
    from tools.workload import adjust_threshold

    L = _lib.load()
    pmc = {}
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_exact_pmc.json"))):
        try:
            pmc.update(json.load(open(path)))
        except (OSError, ValueError):
            pass
    out = {}
    with ac.ApproxCounter(dev_index) as c:
        for name, cfg in EXACT_CONFIGS.items():
            k, lim = cfg["k"], cfg["lim"]
            w2d, _ = make_windows_fast(cfg["n"], cfg["L"], seed=1)
            sample = ac.pack_windows(w2d)
            del w2d
            hw, dw = sample.as_struct(), _lib.ACWindows()
            ac.counter.check(L.ac_sample_upload(c.handle, ctypes.byref(hw), ctypes.byref(dw)), c.handle)
            thr = float(adjust_threshold(1.0, 16, k))
            km, ct = np.zeros(lim, np.uint64), np.zeros(lim, np.uint64)
            fb = np.zeros(1, np.uint64)
            n_out, n_dist, had_n = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()

            def once():
                ac.counter.check(L.ac_exact_count_device(
                    c.handle, k, ctypes.byref(dw), thr, _ptr(fb, ctypes.c_uint64), 0, lim, 0, _ptr(km, ctypes.c_uint64),
                    _ptr(ct, ctypes.c_uint64), lim, ctypes.byref(n_out), ctypes.byref(n_dist), ctypes.byref(had_n)),
                    c.handle)

            for _ in range(3):
                once()
            times = []
            for _ in range(calls):
                t0 = time.perf_counter()
                once()
                times.append(time.perf_counter() - t0)
            ms = float(np.median(times)) * 1e3
            n_pos = cfg["n"] * max(0, cfg["L"] - k + 1)
            key_b = 4 if k <= 16 else 8
            alg = SAMPLE_BYTES_PER_BASE * sample.n_bases + 8 * key_b * n_pos
            row = {"ms": ms, "ms_min": float(min(times)) * 1e3, "path": {1: "partitioned", 0: "hash table"}.get(
                       c.exact_path(), "?"), "windows": cfg["n"], "L": cfg["L"], "k": k, "lim": lim,
                   "kmer_positions": n_pos, "distinct": int(n_dist.value),
                   "algorithmic_bytes": alg, "achieved_GBps": alg / (ms * 1e-3) / 1e9,
                   "frac_hbm": alg / (ms * 1e-3) / HBM_PEAK}
            if name in pmc:
                row["pmc"] = pmc[name]
                tb = pmc[name].get("traffic_bytes_per_call")
                if tb:
                    row["traffic_GBps"] = tb / (ms * 1e-3) / 1e9
            out[name] = row
    out["note"] = ("ac_exact_count_device, sample resident in HBM (synthetic start windows, tools/synth."
                   "make_windows_fast seed 1), median of %d synchronous calls incl. the host's CompareCount "
                   "ranking of the short list; algorithmic bytes = 0.375 B/base + 8 streaming touches x key "
                   "bytes per k-mer position (DESIGN.md 4b); peak 8 TB/s" % calls)
    return out


def load_pmc(workload: str):
    """PMC summary (HBM bytes, VALU instructions per launch) of the count kernel
    for this workload from the committed profiles/*_pmc_traffic.json files."""
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json"))):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if d.get("workload") == workload:
            best = d if best is None else {**best, **d}
    return best


def stage_text(stage_path: str, world: int) -> str:
    """config.stage: what one timed step runs, from host Dna5 buffers to counts."""
    if stage_path == "early-launch-device-pack":
        body = ("1 fused count launch; the Dna5 sample sits in pinned host memory (ac_host_alloc) and 16 copier "
                "workgroups of the kernel read it over PCIe and pack each 4 KB chunk of 2-bit codes (N positions "
                "inline) into HBM while the others count a window as soon as its chunk is in; the host packs "
                "nothing")
    elif stage_path == "early-launch":
        body = ("1 fused count launch issued first in the call, then both read ends packed (host pool, pinned; "
                "N positions inline in each window's slot) with progress records; 16 copier workgroups of the "
                "kernel pull each 4 KB chunk into HBM as it is packed while the others count a window as soon "
                "as its chunk is in")
    else:
        body = ("per part (>= 2^17 windows: 2 parts, >= 2^19: 4): pack (host pool, pinned), copy-engine DMA into "
                "HBM while the previous part counts")
    if world > 1:
        tail = " -> RCCL all-reduce -> counts D2H"
    elif stage_path.startswith("early-launch"):
        tail = (" -> counts tagged with the call's generation stored to pinned host memory by each candidate "
                "group, polled")
    else:
        tail = " -> counts stored to pinned host memory by the kernel"
    return "Dna5 host buffers -> " + body + " (both ends)" + tail


def build_workload(args, rank, world):
    """This rank's {end: {kmers, windows}} and the units of the whole job per step."""
    from approx_counter_amd.shard import shard_bounds
    from tools import workload

    ends = ("start", "end")
    if args.scaling == "strong" or world == 1:
        if args.sn >= 500_000:
            full = workload.build_fast(n_reads=args.sn, k=args.k, sl=args.sl, lim=args.lim, seed=args.seed)
        else:
            full, _ = workload.build(n_reads=args.sn, read_len=args.read_len, k=args.k, sl=args.sl,
                                     lim=args.lim, seed=args.seed)
        units_job = sum(full[e]["kmers"].size * sum(int(w.size) for w in full[e]["windows"]) for e in ends)
        if world == 1:
            return full, units_job
        wl = {}
        for e in ends:
            w = full[e]["windows"]
            c = shard_bounds([len(x) for x in w], world)
            wl[e] = {"kmers": full[e]["kmers"], "windows": w[c[rank]:c[rank + 1]]}
        return wl, units_job
    if args.sn >= 500_000:
        wl = workload.build_fast(n_reads=args.sn, k=args.k, sl=args.sl, lim=args.lim, seed=args.seed + 7919 * rank)
        if rank:  # the same candidates on every rank (rank 0's)
            c0 = workload.build_fast(n_reads=20_000, k=args.k, sl=args.sl, lim=args.lim, seed=args.seed)
            for e in ends:
                wl[e]["kmers"] = c0[e]["kmers"]
    else:
        wl, _ = workload.build(n_reads=args.sn, read_len=args.read_len, k=args.k, sl=args.sl, lim=args.lim,
                               seed=args.seed, shard=rank, n_shards=world)
    units_rank = sum(wl[e]["kmers"].size * sum(int(w.size) for w in wl[e]["windows"]) for e in ends)
    return wl, units_rank * world


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # AC_BENCH_BACKEND=gloo rehearses the N > 1 code path on a box with fewer
    # GPUs than ranks (ranks share devices, the count vector is reduced on the
    # host); the real multi-GPU run uses RCCL ("nccl") over xGMI.
    backend = os.environ.get("AC_BENCH_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count()) if backend != "nccl" else local
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    import approx_counter_amd as ac

    if args.shard:  # one rank's shard of an N-rank strong run, timed alone (a projection, not a scaling run)
        r_s, n_s = (int(x) for x in args.shard.split("/"))
        args.scaling = "strong"
        wl, _ = build_workload(args, r_s, n_s)
        units_job = sum(wl[e]["kmers"].size * sum(int(w.size) for w in wl[e]["windows"]) for e in ("start", "end"))
    else:
        wl, units_job = build_workload(args, rank, world)
    from approx_counter_amd.counter import host_pool_cpus
    ends = ("start", "end")
    n_c = [int(wl[e]["kmers"].size) for e in ends]
    bases = [sum(int(w.size) for w in wl[e]["windows"]) for e in ends]
    units_rank = sum(n * b for n, b in zip(n_c, bases))
    samples = [ac.Dna5Sample.from_windows(wl[e]["windows"]) for e in ends]
    if args.sample == "pinned":  # the sample built in ac_host_alloc memory (outside the timed steps, like sampling)
        samples = [smp.pinned() for smp in samples]
    jobs = ac.Jobs([(wl[e]["kmers"], smp) for e, smp in zip(ends, samples)])
    counter = ac.ApproxCounter(local)
    stream = torch.cuda.current_stream(dev)
    d_counts = torch.zeros(max(1, jobs.n_counts), dtype=torch.int32, device=dev)
    h_counts = torch.zeros(max(1, jobs.n_counts), dtype=torch.int32).pin_memory()
    # one stage call on a cold context and device (first allocations included), for the record
    t_cold = time.perf_counter()
    counter.count_jobs(args.k, jobs) if world == 1 else None
    torch.cuda.synchronize(dev)
    cold_ms = (time.perf_counter() - t_cold) * 1e3

    # ---- kernel-only leg (device-resident inputs; the roofline's basis), max(steps, 100)
    # launches.  Run first: a cold GPU runs the kernel ~8 % slower for its first ~10 ms of load
    # (profiles/r02_trace_percall.log), so the stage's warmup then starts at the sustained clock.
    kern_ms = None
    geo = None
    wlen = None
    if not args.no_kernel_leg:
        packed = [ac.pack_windows(wl[e]["windows"]) for e in ends]
        segs = [ac.DeviceSegment.upload(wl[e]["kmers"], packed[i], device=dev) for i, e in enumerate(ends)]
        arr = ac.ApproxCounter.segment_array(segs)
        # equal windows (every start window sl bases, every end window sl + 1): the launch form the
        # stage's kernel uses (window places computed, not loaded; ac_error_count_device with window_len)
        eq = [p.equal_window_len() for p in packed]
        wlen = eq if all(x is not None for x in eq) else None
        kc = ac.ApproxCounter(local)
        # >= 150 untimed launches (>= 15 ms of load at cfg2): the timed ones then run at the
        # sustained clock, like the stage's steps after them (last 50 of 210 launches:
        # 94.6 us against 98.2 for all 210, profiles/r03_staged_cost_early3.md)
        for _ in range(max(args.warmup, 150)):
            kc.count_device(args.k, arr, stream=stream.cuda_stream, window_len=wlen)
        every = max(1, args.event_every)
        n_kernel = max(args.steps, args.kernel_launches)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(0, n_kernel, every)]
        for i in range(n_kernel):
            if i % every == 0:
                evs[i // every][0].record(stream)
            kc.count_device(args.k, arr, stream=stream.cuda_stream, window_len=wlen)
            if i % every == 0:
                evs[i // every][1].record(stream)
        torch.cuda.synchronize(dev)
        kc.check(stream=stream.cuda_stream)
        kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
        geo = kc.last_launch()
        kc.close()

    # ---- the stage's path (ac_stage_mode, after the cold call above): the early launch at every
    # size (the count kernel launched first, its copier workgroups staging each read end as the host
    # packs it); the DMA path (copy engine, 2-4 parts) only with AC_STAGE_EARLY=0.
    tune_calls = 0
    while counter.stage_mode() < 0 and tune_calls < 4:
        counter.count_jobs(args.k, jobs)
        tune_calls += 1
    stage_path = {3: "early-launch-device-pack", 2: "early-launch", 0: "dma"}.get(counter.stage_mode(), "undecided")

    # ---- pipelined leg (informational, 1 GPU): host-buffer steps back to back, max(steps, 100)
    # of them.  Run before the stage, so the stage is timed in steady state; one stage call on
    # the cold context is reported as stage_cold_call_ms. ------------------------------------
    pipelined = None
    if world == 1 and not args.no_pipelined:
        bufs = [torch.zeros(max(1, jobs.n_counts), dtype=torch.int32, device=dev) for _ in range(2)]
        hosts = [torch.zeros(max(1, jobs.n_counts), dtype=torch.int32).pin_memory() for _ in range(2)]

        def pstep(i):
            counter.submit_jobs(args.k, jobs, bufs[i % 2], stream=stream.cuda_stream)
            hosts[i % 2].copy_(bufs[i % 2], non_blocking=True)

        n_pipe = max(args.steps, args.kernel_launches)
        for i in range(args.warmup):
            pstep(i)
        torch.cuda.synchronize(dev)
        tp = time.perf_counter()
        for i in range(n_pipe):
            pstep(i)
        torch.cuda.synchronize(dev)
        elp = time.perf_counter() - tp
        counter.check(stream=stream.cuda_stream)
        pipelined = {"value": units_rank * n_pipe / elp, "unit": "kmer*bp/s", "ms_per_step": elp / n_pipe * 1e3,
                     "steps": n_pipe,
                     "note": "same host-buffer steps via ac_error_count_jobs_submit + async D2H, not synchronised per "
                             "step: step i+1's packing overlaps step i's kernel (independent -mr runs)"}

    # ---- the count all-reduce of N > 1 (RCCL over xGMI): the library's own communicator
    # (ac_comm_init, id from rank 0 over the process group); if it cannot be set up, torch's
    # RCCL process group does the same all-reduce and the line says so.
    allreduce_by = None
    submit_form = world > 1 or args.step_form == "submit"
    if submit_form and backend == "nccl":
        try:
            uid = [counter.comm_unique_id() if rank == 0 else None]
            if world > 1:
                dist.broadcast_object_list(uid, src=0)
            counter.comm_init(world, rank, uid[0])
            allreduce_by = "library (ac_allreduce_counts, RCCL)"
        except Exception as exc:  # noqa: BLE001 -- reported on the line, the run continues on torch's RCCL
            print(f"[bench] library RCCL communicator unavailable ({exc}); using torch.distributed", file=sys.stderr)
            allreduce_by = (f"torch.distributed RCCL (library communicator failed: {exc})" if world > 1 else
                            f"none: one rank and no library communicator ({exc}); the step skips the all-reduce")
    elif world > 1:
        allreduce_by = f"torch.distributed {backend} on host copies (rehearsal)"

    # ---- the stage (value): host Dna5 buffers -> host counts ---------------------------------
    if not submit_form:
        def step():
            counter.count_jobs(args.k, jobs)  # pack, one fused launch, counts back (synchronous)
    else:
        def step():
            counter.submit_jobs(args.k, jobs, d_counts, stream=stream.cuda_stream)
            if backend == "nccl":
                if allreduce_by.startswith("library"):
                    counter.allreduce_counts(d_counts, stream=stream.cuda_stream)  # RCCL over xGMI
                elif world > 1:
                    dist.all_reduce(d_counts)  # torch's RCCL, on the current stream
                # (world 1 without the library communicator: no process group, so no all-reduce;
                # the line's `allreduce` field says so)
                h_counts.copy_(d_counts, non_blocking=True)
                stream.synchronize()
            else:
                stream.synchronize()
                host = d_counts.cpu()
                if world > 1:
                    dist.all_reduce(host)
                h_counts.copy_(host)

    for _ in range(args.warmup):
        step()
    # the pool that packs the timed steps: made by the first stage call (its size is the plan's, or
    # AC_HOST_THREADS when set), so read after that call, not from the plan before it
    pool_participants, pool_cpus = host_pool_cpus()
    if world > 1:
        print(f"[bench] rank {rank} (local {local}): host pool {pool_participants} participants on CPUs "
              f"{_ranges(pool_cpus)}", file=sys.stderr, flush=True)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    cg0 = cgroup_cpu_stat()  # CPU-quota throttling over the timed steps
    t0 = time.perf_counter()
    marks = []
    for _ in range(args.steps):
        step()
        marks.append(time.perf_counter())
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    cg1 = cgroup_cpu_stat()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    if args.verify and world == 1:  # (N > 1: tests/test_gpu_multirank.py covers the sharded path)
        import oracle

        got = counter.count_jobs(args.k, jobs)
        for e, g in zip(ends, got):
            assert np.array_equal(g, oracle.count_myers(args.k, wl[e]["kmers"], wl[e]["windows"])), e
        print("verify ok: the stage's counts equal the oracle's", file=sys.stderr, flush=True)

    if rank == 0:
        P = min(32 // args.k, 4)
        reads_note = (f"{args.sn} reads sharded over {world} ranks" if world > 1 and args.scaling == "strong"
                      else f"shard {args.shard} of {args.sn} reads (rehearsal: one rank's share, timed alone)"
                      if args.shard else f"{args.sn} reads/rank")
        workload_name = (f"{args.config}: k={args.k} sn={args.sn} sl={args.sl} lim={args.lim}, "
                         f"start+end ends fused, {reads_note}")
        out = {
            "metric": METRIC,
            "value": units_job * args.steps / elapsed,
            "unit": "kmer*bp/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": args.scaling if world > 1 else "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": DATA_NOTE,
            "config": {"workload": workload_name, "k": args.k, "sn": args.sn, "sl": args.sl, "lim": args.lim,
                       "candidates": n_c, "kmer_bp_per_step": units_job, "kmer_bp_per_rank_step": units_rank,
                       "stage": stage_text(stage_path, world),
                       "stage_path": stage_path,
                       "parallelism": (f"{args.scaling} window shards x{world}, "
                                       f"{'RCCL' if backend == 'nccl' else backend} all-reduce of counts")
                       if world > 1 else "1 GPU"},
            **({"allreduce": allreduce_by} if allreduce_by else {}),
        }
        if world == 1 and submit_form:
            out["step_form"] = ("submit: the N > 1 step (ac_error_count_jobs_submit -> RCCL all-reduce on a one-rank "
                                "communicator -> counts D2H -> stream sync) on one GPU: a rehearsal of its costs")
        if world == 1:  # each step is synchronous at N = 1: its own duration
            d = np.diff(np.array([t0] + marks)) * 1e3
            out["step_ms"] = {"min": float(d.min()), "p50": float(np.median(d)), "p99": float(np.percentile(d, 99)),
                              "p99.9": float(np.percentile(d, 99.9)), "max": float(d.max())}
        out["stage_cold_call_ms"] = cold_ms
        if cg1:
            dl = {key: cg1[key] - cg0.get(key, 0) for key in ("nr_periods", "nr_throttled", "throttled_usec", "usage_usec")
                  if key in cg1}
            out["cgroup_cpu"] = {**dl, "cpus_used_per_wall_s": dl.get("usage_usec", 0) / 1e6 / elapsed,
                                 "quota_cpus": cpu_share()[1],
                                 "note": "rank 0's cgroup cpu.stat deltas over the timed steps: a throttled period "
                                         "stalls every thread of the cgroup until the next 100 ms period"}
        out["host_pool"] = {"participants": pool_participants, "cpus": _ranges(pool_cpus),
                            "note": "rank 0's pack pool as it ran the timed steps (read after the first stage call "
                                    "made it): GPU-local CPUs split among the local ranks, at most its share of the "
                                    "cgroup CPU quota, or AC_HOST_THREADS when set (ac_host_pool_cpus)"}
        out["stage_path_choice"] = {"path": stage_path, "untimed_calls": tune_calls,
                                    "note": "ac_stage_mode: the early launch at every size since round 4 (DMA parts "
                                            "only with AC_STAGE_EARLY=0)"}
        if kern_ms is not None:
            ops = OPS_PER_BASE_WORD / P * units_rank  # algorithmic lane-ops per launch (this rank)
            achieved = ops / (kern_ms * 1e-3)
            pmc = load_pmc(workload_name.replace(reads_note, f"{args.sn} reads/rank")) if world == 1 else None
            sample_bytes = SAMPLE_BYTES_PER_BASE * sum(bases) + 12 * sum(n_c)  # sample + kmers in + counts out
            roof = {"bound": "valu", "achieved": achieved / 1e12, "peak": VALU_PEAK_OPS / 1e12, "unit": "Tops/s",
                    "frac": achieved / VALU_PEAK_OPS,
                    "traffic": pmc.get("hbm_bytes_per_launch") if pmc else None,
                    "frac_survey_basis": SURVEY_OPS_PER_UNIT * units_rank / (kern_ms * 1e-3) / VALU_PEAK_OPS,
                    "note": f"int32 VALU lane-ops, {OPS_PER_BASE_WORD}/P per kmer*bp (P={P}) over the kernel-only "
                            f"time (HIP events around every {max(1, args.event_every)}th launch); frac_survey_basis = "
                            f"the same time on SURVEY.md 8(d)'s 20 ops per kmer*bp (> 1 means that op model "
                            f"overestimates a P-packed NFA, not skipped work: counts are bit-exact); PMC from "
                            f"{pmc.get('source') if pmc else 'n/a'}"}
            if pmc and pmc.get("sq_insts_valu_per_launch"):
                model = OPS_PER_BASE_WORD / P * units_rank / 64.0  # wave instructions
                roof["sq_insts_valu"] = {"measured_per_launch": pmc["sq_insts_valu_per_launch"],
                                         "model_per_launch": model,
                                         "ratio": pmc["sq_insts_valu_per_launch"] / model}
            out["kernel_ms"] = kern_ms
            out["kernel_kmer_bp_per_s"] = units_rank / (kern_ms * 1e-3)
            out["kernel_leg"] = ("ac_error_count_device with window_len (equal windows: places computed, as in the stage)"
                                 if wlen else "ac_error_count_device (window descriptors loaded)")
            out["launch"] = geo
            out["roofline"] = roof
            out["roofline_hbm"] = {"bound": "hbm (informational)",
                                   "achieved": sample_bytes / (kern_ms * 1e-3) / 1e9, "peak": HBM_PEAK / 1e9,
                                   "unit": "GB/s", "frac": sample_bytes / (kern_ms * 1e-3) / HBM_PEAK,
                                   "algorithmic_bytes_per_launch": sample_bytes}
        if pipelined:
            out["pipelined"] = pipelined
        if not args.no_exact and world == 1 and not args.shard:
            out["exact"] = exact_block(local)
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(wl, args.k, args.cpu_seconds)
        print(json.dumps(out), flush=True)
    counter.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
