#!/usr/bin/env python3
"""Step-time tail of the host-buffer stage (ac_error_count_jobs) against the
cgroup's CPU-quota throttling.

    python tools/stall_check.py [--config cfg2] [--seconds 10 | --steps N] [--pinned]

Runs the bench's workload through synchronous stage calls for `--seconds` (or `--steps`),
records every step's duration and reads /sys/fs/cgroup/cpu.stat (nr_periods, nr_throttled,
throttled_usec) before and after, plus every ~100 ms in between, so throttled periods can be
lined up with slow steps.  Prints one JSON line.  The pool's size and spin come from the
library's own knobs (AC_HOST_THREADS, AC_HOST_SPIN_US); `--pinned` builds the sample in
ac_host_alloc memory (the device-packing path)."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def cpu_stat():
    """cgroup v2 cpu.stat as a dict of ints ({} when unreadable)."""
    out = {}
    try:
        for ln in open("/sys/fs/cgroup/cpu.stat"):
            k, v = ln.split()
            out[k] = int(v)
    except (OSError, ValueError):
        pass
    return out


def delta(a, b):
    return {k: b[k] - a.get(k, 0) for k in ("nr_periods", "nr_throttled", "throttled_usec", "usage_usec") if k in b}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--steps", type=int, default=0, help="a fixed number of steps instead of --seconds")
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--pinned", action="store_true", help="sample in ac_host_alloc memory (device packing)")
    a = ap.parse_args()
    import bench

    sys.argv = [sys.argv[0], "--config", a.config]
    args = bench.parse()
    import approx_counter_amd as ac

    wl, _ = bench.build_workload(args, 0, 1)
    ends = ("start", "end")
    counter = ac.ApproxCounter(0)
    samples = [ac.Dna5Sample.from_windows(wl[e]["windows"]) for e in ends]
    if a.pinned:
        samples = [s.pinned() for s in samples]
    jobs = ac.Jobs([(wl[e]["kmers"], s) for e, s in zip(ends, samples)])
    for _ in range(a.warmup):
        counter.count_jobs(args.k, jobs)
    durs, stats = [], []
    s0 = cpu_stat()
    t_end = time.perf_counter() + a.seconds
    t0 = last_stat = time.perf_counter()
    stats.append((0.0, s0))
    n = 0
    while (n < a.steps) if a.steps else (time.perf_counter() < t_end):
        t = time.perf_counter()
        counter.count_jobs(args.k, jobs)
        e = time.perf_counter()
        durs.append((t - t0, (e - t) * 1e3))
        n += 1
        if e - last_stat > 0.1:
            stats.append((e - t0, cpu_stat()))
            last_stat = time.perf_counter()
    s1 = cpu_stat()
    el = time.perf_counter() - t0
    stats.append((el, s1))
    d = np.array([x[1] for x in durs])
    p50 = float(np.median(d))
    # throttled sampling intervals and the slow steps inside them
    thr = []
    for (ta, sa), (tb, sb) in zip(stats, stats[1:]):
        if sb.get("nr_throttled", 0) > sa.get("nr_throttled", 0):
            thr.append((ta, tb, sb["throttled_usec"] - sa.get("throttled_usec", 0)))
    slow = [(t, ms) for t, ms in durs if ms > 2 * p50]
    slow_in_thr = sum(1 for t, _ in slow if any(ta <= t <= tb for ta, tb, _ in thr))
    from approx_counter_amd.counter import host_pool_cpus

    pool = host_pool_cpus()
    out = {
        "config": a.config, "pinned": a.pinned, "steps": len(durs), "seconds": el,
        "stage_mode": counter.stage_mode(),
        "step_ms": {"p50": p50, "p90": float(np.percentile(d, 90)), "p99": float(np.percentile(d, 99)),
                    "p99.9": float(np.percentile(d, 99.9)), "max": float(d.max()),
                    "p99_over_p50": float(np.percentile(d, 99)) / p50},
        "steps_over_2x_p50": len(slow), "of_them_in_throttled_intervals": slow_in_thr,
        "cpu_stat_delta": delta(s0, s1),
        "cpu_per_wall": (s1.get("usage_usec", 0) - s0.get("usage_usec", 0)) / 1e6 / el if s1 else None,
        "throttled_intervals": len(thr),
        "pool": {"participants": pool[0], "AC_HOST_THREADS": os.environ.get("AC_HOST_THREADS"),
                 "AC_HOST_SPIN_US": os.environ.get("AC_HOST_SPIN_US")},
        "quota_cpus": bench.cpu_share()[1],
    }
    print(json.dumps(out), flush=True)
    counter.close()


if __name__ == "__main__":
    main()
