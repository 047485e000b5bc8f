#!/usr/bin/env python3
"""Timeline of one early-launch stage call (ac_error_count_jobs) from a
-DAC_STAMPS diagnostic build:

    APPROX_COUNTER_AMD_LIB=build/var/stamps/libapprox_counter_amd.so python tools/stage_stamps.py [--sn N]

Per segment (read end), in us relative to the first wave's entry: when the segment's
host poller saw the host's first progress record and its final header, when the last
chunk was in device memory, and the spread of wave
entry, counting start (after the staging wait and the table barrier), counting end and
exit.  No output value is computed from the stamps."""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sn", type=int, default=10000)
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--lim", type=int, default=500)
    ap.add_argument("--calls", type=int, default=60)
    ap.add_argument("--t0", choices=("entry", "progress"), default="entry",
                    help="progress: time from segment 0's poller first seeing the call's first progress record "
                         "(round 4's armed launches and their AC_ARM_US were removed in round 5)")
    a = ap.parse_args()
    import approx_counter_amd as ac
    from approx_counter_amd import _lib
    from tools import workload

    wl, _ = workload.build(n_reads=a.sn, k=a.k, lim=a.lim)
    ends = ("start", "end")
    jobs = ac.Jobs([(wl[e]["kmers"], ac.Dna5Sample.from_windows(wl[e]["windows"])) for e in ends])
    c = ac.ApproxCounter(0)
    L = _lib.load()
    L.ac_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    pct = lambda x: " ".join(f"{np.percentile(x, q):7.1f}" for q in (0, 10, 50, 90, 100))  # noqa: E731
    for call in range(a.calls):
        c.count_jobs(a.k, jobs)
        if call < a.calls - 3:
            continue
        geo = c.last_launch()
        n = int(geo["waves"])
        buf = np.zeros(8 * (1 << 18) + 64, dtype=np.uint64)
        assert L.ac_debug_stamps(buf.ctypes.data, buf.nbytes) == 0
        raw = buf[: 8 * n].reshape(n, 8).astype(np.int64)
        stage = buf[8 * (1 << 18):].astype(np.int64)
        t0 = raw[:, 0].min() if a.t0 == "entry" else int(stage[1])
        us = (raw[:, :4] - t0) / 100.0
        seg = raw[:, 6] >> 32
        print(f"call {call}: mode {c.stage_mode()} waves={n} kernel span {us[:, 3].max():.1f} us")
        print("                          p0      p10     p50     p90    p100  (us)")
        for s in np.unique(seg):
            m = seg == s
            us_of = lambda i: (stage[8 * s + i] - t0) / 100  # noqa: E731
            print(f" seg {s}: first progress seen {us_of(1):7.1f}, first codes progress {us_of(3):7.1f}, first codes "
                  f"chunk in {us_of(4):7.1f}, final header seen {us_of(0):7.1f}, last chunk in {us_of(2):7.1f}")
            print("   entry           ", pct(us[m, 0]))
            wait_end = (raw[:, 7] - t0) / 100.0
            w0 = m & (np.arange(n) % 4 == 0)
            print("   staging waited  ", pct(wait_end[w0]), "(wave 0 of each workgroup)")
            print("   counting starts ", pct(us[m, 1]))
            print("   counting ends   ", pct(us[m, 2]))
            print("   exit            ", pct(us[m, 3]))
            print("   gate slow path us", pct(raw[m, 4] / 100.0), " calls", pct(raw[m, 5]))
            grp = (raw[:, 6] >> 16) & 0xffff
            for gv in np.unique(grp[m]):
                mg = m & (grp == gv)
                print(f"   group {int(gv)}: {int(mg.sum())} waves; counting ends p0/p50/p100 "
                      f"{us[mg, 2].min():.1f} {np.median(us[mg, 2]):.1f} {us[mg, 2].max():.1f}; exit max {us[mg, 3].max():.1f}")


if __name__ == "__main__":
    main()
