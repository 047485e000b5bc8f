#!/usr/bin/env python3
"""Consecutive-launch timing of one kernel from a rocprofv3 --kernel-trace database (run_results.db):
per launch its duration and the idle gap since the previous launch of ANY kernel ended, and the
start-to-start period -- the GPU side of a step.

    python3 tools/kernel_gaps.py DB [name-substring] [--last N]"""
import sqlite3
import sys

import numpy as np


def main():
    db = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else "wm2_count_kernel"
    last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 300
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    prev_end = None
    dur, gap, period, names = [], [], [], []
    prev_start = None
    for name, s, e in rows:
        if pat in name and prev_end is not None:
            dur.append((e - s) / 1e3)
            gap.append((s - prev_end) / 1e3)
            if prev_start is not None:
                period.append((s - prev_start) / 1e3)
            names.append(name)
        if pat in name:
            prev_start = s
        prev_end = e if prev_end is None else max(prev_end, e)
    dur, gap, period = (np.array(x[-last:]) for x in (dur, gap, period))
    pct = lambda x: " ".join(f"{np.percentile(x, q):8.1f}" for q in (0, 10, 50, 90, 100))  # noqa: E731
    print(f"{len(dur)} launches matching {pat!r} (last {last}); us p0 p10 p50 p90 p100")
    print(f"  duration       {pct(dur)}")
    print(f"  idle gap       {pct(gap)}")
    print(f"  start-to-start {pct(period)}")
    print(f"  kernels: {sorted(set(n.split('(')[0][-60:] for n in names[-last:]))}")


if __name__ == "__main__":
    main()
