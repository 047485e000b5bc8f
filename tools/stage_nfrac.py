#!/usr/bin/env python3
"""Stage step time vs N content of the sample (cfg2 shape), interleaved on one box.

    python tools/stage_nfrac.py [--steps 400] [--reps 3]

Variants of the same cfg2 workload (tools/workload.build): `orig` (0.1 % N per base,
the bench's data), `nfree` (every N replaced by A), `nlast` (N-free except the last 2 %
of each end's windows, which keep their N).  Prints p50/p10/p90 of the synchronous
ac_error_count_jobs step per variant.  Diagnostic only (not part of the product).
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--variants", default="orig,nfree,nlast")
    a = ap.parse_args()
    import approx_counter_amd as ac
    from tools import workload

    wl, _ = workload.build(n_reads=10_000, read_len=400, k=16, sl=100, lim=500, seed=1)
    ends = ("start", "end")

    def variant(name):
        out = []
        for e in ends:
            ws = [w.copy() for w in wl[e]["windows"]]
            if name in ("nfree", "nlast"):
                keep = len(ws) - len(ws) // 50 if name == "nlast" else len(ws)
                for w in ws[:keep]:
                    w[w > 3] = 0
            out.append((wl[e]["kmers"], ac.Dna5Sample.from_windows(ws)))
        return ac.Jobs(out)

    names = a.variants.split(",")
    jobs = {n: variant(n) for n in names}
    c = ac.ApproxCounter(0)
    ref = {n: [r.copy() for r in c.count_jobs(16, jobs[n])] for n in names}
    for _ in range(300):
        c.count_jobs(16, jobs[names[0]])
    for rep in range(a.reps):
        for n in names:
            for _ in range(10):
                c.count_jobs(16, jobs[n])
            ts = []
            for _ in range(a.steps):
                t = time.perf_counter()
                r = c.count_jobs(16, jobs[n])
                ts.append(time.perf_counter() - t)
            ok = all(np.array_equal(x, y) for x, y in zip(r, ref[n]))
            ts = np.array(ts) * 1e3
            print(f"rep {rep} {n:6s}: p10 {np.percentile(ts, 10):.4f} p50 {np.median(ts):.4f} "
                  f"p90 {np.percentile(ts, 90):.4f} max {ts.max():.3f} ms  stable={ok}", flush=True)
    c.close()


if __name__ == "__main__":
    main()
