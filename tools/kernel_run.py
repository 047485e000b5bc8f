#!/usr/bin/env python3
"""Device-resident count-kernel launches of one BASELINE configuration, for
rocprofv3 PMC passes and kernel traces that must see only the kernel (the
bench's stage reads its inputs from pinned host memory, which changes the
memory counters).  Same workload and launch as bench.py's kernel leg.

    rocprofv3 --pmc SQ_INSTS_VALU -d gpurun_out/pmc_valu -o run -- \
        python3 tools/kernel_run.py --config cfg2 --launches 20
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=0,
                    help="launches before the counted ones (a cold GPU runs its first ~10 ms below the "
                         "sustained clock; kernel traces then leave them out: prof_summary.py --skip)")
    ap.add_argument("--descriptors", action="store_true",
                    help="load every window's start / length (ac_error_count_device) even for equal windows")
    ap.add_argument("--staged", action="store_true",
                    help="the early launch's staged instantiation on resident input instead: ac_error_count_jobs "
                         "with every job sent ahead of the launch (AC_TESTING_ALL_AHEAD), so a kernel trace shows "
                         "its own cost against the plain kernel's")
    a = ap.parse_args()
    import torch

    import approx_counter_amd as ac
    import bench

    sys.argv = ["bench.py", "--config", a.config]
    args = bench.parse()
    wl, _ = bench.build_workload(args, 0, 1)
    if a.staged:
        from approx_counter_amd._lib import load

        L = load()
        jobs = [(wl[e]["kmers"], ac.Dna5Sample.from_windows(wl[e]["windows"])) for e in ("start", "end")]
        with ac.ApproxCounter(0) as c:
            prev = L.ac_testing_stage_hooks(2)  # AC_TESTING_ALL_AHEAD
            try:
                for _ in range(a.warmup + a.launches):
                    c.count_jobs(args.k, jobs)
            finally:
                L.ac_testing_stage_hooks(prev)
            print(f"{a.launches} staged launches of {a.config} on resident input (stage mode {c.stage_mode()}); "
                  f"geometry {c.last_launch()}")
        return
    packed = [ac.pack_windows(wl[e]["windows"]) for e in ("start", "end")]
    segs = [ac.DeviceSegment.upload(wl[e]["kmers"], packed[i]) for i, e in enumerate(("start", "end"))]
    arr = ac.ApproxCounter.segment_array(segs)
    eq = [p.equal_window_len() for p in packed]
    wlen = eq if all(x is not None for x in eq) and not a.descriptors else None
    with ac.ApproxCounter(0) as c:
        for _ in range(a.warmup + a.launches):
            c.count_device(args.k, arr, window_len=wlen)
        torch.cuda.synchronize()
        c.check()
        print(f"{a.launches} launches of {a.config} ({'equal windows' if wlen else 'descriptors'}); "
              f"geometry {c.last_launch()}")


if __name__ == "__main__":
    main()
