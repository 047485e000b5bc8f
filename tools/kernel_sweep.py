#!/usr/bin/env python3
"""Count-kernel time on device-resident input against the windows each wave gets: one cfg2-shaped
workload (k=16, 100 / 101-bp read ends, `--lim` candidates per end) cut to several sample sizes, the
kernel timed with HIP events around every launch after a warm-up (the bench's kernel leg, bench.py).
The per-window cost at large samples is the steady state; the excess at cfg2's 10k reads is the
launch's fixed cost (prologue, tail, hand-off).

    python3 tools/kernel_sweep.py [--sn 10000,20000,40000,100000] [--lim 500] [--launches 100]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sn", default="10000,20000,40000,100000")
    ap.add_argument("--lim", type=int, default=500)
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--sl", type=int, default=100)
    ap.add_argument("--launches", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=150)
    ap.add_argument("--every", type=int, default=1,
                    help="events around every n-th launch only (the bench's kernel leg: 5); the launches between "
                         "run back to back")
    a = ap.parse_args()
    import torch

    import approx_counter_amd as ac
    import bench

    sns = [int(x) for x in a.sn.split(",")]
    sys.argv = ["bench.py", "--sn", str(max(sns)), "--lim", str(a.lim), "--k", str(a.k), "--sl", str(a.sl)]
    args = bench.parse()
    full, _ = bench.build_workload(args, 0, 1)
    ends = ("start", "end")
    stream = torch.cuda.current_stream()
    with ac.ApproxCounter(0) as c:
        for sn in sns:
            wl = {e: {"kmers": full[e]["kmers"], "windows": full[e]["windows"][:sn]} for e in ends}
            packed = [ac.pack_windows(wl[e]["windows"]) for e in ends]
            segs = [ac.DeviceSegment.upload(wl[e]["kmers"], packed[i]) for i, e in enumerate(ends)]
            arr = ac.ApproxCounter.segment_array(segs)
            wlen = [p.equal_window_len() for p in packed]
            for _ in range(a.warmup):
                c.count_device(a.k, arr, stream=stream.cuda_stream, window_len=wlen)
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(0, a.launches, a.every)]
            for i in range(a.launches):
                if i % a.every == 0:
                    evs[i // a.every][0].record(stream)
                c.count_device(a.k, arr, stream=stream.cuda_stream, window_len=wlen)
                if i % a.every == 0:
                    evs[i // a.every][1].record(stream)
            torch.cuda.synchronize()
            c.check(stream=stream.cuda_stream)
            t = np.array([b.elapsed_time(e) for b, e in evs]) * 1e3
            geo = c.last_launch()
            units = sum(wl[e]["kmers"].size * sum(int(w.size) for w in wl[e]["windows"]) for e in ends)
            print(f"sn {sn:7d}: kernel mean {t.mean():9.2f} us  p50 {np.median(t):9.2f}  min {t.min():9.2f}  "
                  f"per 10k reads {t.mean() * 1e4 / sn:8.2f} us  kmer*bp/s {units / (t.mean() * 1e-6):.3e}  "
                  f"geometry {geo}", flush=True)
            del segs, arr


if __name__ == "__main__":
    main()
