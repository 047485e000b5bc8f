#!/usr/bin/env python3
"""Per-wave timeline of one count launch from a -DAC_STAMPS diagnostic build.

    APPROX_COUNTER_AMD_LIB=build/var/stamps/libapprox_counter_amd.so python tools/stamps.py [--sn N]

Prints, in µs relative to the first wave's entry: the spread of wave start
times (dispatch ramp), prologue length, main-loop length and end times.
"""
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
    a = ap.parse_args()
    import torch

    import approx_counter_amd as ac
    from approx_counter_amd import _lib
    from tools import workload

    wl, _ = workload.build(n_reads=a.sn, k=a.k, lim=a.lim)
    c = ac.ApproxCounter(0)
    segs = [ac.DeviceSegment.upload(wl[e]["kmers"], ac.pack_windows(wl[e]["windows"])) for e in ("start", "end")]
    for _ in range(5):
        c.count_device(a.k, segs)
    torch.cuda.synchronize()
    geo = c.last_launch()
    n = int(geo["waves"])
    buf = np.zeros(4 * (1 << 18), dtype=np.uint64)
    L = _lib.load()
    L.ac_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    assert L.ac_debug_stamps(buf.ctypes.data, buf.nbytes) == 0
    st = buf[: 4 * n].reshape(n, 4).astype(np.int64)
    t0 = st[:, 0].min()
    us = (st - t0) / 100.0  # 100 MHz
    pct = lambda x: " ".join(f"{np.percentile(x, q):7.1f}" for q in (0, 10, 50, 90, 100))
    print(f"waves={n} geometry={geo}")
    print("                 p0      p10     p50     p90    p100  (us)")
    print("start        ", pct(us[:, 0]))
    print("prologue len ", pct(us[:, 1] - us[:, 0]))
    print("main len     ", pct(us[:, 2] - us[:, 1]))
    print("atomics len  ", pct(us[:, 3] - us[:, 2]))
    print("end          ", pct(us[:, 3]))


if __name__ == "__main__":
    main()
