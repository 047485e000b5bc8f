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
    buf = np.zeros(8 * (1 << 18), dtype=np.uint64)
    L = _lib.load()
    L.ac_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    assert L.ac_debug_stamps(buf.ctypes.data, buf.nbytes) == 0
    raw = buf[: 8 * n].reshape(n, 8).astype(np.int64)
    st = raw[:, :4]
    t0 = st[:, 0].min()
    us = (st - t0) / 100.0  # 100 MHz
    pct = lambda x: " ".join(f"{np.percentile(x, q):7.1f}" for q in (0, 10, 50, 90, 100))
    print(f"waves={n} geometry={geo}")
    print("                 p0      p10     p50     p90    p100  (us)")
    print("start        ", pct(us[:, 0]))
    pre = (raw[:, 7] - t0) / 100.0
    wib = np.arange(n) % 4  # wave in workgroup (waves are numbered blockIdx * 4 + wib)
    print("prologue len ", pct(us[:, 1] - us[:, 0]))
    print("  own part   ", pct(pre - us[:, 0]), "(entry -> before the barrier)")
    print("  own, wave 0", pct((pre - us[:, 0])[wib == 0]), "(k-mer loads + ~Eq table)")
    print("  own, others", pct((pre - us[:, 0])[wib != 0]))
    print("  barrier    ", pct(us[:, 1] - pre))
    print("main len     ", pct(us[:, 2] - us[:, 1]))
    print("atomics len  ", pct(us[:, 3] - us[:, 2]))
    print("main end     ", pct(us[:, 2]))
    print("end          ", pct(us[:, 3]))
    # per candidate group: end times (a group's waves only steal within the group)
    grp = raw[:, 6] >> 16
    print("per group (seg<<16|g): waves, end p0/p50/p100 us")
    for gv in np.unique(grp):
        e = us[grp == gv, 3]
        print(f"  {int(gv):#8x} {e.size:5d}  {e.min():7.1f} {np.median(e):7.1f} {e.max():7.1f}")
    # per-SIMD view: HW_ID (gfx9 layout) wave[3:0] simd[5:4] cu[11:8] sh[12] se[15:13]; + XCC id
    hw, xcc = raw[:, 4], raw[:, 5]
    simd_key = xcc * 100000 + ((hw >> 13) & 7) * 10000 + ((hw >> 12) & 1) * 1000 + ((hw >> 8) & 15) * 10 + ((hw >> 4) & 3)
    keys, inv, cnt = np.unique(simd_key, return_inverse=True, return_counts=True)
    print(f"SIMDs used: {keys.size}; waves per SIMD: min {cnt.min()} max {cnt.max()} mean {cnt.mean():.2f}")
    span = np.zeros(keys.size)
    last = np.zeros(keys.size)
    first = np.full(keys.size, 1e18)
    for i in range(n):
        first[inv[i]] = min(first[inv[i]], us[i, 0])
        last[inv[i]] = max(last[inv[i]], us[i, 3])
    span = last - first
    print("SIMD span    ", pct(span))
    # active-wave profile of the slowest SIMD
    j = int(np.argmax(last))
    w = np.nonzero(inv == j)[0]
    print(f"slowest SIMD {keys[j]}: {w.size} waves, (start, end) us:",
          sorted((round(float(us[i, 0]), 1), round(float(us[i, 3]), 1)) for i in w))
    # time-weighted number of resident waves per SIMD, over the kernel
    T = us[:, 3].max()
    grid = np.linspace(0, T, 200)
    active = np.zeros((keys.size, grid.size))
    for i in range(n):
        active[inv[i]] += (grid >= us[i, 0]) & (grid < us[i, 3])
    # waves past the prologue (counting) per SIMD during the launch ramp
    for t in (2, 5, 10, 20, 30):
        counting = ((us[:, 1] <= t) & (us[:, 2] > t)).sum() / keys.size
        print(f"t={t:3d} us: counting waves per SIMD {counting:.2f}")
    print("mean resident waves per SIMD at 10%..90% of the kernel:",
          [round(float(active[:, int(f * 199)].mean()), 2) for f in (0.1, 0.3, 0.5, 0.7, 0.8, 0.9, 0.95)])


if __name__ == "__main__":
    main()
