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
    packed = [ac.pack_windows(wl[e]["windows"]) for e in ("start", "end")]
    segs = [ac.DeviceSegment.upload(wl[e]["kmers"], packed[i]) for i, e in enumerate(("start", "end"))]
    # the equal-window launch, as the bench's kernel leg and the stage run it
    wlen = [p.equal_window_len() for p in packed]
    wlen = wlen if all(x is not None for x in wlen) else None
    for _ in range(5):
        c.count_device(a.k, segs, window_len=wlen)
    torch.cuda.synchronize()
    geo = c.last_launch()
    n = int(geo["waves"])
    N_ST, N_SG, N_WIN = 1 << 21, 64, 1 << 20  # g_stamps, g_stage_stamps, g_win_stamps (wm_count.hip)
    buf = np.zeros(N_ST + N_SG + N_WIN, dtype=np.uint64)
    L = _lib.load()
    L.ac_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    assert L.ac_debug_stamps(buf.ctypes.data, buf.nbytes) == 0
    raw = buf[: 8 * n].reshape(n, 8).astype(np.int64)
    win = buf[N_ST + N_SG:].reshape(1 << 15, 32)[:n].astype(np.int64)
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
    print("mean resident waves per SIMD at 10/30/50/70/80/90/95 % of the kernel:",
          [round(float(active[:, int(f * 199)].mean()), 2) for f in (0.1, 0.3, 0.5, 0.7, 0.8, 0.9, 0.95)])
    # Per-window stamps (the end of each window a wave counted): window durations against the
    # number of waves resident on the wave's SIMD at the window's midpoint, i.e. the SIMD's
    # throughput as waves leave it (the launch tail), and the launch an even end would give.
    if n <= (1 << 15):
        ends = (win - t0) / 100.0
        per_n = {}
        by_t = {}  # 10-us bins of the window's start: (durations with 4 waves resident)
        tot_windows = np.zeros(keys.size)
        for i in range(n):
            e = ends[i][(ends[i] > us[i, 1]) & (ends[i] <= us[i, 2] + 1e-9)]  # this launch's stamps only
            e = np.sort(e)
            if e.size == 0:
                continue
            tot_windows[inv[i]] += e.size
            prev = np.concatenate([[us[i, 1]], e[:-1]])
            mid = (prev + e) / 2
            gi = np.clip(np.searchsorted(grid, mid), 0, grid.size - 1)
            nres = active[inv[i], gi].astype(int)
            for d, r, p0 in zip(e - prev, nres, prev):
                per_n.setdefault(int(r), []).append(d)
                if r == 4:
                    by_t.setdefault(int(p0 // 10), []).append(d)
        print("4-wave SIMD rate by the window's start time (10-us bins): " + " ".join(
            f"{b * 10}:{4 / np.mean(v):.3f}" for b, v in sorted(by_t.items()) if len(v) > 200))
        print("window durations by waves resident on the SIMD (n: windows, mean us, SIMD windows/us):")
        for r in sorted(per_n):
            d = np.array(per_n[r])
            print(f"  n={r}: {d.size:6d} windows  mean {d.mean():6.2f} us  p50 {np.median(d):6.2f}  "
                  f"SIMD rate {r / d.mean():.3f} windows/us")
        # per SIMD: its waves' exits in order (intra-SIMD spread: the last wave alone after the others)
        ex = {}
        for i in range(n):
            ex.setdefault(inv[i], []).append(us[i, 3])
        ex = {kk: sorted(v) for kk, v in ex.items()}
        lone = np.array([v[-1] - v[-2] for v in ex.values() if len(v) > 1])
        spread = np.array([v[-1] - v[0] for v in ex.values()])
        print("per SIMD: last exit - second-to-last exit (the last wave alone)", pct(lone))
        print("per SIMD: last exit - first exit                              ", pct(spread))
        print("per SIMD: windows counted                                     ", pct(tot_windows))
        cc = np.corrcoef(tot_windows, last)[0, 1]
        print(f"corr(windows on the SIMD, SIMD end) = {cc:.2f}")
        # per group: the last window start (~ the moment its queue ran dry) and its last exit
        print("per group: last window start / last main end / last exit (us)")
        for gv in np.unique(grp):
            sel = np.nonzero(grp == gv)[0]
            starts = []
            for i in sel:
                e = np.sort(ends[i][(ends[i] > us[i, 1]) & (ends[i] <= us[i, 2] + 1e-9)])
                prev = np.concatenate([[us[i, 1]], e[:-1]])
                if prev.size:
                    starts.append(prev.max())
            print(f"  {int(gv):#8x}  {max(starts):7.1f} {us[sel, 2].max():7.1f} {us[sel, 3].max():7.1f}")
        if 4 in per_n:
            r4 = 4 / np.mean(per_n[4])
            ideal = np.median(first) + np.median(us[:, 1] - us[:, 0]) + tot_windows.mean() / r4
            print(f"windows per SIMD: mean {tot_windows.mean():.1f}; at the full-residency rate "
                  f"({r4:.3f}/us) they end at {ideal:.1f} us (even end); SIMDs actually end "
                  f"p50 {np.median(last):.1f} / max {last.max():.1f} us")


if __name__ == "__main__":
    main()
