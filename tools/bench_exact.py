"""Exact-count stage benchmark: ac_exact_count_device
(count_kmers + get_most_frequent, approx_counter.cpp:487-519 / 396-405) on a
sample already resident in HBM, beside the host stage the CLI's --host-exact
runs (libac_host: ach_count_kmers + ach_rank, one thread like the reference).
Both results are compared; the GPU stage time includes its small D2H copies
and the host ranking of the gathered short list (the call is synchronous).

    python tools/bench_exact.py [--reads 100000] [--sl 100] [--k 16] [--lim 2000] [--steps 20]

Prints one JSON line.  Windows are the start windows of synthetic reads
(tools/synth.make_reads, adapters planted), 'data': 'synthetic'."""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import approx_counter_amd as ac  # noqa: E402
from approx_counter_amd import _lib  # noqa: E402
from approx_counter_amd.counter import _ptr  # noqa: E402
from tools.synth import make_reads  # noqa: E402
from tools.workload import windows_from_reads  # noqa: E402

HOST_LIB = os.path.join(ROOT, "approx_counter_amd", "lib", "libac_host.so")


def host_lib():
    L = ctypes.CDLL(HOST_LIB)
    u8p, u64p, u32p = (ctypes.POINTER(t) for t in (ctypes.c_uint8, ctypes.c_uint64, ctypes.c_uint32))
    L.ach_count_kmers.argtypes = [u8p, u64p, u32p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_float, u64p,
                                  ctypes.c_uint32, u64p, u64p, ctypes.c_uint64, u64p, u64p]
    L.ach_count_kmers.restype = ctypes.c_int
    L.ach_rank.argtypes = [u64p, u64p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, u64p, u64p]
    L.ach_rank.restype = ctypes.c_uint64
    L.ach_adjust_threshold.argtypes = [ctypes.c_float, ctypes.c_uint32, ctypes.c_uint32]
    L.ach_adjust_threshold.restype = ctypes.c_float
    return L


def host_stage(H, windows, k, thr, lim):
    lens = np.array([w.size for w in windows], np.uint32)
    offs = np.zeros(len(windows), np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    flat = np.concatenate(windows).astype(np.uint8)
    cap = int(lens.sum()) + 1
    ok, oc = np.zeros(cap, np.uint64), np.zeros(cap, np.uint64)
    n_out, had_n = ctypes.c_uint64(), ctypes.c_uint64()
    fb = np.zeros(1, np.uint64)
    t0 = time.perf_counter()
    rc = H.ach_count_kmers(_ptr(flat, ctypes.c_uint8), _ptr(offs, ctypes.c_uint64), _ptr(lens, ctypes.c_uint32),
                           len(windows), k, thr, _ptr(fb, ctypes.c_uint64), 0, _ptr(ok, ctypes.c_uint64),
                           _ptr(oc, ctypes.c_uint64), cap, ctypes.byref(n_out), ctypes.byref(had_n))
    assert rc == 0
    n = n_out.value
    rk, rc_ = np.zeros(lim, np.uint64), np.zeros(lim, np.uint64)
    m = H.ach_rank(_ptr(ok, ctypes.c_uint64), _ptr(oc, ctypes.c_uint64), n, lim, 0, k,
                   _ptr(rk, ctypes.c_uint64), _ptr(rc_, ctypes.c_uint64))
    dt = time.perf_counter() - t0
    return list(zip(rk[:m].tolist(), rc_[:m].tolist())), n, had_n.value, dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=100_000)
    ap.add_argument("--read-len", type=int, default=400)
    ap.add_argument("--sl", type=int, default=100)
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--lim", type=int, default=2000)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-host", action="store_true")
    ap.add_argument("--forbidden", type=int, default=0,
                    help="pass N random k-mers as the forbidden set (timing of the forbidden filter; use with --no-host)")
    ap.add_argument("--fast", action="store_true",
                    help="vectorised equal-length windows (tools/synth.make_windows_fast) instead of make_reads: "
                         "for the 10^6-window (cfg4) sample")
    a = ap.parse_args()

    import torch  # noqa: F401  (device runtime first, see _lib.load)

    if a.fast:
        from tools.synth import make_windows_fast

        w2d, _ = make_windows_fast(a.reads, a.sl, seed=1)
        windows = list(w2d)
    else:
        reads, _ = make_reads(a.reads, read_len=a.read_len, seed=1)
        windows = windows_from_reads(reads, a.sl, False)
    H = host_lib()
    thr = float(H.ach_adjust_threshold(1.0, 16, a.k))
    sample = ac.pack_windows(windows)
    n_pos = sum(max(0, w.size - a.k + 1) for w in windows)

    L = _lib.load()
    with ac.ApproxCounter(0) as c:
        hw = sample.as_struct()
        dw = _lib.ACWindows()
        ac.counter.check(L.ac_sample_upload(c.handle, ctypes.byref(hw), ctypes.byref(dw)), c.handle)
        km, ct = np.zeros(a.lim, np.uint64), np.zeros(a.lim, np.uint64)
        fb = np.zeros(1, np.uint64)
        if a.forbidden:
            rng = np.random.default_rng(7)
            fb = rng.integers(0, 1 << min(63, 2 * a.k), size=a.forbidden, dtype=np.uint64)
        n_out, n_dist, had_n = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()

        def once():
            st = L.ac_exact_count_device(c.handle, a.k, ctypes.byref(dw), thr, _ptr(fb, ctypes.c_uint64), a.forbidden, a.lim,
                                         0, _ptr(km, ctypes.c_uint64), _ptr(ct, ctypes.c_uint64), a.lim,
                                         ctypes.byref(n_out), ctypes.byref(n_dist), ctypes.byref(had_n))
            ac.counter.check(st, c.handle)

        for _ in range(a.warmup):
            once()
        times = []
        for _ in range(a.steps):
            t0 = time.perf_counter()
            once()
            times.append(time.perf_counter() - t0)
        gpu = list(zip(km[: n_out.value].tolist(), ct[: n_out.value].tolist()))
        path = {1: "partitioned", 0: "hash table"}.get(c.exact_path(), "?")

    gpu_s = float(np.median(times))
    out = {"metric": "exact_count_kmer_positions_per_s", "value": n_pos / gpu_s, "unit": "kmer positions/s",
           "ms_per_call": gpu_s * 1e3, "ms_min": min(times) * 1e3, "steps": a.steps,
           "config": {"workload": "exact count + top-lim, start windows", "reads": len(windows), "sl": a.sl,
                      "k": a.k, "lim": a.lim, "kmer_positions": n_pos, "distinct": n_dist.value}, "path": path,
           "data": "synthetic"}
    if not a.no_host:
        host, n_host, hn, host_s = host_stage(H, windows, a.k, thr, a.lim)
        out["host"] = {"value": n_pos / host_s, "ms": host_s * 1e3, "cores": 1,
                       "kind": "CLI --host-exact stage (libac_host)"}
        out["parity"] = bool(host == gpu and n_host == n_dist.value and hn == had_n.value)
        if not out["parity"]:
            print(json.dumps(out))
            raise SystemExit("GPU exact count differs from the host stage")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
