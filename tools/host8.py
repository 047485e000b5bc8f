#!/usr/bin/env python3
"""The host-side work of one rank's step at 8 ranks, eight processes at once.

    python tools/host8.py [--sample pinned|heap] [--ranks 8] [--calls 200] [--config cfg4|cfg2]

Each process takes LOCAL_RANK r of LOCAL_WORLD_SIZE 8 (so the library plans its host pool as an
8-rank node would: disjoint CPUs, the rank's share of the cgroup quota) and submits its 1/8 shard
of cfg4 (2 x 125k windows, strong scaling, bench.build_workload; or with --config cfg2 its own
2 x 10k windows, weak scaling as bench.py's cfg2 line) with ac_error_count_jobs_submit
-- bench.py's N > 1 step -- timing the submit call alone: everything the host does before the
count kernel owns the step (layout, and with a heap sample the host pool's packing; with a
pinned sample the kernel packs).  The device work then completes untimed (one GPU
serves all eight processes here, so device time is not a rank's).  Prints per-rank p50 / p90 /
max and one JSON line with the max over ranks."""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(rank, ranks, sample, calls, warmup, go_file, config="cfg4"):
    import torch

    import approx_counter_amd as ac
    import bench
    from approx_counter_amd.counter import host_pool_cpus

    sys.argv = ["bench.py", "--config", config]
    args = bench.parse()
    args.scaling = "strong" if config == "cfg4" else "weak"
    wl, _ = bench.build_workload(args, rank, ranks)
    ends = ("start", "end")
    smp = [ac.Dna5Sample.from_windows(wl[e]["windows"]) for e in ends]
    if sample == "pinned":
        smp = [s.pinned() for s in smp]
    jobs = ac.Jobs([(wl[e]["kmers"], s) for e, s in zip(ends, smp)])
    c = ac.ApproxCounter(0)
    st = torch.cuda.current_stream()
    d = torch.zeros(jobs.n_counts, dtype=torch.int32, device="cuda")
    for _ in range(warmup):
        c.submit_jobs(16, jobs, d, stream=st.cuda_stream)
        st.synchronize()
    open(go_file + f".ready{rank}", "w").close()
    while not os.path.exists(go_file):  # all ranks start their timed calls together
        time.sleep(0.001)
    t = []
    for _ in range(calls):
        t0 = time.perf_counter()
        c.submit_jobs(16, jobs, d, stream=st.cuda_stream)
        t.append(time.perf_counter() - t0)
        st.synchronize()
    c.check(stream=st.cuda_stream)
    part, cpus = host_pool_cpus()
    t = np.array(t) * 1e6
    print(json.dumps({"rank": rank, "mode": c.stage_mode(), "participants": part, "n_cpus": len(cpus),
                      "p50_us": float(np.median(t)), "p90_us": float(np.percentile(t, 90)), "max_us": float(t.max())}),
          flush=True)
    c.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sample", choices=("pinned", "heap"), default="pinned")
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--worker", type=int, default=-1)
    ap.add_argument("--go", default="")
    ap.add_argument("--config", choices=("cfg4", "cfg2"), default="cfg4")
    a = ap.parse_args()
    if a.worker >= 0:
        worker(a.worker, a.ranks, a.sample, a.calls, a.warmup, a.go, a.config)
        return
    go = f"/tmp/host8_go_{os.getpid()}"
    procs = []
    for r in range(a.ranks):
        env = dict(os.environ, LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(a.ranks))
        procs.append(subprocess.Popen([sys.executable, __file__, "--worker", str(r), "--ranks", str(a.ranks),
                                       "--sample", a.sample, "--calls", str(a.calls), "--warmup", str(a.warmup),
                                       "--config", a.config,
                                       "--go", go], env=env, stdout=subprocess.PIPE, text=True))
    t0 = time.time()
    while not all(os.path.exists(go + f".ready{r}") for r in range(a.ranks)):
        if any(p.poll() not in (None, 0) for p in procs) or time.time() - t0 > 300:
            break
        time.sleep(0.05)
    open(go, "w").close()
    rows = []
    for p in procs:
        out, _ = p.communicate(timeout=600)
        for ln in out.splitlines():
            if ln.startswith("{"):
                rows.append(json.loads(ln))
                print(ln)
    for f in [go] + [go + f".ready{r}" for r in range(a.ranks)]:
        if os.path.exists(f):
            os.remove(f)
    if len(rows) != a.ranks:
        raise SystemExit(f"only {len(rows)} of {a.ranks} ranks reported")
    print(json.dumps({"ranks": a.ranks, "sample": a.sample, "config": a.config, "modes": sorted({r["mode"] for r in rows}),
                      "participants": sorted({r["participants"] for r in rows}),
                      "max_over_ranks_p50_us": max(r["p50_us"] for r in rows),
                      "max_over_ranks_p90_us": max(r["p90_us"] for r in rows),
                      "median_rank_p50_us": float(np.median([r["p50_us"] for r in rows]))}))


if __name__ == "__main__":
    main()
