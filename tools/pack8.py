#!/usr/bin/env python3
"""Host-side evidence for the 8-GPU projection: eight concurrent pack-only processes,
each one rank's share of one node -- LOCAL_RANK r of LOCAL_WORLD_SIZE 8, its host pool planned by the
library exactly as the bench's ranks plan it (ac_create -> plan_host_pool: the GPU-local CPUs split
among the local ranks by physical core, at most its share of the cgroup CPU quota) -- packing one rank's
1/8 cfg4 shard (2 x 125,000 windows of 100 / 101 bases, the stage's equal-window record form) with the
stage's packer (tools/pack_bench.cpp, host_pack.cpp).  Reports each process's per-call pack time, alone
and with all eight packing at once (the host DRAM bandwidth and CPU quota they share).

    python3 tools/pack8.py [--ranks 8] [--n 125000] [--iters 400]
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def plan(rank, ranks):
    """(participants, cpulist) the library plans for local rank `rank` of `ranks` (creates a context)."""
    code = ("import json, approx_counter_amd as ac\n"
            "from approx_counter_amd.counter import host_pool_cpus\n"
            "c = ac.ApproxCounter(0)\n"
            "print(json.dumps(host_pool_cpus()))\n"
            "c.close()\n")
    env = dict(os.environ, LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(ranks), PYTHONPATH=ROOT)
    env.pop("AC_HOST_THREADS", None)
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    if out.returncode:
        sys.exit(f"plan for rank {rank} failed: {out.stderr[-2000:]}")
    part, cpus = json.loads(out.stdout.strip().splitlines()[-1])
    return part, cpus


def cpulist(cpus):
    return ",".join(str(c) for c in cpus)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--n", type=int, default=125_000, help="windows per read end of one rank's shard")
    ap.add_argument("--iters", type=int, default=400)
    a = ap.parse_args()
    exe = os.path.join(ROOT, "build", "pack_bench")
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    subprocess.run(["g++", "-O3", "-std=c++17", "-pthread", "-I" + os.path.join(ROOT, "approx_counter_amd", "csrc"),
                    os.path.join(ROOT, "tools", "pack_bench.cpp"),
                    os.path.join(ROOT, "approx_counter_amd", "csrc", "host_pack.cpp"), "-o", exe], check=True)
    plans = [plan(r, a.ranks) for r in range(a.ranks)]
    for r, (part, cpus) in enumerate(plans):
        print(f"rank {r}: {part} participants on CPUs {cpulist(cpus) or 'unpinned'}", flush=True)
    allc = [c for _, cpus in plans for c in cpus]
    print(f"plans disjoint: {len(allc) == len(set(allc))}", flush=True)

    def launch(r):
        part, cpus = plans[r]
        env = dict(os.environ, AC_HOST_THREADS=str(part))
        if cpus:
            env["AC_PACK_CPUS"] = cpulist(cpus)
        # tasks of 2,048 windows: the early launch's task size for a call this large (capi.cpp)
        return subprocess.Popen([exe, str(a.n), str(a.iters), "2048", "1"], env=env, stdout=subprocess.PIPE,
                                stderr=subprocess.STDOUT, text=True)

    def result(p):
        out = p.communicate(timeout=600)[0]
        if p.returncode:
            sys.exit(f"pack_bench failed: {out[-2000:]}")
        return json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])

    alone = result(launch(0))
    print(f"alone (rank 0's plan): both ends packed p50 {alone['both_p50_us']:.1f} us, p90 {alone['both_p90_us']:.1f}, "
          f"max {alone['both_max_us']:.1f} ({alone['participants']} participants)", flush=True)
    procs = [launch(r) for r in range(a.ranks)]
    res = [result(p) for p in procs]
    for r, x in enumerate(res):
        print(f"concurrent rank {r}: both ends packed p50 {x['both_p50_us']:.1f} us, p90 {x['both_p90_us']:.1f}, "
              f"max {x['both_max_us']:.1f} ({x['participants']} participants)", flush=True)
    p50 = sorted(x["both_p50_us"] for x in res)
    print(json.dumps({"ranks": a.ranks, "windows_per_end": a.n, "alone_p50_us": alone["both_p50_us"],
                      "concurrent_p50_us": {"min": p50[0], "median": p50[len(p50) // 2], "max": p50[-1]},
                      "concurrent_p90_max_us": max(x["both_p90_us"] for x in res)}), flush=True)


if __name__ == "__main__":
    main()
