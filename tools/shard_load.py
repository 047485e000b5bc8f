#!/usr/bin/env python3
"""One rank's step of an 8-rank node, on one GPU, with the other seven ranks' host load beside it
(VERDICT r5 item 1): bench.py --config cfg4 --shard 0/8 (rank 0's 1/8 shard, 2 x 125k windows,
timed alone on the GPU) while seven pack-only processes (tools/pack_bench.cpp: the host pool's
packer on their own 1/8 shards, 2 threads each, LOCAL_RANK 1..7's CPU plans) load the host's CPUs
and DRAM as seven host-packing ranks would -- the heaviest host load an 8-rank node can carry.

    python3 tools/shard_load.py [--sample pinned|heap] [--loads 7] [--steps 200]
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sample", choices=("pinned", "heap"), default="pinned")
    ap.add_argument("--loads", type=int, default=7)
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args()
    import pack8

    exe = os.path.join(ROOT, "build", "pack_bench")
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    subprocess.run(["g++", "-O3", "-std=c++17", "-pthread", "-I" + os.path.join(ROOT, "approx_counter_amd", "csrc"),
                    os.path.join(ROOT, "tools", "pack_bench.cpp"),
                    os.path.join(ROOT, "approx_counter_amd", "csrc", "host_pack.cpp"), "-o", exe], check=True)
    loads = []
    for r in range(1, a.loads + 1):
        part, cpus = pack8.plan(r, 8)
        env = dict(os.environ, AC_HOST_THREADS=str(max(2, part)))
        if cpus:
            env["AC_PACK_CPUS"] = pack8.cpulist(cpus)
        loads.append(subprocess.Popen([exe, "125000", "100000", "2048", "1"], env=env, stdout=subprocess.DEVNULL,
                                      stderr=subprocess.DEVNULL))
    try:
        env = dict(os.environ, LOCAL_RANK="0", LOCAL_WORLD_SIZE="8")
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "cfg4", "--shard", "0/8",
                            "--steps", str(a.steps), "--warmup", "10", "--no-cpu-baseline", "--no-pipelined",
                            "--no-kernel-leg", "--no-exact", "--sample", a.sample],
                           env=env, capture_output=True, text=True, timeout=400)
    finally:
        running = sum(1 for p in loads if p.poll() is None)
        for p in loads:
            p.terminate()
        for p in loads:
            p.wait(timeout=30)
    if r.returncode:
        raise SystemExit(r.stderr[-3000:])
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    print(json.dumps({"sample": a.sample, "loads_running_at_end": running, "loads": a.loads,
                      "ms_per_step": line["ms_per_step"], "step_ms": line.get("step_ms"),
                      "stage_path": line["config"]["stage_path"], "host_pool": line.get("host_pool"),
                      "cgroup_cpu": line.get("cgroup_cpu")}))


if __name__ == "__main__":
    main()
