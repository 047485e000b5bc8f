#!/usr/bin/env python3
"""Benchmark of the approximate-count stage (errorCount, approx_counter.cpp:531-601).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2|cfg3|cfg4|cfg5]

A step is one pass of the hot path over one batch: both read ends of one run
(start + end windows, approx_counter.cpp:858) counted against their own
top-`lim` candidates in ONE fused kernel launch, which also stores the count
vector (no separate zeroing dispatch), inputs already resident in HBM.  Default workload = BASELINE.json
configs[1] (k=16, sn=10,000, sl=100, lim=500), the configuration the metric is
quoted on, on seeded synthetic reads.  With N > 1 ranks (one
process per GPU, torchrun) every rank counts its own sn reads against the same
candidates and the per-candidate count vector is summed with one RCCL
all-reduce per step (weak scaling); the all-reduce of step i overlaps the
count launch of step i+1 (two count buffers, async_op).  Rank 0 prints ONE JSON line.

Roofline: the count kernel is bound by integer VALU
issue, not HBM and not MFMA.  `roofline.achieved` = algorithmic VALU lane-ops
per launch / mean kernel duration (HIP events around every 5th timed launch,
on the launch stream, inside the timed loop: an event is a queue packet of its
own and bracketing every launch adds ~3 us between launches); algorithmic work = 9.5 full-rate lane
ops per text base per lane word of P candidates (P = 2 at k=16, 1 at k=22):
the 8 ops of the Wu-Manber NFA for 3 rows + 1.5 of hit accumulation, with ~Eq
a table lookup as in the textbook algorithm;
`peak` = 256 CU x 4 SIMD x 32 lanes x 2.4 GHz (MI355X_MICROARCH.md: SIMD-32,
2-cycle wave64 VALU issue).  `traffic` = HBM bytes per launch from the
committed rocprofv3 PMC passes (profiles/*_pmc_traffic.json) for the same
workload, FETCH_SIZE doubled per the gfx950 correction, or null.
"""
from __future__ import annotations

import argparse
import copy
import glob
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "approx-count kmer×base pairs/sec (k=16, lim=500, 10k×100bp ends)"
VALU_PEAK_OPS = 256 * 4 * 32 * 2.4e9       # int32 lane-ops/s (2-cycle wave64 issue per SIMD-32)
HBM_PEAK = 8.0e12                           # B/s (MI355X_MICROARCH.md, spec)
OPS_PER_BASE_WORD = 9.5                     # 8 NFA + 1.5 hit accumulation (~Eq: LDS table)
SAMPLE_BYTES_PER_BASE = 0.375               # 2-bit code + 1-bit N mask, read once

CONFIGS = {  # BASELINE.json configs (sn per rank for the bench)
    "cfg2": dict(k=16, sn=10_000, sl=100, lim=500),
    "cfg3": dict(k=16, sn=100_000, sl=100, lim=2000),
    "cfg4": dict(k=16, sn=1_000_000, sl=100, lim=500),
    "cfg5": dict(k=22, sn=100_000, sl=150, lim=1000),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="cfg2", choices=sorted(CONFIGS))
    ap.add_argument("--k", type=int)
    ap.add_argument("--sn", type=int)
    ap.add_argument("--sl", type=int)
    ap.add_argument("--lim", type=int)
    ap.add_argument("--read-len", type=int, default=400)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="target duration of the bounded CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-boundary", action="store_true",
                    help="skip the PCIe-inclusive host-buffer timing (keeps a rocprof trace to the timed launches)")
    ap.add_argument("--inflight", type=int, default=1,
                    help="batches in flight: independent counter contexts on their own HIP streams, "
                         "steps dealt round-robin, so one batch's launch tail overlaps the next one's start")
    ap.add_argument("--no-inflight-probe", action="store_true",
                    help="skip the informational two-batches-in-flight timing of a 1-GPU run")
    ap.add_argument("--verify", action="store_true", help="check counts against the oracle (slow)")
    ap.add_argument("--event-every", type=int, default=5,
                    help="bracket every N-th timed launch with HIP events (the kernel-duration sample); "
                         "each event is a queue packet of its own, ~3 us between launches when every "
                         "launch is bracketed")
    a = ap.parse_args()
    for key, v in CONFIGS[a.config].items():
        if getattr(a, key) is None:
            setattr(a, key, v)
    a.read_len = max(a.read_len, 2 * a.sl)
    return a


def cpu_baseline(wl, k, seconds):
    """The oracle's OpenMP Myers restatement (the 'port' CPU path) timed on this
    host's cores over the same workload (both ends), repeated to fill ~`seconds`."""
    import oracle

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    units_rep = sum(wl[e]["kmers"].size * sum(int(w.size) for w in wl[e]["windows"]) for e in ("start", "end"))

    def one():
        for e in ("start", "end"):
            oracle.count_myers(k, wl[e]["kmers"], wl[e]["windows"], threads)

    t = time.perf_counter()
    one()
    dt1 = max(time.perf_counter() - t, 1e-6)
    reps = max(1, int(seconds / dt1))
    t = time.perf_counter()
    for _ in range(reps):
        one()
    dt = time.perf_counter() - t
    return {"value": units_rep * reps / dt, "unit": "kmer*bp/s", "cores": threads, "kind": "port",
            "sample": f"the full workload (both ends, {units_rep:.4g} kmer*bp) x {reps} repetitions = {dt:.1f} s; "
                      f"oracle/ac_oracle.c Myers bit-vector, OpenMP over candidates (the reference's SeqAn "
                      f"FM-index path cannot be built here: SURVEY.md 8(c))"}


def load_traffic(workload: str):
    """HBM bytes per launch of the count kernel from committed PMC summaries."""
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json"))):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if d.get("workload") == workload:
            best = d
    return best


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # AC_BENCH_BACKEND=gloo rehearses the N > 1 code path on a box with fewer
    # GPUs than ranks (ranks share devices, the count vector is reduced on the
    # host); the real multi-GPU run uses RCCL ("nccl") over xGMI.
    backend = os.environ.get("AC_BENCH_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count()) if backend != "nccl" else local
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    import approx_counter_amd as ac
    from tools import workload

    wl, _ = workload.build(n_reads=args.sn, read_len=args.read_len, k=args.k, sl=args.sl,
                           lim=args.lim, seed=args.seed, shard=rank, n_shards=world)
    ends = ("start", "end")
    n_c = [int(wl[e]["kmers"].size) for e in ends]
    packed = {e: ac.pack_windows(wl[e]["windows"]) for e in ends}
    base_segs = [ac.DeviceSegment.upload(wl[e]["kmers"], packed[e], device=dev) for e in ends]
    n_slots = max(1, args.inflight)
    # rank 0 of a 1-GPU run also times two batches in flight (informational `inflight_2`)
    extra_slot = world == 1 and n_slots == 1 and not args.no_inflight_probe
    n_build = n_slots + (1 if extra_slot else 0)
    # One slot per batch in flight: its own counter context (device scratch, queue counters),
    # its own stream and two count vectors.  With N > 1 ranks the RCCL all-reduce of a slot's
    # step runs on the communicator's stream while that slot counts its next step into the
    # other vector.
    slots = []
    for si in range(n_build):
        counter_s = ac.ApproxCounter(local)
        st = torch.cuda.current_stream(dev) if si == 0 else torch.cuda.Stream(dev)
        bufs = [torch.zeros(sum(n_c), dtype=torch.int32, device=dev) for _ in range(2)]
        seg_sets = []
        for buf in bufs:
            off, ss = 0, []
            for seg, n in zip(base_segs, n_c):
                s2 = copy.copy(seg)
                s2.counts = buf[off:off + n]
                off += n
                ss.append(s2)
            seg_sets.append(ss)
        slots.append(dict(counter=counter_s, stream=st, bufs=bufs, seg_sets=seg_sets,
                          arrays=[ac.ApproxCounter.segment_array(ss) for ss in seg_sets],
                          pending=[None, None], n=0))
    counter = slots[0]["counter"]
    segs = slots[0]["seg_sets"][0]
    bases = [sum(int(w.size) for w in wl[e]["windows"]) for e in ends]
    units = sum(n * b for n, b in zip(n_c, bases))
    sp = slots[0]["stream"].cuda_stream
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]

    n_step = [0]

    active = [n_slots]

    def step(i=None):
        sl = slots[n_step[0] % active[0]]
        n_step[0] += 1
        b = sl["n"] % 2
        sl["n"] += 1
        buf = sl["bufs"][b]
        st = sl["stream"]
        if sl["pending"][b] is not None:  # the buffer's previous all-reduce must finish first
            with torch.cuda.stream(st):
                sl["pending"][b].wait()
            sl["pending"][b] = None
        if i is not None:
            evs[i][0].record(st)
        # ac_error_count_device: the counts are stored by the launch itself (no memset)
        sl["counter"].count_device(args.k, sl["arrays"][b], stream=st.cuda_stream)
        if i is not None:
            evs[i][1].record(st)
        if world > 1:
            if backend == "nccl":
                with torch.cuda.stream(st):
                    sl["pending"][b] = dist.all_reduce(buf, async_op=True)
            else:
                st.synchronize()
                host = buf.cpu()
                dist.all_reduce(host)
                buf.copy_(host)

    def drain():
        for sl in slots:
            for b in range(2):
                if sl["pending"][b] is not None:
                    sl["pending"][b].wait()
                    sl["pending"][b] = None

    for _ in range(args.warmup):
        step()
    drain()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i if i % max(1, args.event_every) == 0 else None)
    t_enq = time.perf_counter() - t0  # host enqueue time of the K steps (diagnostic)
    drain()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kern_ms = float(np.mean([evs[i][0].elapsed_time(evs[i][1])
                             for i in range(0, args.steps, max(1, args.event_every))]))
    geo = counter.last_launch()

    if args.verify:
        import oracle

        counter.count_device(args.k, segs, stream=sp)
        torch.cuda.synchronize(dev)
        for e, seg in zip(ends, segs):
            exp = oracle.count_myers(args.k, wl[e]["kmers"], wl[e]["windows"])
            assert np.array_equal(seg.counts_numpy(), exp), f"parity failure on {e}"

    if rank == 0:
        P = min(32 // args.k, 4)
        workload_name = (f"{args.config}: k={args.k} sn={args.sn} sl={args.sl} lim={args.lim}, "
                         f"start+end ends fused, {args.sn} reads/rank")
        ops = OPS_PER_BASE_WORD / P * units  # algorithmic lane-ops per launch (one rank)
        achieved = ops / (kern_ms * 1e-3)
        sample_bytes = SAMPLE_BYTES_PER_BASE * sum(bases) + 12 * sum(n_c)  # sample + kmers in + counts out
        tr = load_traffic(workload_name)
        out = {
            "metric": METRIC,
            "value": units * args.steps * world / elapsed,
            "unit": "kmer*bp/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (seeded reads, SURVEY.md 8(d)); inputs resident in HBM",
            "config": {"workload": workload_name, "k": args.k, "sn_per_rank": args.sn, "sl": args.sl,
                       "lim": args.lim, "candidates": n_c, "kmer_bp_per_rank_step": units,
                       "batches_in_flight": n_slots,
                       "parallelism": f"window shards x{world}, {'RCCL' if backend == 'nccl' else backend} "
                                      f"all-reduce of counts" if world > 1 else "1 GPU"},
            "kernel_ms": kern_ms,
            "host_enqueue_ms_per_step": t_enq / args.steps * 1e3,
            "kernel_kmer_bp_per_s": units / (kern_ms * 1e-3),
            "launch": geo,
            "roofline": {"bound": "valu", "achieved": achieved / 1e12, "peak": VALU_PEAK_OPS / 1e12,
                         "unit": "Tops/s", "frac": achieved / VALU_PEAK_OPS,
                         "traffic": tr["hbm_bytes_per_launch"] if tr else None,
                         "note": f"int32 VALU lane-ops, {OPS_PER_BASE_WORD}/P per kmer*bp (P={P}); HIP events "
                                 f"around every {max(1, args.event_every)}th timed launch; traffic from "
                                 f"{os.path.basename(tr['source']) if tr else 'n/a'}"},
            "roofline_hbm": {"bound": "hbm (informational)", "achieved": sample_bytes / (kern_ms * 1e-3) / 1e9,
                             "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                             "frac": sample_bytes / (kern_ms * 1e-3) / HBM_PEAK,
                             "algorithmic_bytes_per_launch": sample_bytes},
        }
        if world == 1 and not args.no_host_boundary:
            # The drop-in entry point hands over host buffers (ac_error_count: H2D of the packed
            # sample and candidates, the kernel, D2H of the counts), one call per read end.  Reported
            # beside `value`, never as it.
            reps = max(5, args.steps // 5)
            for e in ends:
                counter.count(args.k, wl[e]["kmers"], packed[e])
            t_h = time.perf_counter()
            for _ in range(reps):
                for e in ends:
                    counter.count(args.k, wl[e]["kmers"], packed[e])
            host_s = (time.perf_counter() - t_h) / reps
            out["host_boundary"] = {"value": units / host_s, "unit": "kmer*bp/s", "ms_per_step": host_s * 1e3,
                                    "note": "ac_error_count with host buffers (PCIe-inclusive: H2D of the 2-bit "
                                            "sample + candidates, kernel, D2H of counts), both ends, synchronous"}
        if extra_slot:
            # Two batches in flight: the same steps dealt alternately to two counter contexts on
            # two streams, so one launch's tail overlaps the next one's start.
            # Reported beside `value` (which keeps one batch in flight and per-launch kernel
            # times), never as it.
            active[0] = 2
            for _ in range(args.warmup):
                step()
            torch.cuda.synchronize(dev)
            t2 = time.perf_counter()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize(dev)
            el2 = time.perf_counter() - t2
            active[0] = n_slots
            out["inflight_2"] = {"value": units * args.steps / el2, "unit": "kmer*bp/s",
                                 "ms_per_step": el2 / args.steps * 1e3,
                                 "note": "2 batches in flight (2 contexts, 2 streams), same steps and workload"}
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(wl, args.k, args.cpu_seconds)
        print(json.dumps(out), flush=True)
    for sl in slots:
        sl["counter"].close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
