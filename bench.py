#!/usr/bin/env python3
"""Benchmark of the approximate-count stage (errorCount, approx_counter.cpp:531-601).

    python bench.py [--gpus N] [--steps K] [--warmup W]

A step is one pass of the hot path over one batch: both read ends of one run
(start + end windows, approx_counter.cpp:858) counted against their own
top-`lim` candidates in ONE fused kernel launch, inputs already resident in
HBM.  Workload = BASELINE config 2 (k=16, sn=10,000, sl=100, lim=500) on
seeded synthetic reads.  With N > 1 ranks (one process per
GPU, torchrun) every rank counts its own 10,000 reads against the same
candidates and the per-candidate count vector is summed with one RCCL
all-reduce per step (weak scaling).  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "approx-count kmer×base pairs/sec (k=16, lim=500, 10k×100bp ends)"
# int32 VALU peak: 256 CU x 4 SIMD x 32 lanes/clk x 2.4 GHz (MI355X_MICROARCH.md:28-34,54)
VALU_PEAK_OPS = 256 * 4 * 32 * 2.4e9
# VALU lane-ops per text base per lane word (kernel section): 2 (Eq) + 10
# (three NFA rows) + 1.5 (hit accumulators, v_or3 over two bases).
OPS_PER_BASE_WORD = 13.5


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--sn", type=int, default=10_000)
    ap.add_argument("--sl", type=int, default=100)
    ap.add_argument("--lim", type=int, default=500)
    ap.add_argument("--read-len", type=int, default=400)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="target duration of the bounded CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verify", action="store_true", help="check counts against the oracle (slow)")
    return ap.parse_args()


def cpu_baseline(wl, k, seconds):
    """Oracle Myers (OpenMP C, the restated CPU path) on a bounded sample of the same
    workload: all start candidates against the first W start windows."""
    import oracle

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    kmers = wl["start"]["kmers"]
    wins = wl["start"]["windows"]
    probe = wins[:200]
    t = time.perf_counter()
    oracle.count_myers(k, kmers, probe, threads)
    dt = max(time.perf_counter() - t, 1e-6)
    n_win = int(min(len(wins), max(200, 200 * seconds / dt)))
    sample = wins[:n_win]
    units = len(kmers) * sum(int(w.size) for w in sample)
    t = time.perf_counter()
    oracle.count_myers(k, kmers, sample, threads)
    dt = time.perf_counter() - t
    return {"value": units / dt, "unit": "kmer*bp/s", "cores": threads, "kind": "port",
            "sample": f"{len(kmers)} start candidates x {n_win} start windows ({units:.3g} kmer*bp), "
                      f"oracle Myers 64-bit OpenMP, {dt:.2f} s"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    import approx_counter_amd as ac
    from tools import workload

    wl, _ = workload.build(n_reads=args.sn, read_len=args.read_len, k=args.k, sl=args.sl,
                           lim=args.lim, seed=args.seed, shard=rank, n_shards=world)
    counter = ac.ApproxCounter(local)
    ends = ("start", "end")
    n_c = [int(wl[e]["kmers"].size) for e in ends]
    counts = torch.zeros(sum(n_c), dtype=torch.int32, device=dev)
    segs = []
    off = 0
    for e, n in zip(ends, n_c):
        seg = ac.DeviceSegment.upload(wl[e]["kmers"], ac.pack_windows(wl[e]["windows"]), device=dev)
        seg.counts = counts[off:off + n]
        off += n
        segs.append(seg)
    units = sum(n * sum(int(w.size) for w in wl[e]["windows"]) for e, n in zip(ends, n_c))
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream

    def step():
        counter.count_device(args.k, segs, stream=sp)
        if world > 1:
            dist.all_reduce(counts)

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # Kernel-only duration with HIP events on the launch stream (counts zeroed outside).
    n_ev = max(10, min(args.steps, 200))
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n_ev)]
    for a, b in evs:
        counts.zero_()
        a.record(stream)
        counter.count_device(args.k, segs, stream=sp, accumulate=True)
        b.record(stream)
    torch.cuda.synchronize(dev)
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    geo = counter.last_launch()

    if args.verify:
        import oracle

        counts.zero_()
        counter.count_device(args.k, segs, stream=sp)
        torch.cuda.synchronize(dev)
        for e, seg in zip(ends, segs):
            exp = oracle.count_myers(args.k, wl[e]["kmers"], wl[e]["windows"])
            assert np.array_equal(seg.counts_numpy(), exp), f"parity failure on {e}"

    if rank == 0:
        P = min(32 // args.k, 4)
        base_words = sum(((n + 64 * P - 1) // (64 * P)) * 64 * sum(int(w.size) for w in wl[e]["windows"])
                         for e, n in zip(ends, n_c))
        ops = OPS_PER_BASE_WORD * base_words  # lane-ops per launch (all lane words, incl. padding)
        achieved = ops / (kern_ms * 1e-3) / 1e9
        peak = VALU_PEAK_OPS / 1e9
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
            "config": {"workload": f"cfg2: k={args.k} sn={args.sn} sl={args.sl} lim={args.lim}, "
                                   f"start+end ends fused, {args.sn} reads/rank",
                       "k": args.k, "sn_per_rank": args.sn, "sl": args.sl, "lim": args.lim,
                       "candidates": n_c, "kmer_bp_per_rank_step": units,
                       "parallelism": f"window shards x{world}, all-reduce of counts"},
            "kernel_ms": kern_ms,
            "kernel_kmer_bp_per_s": units / (kern_ms * 1e-3),
            "launch": geo,
            "roofline": {"bound": "valu", "achieved": achieved, "peak": peak, "unit": "Gop/s",
                         "frac": achieved / peak, "traffic": None,
                         "note": f"int32 VALU lane-ops: {OPS_PER_BASE_WORD} per base per lane word "
                                 f"({P} candidates per lane word)"},
        }
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(wl, args.k, args.cpu_seconds)
        print(json.dumps(out), flush=True)
    counter.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
