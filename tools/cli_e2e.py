"""End-to-end timing of the drop-in CLI (bin/adaptFinder) on a synthetic FASTA:
the default pipeline (fused reader, GPU exact count + selection, GPU approximate
count on one upload) against --host-exact (whole reads, host exact count, GPU
approximate count).  Both must write identical files.

    python tools/cli_e2e.py [--reads 10000] [--lim 500] [--read-len 400]

Prints one JSON line with the wall times and the stage timestamps of the
default run (the CLI's own "[ms]" log lines), plus the same parse + sampling
with --dump-sample (no GPU stage) and a 100-read run (the fixed cost)."""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tools.synth import make_reads, write_fasta  # noqa: E402

CLI = os.path.join(ROOT, "approx_counter_amd", "bin", "adaptFinder")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=10_000)
    ap.add_argument("--read-len", type=int, default=400)
    ap.add_argument("--lim", type=int, default=500)
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--sl", type=int, default=100)
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as d:
        reads, _ = make_reads(a.reads, read_len=a.read_len, seed=1)
        fa = os.path.join(d, "reads.fa")
        write_fasta(fa, reads, width=80)
        base = [CLI, fa, "-k", str(a.k), "-sn", str(a.reads), "-sl", str(a.sl), "-lim", str(a.lim), "--seed", "1"]
        out = {"config": {"reads": a.reads, "read_len": a.read_len, "k": a.k, "sl": a.sl, "lim": a.lim,
                          "fasta_MB": round(os.path.getsize(fa) / 1e6, 1)}, "data": "synthetic"}
        for tag, extra in (("default", []), ("host_exact", ["--host-exact"])):
            cmd = base + ["-o", os.path.join(d, tag), "-e", os.path.join(d, tag + "_exact")] + extra
            t = time.perf_counter()
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
            dt = time.perf_counter() - t
            if r.returncode != 0:
                raise SystemExit(f"{tag} failed ({r.returncode}): {r.stderr[-2000:]}")
            out[tag + "_s"] = round(dt, 4)
            if tag == "default":
                out["default_log"] = [ln.strip() for ln in r.stdout.splitlines() if ln.startswith("[")]
        # the same parse + sampling without any GPU stage (--dump-sample), and the
        # whole pipeline on 100 reads: the fixed cost (process, HIP runtime, device)
        t = time.perf_counter()
        r = subprocess.run(base + ["--dump-sample", os.path.join(d, "dump")], capture_output=True, text=True,
                           timeout=600)
        out["dump_sample_s"] = round(time.perf_counter() - t, 4)
        if r.returncode != 0:
            raise SystemExit(f"--dump-sample failed ({r.returncode}): {r.stderr[-2000:]}")
        tiny = os.path.join(d, "tiny.fa")
        write_fasta(tiny, reads[:100], width=80)
        t = time.perf_counter()
        r = subprocess.run([CLI, tiny, "-k", str(a.k), "-sl", str(a.sl), "-lim", str(a.lim), "--seed", "1", "-o",
                            os.path.join(d, "tiny")], capture_output=True, text=True, timeout=600)
        out["tiny_100_reads_s"] = round(time.perf_counter() - t, 4)
        if r.returncode != 0:
            raise SystemExit(f"tiny run failed ({r.returncode}): {r.stderr[-2000:]}")
        same = all(open(os.path.join(d, f"default{s}_0.{e}")).read() == open(os.path.join(d, f"host_exact{s}_0.{e}")).read()
                   for s in ("", "_exact") for e in ("start", "end"))
        out["identical_outputs"] = same
        print(json.dumps(out))
        if not same:
            raise SystemExit("outputs differ")


if __name__ == "__main__":
    main()
