#!/usr/bin/env python3
"""Summarise rocprofv3 output (the .db written by ``--kernel-trace [--pmc ...]``).

    python tools/prof_summary.py gpurun_out/<tag>/prof [--out profiles/<name>.md]

Writes a markdown table per kernel: calls, total / average / min / max duration
(µs) and share of GPU time; and, when PMC counters were collected, the mean
value of every counter per dispatch of each kernel.  Used to turn the scratch
output under gpurun_out/ into the summaries committed under profiles/.
"""
from __future__ import annotations

import argparse
import glob
import os
import sqlite3
import statistics
from collections import defaultdict


def find_dbs(path):
    if os.path.isfile(path):
        return [path]
    return sorted(glob.glob(os.path.join(path, "**", "*.db"), recursive=True))


def short(name: str, n: int = 70) -> str:
    return name if len(name) <= n else name[: n - 3] + "..."


def kernel_rows(con, skip=0):
    """Durations per kernel name in dispatch order, the first `skip` of each left out (a cold
    GPU runs its first ~10 ms of dense load below the sustained clock)."""
    dur = defaultdict(list)
    for name, d in con.execute("select name, duration from kernels order by start"):
        dur[name].append(d)
    return {k: v[skip:] for k, v in dur.items() if len(v) > skip}


def pmc_rows(con):
    vals = defaultdict(lambda: defaultdict(list))
    try:
        cur = con.execute("select kernel_name, counter_name, dispatch_id, value from counters_collection")
    except sqlite3.Error:
        return vals
    per = defaultdict(float)
    names = {}
    for kname, cname, did, v in cur:
        per[(kname, cname, did)] += float(v)
        names[(kname, cname, did)] = (kname, cname)
    for key, v in per.items():
        kname, cname = names[key]
        vals[kname][cname].append(v)
    return vals


def summarise(dbs, skip=0):
    dur = defaultdict(list)
    pmc = defaultdict(lambda: defaultdict(list))
    for db in dbs:
        con = sqlite3.connect(db)
        for k, v in kernel_rows(con, skip).items():
            dur[k] += v
        for k, cs in pmc_rows(con).items():
            for c, v in cs.items():
                pmc[k][c] += v
        con.close()
    lines = []
    total = sum(sum(v) for v in dur.values()) or 1
    if dur:
        lines.append("| kernel | calls | total µs | avg µs | min µs | max µs | % |")
        lines.append("|---|---|---|---|---|---|---|")
        for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
            lines.append(f"| `{short(k)}` | {len(v)} | {sum(v) / 1e3:.1f} | {statistics.mean(v) / 1e3:.2f} | "
                         f"{min(v) / 1e3:.2f} | {max(v) / 1e3:.2f} | {100 * sum(v) / total:.1f} |")
    if pmc:
        lines.append("")
        lines.append("| kernel | counter | dispatches | mean per dispatch |")
        lines.append("|---|---|---|---|")
        for k, cs in pmc.items():
            for c, v in sorted(cs.items()):
                lines.append(f"| `{short(k, 50)}` | {c} | {len(v)} | {statistics.mean(v):.6g} |")
    return "\n".join(lines) + "\n"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--out")
    ap.add_argument("--title", default="")
    ap.add_argument("--skip", type=int, default=0, help="leave out each kernel's first N dispatches (warm-up)")
    a = ap.parse_args()
    dbs = find_dbs(a.path)
    if not dbs:
        raise SystemExit(f"no rocprofv3 .db under {a.path}")
    text = summarise(dbs, a.skip)
    if a.skip:
        text = f"(each kernel's first {a.skip} dispatches left out: warm-up)\n\n" + text
    if a.title:
        text = f"## {a.title}\n\n" + text
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
