#!/usr/bin/env python3
"""One exact-count call's timeline from a rocprofv3 --hip-trace --kernel-trace --memory-copy-trace
output dir: HIP API calls (host), kernels and copies (device) between the fill that starts the call
and the next call's fill, in start order, with durations and gaps -- where a call's non-kernel time
goes.  Prints text (the .db files are large: the caller deletes them after).

    python tools/host_gaps.py DIR [--call -2]
"""
import argparse
import os
import re
import sqlite3
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import find_dbs  # noqa: E402


def short(n):
    m = re.search(r"::(\w+)(?:<[^(]*>)?\(", n) or re.search(r"(\w+)", n)
    return m.group(1) if m else n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--call", type=int, default=-2, help="which call (by its keys kernel), -2 = the next to last")
    a = ap.parse_args()
    ev = []
    for db in find_dbs(a.dir):
        con = sqlite3.connect(db)
        names = {r[0] for r in con.execute("select name from sqlite_master where type in ('table','view')")}
        for n, s, e in con.execute("select name, start, end from kernels"):
            ev.append((s, e, "K", short(n)))
        if "memory_copies" in names:
            cols = [r[1] for r in con.execute("pragma table_info(memory_copies)")]
            sz = "size" if "size" in cols else None
            q = f"select name, start, end{', ' + sz if sz else ''} from memory_copies"
            for r in con.execute(q):
                ev.append((r[1], r[2], "C", f"{r[0]} {r[3] if sz else ''}"))
        for t in ("regions", "region"):
            if t in names:
                for n, s, e in con.execute(f"select name, start, end from {t}"):
                    if n.startswith("hip") or n.startswith("__hip"):
                        ev.append((s, e, "A", n))
                break
        con.close()
    ev.sort()
    keys = [i for i, x in enumerate(ev) if x[2] == "K" and "part_keys" in x[3]]
    if len(keys) < 2:
        sys.exit("fewer than two calls in the trace")
    i0 = keys[a.call]
    # the call's first event: the last fill / memset API before its keys kernel
    j = i0
    while j > 0 and not (ev[j][2] in ("K", "A") and ("fill" in ev[j][3].lower() or "Memset" in ev[j][3])):
        j -= 1
    nxt = keys[a.call + 1] if a.call + 1 < 0 or a.call + 1 < len(keys) else len(ev)
    t0 = ev[j][0]
    for s, e, kind, n in ev[j:nxt]:
        print(f"{kind} {(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {n[:90]}")


if __name__ == "__main__":
    main()
