#!/usr/bin/env python3
"""Mean of every collected PMC counter per kernel, from rocprofv3 `--pmc` output dirs.

    python tools/pmc_kernels.py DIR [DIR ...] [--match SUBSTR]
"""
import argparse
import collections
import os
import re
import sqlite3
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import find_dbs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    per = collections.defaultdict(dict)  # (kernel, counter) -> {(db, dispatch): value}
    for d in a.dirs:
        for db in find_dbs(d):
            con = sqlite3.connect(db)
            for kname, cname, did, v in con.execute(
                    "select kernel_name, counter_name, dispatch_id, value from counters_collection"):
                if a.match in kname:
                    m = re.search(r"::(\w+)(?:<[^(]*>)?\(", kname) or re.search(r"(\w+)\(", kname)
                    key = (m.group(1) if m else kname, cname)
                    per[key][(db, did)] = per[key].get((db, did), 0.0) + float(v)
            con.close()
    for (k, c) in sorted(per):
        vals = list(per[(k, c)].values())
        print(f"{k:32s} {c:24s} {statistics.mean(vals):14.4g}  (n={len(vals)})")


if __name__ == "__main__":
    main()
