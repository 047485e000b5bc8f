#!/usr/bin/env python3
"""HBM traffic per exact-count call (row f1) from two rocprofv3 PMC passes over
tools/bench_exact.py, for bench.py's `exact` block.

    python tools/exact_pmc.py --config cfg4 --fetch DIR --write DIR --calls N --out profiles/rNN_cfg4_exact_pmc.json

Every kernel of the partitioned path (part_*) and the selection (exact_*) is summed per call:
FETCH_SIZE doubled (MI355X_MICROARCH.md §HBM: gfx950 counts half the bytes of a wide streaming
read), WRITE_SIZE as is, KB -> B; divided by the calls the run made (part_keys_kernel dispatches).
The file maps the config name to its figures, so several configs can be merged by bench.py."""
import argparse
import json
import os
import re
import sqlite3
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import find_dbs  # noqa: E402

MATCH = ("part_", "exact_")


def totals(path, counter):
    """(sum of `counter` over the exact-count kernels, calls = part_keys_kernel dispatches, per-kernel sums)."""
    per, calls = {}, set()
    for db in find_dbs(path):
        con = sqlite3.connect(db)
        for kname, cname, did, v in con.execute(
                "select kernel_name, counter_name, dispatch_id, value from counters_collection"):
            if cname != counter or not any(m in kname for m in MATCH):
                continue
            m = re.search(r"::(\w+)(?:<[^(]*>)?\(", kname)
            short = m.group(1) if m else kname
            per[short] = per.get(short, 0.0) + float(v)
            if "part_keys_kernel" in kname:
                calls.add((db, did))
        con.close()
    if not per:
        raise SystemExit(f"no {counter} samples of the exact-count kernels under {path}")
    return sum(per.values()), len(calls), per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    f, nf, fper = totals(a.fetch, "FETCH_SIZE")
    w, nw, wper = totals(a.write, "WRITE_SIZE")
    fetch_b, write_b = 2.0 * f * 1024.0 / nf, w * 1024.0 / nw
    d = {a.config: {
        "fetch_bytes_per_call": fetch_b, "write_bytes_per_call": write_b, "traffic_bytes_per_call": fetch_b + write_b,
        "calls": [nf, nw],
        "per_kernel_MB_per_call": {k: {"fetch": 2.0 * fper[k] * 1024.0 / nf / 1e6, "write": wper.get(k, 0.0) * 1024.0 / nw / 1e6}
                                   for k in sorted(fper)},
        "correction": "2 x FETCH_SIZE (gfx950 half-count, MI355X_MICROARCH.md HBM) + WRITE_SIZE, KB -> B",
        "source": os.path.basename(a.out)}}
    with open(a.out, "w") as fh:
        json.dump(d, fh, indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
