#!/usr/bin/env python3
"""HBM traffic per launch of the count kernel from two rocprofv3 PMC passes.

    python tools/pmc_traffic.py --fetch DIR --write DIR --workload "<bench workload string>" \
        --out profiles/rNN_<cfg>_pmc_traffic.json

FETCH_SIZE and WRITE_SIZE (KB per dispatch) come from separate `--pmc` passes
(they do not fit one TCC pass on gfx950).  Per MI355X_MICROARCH.md §HBM,
FETCH_SIZE reads half the bytes of a wide streaming read on gfx950, so it is
doubled; WRITE_SIZE is taken as is (it counts the kernel's atomic requests).
bench.py picks the file whose `workload` equals its own config string.
"""
import argparse
import json
import os
import sqlite3
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import find_dbs  # noqa: E402

KERNEL = "wm2_count_kernel"


def mean_counter(path, counter):
    vals = {}
    for db in find_dbs(path):
        con = sqlite3.connect(db)
        for kname, cname, did, v in con.execute(
                "select kernel_name, counter_name, dispatch_id, value from counters_collection"):
            if KERNEL in kname and cname == counter:
                vals[(db, did)] = vals.get((db, did), 0.0) + float(v)
        con.close()
    if not vals:
        raise SystemExit(f"no {counter} samples for {KERNEL} under {path}")
    return statistics.mean(vals.values()), len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--workload", required=True)
    ap.add_argument("--valu", help="directory of a SQ_INSTS_VALU pass (optional)")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    fetch, nf = mean_counter(a.fetch, "FETCH_SIZE")
    write, nw = mean_counter(a.write, "WRITE_SIZE")
    d = {"workload": a.workload, "kernel": KERNEL, "fetch_size_kb": fetch, "write_size_kb": write,
         "dispatches": [nf, nw], "hbm_bytes_per_launch": (2.0 * fetch + write) * 1024.0,
         "correction": "2 x FETCH_SIZE (gfx950 half-count, MI355X_MICROARCH.md HBM) + WRITE_SIZE, KB -> B",
         "source": os.path.basename(a.out)}
    if a.valu:  # wave-level VALU instructions per launch (bench.py compares them with the 9.5/P model)
        valu, nv = mean_counter(a.valu, "SQ_INSTS_VALU")
        d["sq_insts_valu_per_launch"] = valu
        d["dispatches"].append(nv)
    with open(a.out, "w") as fh:
        json.dump(d, fh, indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
