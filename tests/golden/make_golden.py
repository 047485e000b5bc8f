"""Regenerate the committed golden fixtures (run from the repo root):

    python tests/golden/make_golden.py

1. tests/golden/vectors.json -- small (k, kmers, windows) cases with expected
   counts.  Each expected vector is computed three ways by the CPU oracle:
   the SeqAn 2.4 find<0,2> scheme simulator (approx_counter.cpp:586 restated),
   plain DP and Myers (model M1); the script refuses to write unless all agree
   (k >= 4; for k in {2, 3} the scheme has zero-length blocks and M1 is the
   contract).
2. tests/golden/cfg1/ -- BASELINE config 1 (k=16, sn=1000, sl=100, lim=100):
   a seeded 1000-read FASTA and the files the reference CLI would write
   (``-e exact -o out.txt``): exact_0.start/.end and out.txt_0.start/.end,
   produced by oracle.host_ref (host stages restated in Python) + the oracle
   approximate counts, cross-checked against the scheme simulator.

The reference itself cannot be built here (SeqAn absent), so these fixtures
pin the product to the oracle, not to a reference run: parity unpinned.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from oracle import host_ref  # noqa: E402
from tests import cases  # noqa: E402
from tools.synth import make_reads, write_fasta  # noqa: E402

HERE = os.path.join(ROOT, "tests", "golden")


def vectors():
    out = []
    specs = [(s, k, nk, nw) for s, (k, nk, nw) in enumerate(
        [(4, 6, 12), (5, 5, 10), (8, 8, 15), (10, 7, 12), (12, 10, 20), (13, 9, 15), (16, 12, 25),
         (16, 70, 18), (17, 8, 20), (20, 6, 15), (22, 10, 20), (25, 5, 12), (31, 6, 10), (32, 8, 16)],
        start=100)]
    for seed, k, nk, nw in specs:
        kmers, wins = cases.planted_case(seed, k, nk, nw, win_len=(max(1, k - 4), k + 40))
        out.append(("planted_s%d_k%d" % (seed, k), k, kmers, wins))
    out += cases.edge_cases()
    result = []
    for name, k, kmers, wins in out:
        dp = oracle.count_dp(k, kmers, wins)
        my = oracle.count_myers(k, kmers, wins, 1)
        assert np.array_equal(dp, my), name
        source = "dp==myers"
        if k >= 4:
            sc = oracle.count_scheme(k, kmers, wins)
            assert np.array_equal(dp, sc), (name, dp, sc)
            source = "scheme==dp==myers"
        result.append({"name": name, "k": k, "kmers": [int(x) for x in kmers], "windows": wins,
                       "counts": [int(x) for x in dp], "source": source})
    with open(os.path.join(HERE, "vectors.json"), "w") as fh:
        json.dump(result, fh, indent=0)
    print("vectors.json:", len(result), "cases")


CFG1 = dict(n_reads=1000, read_len=210, seed=1, k=16, sl=100, lim=100, lc=1.0)


def cfg1():
    d = os.path.join(HERE, "cfg1")
    os.makedirs(d, exist_ok=True)
    reads, _ = make_reads(CFG1["n_reads"], read_len=CFG1["read_len"], seed=CFG1["seed"])
    fasta = os.path.join(d, "reads.fa")
    write_fasta(fasta, reads, width=80)
    _, seqs = host_ref.read_fasta(fasta)
    k, sl, lim = CFG1["k"], CFG1["sl"], CFG1["lim"]
    for end, bottom in (("start", False), ("end", True)):
        exact, approx, windows = host_ref.run_end(seqs, k, sl, lim, CFG1["lc"], bottom)
        kmers = [km for km, _ in exact]
        sc = oracle.count_scheme(k, kmers, windows)
        my = oracle.count_myers(k, kmers, windows)
        assert np.array_equal(sc, my), end
        with open(os.path.join(d, "exact_0." + end), "w") as fh:
            fh.write(host_ref.export_lines(exact, k))
        with open(os.path.join(d, "out.txt_0." + end), "w") as fh:
            fh.write(host_ref.export_lines(approx, k))
        print(end, "top:", host_ref.export_lines(approx[:3], k).replace("\n", " | "))
    with open(os.path.join(d, "params.json"), "w") as fh:
        json.dump(CFG1, fh)


if __name__ == "__main__":
    vectors()
    cfg1()
