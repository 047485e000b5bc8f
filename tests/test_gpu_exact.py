"""GPU exact count + selection (ac_exact_count) against the
host restatement: count_kmers (approx_counter.cpp:487-519) with the N, float
low-complexity and forbidden filters, then get_most_frequent / get_solid_kmers
in CompareCount order.  Bit-exact lists, distinct counts and N-skip counts."""
import json
import os
import random

import numpy as np
import pytest

import approx_counter_amd as ac
from oracle import host_ref
from tests import cases

pytestmark = pytest.mark.gpu
CFG1 = os.path.join(os.path.dirname(__file__), "golden", "cfg1")


def expected(windows, k, thr, forbidden=frozenset(), limit=500, solid=0):
    counter, had_n = host_ref.count_kmers(windows, k, thr, forbidden)
    ranked = host_ref.get_solid_kmers(counter, solid, k) if solid else host_ref.get_most_frequent(counter, limit, k)
    return ranked, len(counter), had_n


def check(counter, windows, k, thr, forbidden=frozenset(), limit=500, solid=0):
    got, n_dist, had_n = counter.exact_count(k, ac.pack_windows(windows), thr, forbidden, limit, solid)
    exp, exp_dist, exp_n = expected(windows, k, thr, forbidden, limit, solid)
    assert got == exp
    assert (n_dist, had_n) == (exp_dist, exp_n)


def test_cfg1_exact_files(counter):
    p = json.load(open(os.path.join(CFG1, "params.json")))
    _, seqs = host_ref.read_fasta(os.path.join(CFG1, "reads.fa"))
    for end, bottom in (("start", False), ("end", True)):
        wins = host_ref.sample_all(seqs, p["sl"], bottom)
        got, _, _ = counter.exact_count(p["k"], ac.pack_windows(wins), float(host_ref.adjust_threshold(p["lc"], 16, p["k"])),
                                        (), p["lim"])
        assert host_ref.export_lines(got, p["k"]) == open(os.path.join(CFG1, "exact_0." + end)).read()


@pytest.mark.parametrize("k", [2, 3, 5, 8, 11, 16, 17, 22, 31, 32])
def test_random_windows_every_regime(counter, k):
    rng = random.Random(k)
    wins = [cases.rand_seq(rng, rng.randint(0, 300), p_n=0.01) for _ in range(300)]
    wins += ["A" * 60, "ACACACACACACACACACACACACACAC", "T" * 40]  # low-complexity and all-T runs
    thr = float(host_ref.adjust_threshold(1.0, 16, k))
    check(counter, wins, k, thr, limit=200)
    check(counter, wins, k, float(host_ref.adjust_threshold(1.5, 16, k)), limit=10**6)  # everything kept, ranked


def test_forbidden_solid_and_limits(counter):
    from tools.synth import make_reads

    reads, _ = make_reads(2000, read_len=220, seed=5)
    wins = host_ref.sample_all([r.decode() for r in reads], 100, False)
    top, _, _ = expected(wins, 16, 1.0, limit=20)
    forbidden = {top[0][0], top[5][0], 12345}
    check(counter, wins, 16, 1.0, forbidden, limit=100)
    check(counter, wins, 16, 1.0, limit=1)
    check(counter, wins, 16, 1.0, limit=0)
    check(counter, wins, 16, 1.0, solid=30)
    check(counter, wins, 16, 1.0, solid=10**6)  # nothing that solid


@pytest.mark.parametrize("k", [16, 22])
def test_overlapping_windows_more_positions_than_bases(counter, k):
    """ac_windows allows overlapping windows: here every window starts at image base 0,
    so the sample holds 6x more k-mer positions than the image has bases.  The
    partitioned path's dense key arrays are sized by the image, so it must detect the
    excess and recount on the hash table, not return short counts."""
    rng = random.Random(77 + k)
    w = cases.rand_seq(rng, 100, p_n=0.0)
    img = ac.pack_windows([w])
    dup = ac.PackedSample(img.codes, img.nmask, np.zeros(6, np.uint64), np.full(6, 100, np.uint32), img.n_bases)
    thr = float(host_ref.adjust_threshold(1.5, 16, k))
    got, n_dist, had_n = counter.exact_count(k, dup, thr, (), 10**6)
    exp, exp_dist, exp_n = expected([w] * 6, k, thr, limit=10**6)
    assert got == exp and (n_dist, had_n) == (exp_dist, exp_n)
    assert all(c >= 6 for _, c in got)


def test_edge_windows(counter):
    check(counter, [], 16, 1.0)
    check(counter, ["", "ACG", "N" * 40], 16, 1.0)
    check(counter, ["T" * 80, "T" * 32 + "A", "NTTTT" + "T" * 40], 32, 1.0, limit=50)  # all-T 32-mer (table sentinel)
    # all-T 16-mer: the compact layout's sentinel (its stored key wraps to 0); the
    # threshold keeps the low-complexity run so the sentinel reaches the output
    check(counter, ["T" * 40, "T" * 16 + "A", "ACGT" * 10 + "T" * 20], 16, 100.0, limit=50)
    check(counter, ["T" * 40, "GT" * 30], 15, 100.0, limit=50)  # all-T 15-mer: an ordinary compact key
    check(counter, ["ACGT" * 300], 16, 1.0)  # a window longer than the LDS staging


def test_cfg3_scale(counter):
    """100k windows of 100 bp (BASELINE config 3 sample size), lim=2000."""
    from tools import workload

    w = workload.windows_from_reads(__import__("tools.synth", fromlist=["make_reads"]).make_reads(
        100_000, read_len=400, seed=9)[0], 100, False)
    got, n_dist, _ = counter.exact_count(16, ac.pack_windows(w), 1.0, (), 2000)
    exp = workload.exact_topk(w, 16, 2000, 1.0)
    assert got == exp
    assert n_dist > 1_000_000
