"""CPU tests of the oracle (the checker): its three restatements agree, it reproduces
the committed golden fixtures, and hand-computable known answers hold."""
import json
import os

import numpy as np
import pytest

import oracle
from oracle import host_ref
from tests import cases

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("seed", range(6))
def test_three_restatements_agree(seed):
    for k in (4, 7, 9, 11, 16, 19, 22, 28, 32):
        kmers, wins = cases.planted_case(1000 * seed + k, k, 5, 8, win_len=(max(1, k - 3), k + 30))
        dp = oracle.count_dp(k, kmers, wins)
        assert np.array_equal(dp, oracle.count_myers(k, kmers, wins, 2))
        assert np.array_equal(dp, oracle.count_scheme(k, kmers, wins)), (k, seed)


def test_scheme_levels_are_d_to_2():
    """SeqAn's per-read error levels (tcount[e], approx_counter.cpp:563) are {d..2}."""
    for k in (4, 6, 16, 21):
        kmers, wins = cases.planted_case(77 + k, k, 4, 10, win_len=(k - 2, k + 20))
        _, levels = oracle.count_scheme(k, kmers, wins, return_levels=True)
        for i, km in enumerate(kmers):
            for j, w in enumerate(wins):
                d = oracle.distance(km, k, w)
                assert levels[i, j] == sum(1 << e for e in range(d, 3)), (k, i, j, d)


def test_strict_variant_is_a_real_alternative():
    """The SeqAn3-style end-indel pruning changes results (residual risk)."""
    diff = 0
    for s in range(20):
        kmers, wins = cases.planted_case(s, 12, 4, 6, win_len=(10, 40))
        diff += int(not np.array_equal(oracle.count_scheme(12, kmers, wins),
                                       oracle.count_scheme(12, kmers, wins, strict=True)))
    assert diff > 0


def test_strict_levels_depend_on_context():
    """Why `strict` is not a flag flip on the GPU's <= d NFA rows: an exact
    occurrence reports {0, 1, 2} under M1 wherever it sits, but under strict {0, 2} when it
    starts the window (no leading base for scheme 2's e = 1) and {0, 1, 2} otherwise."""
    p = "ACGTTGCAAGTCCGTA"
    km = np.array([cases.kmer_value(p)], dtype=np.uint64)
    for w, m1, strict in (("GG" + p + "TT", 7, 7), (p + "TT", 7, 5), ("GG" + p, 7, 7), (p, 7, 5)):
        assert oracle.count_scheme(16, km, [w], return_levels=True)[1][0][0] == m1
        assert oracle.count_scheme(16, km, [w], strict=True, return_levels=True)[1][0][0] == strict


def test_known_answers():
    km = "ACGTACGTTGCAAGCT"
    v = cases.kmer_value(km)
    assert oracle.distance(v, 16, km) == 0
    assert oracle.distance(v, 16, "GG" + km + "GG") == 0
    assert oracle.distance(v, 16, km[:7] + "A" + km[8:]) == 1        # substitution
    assert oracle.distance(v, 16, km[:7] + "N" + km[8:]) == 1        # N never matches
    assert oracle.distance(v, 16, km[:15]) == 1                      # truncated at the window end
    assert oracle.distance(v, 16, km[1:]) == 1                       # truncated at the window start
    assert oracle.distance(v, 16, km[:5] + "T" + km[5:]) == 1        # insertion in the text
    assert oracle.distance(v, 16, km[:3] + km[4:12] + km[13:]) == 2  # two deletions
    assert oracle.distance(v, 16, "") == 3                            # capped
    assert list(oracle.count_dp(16, [v], [km, km[:15], "T" * 30, ""])) == [3 + 2 + 0 + 0]


def test_golden_vectors_reproduce():
    with open(os.path.join(GOLDEN, "vectors.json")) as fh:
        vecs = json.load(fh)
    assert len(vecs) >= 20
    for vec in vecs:
        got = oracle.count_myers(vec["k"], vec["kmers"], vec["windows"], 1)
        assert [int(x) for x in got] == vec["counts"], vec["name"]


def test_host_ref_known_answers():
    # poly-A: 15 dimers AA -> 15*14 = 210, s = 210/28 = 7.5 >= 1.0
    assert host_ref.get_complexity(0, 16) == np.float32(7.5)
    assert host_ref.have_low_complexity(0, 16, 1.0)
    assert host_ref.adjust_threshold(1.0, 16, 16) == np.float32(1.0)
    assert host_ref.adjust_threshold(1.0, 16, 22) == np.float32(441.0 / 225.0)
    # CompareCount: count desc, then complexity asc, then value desc
    k = 4
    a, b = cases.kmer_value("ACGT"), cases.kmer_value("AAAA")
    ranked = host_ref.get_most_frequent({a: 5, b: 5, 7: 9}, 10, k)
    assert ranked[0] == (7, 9) and ranked[1][0] == a
    x, y = cases.kmer_value("ACGT"), cases.kmer_value("TGCA")
    assert host_ref.get_complexity(x, 4) == host_ref.get_complexity(y, 4)
    assert [km for km, _ in host_ref.get_most_frequent({x: 1, y: 1}, 2, 4)] == [max(x, y), min(x, y)]
    # end windows are sl+1 bases (approx_counter.cpp:463)
    assert [len(w) for w in host_ref.sample_all(["A" * 250], 100, True)] == [101]
    assert [len(w) for w in host_ref.sample_all(["A" * 199, "C" * 200], 100, False)] == [100]


def test_cfg1_fixture_reproduces():
    d = os.path.join(GOLDEN, "cfg1")
    params = json.load(open(os.path.join(d, "params.json")))
    _, seqs = host_ref.read_fasta(os.path.join(d, "reads.fa"))
    assert len(seqs) == params["n_reads"]
    k = params["k"]
    for end, bottom in (("start", False), ("end", True)):
        exact, approx, _ = host_ref.run_end(seqs, k, params["sl"], params["lim"], params["lc"], bottom)
        assert host_ref.export_lines(exact, k) == open(os.path.join(d, "exact_0." + end)).read()
        assert host_ref.export_lines(approx, k) == open(os.path.join(d, "out.txt_0." + end)).read()
