"""The CLI's host stages (libac_host.so: count_kmers + get_most_frequent / get_solid_kmers,
approx_counter.cpp:487-519, 396-405, 372-388, CompareCount 275-305) against the oracle's
restatement (oracle/host_ref.py) at the BASELINE sample sizes -- cfg4's 10^6 windows of 100 bases
at k = 16 and cfg5's 10^5 windows of 151 bases at k = 22 -- on the very samples the -m gpu
full-scale exact-count tests use (tests/test_gpu_exact.py::test_full_scale_partitioned compares
the GPU with libac_host.so there, so that checker is tied to the oracle at the size it runs).

The restatement here is host_ref's vectorised form (count_kmers_dense / rank_dense), itself
checked against host_ref's loop restatement at small sizes (test_dense_restatement_is_the_loop_one)."""
import random

import numpy as np
import pytest

from oracle import encode_dna5, host_ref
from tests import cases
from tests.test_gpu_exact import _host_topk


@pytest.mark.parametrize("k", [2, 3, 4, 9, 16, 22, 32])
def test_dense_restatement_is_the_loop_one(k):
    rng = random.Random(100 + k)
    L = 70
    wins = [cases.rand_seq(rng, L, p_n=0.02) for _ in range(90)]
    wins[3], wins[4], wins[5] = "A" * L, ("AC" * L)[:L], ("ACGT" * L)[:L]
    w2 = np.stack([encode_dna5(x) for x in wins])
    thr = host_ref.adjust_threshold(1.0, 16, k)
    forb = {cases.kmer_value(wins[7][:k])} if "N" not in wins[7][:k] else set()
    exp, exp_n = host_ref.count_kmers(wins, k, thr, forb)
    uk, c, hn = host_ref.count_kmers_dense(w2, k, thr, forb)
    assert {int(a): int(b) for a, b in zip(uk, c)} == exp and hn == exp_n
    if k == 2:  # getComplexity is 0/0 = NaN for every 2-mer: CompareCount's order is undefined there
        return
    for lim in (1, 7, 50, 10**6):
        assert host_ref.rank_dense(uk, c, lim, 0, k) == host_ref.get_most_frequent(exp, lim, k)
    assert host_ref.rank_dense(uk, c, 0, 2, k) == host_ref.get_solid_kmers(exp, 2, k)


@pytest.mark.slow  # (~40 s and a few GB for cfg4: out of the quick suite, in the full CPU suite)
@pytest.mark.parametrize("cfg", [dict(k=16, n=1_000_000, L=100, lim=500), dict(k=22, n=100_000, L=151, lim=1000)],
                         ids=["cfg4", "cfg5"])
def test_host_stages_full_scale_vs_oracle(cfg):
    """Same sample, threshold and limit as test_gpu_exact.py::test_full_scale_partitioned: the host
    stages' top-`lim` list, distinct kept k-mers and N-skipped positions equal the restatement's."""
    from tools.synth import make_windows_fast

    k = cfg["k"]
    w, _ = make_windows_fast(cfg["n"], cfg["L"], seed=k, at_end=False)
    got, n_dist, had_n = _host_topk(w, k, cfg["lim"], 1.0)
    uk, c, exp_n = host_ref.count_kmers_dense(w, k, host_ref.adjust_threshold(1.0, 16, k))
    assert (n_dist, had_n) == (uk.size, exp_n)
    assert got == host_ref.rank_dense(uk, c, cfg["lim"], 0, k)
    assert got[0][1] > cfg["n"] // 4  # the planted adapter's k-mers lead


@pytest.mark.slow
def test_host_stages_full_scale_solid_and_forbidden():
    """cfg5's sample in solid mode (-sk) with a forbidden set (-fk) taken from its own top list."""
    from tools.synth import make_windows_fast

    k, n, L = 22, 100_000, 151
    w, _ = make_windows_fast(n, L, seed=k, at_end=True)
    thr = host_ref.adjust_threshold(1.0, 16, k)
    uk, c, _ = host_ref.count_kmers_dense(w, k, thr)
    top = host_ref.rank_dense(uk, c, 40, 0, k)
    forbidden = sorted(km for km, _ in top[::3])
    got = _host_rank(w, k, thr, forbidden, solid=500)
    uk2, c2, _ = host_ref.count_kmers_dense(w, k, thr, forbidden)
    exp = host_ref.rank_dense(uk2, c2, 0, 500, k)
    assert got == exp and len(exp) > 5
    assert not set(forbidden) & {km for km, _ in got}


def _host_rank(win2d, k, thr, forbidden, solid):
    """libac_host.so count_kmers (with a forbidden set) + rank in solid mode."""
    import ctypes
    import os

    lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "approx_counter_amd",
                                   "lib", "libac_host.so"))
    u8p, u32p, u64p = (ctypes.POINTER(t) for t in (ctypes.c_uint8, ctypes.c_uint32, ctypes.c_uint64))
    lib.ach_count_kmers.argtypes = [u8p, u64p, u32p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_float, u64p,
                                    ctypes.c_uint32, u64p, u64p, ctypes.c_uint64, u64p, u64p]
    lib.ach_rank.restype = ctypes.c_uint64
    lib.ach_rank.argtypes = [u64p, u64p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, u64p, u64p]
    P = lambda a, t: a.ctypes.data_as(t)  # noqa: E731
    n, L = win2d.shape
    flat = np.ascontiguousarray(win2d).reshape(-1)
    off = np.arange(n, dtype=np.uint64) * np.uint64(L)
    ln = np.full(n, L, dtype=np.uint32)
    fb = np.array(forbidden or [0], np.uint64)
    cap = n * max(1, L - k + 1)
    km, ct = np.zeros(cap, np.uint64), np.zeros(cap, np.uint64)
    n_out, had = ctypes.c_uint64(), ctypes.c_uint64()
    assert lib.ach_count_kmers(P(flat, u8p), P(off, u64p), P(ln, u32p), n, k, float(thr), P(fb, u64p), len(forbidden),
                               P(km, u64p), P(ct, u64p), cap, ctypes.byref(n_out), ctypes.byref(had)) == 0
    m = int(n_out.value)
    ok, oc = np.zeros(m, np.uint64), np.zeros(m, np.uint64)
    r = lib.ach_rank(P(km, u64p), P(ct, u64p), m, 2**63, solid, k, P(ok, u64p), P(oc, u64p))
    return [(int(a), int(b)) for a, b in zip(ok[:r], oc[:r])]
