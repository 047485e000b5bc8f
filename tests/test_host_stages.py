"""The CLI's host stages (libac_host.so, include/approx_counter_host.h) against
the oracle's restatement (oracle.host_ref): exact count with the N and
low-complexity filters, the float DUST score, CompareCount ranking."""
import ctypes
import os
import random

import numpy as np
import pytest

from oracle import encode_dna5, host_ref
from tests import cases

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "approx_counter_amd", "lib", "libac_host.so")


@pytest.fixture(scope="module")
def H():
    L = ctypes.CDLL(LIB)
    u8p, u64p, u32p = (ctypes.POINTER(t) for t in (ctypes.c_uint8, ctypes.c_uint64, ctypes.c_uint32))
    L.ach_complexity.argtypes = [ctypes.c_uint64, ctypes.c_uint32]
    L.ach_complexity.restype = ctypes.c_float
    L.ach_adjust_threshold.argtypes = [ctypes.c_float, ctypes.c_uint32, ctypes.c_uint32]
    L.ach_adjust_threshold.restype = ctypes.c_float
    L.ach_count_kmers.argtypes = [u8p, u64p, u32p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_float, u64p,
                                  ctypes.c_uint32, u64p, u64p, ctypes.c_uint64, u64p, u64p]
    L.ach_count_kmers.restype = ctypes.c_int
    L.ach_rank.argtypes = [u64p, u64p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, u64p, u64p]
    L.ach_rank.restype = ctypes.c_uint64
    return L


def p(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


def count(H, windows, k, thr, forbidden=()):
    arrs = [encode_dna5(w) for w in windows]
    lens = np.array([a.size for a in arrs], np.uint32)
    offs = np.zeros(len(arrs), np.uint64)
    if len(arrs) > 1:
        offs[1:] = np.cumsum(lens[:-1])
    flat = np.concatenate(arrs + [np.zeros(1, np.uint8)]).astype(np.uint8)
    fb = np.array(sorted(forbidden) or [0], np.uint64)
    cap = int(lens.sum()) + 1
    ok, oc = np.zeros(cap, np.uint64), np.zeros(cap, np.uint64)
    n_out, had_n = ctypes.c_uint64(), ctypes.c_uint64()
    rc = H.ach_count_kmers(p(flat, ctypes.c_uint8), p(offs, ctypes.c_uint64), p(lens, ctypes.c_uint32), len(arrs), k,
                           thr, p(fb, ctypes.c_uint64), len(forbidden), p(ok, ctypes.c_uint64),
                           p(oc, ctypes.c_uint64), cap, ctypes.byref(n_out), ctypes.byref(had_n))
    assert rc == 0
    n = n_out.value
    return {int(a): int(b) for a, b in zip(ok[:n], oc[:n])}, had_n.value


@pytest.mark.parametrize("k", [4, 9, 13, 16, 22, 32])
def test_count_kmers_matches_restatement(H, k):
    rng = random.Random(k)
    wins = [cases.rand_seq(rng, rng.randint(0, 120), p_n=0.02) for _ in range(60)]
    wins += ["A" * 50, "ACACACACACACACACACACACAC", "ACGT" * 20]  # low-complexity material
    thr = float(host_ref.adjust_threshold(1.0, 16, k))
    forbidden = {cases.kmer_value(wins[5][:k])} if len(wins[5]) >= k and "N" not in wins[5][:k] else set()
    got, had_n = count(H, wins, k, thr, forbidden)
    exp, exp_n = host_ref.count_kmers(wins, k, thr, forbidden)
    assert got == exp and had_n == exp_n


def test_complexity_and_threshold(H):
    rng = np.random.default_rng(5)
    for k in (2, 3, 4, 9, 16, 22, 32):
        for km in rng.integers(0, 4 ** min(k, 31), size=300, dtype=np.uint64):
            a = np.float32(H.ach_complexity(int(km), k))
            b = host_ref.get_complexity(int(km), k)
            assert (np.isnan(a) and np.isnan(b)) or a == b
        assert np.float32(H.ach_adjust_threshold(1.0, 16, k)) == host_ref.adjust_threshold(1.0, 16, k)
        assert np.float32(H.ach_adjust_threshold(1.5, 16, k)) == host_ref.adjust_threshold(1.5, 16, k)


@pytest.mark.parametrize("k", [5, 16])
def test_rank_matches_compare_count(H, k):
    rng = np.random.default_rng(k)
    n = 3000
    kmers = np.unique(rng.integers(0, 4 ** k, size=n, dtype=np.uint64))
    counts = rng.integers(1, 6, size=kmers.size).astype(np.uint64)  # many ties
    d = {int(a): int(b) for a, b in zip(kmers, counts)}
    for limit in (1, 50, 10**9):
        ok, oc = np.zeros(kmers.size, np.uint64), np.zeros(kmers.size, np.uint64)
        m = H.ach_rank(p(kmers, ctypes.c_uint64), p(counts, ctypes.c_uint64), kmers.size, min(limit, 2**63),
                       0, k, p(ok, ctypes.c_uint64), p(oc, ctypes.c_uint64))
        exp = host_ref.get_most_frequent(d, limit, k)
        assert [(int(a), int(b)) for a, b in zip(ok[:m], oc[:m])] == exp
    # solid mode: counts >= 4, CompareCount order
    m = H.ach_rank(p(kmers, ctypes.c_uint64), p(counts, ctypes.c_uint64), kmers.size, 2**63, 4, k,
                   p(ok, ctypes.c_uint64), p(oc, ctypes.c_uint64))
    assert [(int(a), int(b)) for a, b in zip(ok[:m], oc[:m])] == host_ref.get_solid_kmers(d, 4, k)
