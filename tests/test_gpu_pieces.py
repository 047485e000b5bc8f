"""The launch tail's pieces: in equal-window launches the last windows of every
candidate group are counted as two pieces of text -- bases [0, cut + k + 1) and [cut, L) -- whose
level bits are OR-ed in a meeting line before the window is counted.  Exact because an alignment
of a k-mer with <= 2 edits spans at most k + 2 bases (errorCount's find<0,2>, approx_counter.cpp:586;
level sets approx_counter.cpp:553-565).  These tests plant occurrences across the cut, at both
ends and with N bases around it, for every k and the window lengths the configurations use, and
compare both launch forms (device-resident equal windows, and the early launch of the host-buffer
stage) with the oracle."""
import random

import numpy as np
import pytest

import approx_counter_amd as ac
import oracle
from approx_counter_amd import _lib
from tests import cases

pytestmark = pytest.mark.gpu


def cut_for(L, k):
    """capi.cpp split_cut_for: the 32-aligned cut whose longer piece is shortest (0: no cut)."""
    best, best_max = 0, L
    if L > 256:
        return 0
    for cut in range(32, L, 32):
        a, b = cut + k + 1, L - cut
        if a >= L:
            break
        if max(a, b) < best_max:
            best, best_max = cut, max(a, b)
    return best


def straddle_case(seed, k, L, n_kmers, n_windows, p_n=0.01):
    """Equal windows of L bases; most carry a candidate with 0-3 edits planted so that it crosses or
    touches the cut (either side, by up to k + 3 bases), or at either end; some have N right at the
    cut."""
    rng = random.Random(seed)
    kmers = [cases.kmer_value(cases.rand_seq(rng, k)) for _ in range(n_kmers)]
    cut = cut_for(L, k)
    wins = []
    for _ in range(n_windows):
        w = list(cases.rand_seq(rng, L, p_n))
        if rng.random() < 0.8:
            pl = cases.mutate(rng, cases.kmer_string(rng.choice(kmers), k), rng.randint(0, 3))
            where = rng.randrange(4)
            if where == 0 and cut:
                p = max(0, min(L - len(pl), cut + rng.randint(-len(pl) - 3, k + 3)))
            elif where == 1:
                p = 0
            elif where == 2:
                p = max(0, L - len(pl))
            else:
                p = rng.randint(0, max(0, L - len(pl)))
            w[p:p + len(pl)] = list(pl)
            w = w[:L]
        if cut and rng.random() < 0.1:
            w[min(L - 1, cut + rng.randint(-2, k + 2))] = "N"
        wins.append("".join(w)[:L].ljust(L, "A"))
    return kmers, wins


# (k, L): the configurations' windows (100 / 101 at k = 16, 150 / 151 at k = 22), short and long
# ones, and every k at L = 100
CASES = sorted({(16, 100), (16, 101), (22, 150), (22, 151), (16, 64), (16, 256), (9, 200), (32, 96), (2, 70),
                (27, 255)} | {(k, 100) for k in range(2, 33)})


@pytest.mark.parametrize("k,L", CASES)
def test_pieces_device_equal_windows(counter, k, L):
    import torch

    km0, w0 = straddle_case(1000 * k + L, k, L, 150, 400)
    km1, w1 = straddle_case(7 + 1000 * k + L, k, L, 70, 250)
    packed = [ac.pack_windows(w0), ac.pack_windows(w1)]
    segs = [ac.DeviceSegment.upload(km0, packed[0]), ac.DeviceSegment.upload(km1, packed[1])]
    counter.count_device(k, segs, window_len=[L, L])
    torch.cuda.synchronize()
    counter.check()
    if cut_for(L, k):
        assert _lib.load().ac_testing_last_pieces(counter._h) > 0, "no window was counted in pieces"
    assert np.array_equal(segs[0].counts_numpy(), oracle.count_myers(k, km0, w0))
    assert np.array_equal(segs[1].counts_numpy(), oracle.count_myers(k, km1, w1))


@pytest.mark.parametrize("k,L", [(16, 100), (22, 151), (11, 160), (32, 100)])
def test_pieces_early_launch(counter, k, L):
    """The host-buffer stage (early launch, equal windows with inline N records), repeated so both
    queue banks -- each with its own meeting lines, zeroed by the launch on the other bank -- are used
    twice, with different data every call."""
    for rep in range(4):
        km0, w0 = straddle_case(50 * rep + k, k, L, 300, 1500, p_n=0.004)
        km1, w1 = straddle_case(50 * rep + k + 1, k, L + 1 if L < 256 else L, 200, 1200, p_n=0.004)
        got = counter.count_jobs(k, ac.Jobs([(km0, ac.Dna5Sample.from_windows(w0)),
                                             (km1, ac.Dna5Sample.from_windows(w1))]))
        assert counter.stage_mode() == 2
        assert _lib.load().ac_testing_last_pieces(counter._h) > 0
        assert np.array_equal(got[0], oracle.count_myers(k, km0, w0)), rep
        assert np.array_equal(got[1], oracle.count_myers(k, km1, w1)), rep


def test_pieces_then_ragged_then_pieces(counter):
    """A ragged launch (window descriptors: no pieces, and it does not zero the meeting lines of the
    other bank) between equal-window launches on the same scratch: the lines it leaves to the next
    equal-window launches are clean."""
    import torch

    k, L = 16, 100
    for rep in range(3):
        km, w = straddle_case(900 + rep, k, L, 200, 600)
        seg = ac.DeviceSegment.upload(km, ac.pack_windows(w))
        counter.count_device(k, [seg], window_len=[L])
        torch.cuda.synchronize()
        assert np.array_equal(seg.counts_numpy(), oracle.count_myers(k, km, w)), rep
        km2, w2 = cases.planted_case(77 + rep, k, 100, 300, win_len=(60, 140))
        seg2 = ac.DeviceSegment.upload(km2, ac.pack_windows(w2))
        counter.count_device(k, [seg2])
        torch.cuda.synchronize()
        assert np.array_equal(seg2.counts_numpy(), oracle.count_myers(k, km2, w2)), rep
    counter.check()
