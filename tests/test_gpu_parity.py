"""GPU parity: the HIP kernel (through the C ABI) against the CPU oracle.

Bit-exact integer equality everywhere; the oracle is the
checker only.  Run with ``pytest -m gpu`` on an MI355X.
"""
import json
import os

import numpy as np
import pytest

import approx_counter_amd as ac
import oracle
from oracle import host_ref
from tests import cases

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def gpu_counts(counter, k, kmers, windows):
    return counter.count(k, kmers, ac.pack_windows(windows))


def test_golden_vectors(counter):
    with open(os.path.join(GOLDEN, "vectors.json")) as fh:
        vecs = json.load(fh)
    for vec in vecs:
        got = gpu_counts(counter, vec["k"], vec["kmers"], vec["windows"])
        assert [int(x) for x in got] == vec["counts"], vec["name"]


@pytest.mark.parametrize("k", list(range(2, 33)))
def test_every_k_planted(counter, k):
    for seed in range(3):
        kmers, wins = cases.planted_case(10_000 * k + seed, k, 150, 60,
                                         win_len=(max(0, k - 5), k + 140), p_n=0.02)
        exp = oracle.count_myers(k, kmers, wins)
        got = gpu_counts(counter, k, kmers, wins)
        assert np.array_equal(got, exp), (k, seed, np.nonzero(got != exp)[0][:10])


def test_every_k_dp_crosscheck(counter):
    for k in range(2, 33):
        kmers, wins = cases.planted_case(555 + k, k, 20, 25, win_len=(0, k + 30), p_n=0.05)
        assert np.array_equal(gpu_counts(counter, k, kmers, wins), oracle.count_dp(k, kmers, wins)), k


@pytest.mark.parametrize("name,k,kmers,windows", cases.edge_cases(), ids=lambda x: x if isinstance(x, str) else "")
def test_edge_cases(counter, name, k, kmers, windows):
    exp = oracle.count_dp(k, kmers, windows)
    assert np.array_equal(gpu_counts(counter, k, kmers, windows), exp), name


@pytest.mark.parametrize("n_kmers", [1, 63, 64, 65, 127, 128, 129, 255, 256, 257, 500, 1000])
def test_ragged_candidate_groups(counter, n_kmers):
    for k in (16, 10, 22):
        kmers, wins = cases.planted_case(n_kmers * 31 + k, k, n_kmers, 40, win_len=(80, 110))
        assert np.array_equal(gpu_counts(counter, k, kmers, wins), oracle.count_myers(k, kmers, wins)), k


def test_many_windows_ragged_lengths(counter):
    kmers, wins = cases.planted_case(4242, 16, 300, 5000, win_len=(0, 300), p_n=0.01)
    assert np.array_equal(gpu_counts(counter, 16, kmers, wins), oracle.count_myers(16, kmers, wins))


def test_config2_scale_bit_exact(counter):
    """BASELINE config 2 shape: k=16, 10k windows of 100/101 bp, 500 candidates."""
    from tools.synth import make_reads

    reads, _ = make_reads(10_000, read_len=400, seed=1)
    seqs = [r.decode() for r in reads]
    for bottom in (False, True):
        wins = host_ref.sample_all(seqs, 100, bottom)
        # candidates: the adapter-rich top of a quick exact count on a subset + random ones
        counter_exact, _ = host_ref.count_kmers(wins[:1500], 16, 1.0)
        cands = [km for km, _ in host_ref.get_most_frequent(counter_exact, 500, 16)]
        exp = oracle.count_myers(16, cands, wins)
        got = gpu_counts(counter, 16, cands, wins)
        assert np.array_equal(got, exp)
        assert got.max() > 1000  # adapter k-mers are found in most windows


def _device_segments(k, parts):
    return [ac.DeviceSegment.upload(km, ac.pack_windows(w)) for km, w in parts]


def test_fused_segments_one_launch(counter):
    import torch

    parts = [cases.planted_case(s, 16, n, 200, win_len=(90, 110)) for s, n in ((1, 500), (2, 77), (3, 300))]
    segs = _device_segments(16, parts)
    counter.count_device(16, segs)
    torch.cuda.synchronize()
    for (km, w), seg in zip(parts, segs):
        assert np.array_equal(seg.counts_numpy(), oracle.count_myers(16, km, w))


@pytest.mark.parametrize("k,lens", [(16, (100, 101)), (22, (151, 151)), (9, (300, 37))])
def test_device_equal_windows(counter, k, lens):
    """ac_error_count_device with window_len: windows back to back at ceil32 strides, places
    computed instead of loaded (start / length not read) -- both ends fused, bit-exact; with
    AC_DEVICE_ACCUMULATE too (ABI 8: the equal and accumulate forms combine)."""
    import torch

    parts = []
    for s, L in enumerate(lens):
        km, w = cases.planted_case(700 + s + k, k, 300, 900, win_len=(L, L), p_n=0.01)
        parts.append((km, [(x + "A" * L)[:L] for x in w]))  # truly equal (a plant may grow one)
    packed = [ac.pack_windows(w) for _, w in parts]
    assert [p.equal_window_len() for p in packed] == list(lens)
    segs = [ac.DeviceSegment.upload(km, p) for (km, _), p in zip(parts, packed)]
    counter.count_device(k, segs, window_len=list(lens))
    torch.cuda.synchronize()
    counter.check()
    exp = [oracle.count_myers(k, km, w) for km, w in parts]
    for e, seg in zip(exp, segs):
        assert np.array_equal(seg.counts_numpy(), e)
    counter.count_device(k, segs, window_len=list(lens), accumulate=True)
    torch.cuda.synchronize()
    counter.check()
    for e, seg in zip(exp, segs):
        assert np.array_equal(seg.counts_numpy(), 2 * e)
    # windows that would reach past n_bases are refused on the host
    with pytest.raises(ac.ApproxCounterError):
        counter.count_device(k, segs[:1], window_len=[lens[0] + 64])


def test_sharded_accumulate_equals_whole(counter):
    """Windows split into shards and accumulated == one launch (multi-GPU identity)."""
    import torch

    kmers, wins = cases.planted_case(99, 16, 500, 1200, win_len=(100, 101))
    exp = oracle.count_myers(16, kmers, wins)
    whole = ac.DeviceSegment.upload(kmers, ac.pack_windows(wins))
    counter.count_device(16, [whole])
    for n_shards in (2, 3, 8):
        bounds = np.linspace(0, len(wins), n_shards + 1).astype(int)
        seg0 = ac.DeviceSegment.upload(kmers, ac.pack_windows(wins[bounds[0]:bounds[1]]))
        counter.count_device(16, [seg0])
        for i in range(1, n_shards):
            part = ac.DeviceSegment.upload(kmers, ac.pack_windows(wins[bounds[i]:bounds[i + 1]]))
            part.counts = seg0.counts
            counter.count_device(16, [part], accumulate=True)
        torch.cuda.synchronize()
        assert np.array_equal(seg0.counts_numpy(), exp), n_shards
    torch.cuda.synchronize()
    assert np.array_equal(whole.counts_numpy(), exp)


def test_repeatable(counter):
    kmers, wins = cases.planted_case(5, 16, 500, 800, win_len=(100, 101))
    s = ac.pack_windows(wins)
    a = counter.count(16, kmers, s)
    b = counter.count(16, kmers, s)
    assert np.array_equal(a, b)


def test_invalid_k_rejected(counter):
    s = ac.pack_windows(["ACGT" * 10])
    for k in (0, 1, 33, 64):
        with pytest.raises(ac.ApproxCounterError) as ei:
            counter.count(k, [1, 2], s)
        assert ei.value.status == 1


def test_error_count_mirror_cfg1(counter):
    """errorCount mirror on the config-1 fixture reproduces out.txt_0.<end>."""
    d = os.path.join(GOLDEN, "cfg1")
    params = json.load(open(os.path.join(d, "params.json")))
    _, seqs = host_ref.read_fasta(os.path.join(d, "reads.fa"))
    k = params["k"]
    for end, bottom in (("start", False), ("end", True)):
        wins = host_ref.sample_all(seqs, params["sl"], bottom)
        exact = [(cases.kmer_value(ln.split("\t")[0]), int(ln.split("\t")[1]))
                 for ln in open(os.path.join(d, "exact_0." + end)).read().splitlines()]
        res = ac.error_count(wins, exact, 4, k, 0)
        ranked = host_ref.get_most_frequent(res, params["lim"], k)
        assert host_ref.export_lines(ranked, k) == open(os.path.join(d, "out.txt_0." + end)).read()


def test_survey_ac_count_layout(counter):
    """ac_count (SURVEY.md 8(b) argument list): the same counts as ac_error_count on
    the same image, with word offsets and uint16 lengths."""
    kmers, wins = cases.planted_case(8080, 16, 200, 700, win_len=(0, 260), p_n=0.02)
    ps = ac.pack_windows(wins)
    got = counter.count_words(16, kmers, ps.codes, ps.nmask, ps.start // 16, ps.length.astype(np.uint16))
    assert np.array_equal(got, oracle.count_myers(16, kmers, wins))
    with pytest.raises(ac.ApproxCounterError):  # odd word offset: not 32-base aligned
        counter.count_words(16, kmers, ps.codes, ps.nmask, ps.start // 16 + 1, ps.length.astype(np.uint16))


@pytest.mark.parametrize("shards", [2, 3, 7])
def test_multi_gpu_context_shards_equal_one(shards):
    """ac_create_multi: windows split into `shards` slices (wrapping onto this box's
    GPUs), counted concurrently, summed on the host: identical to one device,
    including shards holding only empty windows."""
    kmers, wins = cases.planted_case(9090 + shards, 13, 150, 40, win_len=(0, 200), p_n=0.01)
    wins = wins + ["", "", ""]  # trailing empty windows (start == image end)
    exp = oracle.count_myers(13, kmers, wins)
    with ac.ApproxCounter(n_gpus=shards) as multi:
        assert np.array_equal(multi.count(13, kmers, ac.pack_windows(wins)), exp)
        assert np.array_equal(multi.count(13, kmers, ac.pack_windows(wins[:2])), oracle.count_myers(13, kmers, wins[:2]))


def test_counts_stored_without_memset(counter):
    """ac_error_count_device stores the counts from inside the launch (the group's
    last workgroup): stale values in the buffer are overwritten, and the hand-off
    scratch is back to zero for the next launch, across launches of varying shape."""
    import torch

    rng = np.random.default_rng(7)
    for trial, (k, n_kmers, n_win) in enumerate([(16, 500, 900), (16, 37, 300), (22, 300, 500),
                                                 (11, 1000, 200), (16, 500, 900), (5, 9, 50)]):
        kmers, wins = cases.planted_case(4242 + trial, k, n_kmers, n_win, win_len=(60, 151), p_n=0.01)
        seg = ac.DeviceSegment.upload(kmers, ac.pack_windows(wins))
        seg.counts.copy_(torch.from_numpy(rng.integers(1, 1 << 30, seg.counts.numel(), dtype=np.int32)))
        counter.count_device(k, [seg])
        torch.cuda.synchronize()
        assert np.array_equal(seg.counts_numpy(), oracle.count_myers(k, kmers, wins)), (trial, k)


def test_accumulate_adds_to_existing(counter):
    import torch

    kmers, wins = cases.planted_case(31337, 16, 300, 400, win_len=(100, 101))
    exp = oracle.count_myers(16, kmers, wins)
    seg = ac.DeviceSegment.upload(kmers, ac.pack_windows(wins))
    base = np.arange(seg.counts.numel(), dtype=np.int32) * 7
    seg.counts.copy_(torch.from_numpy(base))
    counter.count_device(16, [seg], accumulate=True)
    counter.count_device(16, [seg], accumulate=True)
    torch.cuda.synchronize()
    assert np.array_equal(seg.counts_numpy(), base[: len(kmers)].astype(np.uint64) + 2 * exp)


def test_fused_shards_sharing_counts(counter):
    """Window shards of one candidate set fused in one non-accumulate launch, all
    pointing at the same count vector: the launch sums them (zeroing once)."""
    import torch

    kmers, wins = cases.planted_case(2718, 16, 500, 1000, win_len=(90, 110), p_n=0.01)
    exp = oracle.count_myers(16, kmers, wins)
    bounds = np.linspace(0, len(wins), 5).astype(int)
    segs = [ac.DeviceSegment.upload(kmers, ac.pack_windows(wins[bounds[i]:bounds[i + 1]])) for i in range(4)]
    for s in segs[1:]:
        s.counts = segs[0].counts
    segs[0].counts.fill_(12345)
    counter.count_device(16, segs)
    torch.cuda.synchronize()
    assert np.array_equal(segs[0].counts_numpy(), exp)


@pytest.mark.parametrize("k", [5, 11, 16, 22, 32])
def test_long_ragged_windows(counter, k):
    """Windows longer than one 256-base fetch segment (ragged lengths, N's, hits
    planted anywhere incl. across the 256-base seams)."""
    kmers, wins = cases.planted_case(777 + k, k, 150, 120, win_len=(200, 1500), p_n=0.005)
    assert np.array_equal(gpu_counts(counter, k, kmers, wins), oracle.count_myers(k, kmers, wins)), k
