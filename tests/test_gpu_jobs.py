"""GPU parity of the host-buffer stage ac_error_count_jobs / _submit (Dna5 windows
in, packed by the host pool, one DMA, one fused launch, counts back) and of the
device error word (ac_check), against the CPU oracle.  Bit-exact everywhere."""
import json
import os

import numpy as np
import pytest

import approx_counter_amd as ac
import oracle
from tests import cases

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _shuffled_sample(wins, seed):
    """A Dna5 sample whose windows sit at shuffled, partly overlapping offsets of
    one byte buffer (a StringSet's strings need not be in order)."""
    rng = np.random.default_rng(seed)
    arrs = [ac.to_dna5(w) for w in wins]
    order = rng.permutation(len(arrs))
    buf, offs = [], np.zeros(len(arrs), np.uint64)
    pos = 0
    for i in order:
        buf.append(rng.integers(0, 5, size=int(rng.integers(0, 7)), dtype=np.uint8))  # junk between windows
        pos += buf[-1].size
        offs[i] = pos
        buf.append(arrs[i])
        pos += arrs[i].size
    lens = np.array([a.size for a in arrs], np.uint32)
    return ac.Dna5Sample(np.concatenate(buf) if buf else np.zeros(1, np.uint8), offs, lens)


def test_golden_vectors_jobs(counter):
    with open(os.path.join(GOLDEN, "vectors.json")) as fh:
        vecs = json.load(fh)
    for vec in vecs:
        got = counter.count_jobs(vec["k"], [(vec["kmers"], vec["windows"])])[0]
        assert [int(x) for x in got] == vec["counts"], vec["name"]


@pytest.mark.parametrize("k", [2, 3, 7, 11, 16, 17, 22, 31, 32])
def test_two_ends_fused(counter, k):
    """Both read ends in one call, windows at shuffled offsets, ragged lengths incl. 0."""
    a = cases.planted_case(100 + k, k, 300, 400, win_len=(0, 260), p_n=0.02)
    b = cases.planted_case(200 + k, k, 170, 350, win_len=(0, 130), p_n=0.02)
    got = counter.count_jobs(k, [(a[0], _shuffled_sample(a[1], k)), (b[0], _shuffled_sample(b[1], k + 1))])
    assert np.array_equal(got[0], oracle.count_myers(k, *a))
    assert np.array_equal(got[1], oracle.count_myers(k, *b))


def test_four_jobs_with_empty_ones(counter):
    a = cases.planted_case(1, 16, 500, 300, win_len=(90, 110))
    b = cases.planted_case(2, 16, 64, 0)  # candidates, no windows
    c = (np.zeros(0, np.uint64), cases.planted_case(3, 16, 5, 50)[1])  # windows, no candidates
    d = cases.planted_case(4, 16, 1, 70, win_len=(0, 40), p_n=0.2)
    got = counter.count_jobs(16, [a, b, c, d])
    assert np.array_equal(got[0], oracle.count_myers(16, *a))
    assert np.array_equal(got[1], np.zeros(64, np.uint64))
    assert got[2].size == 0
    assert np.array_equal(got[3], oracle.count_myers(16, *d))


def test_dna5_bytes_above_4_are_n(counter):
    """Any ordinal > 3 (SeqAn's N is 4; here also 5..255) matches nothing."""
    kmers = [cases.kmer_value("ACGTACGTACGTACGT")]
    base = ac.to_dna5("ACGTACGTACGTACGT")
    wins = []
    for v in (4, 5, 77, 128, 200, 255):
        w = base.copy()
        w[7] = v
        wins.append(w)
    got = counter.count_jobs(16, [(kmers, wins)])[0]
    exp = oracle.count_myers(16, kmers, [np.where(w > 3, 4, w).astype(np.uint8) for w in wins])
    assert np.array_equal(got, exp) and got[0] == 2 * len(wins)


def test_single_n_anywhere_is_seen(counter):
    """A job is sent and counted without its N bitmap only when none of its windows holds
    an N: a single N in the first, a middle or the last window (a different pool task each)
    must still count as a mismatch; an N-free job fused beside it is counted N-free."""
    rng = np.random.default_rng(41)
    n, L = 6000, 100
    base = rng.integers(0, 4, size=(n, L), dtype=np.uint8)
    pick = base[17, 30:46]
    kmers = np.array([sum(int(b) << (2 * (15 - i)) for i, b in enumerate(pick))], dtype=np.uint64)
    clean = [w for w in base]
    exp_clean = oracle.count_myers(16, kmers, clean, 16)
    for where in (17, n // 2, n - 1):
        wins = base.copy()
        wins[where, 30 + 7 if where == 17 else L - 1] = 4
        got = counter.count_jobs(16, [(kmers, [w for w in wins]), (kmers, clean)])
        assert np.array_equal(got[0], oracle.count_myers(16, kmers, [w for w in wins], 16))
        assert np.array_equal(got[1], exp_clean)
        if where == 17:  # the N sits inside the k-mer's exact occurrence: one level fewer there
            assert got[0][0] < exp_clean[0]


def test_jobs_equal_image_path_and_repeat(counter):
    """Calls alternating between the two staging slots, growing and shrinking."""
    for trial, (n_k, n_w, wl) in enumerate([(500, 2000, (100, 101)), (37, 50, (0, 300)), (1000, 5000, (150, 151)),
                                            (500, 2000, (100, 101)), (3, 3, (0, 5))]):
        kmers, wins = cases.planted_case(77 + trial, 16, n_k, n_w, win_len=wl, p_n=0.01)
        got = counter.count_jobs(16, [(kmers, wins)])[0]
        assert np.array_equal(got, counter.count(16, kmers, ac.pack_windows(wins))), trial
        assert np.array_equal(got, oracle.count_myers(16, kmers, wins)), trial


def test_large_sample_pool_split(counter):
    """Enough windows that the host pool splits them into many tasks."""
    from tools.synth import make_windows_fast

    w, _ = make_windows_fast(60_000, 101, seed=5, at_end=True)
    kmers, _ = cases.planted_case(9, 16, 200, 0)
    from tools import workload

    cand = workload.exact_topk(list(w[:3000]), 16, 100)
    kmers = np.array([c for c, _ in cand] + kmers[:100], np.uint64)
    got = counter.count_jobs(16, [(kmers, ac.Dna5Sample.from_windows(w))])[0]
    assert np.array_equal(got, oracle.count_myers(16, kmers, w, 16))


@pytest.mark.parametrize("shards", [2, 3])
def test_multi_context_jobs_equal_one(shards):
    """ac_create_multi + jobs: each job's windows sharded over the contexts (here on
    one GPU), shard counts summed: identical to one device, k = 2 empty windows too."""
    for k in (16, 2):
        a = cases.planted_case(600 + k, k, 150, 40, win_len=(0, 200), p_n=0.01)
        b = (a[0], ["", "", "", ""])  # only empty windows: k = 2 still counts d = 2 hits
        with ac.ApproxCounter(n_gpus=shards) as multi:
            got = multi.count_jobs(k, [(a[0], _shuffled_sample(a[1], 3)), b])
        assert np.array_equal(got[0], oracle.count_myers(k, *a)), k
        assert np.array_equal(got[1], oracle.count_myers(k, *b)), k


def test_submit_into_device_tensor(counter):
    import torch

    a = cases.planted_case(11, 16, 500, 900, win_len=(100, 101), p_n=0.01)
    b = cases.planted_case(12, 16, 400, 700, win_len=(101, 101), p_n=0.01)
    jobs = ac.Jobs([(a[0], ac.Dna5Sample.from_windows(a[1])), (b[0], ac.Dna5Sample.from_windows(b[1]))])
    out = torch.full((jobs.n_counts,), 7, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream()
    for _ in range(3):  # both staging slots, back to back on one stream
        counter.submit_jobs(16, jobs, out, stream=st.cuda_stream)
    counter.check(stream=st.cuda_stream)
    got = out.cpu().numpy().view(np.uint32).astype(np.uint64)
    assert np.array_equal(got[:500], oracle.count_myers(16, *a))
    assert np.array_equal(got[500:], oracle.count_myers(16, *b))


def test_sync_call_while_submit_in_flight(counter):
    """A synchronous jobs call made while a submit's launch is still running on another
    stream: the two launches use separate count-kernel scratch (queues, sums, tickets),
    so neither corrupts the other."""
    import torch

    a = cases.planted_case(31, 16, 500, 3000, win_len=(100, 101), p_n=0.01)
    b = cases.planted_case(32, 16, 300, 2000, win_len=(100, 101), p_n=0.01)
    ja = ac.Jobs([(a[0], ac.Dna5Sample.from_windows(a[1]))])
    st = torch.cuda.Stream()
    out = torch.zeros(ja.n_counts, dtype=torch.int32, device="cuda")
    exp_a, exp_b = oracle.count_myers(16, *a), oracle.count_myers(16, *b)
    for _ in range(4):
        out.fill_(-1)
        counter.submit_jobs(16, ja, out, stream=st.cuda_stream)  # not synchronised
        got_b = counter.count_jobs(16, [(b[0], ac.Dna5Sample.from_windows(b[1]))])[0]
        st.synchronize()
        assert np.array_equal(got_b, exp_b)
        assert np.array_equal(out.cpu().numpy().view(np.uint32).astype(np.uint64), exp_a)
    counter.check(stream=st.cuda_stream)


def test_device_error_word_reports_malformed_window(counter):
    """A device segment with a misaligned window (and one past the image) is
    skipped by the kernel, which reports it: ac_check returns AC_ERR_INVALID."""
    import torch

    kmers, wins = cases.planted_case(21, 16, 100, 10, win_len=(100, 101))
    seg = ac.DeviceSegment.upload(kmers, ac.pack_windows(wins))
    counter.count_device(16, [seg])
    counter.check()  # clean launch: OK
    bad = seg.start.clone()
    bad[3] += 1  # not 32-aligned
    seg.start = bad
    counter.count_device(16, [seg])
    with pytest.raises(ac.ApproxCounterError) as ei:
        counter.check()
    assert ei.value.status == 1 and "malformed" in str(ei.value)
    counter.check()  # the word was cleared
    bad2 = seg.start.clone()
    bad2[3] = torch.tensor(seg.n_bases + 64, dtype=torch.int64)  # past the image
    seg.start = bad2
    counter.count_device(16, [seg])
    with pytest.raises(ac.ApproxCounterError):
        counter.check()


def test_multi_context_shuffled_overlapping_windows():
    """on an ac_create_multi context a shard's slice of the image spans
    its lowest start to its highest end, so windows in any order, overlapping,
    are counted as on one device (no wrapped start)."""
    kmers, wins = cases.planted_case(4040, 16, 120, 64, win_len=(64, 128), p_n=0.01)
    ps = ac.pack_windows(wins)
    rng = np.random.default_rng(1)
    order = rng.permutation(len(wins))
    start = ps.start[order].copy()
    length = ps.length[order].copy()
    # an overlapping window: bases 32..127 of the image, inside the first windows
    start[1], length[1] = 32, 96
    shuffled = ac.PackedSample(ps.codes, ps.nmask, start, length, ps.n_bases)
    with ac.ApproxCounter(0) as one:
        exp = one.count(16, kmers, shuffled)
    for shards in (2, 3, 5):
        with ac.ApproxCounter(n_gpus=shards) as multi:
            assert np.array_equal(multi.count(16, kmers, shuffled), exp), shards


@pytest.mark.skipif("AC_STAGE_ZEROCOPY" in os.environ, reason="transfer path forced by the environment")
def test_transfer_path_probe_both_ways_bit_exact():
    """A fresh context alternates zero-copy and DMA over its first synchronous calls
    (ac_stage_mode -1 until then), keeps the faster, and every call is bit-exact."""
    a = cases.planted_case(31, 16, 200, 300, win_len=(0, 150), p_n=0.02)
    b = cases.planted_case(32, 16, 90, 260, win_len=(80, 120))
    exp = [oracle.count_myers(16, *a), oracle.count_myers(16, *b)]
    c = ac.ApproxCounter(0)
    try:
        assert c.stage_mode() == -1
        jobs = ac.Jobs([(a[0], _shuffled_sample(a[1], 5)), (b[0], ac.Dna5Sample.from_windows(b[1]))])
        modes = []
        for _ in range(12):
            got = c.count_jobs(16, jobs)
            assert np.array_equal(got[0], exp[0]) and np.array_equal(got[1], exp[1])
            modes.append(c.stage_mode())
        assert modes[8] == -1 and modes[9] in (0, 1) and len(set(modes[9:])) == 1, modes
    finally:
        c.close()


def test_image_size_limit_rejected(counter):
    """The count kernel addresses the image through 32-bit buffer offsets: a device
    segment claiming 2^34 bases or more is refused up front (AC_ERR_INVALID), never
    launched."""
    kmers, wins = cases.planted_case(22, 16, 100, 10, win_len=(100, 101))
    seg = ac.DeviceSegment.upload(kmers, ac.pack_windows(wins))
    seg.n_bases = 1 << 34
    with pytest.raises(ac.ApproxCounterError) as ei:
        counter.count_device(16, [seg])
    assert ei.value.status == 1 and "2^34" in str(ei.value)
    seg.n_bases = ac.pack_windows(wins).n_bases  # the context still counts afterwards
    counter.count_device(16, [seg])
    counter.check()
    assert np.array_equal(seg.counts_numpy(), oracle.count_myers(16, kmers, wins, 16))


@pytest.mark.skipif("AC_STAGE_ZEROCOPY" in os.environ, reason="transfer path forced by the environment")
def test_large_image_takes_dma_path():
    """A call whose zero-copy would move more than 256 MB over PCIe (image x candidate
    groups; zero-copy may read the image once per group) is staged by DMA: a fresh
    context reports DMA at once (ac_stage_mode 0), and the kernel writes the counts into
    the pinned block, bit-exact (checked on a prefix of the candidates)."""
    rng = np.random.default_rng(7)
    n, L = 700_000, 100  # 700k x 128 bases x 3/8 B x 8 groups = 269 MB
    win = rng.integers(0, 4, size=(n, L), dtype=np.uint8)
    win[rng.integers(0, n, size=2000), rng.integers(0, L, size=2000)] = 4  # a few N
    picks = rng.integers(0, n, size=1000)
    kmers = np.array([int(sum(int(b) << (2 * (15 - i)) for i, b in enumerate(win[p, 20:36]))) for p in picks],
                     dtype=np.uint64)
    sample = ac.Dna5Sample(win.reshape(-1), np.arange(n, dtype=np.uint64) * np.uint64(L),
                           np.full(n, L, dtype=np.uint32))
    c = ac.ApproxCounter(0)
    try:
        assert c.stage_mode() == -1
        got = c.count_jobs(16, [(kmers, sample)])[0]
        assert c.stage_mode() == 0
    finally:
        c.close()
    sub = np.r_[0:16, 500:508, 992:1000]  # every candidate group's first and last lanes, and more
    assert np.array_equal(got[sub], oracle.count_myers(16, kmers[sub], win, 16))


def test_rccl_allreduce_single_rank(counter):
    """The library's RCCL path (ac_comm_unique_id / ac_comm_init / ac_allreduce_counts),
    as bench.py's N > 1 steps use it, on a one-rank communicator (this pool has one GPU
    per box; RCCL refuses two ranks on one device): the sum over one rank is the
    identity, so the all-reduced counts equal the oracle's; misuse is refused."""
    import torch

    with pytest.raises(ac.ApproxCounterError):  # no communicator yet
        counter.allreduce_counts(torch.zeros(4, dtype=torch.int32, device="cuda"))
    uid = counter.comm_unique_id()
    assert len(uid) == 128
    counter.comm_init(1, 0, uid)
    with pytest.raises(ac.ApproxCounterError):  # one communicator per context
        counter.comm_init(1, 0, uid)
    a = cases.planted_case(41, 16, 300, 500, win_len=(100, 101), p_n=0.01)
    b = cases.planted_case(42, 16, 200, 400, win_len=(101, 101))
    jobs = ac.Jobs([(a[0], ac.Dna5Sample.from_windows(a[1])), (b[0], ac.Dna5Sample.from_windows(b[1]))])
    out = torch.zeros(jobs.n_counts, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream()
    counter.submit_jobs(16, jobs, out, stream=st.cuda_stream)
    counter.allreduce_counts(out, stream=st.cuda_stream)
    counter.check(stream=st.cuda_stream)
    got = out.cpu().numpy().view(np.uint32).astype(np.uint64)
    assert np.array_equal(got[:300], oracle.count_myers(16, *a))
    assert np.array_equal(got[300:], oracle.count_myers(16, *b))
