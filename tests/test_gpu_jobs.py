"""GPU parity of the host-buffer stage ac_error_count_jobs / _submit (Dna5 windows
in, packed by the host pool, one DMA, one fused launch, counts back) and of the
device error word (ac_check), against the CPU oracle.  Bit-exact everywhere."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import approx_counter_amd as ac
import oracle
from tests import cases

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

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


def _kmers_from(wins, n, seed, k=16):
    """n k-mers cut from random places of random windows (N bases read as random bases)."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        w = wins[int(rng.integers(len(wins)))]
        s0 = int(rng.integers(0, max(1, len(w) - k + 1)))
        v = 0
        for b in w[s0:s0 + k]:
            v = (v << 2) | (int(b) if b < 4 else int(rng.integers(4)))
        out.append(v)
    return np.array(out, np.uint64)


def _n_record_windows(seed, n, L, counts, spots=()):
    """n equal windows of L random bases; window i holds counts[i % len(counts)] N bases,
    the first ones at `spots` (window-relative, clipped to L), the rest at random places."""
    rng = np.random.default_rng(seed)
    w = rng.integers(0, 4, size=(n, L), dtype=np.uint8)
    for i in range(n):
        c = counts[i % len(counts)]
        pos = [p for p in spots if p < L][:c]
        free = np.setdiff1d(np.arange(L), pos)
        pos += list(rng.choice(free, size=c - len(pos), replace=False))
        w[i, pos] = 4 if i % 3 else 9  # (any ordinal > 3 is N)
    return w


@pytest.mark.parametrize("L", [100, 101, 150, 151, 128, 16, 40])
def test_inline_n_records(counter, L):
    """Equal windows carry their N positions in the slot's padding (nrec.h): 4 positions
    at L = 100/101, 2 at 150, 1 at 151, none at 128 (no room: the N bitmap path), 4 at 16 / 40.
    Windows with 0..6 N bases -- records that hold them all and records that overflow (their
    N-bitmap words are used) -- with N on word edges (0, 15, 16, 31, 32, 63, 64, L - 1), in
    one job beside an N-free job and a job whose only N-holders overflow."""
    ws = _n_record_windows(L, 3000, L, [0, 1, 0, 2, 0, 3, 4, 0, 5, 6, 1], spots=(0, 15, 16, 31, 32, 63, 64, L - 1))
    over = _n_record_windows(L + 1, 900, L, [0, 0, 7])
    clean = _n_record_windows(L + 2, 700, L, [0])
    kmers = _kmers_from(ws, 300, seed=L)  # occurrences in the windows, many across an N
    km2 = np.concatenate([_kmers_from(over, 100, seed=L + 1), kmers[:20]])
    jobs = [(kmers, ac.Dna5Sample.from_windows(ws)), (km2, ac.Dna5Sample.from_windows(over)),
            (kmers[:64], ac.Dna5Sample.from_windows(clean))]
    for rep in range(2):  # (both staging slots)
        got = counter.count_jobs(16, jobs)
        assert np.array_equal(got[0], oracle.count_myers(16, kmers, np.minimum(ws, 4), 16)), rep
        assert np.array_equal(got[1], oracle.count_myers(16, km2, np.minimum(over, 4), 16)), rep
        assert np.array_equal(got[2], oracle.count_myers(16, kmers[:64], clean, 16)), rep


def test_inline_n_records_large_call(counter):
    """A large call (150k windows: the early launch with copier workgroups, both jobs packed
    interleaved) with inline N records: the N bitmap is sent only for the job whose records
    overflowed, and its windows with overflowed records wait for it."""
    L = 101
    a = _n_record_windows(7, 90_000, L, [0] * 20 + [1, 2, 3, 4])
    b = _n_record_windows(8, 60_000, L, [0] * 50 + [1, 5])
    kmers = _kmers_from(a, 40, seed=77)
    got = counter.count_jobs(16, [(kmers, ac.Dna5Sample.from_windows(a)), (kmers, ac.Dna5Sample.from_windows(b))])
    assert np.array_equal(got[0], oracle.count_myers(16, kmers, np.minimum(a, 4), 16))
    assert np.array_equal(got[1], oracle.count_myers(16, kmers, np.minimum(b, 4), 16))


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


def _late_n(wins, frac):
    """The windows with N only in the last `frac` of them (the early-counting prefix stops there)."""
    out = [w.replace("N", "A") for w in wins]
    for i in range(int(len(out) * (1 - frac)), len(out)):
        if len(out[i]) > 3:
            out[i] = out[i][:2] + "N" + out[i][3:]
    return out


def early_rotation(calls=30):
    """Rotates different workloads (sizes, N / no N, equal / ragged windows, 1-3 jobs) through
    one context's early-launch stage; every call checked.  Equal-window jobs are counted while
    they arrive (windows gated chunk by chunk): among them jobs whose N sit only in the last
    windows or only in the first, windows longer than one 256-base fetch, and k-mer sets that
    span several staging chunks."""
    rng = np.random.default_rng(5)
    work = []
    for seed, (nw, lens, p_n, n_jobs, n_k, shape) in enumerate([
            (900, (100, 100), 0.0, 2, None, None), (2500, (0, 150), 0.02, 3, None, None),
            (400, (101, 101), 0.01, 1, None, None), (6000, (100, 100), 0.0, 2, 1500, "late_n"),
            (3000, (101, 101), 0.0, 1, None, "first_n"), (700, (600, 600), 0.0, 2, 700, None)]):
        jobs, exp = [], []
        for j in range(n_jobs):
            km, wins = cases.planted_case(300 + 10 * seed + j, 16, n_k or int(rng.integers(60, 400)), nw,
                                          win_len=lens, p_n=p_n)
            if lens[0] == lens[1]:  # truly equal windows (a planted candidate may have grown one)
                wins = [(w + "A" * lens[0])[: lens[0]] for w in wins]
            if shape == "late_n":
                wins = _late_n(wins, 0.02)
            elif shape == "first_n":
                wins = list(wins)
                wins[0] = "N" + wins[0][1:]
            jobs.append((km, ac.Dna5Sample.from_windows(wins)))
            exp.append(oracle.count_myers(16, km, wins))
        work.append((ac.Jobs(jobs), exp))
    c = ac.ApproxCounter(0)
    try:
        for i in range(calls):
            jobs, exp = work[i % len(work)]
            got = c.count_jobs(16, jobs)
            assert c.stage_mode() == 2, c.stage_mode()
            for g, e in zip(got, exp):
                assert np.array_equal(g, e), i
    finally:
        c.close()


@pytest.mark.parametrize("mode", ["1", "2"])
def test_early_launch_rotating_inputs_bit_exact(mode):
    """The early-launch stage (ac_stage_mode 2): the kernel is launched before the host
    packs (mode 2: after the first job, which the copy kernel sends ahead of it), copies
    each later job into device memory itself once the host flags it, and the host polls the
    generation-tagged counts instead of the stream.  Staging slots alternate between calls, so
    rotating three different workloads through one context makes every call land on a slot
    that last held other data: any stale line read or early completion shows up as a wrong
    count.  In a child process per mode (AC_STAGE_EARLY is read once per process)."""
    env = dict(os.environ, AC_STAGE_EARLY=mode, PYTHONPATH=ROOT)
    code = "from tests.test_gpu_jobs import early_rotation; early_rotation(48); print('OK')"
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=200, cwd=ROOT)
    assert r.returncode == 0 and "OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])


def test_early_launch_unflagged_job_recovers():
    """The early-launch kernel's waits are bounded: a job the host never flags (test-only
    hook, include/approx_counter_amd_testing.h) makes its waves give up after 0.5 s without
    progress and report it; the launch still completes, and the synchronous call runs again
    through the DMA path instead of failing or hanging -- exact counts, ac_stage_mode() 0."""
    from approx_counter_amd import _lib

    a = cases.planted_case(41, 16, 100, 200, win_len=(100, 101))
    b = cases.planted_case(42, 16, 100, 200, win_len=(100, 101))
    jobs = [(a[0], ac.Dna5Sample.from_windows(a[1])), (b[0], ac.Dna5Sample.from_windows(b[1]))]
    L = _lib.load()
    with ac.ApproxCounter(0) as c:
        prev = L.ac_testing_stage_hooks(1)  # AC_TESTING_UNFLAG_LAST
        try:
            got = c.count_jobs(16, jobs)
            assert c.stage_mode() == 0  # the retry's path
        finally:
            L.ac_testing_stage_hooks(prev)
        assert np.array_equal(got[0], oracle.count_myers(16, *a))
        assert np.array_equal(got[1], oracle.count_myers(16, *b))
        got = c.count_jobs(16, jobs)  # hooks off: the early launch again, same context
        assert c.stage_mode() == 2
        assert np.array_equal(got[1], oracle.count_myers(16, *b))


def test_early_launch_slow_host_is_not_a_timeout():
    """a staged launch's waits restart their clock whenever the host makes
    progress, so a call whose packing takes longer than the 0.5 s timeout in total -- a
    large call on one or two CPUs -- is counted, not failed.  The test-only hook
    AC_TESTING_SLOW_HOST makes the publishing thread sleep 60 ms after each of the call's
    first 12 progress records (> 0.7 s in all, every gap far below 0.5 s): the early
    launch must complete by itself (ac_stage_mode 2, no retry), bit-exact."""
    import time

    from approx_counter_amd import _lib

    a = cases.planted_case(51, 16, 300, 6000, win_len=(100, 100), p_n=0.0)
    b = cases.planted_case(52, 16, 200, 6000, win_len=(101, 101), p_n=0.002)
    wa = [(w + "A" * 100)[:100] for w in a[1]]
    wb = [(w + "A" * 101)[:101] for w in b[1]]
    jobs = [(a[0], ac.Dna5Sample.from_windows(wa)), (b[0], ac.Dna5Sample.from_windows(wb))]
    L = _lib.load()
    with ac.ApproxCounter(0) as c:
        c.count_jobs(16, jobs)  # (allocations out of the timed call)
        prev = L.ac_testing_stage_hooks(4)  # AC_TESTING_SLOW_HOST
        try:
            t = time.perf_counter()
            got = c.count_jobs(16, jobs)
            dt = time.perf_counter() - t
            assert c.stage_mode() == 2, "the early launch timed out and was retried"
        finally:
            L.ac_testing_stage_hooks(prev)
    assert dt > 0.6, dt
    assert np.array_equal(got[0], oracle.count_myers(16, a[0], wa))
    assert np.array_equal(got[1], oracle.count_myers(16, b[0], wb))


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


def test_window_count_limit_rejected(counter):
    """The count hand-off keeps a candidate's sum (<= 3 per window) in 32 bits beside the arrival
    count: a segment of 2^32 / 3 windows or more is refused before any launch (AC_ERR_INVALID);
    one window fewer passes the check (here: empty equal windows, so nothing reaches the kernel's
    image).  ADVICE r5."""
    import ctypes

    kmers, wins = cases.planted_case(23, 16, 64, 8, win_len=(100, 100))
    seg = ac.DeviceSegment.upload(kmers, ac.pack_windows(wins))
    limit = (1 << 32) // 3 + 1  # 3 * limit >= 2^32 > 3 * (limit - 1)
    seg.n_windows = limit
    arr = ac.ApproxCounter.segment_array([seg])
    wl = np.zeros(1, np.uint32)  # length-0 windows: every one at base 0, inside any image
    L = counter._L
    st = L.ac_error_count_device(counter.handle, 16, arr, 1, wl.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), 0,
                                 None)
    assert st == 1 and "2^32 / 3" in L.ac_last_error(counter.handle).decode()
    seg.n_windows = len(wins)  # the context still counts afterwards
    counter.count_device(16, [seg])
    counter.check()
    assert np.array_equal(seg.counts_numpy(), oracle.count_myers(16, kmers, wins, 16))


def test_large_call_early_launch_copier_workgroups():
    """A large call (700k windows: 22 MB of staging region, ~5,500 chunks, far more than
    half the workgroups) takes the early launch in one part since round 4: a few copier
    workgroups stage every chunk while the others count windows as their chunks land
    (wm_count.h LaunchArgs::copier_wgs).  Tasks of <= 2,048 windows, progress published
    as they finish; bit-exact on every candidate group's first and last lanes."""
    rng = np.random.default_rng(7)
    n, L = 700_000, 100
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
        assert c.stage_mode() == 2
        again = c.count_jobs(16, [(kmers, sample)])[0]  # the other staging slot
        assert np.array_equal(got, again)
    finally:
        c.close()
    sub = np.r_[0:16, 500:508, 992:1000]  # every candidate group's first and last lanes, and more
    assert np.array_equal(got[sub], oracle.count_myers(16, kmers[sub], win, 16))


def test_large_call_four_jobs_mixed():
    """A large early launch with four jobs (segments): the host packs their tasks interleaved
    and each copier workgroup starts on its own segment (blockIdx mod segments).  Equal
    windows with N (inline records), ragged windows (descriptors sent: the segment waits for
    its whole region), a small job and a job without windows, all in one call -- bit-exact
    on every candidate of the small jobs and on a candidate subset of the large ones."""
    rng = np.random.default_rng(17)
    jobs, exp_fn = [], []
    # 1: 70k equal windows of 100 bases, 0.2 % N
    n1 = 70_000
    w1 = rng.integers(0, 4, size=(n1, 100), dtype=np.uint8)
    w1[rng.random((n1, 100)) < 0.002] = 4
    km1 = np.array([int(sum(int(b) << (2 * (15 - i)) for i, b in enumerate(w1[p, 30:46])))
                    for p in rng.integers(0, n1, size=300)], dtype=np.uint64)
    jobs.append((km1, ac.Dna5Sample(w1.reshape(-1), np.arange(n1, dtype=np.uint64) * np.uint64(100),
                                   np.full(n1, 100, np.uint32))))
    exp_fn.append(lambda sub: oracle.count_myers(16, km1[sub], w1, 16))
    # 2: 50k ragged windows (60-140 bases)
    km2, wins2 = cases.planted_case(71, 16, 200, 50_000, win_len=(60, 140), p_n=0.01)
    km2 = np.asarray(km2, dtype=np.uint64)
    jobs.append((km2, ac.Dna5Sample.from_windows(wins2)))
    exp_fn.append(lambda sub: oracle.count_myers(16, km2[sub], wins2, 16))
    # 3: a small job; 4: candidates without windows
    km3, wins3 = cases.planted_case(72, 16, 90, 700, win_len=(101, 101), p_n=0.01)
    km3 = np.asarray(km3, dtype=np.uint64)
    wins3 = [(w + "A" * 101)[:101] for w in wins3]
    jobs.append((km3, ac.Dna5Sample.from_windows(wins3)))
    exp_fn.append(lambda sub: oracle.count_myers(16, km3[sub], wins3, 16))
    km4 = km3[:40].copy()
    jobs.append((km4, ac.Dna5Sample.from_windows([])))
    exp_fn.append(lambda sub: np.zeros(len(km4[sub]), np.uint64))
    with ac.ApproxCounter(0) as c:
        for _ in range(2):  # both staging slots
            got = c.count_jobs(16, ac.Jobs(jobs))
            assert c.stage_mode() == 2
            for j, (g, f) in enumerate(zip(got, exp_fn)):
                sub = np.arange(len(g)) if len(g) <= 200 else np.r_[0:12, len(g) - 12:len(g)]
                assert np.array_equal(g[sub], f(sub)), j


def test_dma_parts_path_without_early_launch():
    """AC_STAGE_EARLY=0 keeps round 2's copy-engine path: a call of >= 2^17 windows cut
    into parts, each packed and sent while the previous part counts (ac_stage_mode 0), for
    the synchronous call and a submit; ragged windows with N.  In a child process
    (AC_STAGE_EARLY is read once per process)."""
    code = (
        "import numpy as np, torch, approx_counter_amd as ac, oracle\n"
        "from tests import cases\n"
        "km, wins = cases.planted_case(61, 16, 300, 140_000, win_len=(90, 110), p_n=0.002)\n"
        "km2, wins2 = cases.planted_case(62, 16, 200, 10_000, win_len=(101, 101), p_n=0.002)\n"
        "jobs = ac.Jobs([(km, ac.Dna5Sample.from_windows(wins)), (km2, ac.Dna5Sample.from_windows(wins2))])\n"
        "exp = [oracle.count_myers(16, km, wins, 16), oracle.count_myers(16, km2, wins2, 16)]\n"
        "with ac.ApproxCounter(0) as c:\n"
        "    got = c.count_jobs(16, jobs)\n"
        "    assert c.stage_mode() == 0, c.stage_mode()\n"
        "    assert all(np.array_equal(g, e) for g, e in zip(got, exp))\n"
        "    d = torch.full((jobs.n_counts,), -1, dtype=torch.int32, device='cuda')\n"
        "    st = torch.cuda.current_stream()\n"
        "    c.submit_jobs(16, jobs, d, stream=st.cuda_stream)\n"
        "    c.check(stream=st.cuda_stream)\n"
        "    assert c.stage_mode() == 0\n"
        "    assert np.array_equal(d.cpu().numpy().view(np.uint32).astype(np.uint64), np.concatenate(exp))\n"
        "print('OK')\n"
    )
    env = dict(os.environ, AC_STAGE_EARLY="0", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=250, cwd=ROOT)
    assert r.returncode == 0 and "OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])


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


def _permuted_image(wins, seed):
    """A packed image whose window descriptors come in shuffled order, plus one window
    listed twice (overlap): (image, the windows in descriptor order)."""
    img = ac.pack_windows(wins)
    rng = np.random.default_rng(seed)
    order = rng.permutation(len(wins))
    order = np.concatenate([order, order[:1]])
    return (ac.PackedSample(img.codes, img.nmask, img.start[order].copy(), img.length[order].copy(), img.n_bases),
            [wins[i] for i in order])


@pytest.mark.parametrize("n_gpus", [0, 3])
def test_images_fused_and_sharded(n_gpus):
    """ac_error_count_images (the CLI's approximate count): both read ends' host images in
    ONE fused launch per device; on an n_gpus context each end's windows are cut into one
    shard per device and the shard counts summed.  Shuffled and repeated descriptors."""
    a = cases.planted_case(51, 16, 300, 700, win_len=(100, 100), p_n=0.01)
    b = cases.planted_case(52, 16, 200, 600, win_len=(0, 101), p_n=0.01)
    ia, wa = _permuted_image(a[1], 1)
    ib, wb = _permuted_image(b[1], 2)
    with ac.ApproxCounter(0, n_gpus=n_gpus) as c:
        got = c.count_images(16, [(a[0], ia), (b[0], ib)])
    assert np.array_equal(got[0], oracle.count_myers(16, a[0], wa))
    assert np.array_equal(got[1], oracle.count_myers(16, b[0], wb))


def test_samples_two_upload_slots_fused(counter):
    """Both ends uploaded once (slots 0 and 1), the exact count run on each upload, then one
    fused approximate launch over the two device samples (ac_error_count_samples)."""
    a = cases.planted_case(61, 16, 250, 500, win_len=(100, 100), p_n=0.01)
    b = cases.planted_case(62, 22, 120, 400, win_len=(151, 151), p_n=0.01)
    for k, (x, y) in ((16, (a, a)), (22, (b, b))):
        ix, iy = ac.pack_windows(x[1]), ac.pack_windows(y[1][::-1])
        dx = counter.upload_sample(ix, 0)
        dy = counter.upload_sample(iy, 1)
        got = counter.count_samples(k, [(x[0], dx), (y[0][::-1].copy(), dy)])
        assert np.array_equal(got[0], oracle.count_myers(k, x[0], x[1]))
        assert np.array_equal(got[1], oracle.count_myers(k, y[0][::-1].copy(), y[1][::-1]))
