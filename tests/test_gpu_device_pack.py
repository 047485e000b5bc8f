"""GPU parity of device packing (ABI 7): a job whose Dna5 bytes and window offsets
lie in ac_host_alloc memory and whose windows have one length of 1..256 bases is packed by the count
kernel's copier workgroups straight from pinned host memory (ac_stage_mode 3) -- the reference's own
sample shape, every start window sl bases and every end window sl + 1 (approx_counter.cpp:415-476) --
instead of by the host pool.  Every count is checked against the oracle (bit-exact), including
inline N records that overflow, windows straddling staging chunks, windows in any order at any byte
offset, mixed host- and device-packed jobs, and windows reaching past their block (an error)."""
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
AC_TESTING_DEVICE_PACK = 8  # include/approx_counter_amd_testing.h: device packing whatever the call's size


@pytest.fixture(autouse=True)
def _device_pack_every_call():
    """These calls are small (the default policy packs calls under 2^16 windows on the host):
    force device packing for every eligible job while a test runs."""
    from approx_counter_amd import _lib

    L = _lib.load()
    prev = L.ac_testing_stage_hooks(AC_TESTING_DEVICE_PACK)
    yield
    L.ac_testing_stage_hooks(prev)


def _equal(wins, L):
    return [(w + "A" * L)[:L] for w in wins]


def _pinned(wins, seed=0, scatter=False):
    """A pinned Dna5 sample of `wins`; scatter: in shuffled order at odd byte offsets with junk between."""
    if not scatter:
        return ac.Dna5Sample.from_windows(wins).pinned()
    rng = np.random.default_rng(seed)
    arrs = [ac.to_dna5(w) for w in wins]
    buf, offs, pos = [], np.zeros(len(arrs), np.uint64), 0
    for i in rng.permutation(len(arrs)):
        junk = rng.integers(0, 256, size=int(rng.integers(0, 7)), dtype=np.uint8)
        buf.append(junk)
        pos += junk.size
        offs[i] = pos
        buf.append(arrs[i])
        pos += arrs[i].size
    s = ac.Dna5Sample(np.concatenate(buf), offs, np.array([a.size for a in arrs], np.uint32))
    return s.pinned()


@pytest.mark.parametrize("L", [1, 16, 31, 32, 33, 64, 96, 100, 101, 127, 128, 150, 151, 160, 200, 255, 256])
def test_device_pack_every_slot_shape(counter, L):
    """Window lengths across every slot shape: with and without room for an inline N record
    (nrec.h), slots of 32..256 bases, slots that straddle 4 KB staging chunks (160, 200 ...)."""
    k = 16 if L >= 16 else 5
    km, wins = cases.planted_case(1000 + L, k, 300, 1500, win_len=(L, L), p_n=0.02)
    wins = _equal(wins, L)
    km2, wins2 = cases.planted_case(2000 + L, k, 200, 900, win_len=(L, L), p_n=0.0)
    wins2 = _equal(wins2, L)
    got = counter.count_jobs(k, ac.Jobs([(km, _pinned(wins)), (km2, _pinned(wins2))]))
    assert counter.stage_mode() == 3
    assert np.array_equal(got[0], oracle.count_myers(k, km, wins))
    assert np.array_equal(got[1], oracle.count_myers(k, km2, wins2))


@pytest.mark.parametrize("L", [100, 101, 150])
def test_device_pack_record_overflow_and_n_runs(counter, L):
    """Windows with more N than their record holds (their N-bitmap words then come from the bitmap
    the packer stores), runs of N, bytes above 4, and windows that are all N."""
    km, wins = cases.planted_case(3000 + L, 16, 400, 2000, win_len=(L, L), p_n=0.06)
    wins = _equal(wins, L)
    wins[5] = "N" * L
    wins[6] = wins[6][:30] + "N" * 40 + wins[6][70:]
    wins[7] = "N" + wins[7][1:-1] + "N"
    s = ac.Dna5Sample.from_windows(wins)
    b = s.bases.copy()
    b[b == 4] = np.array([4, 5, 77, 255], np.uint8)[np.arange(int((b == 4).sum())) % 4]  # any ordinal >= 4 is N
    got = counter.count_jobs(16, ac.Jobs([(km, ac.Dna5Sample(b, s.offset, s.length).pinned())]))
    assert counter.stage_mode() == 3
    assert np.array_equal(got[0], oracle.count_myers(16, km, wins))


def test_device_pack_scattered_offsets(counter):
    """Windows in any order at unaligned byte offsets, junk bytes between them (a StringSet's
    strings need not be contiguous)."""
    km, wins = cases.planted_case(4000, 16, 500, 3000, win_len=(100, 100), p_n=0.01)
    wins = _equal(wins, 100)
    kb, winb = cases.planted_case(4001, 16, 500, 3000, win_len=(101, 101), p_n=0.01)
    winb = _equal(winb, 101)
    got = counter.count_jobs(16, ac.Jobs([(km, _pinned(wins, 1, True)), (kb, _pinned(winb, 2, True))]))
    assert counter.stage_mode() == 3
    assert np.array_equal(got[0], oracle.count_myers(16, km, wins))
    assert np.array_equal(got[1], oracle.count_myers(16, kb, winb))


def test_device_and_host_packed_jobs_in_one_call(counter):
    """Job 0 pinned (packed on the device), job 1 in ordinary memory (host pool), job 2 pinned but
    ragged (host pool too), job 3 pinned with k-mers but no windows: one fused launch."""
    a = cases.planted_case(5000, 16, 300, 1200, win_len=(100, 100), p_n=0.01)
    b = cases.planted_case(5001, 16, 200, 1100, win_len=(101, 101), p_n=0.01)
    c = cases.planted_case(5002, 16, 150, 800, win_len=(0, 180), p_n=0.01)
    wa, wb = _equal(a[1], 100), _equal(b[1], 101)
    got = counter.count_jobs(16, ac.Jobs([(a[0], _pinned(wa)), (b[0], ac.Dna5Sample.from_windows(wb)),
                                          (c[0], _pinned(c[1])), (a[0][:64], _pinned([]))]))
    assert counter.stage_mode() == 3
    assert np.array_equal(got[0], oracle.count_myers(16, a[0], wa))
    assert np.array_equal(got[1], oracle.count_myers(16, b[0], wb))
    assert np.array_equal(got[2], oracle.count_myers(16, c[0], c[1]))
    assert not got[3].any()


def test_device_pack_k22_and_small_k(counter):
    """P = 1 (k = 22, cfg5's windows of 150 / 151 bases) and P = 4 (k = 8)."""
    for k, L in ((22, 150), (22, 151), (8, 100), (32, 101)):
        km, wins = cases.planted_case(6000 + k + L, k, 700, 1500, win_len=(L, L), p_n=0.01)
        wins = _equal(wins, L)
        got = counter.count_jobs(k, ac.Jobs([(km, _pinned(wins))]))
        assert counter.stage_mode() == 3
        assert np.array_equal(got[0], oracle.count_myers(k, km, wins)), (k, L)


def test_device_pack_window_past_block_is_an_error(counter):
    """A window whose offset points past the end of its pinned block is refused on the device
    (AC_ERR_INVALID, "malformed window"): its bytes are never read (range-checked loads)."""
    km, wins = cases.planted_case(7000, 16, 64, 300, win_len=(100, 100), p_n=0.0)
    wins = _equal(wins, 100)
    s = ac.Dna5Sample.from_windows(wins).pinned()
    bad = ac.Dna5Sample.__new__(ac.Dna5Sample)  # (the constructor's host-side check would refuse it)
    bad.bases, bad.length = s.bases, s.length
    off = ac.pinned_copy(s.offset)
    off[17] = s.bases.size - 50  # reaches 50 bytes past the block
    bad.offset = off
    with pytest.raises(ac.ApproxCounterError) as ei:
        counter.count_jobs(16, ac.Jobs([(km, bad)]))
    assert ei.value.status == 1
    got = counter.count_jobs(16, ac.Jobs([(km, s)]))  # the context still counts afterwards
    assert np.array_equal(got[0], oracle.count_myers(16, km, wins))


def test_device_pack_submit_into_device_tensor(counter):
    import torch

    a = cases.planted_case(8000, 16, 500, 4000, win_len=(100, 100), p_n=0.01)
    b = cases.planted_case(8001, 16, 500, 4000, win_len=(101, 101), p_n=0.01)
    wa, wb = _equal(a[1], 100), _equal(b[1], 101)
    jobs = ac.Jobs([(a[0], _pinned(wa)), (b[0], _pinned(wb))])
    d = torch.zeros(1000, dtype=torch.int32, device="cuda")
    for _ in range(3):
        counter.submit_jobs(16, jobs, d)
    torch.cuda.synchronize()
    counter.check()
    assert counter.stage_mode() == 3
    got = d.cpu().numpy().view(np.uint32).astype(np.uint64)
    assert np.array_equal(got[:500], oracle.count_myers(16, a[0], wa))
    assert np.array_equal(got[500:], oracle.count_myers(16, b[0], wb))


def test_device_pack_large_call():
    """300k windows per end (each end ~30 MB of Dna5 bytes, ~2,300 staging chunks): the copier
    workgroups pack while the others count as chunks land; bit-exact on every candidate group's
    first and last lanes (the oracle over all 500 candidates would take minutes)."""
    from tools.synth import make_windows_fast

    n = 300_000
    wa, _ = make_windows_fast(n, 100, seed=11, at_end=False)
    wb, _ = make_windows_fast(n, 101, seed=12, at_end=True)
    rng = np.random.default_rng(3)
    kms = [rng.integers(0, 1 << 32, size=500, dtype=np.uint64) for _ in range(2)]
    for km, w in zip(kms, (wa, wb)):  # a few real k-mers of the sample among the candidates
        for i in range(0, 500, 50):
            sub = w[i * 7, 10:26]
            if (sub < 4).all():
                km[i] = sum(int(b) << (2 * (15 - j)) for j, b in enumerate(sub))
    jobs = ac.Jobs([(kms[0], ac.Dna5Sample.from_windows(wa).pinned()),
                    (kms[1], ac.Dna5Sample.from_windows(wb).pinned())])
    with ac.ApproxCounter(0) as c:
        got = c.count_jobs(16, jobs)
        assert c.stage_mode() == 3
    pick = sorted({i for g in range(0, 500, 256) for i in (g, g + 1, g + 254, g + 255) if i < 500} | set(range(0, 500, 50)))
    for e, (km, w) in enumerate(zip(kms, (wa, wb))):
        exp = oracle.count_myers(16, km[pick], w, 16)
        assert np.array_equal(got[e][pick], exp), e


def pinned_rotation(calls=24):
    """Rotates pinned (device-packed) and ordinary (host-packed) workloads of different sizes,
    N patterns and lengths through one context, alternating staging slots: a stale line, an early
    completion or a wrong N decision shows up as a wrong count."""
    from approx_counter_amd import _lib

    _lib.load().ac_testing_stage_hooks(AC_TESTING_DEVICE_PACK)
    work = []
    for seed, (nw, L, p_n, pin) in enumerate([(900, 100, 0.0, True), (2500, 101, 0.02, True), (400, 100, 0.01, False),
                                              (6000, 100, 0.07, True), (3000, 150, 0.0, True),
                                              (700, 33, 0.01, False), (5000, 256, 0.03, True)]):
        km, wins = cases.planted_case(9000 + seed, 16, 100 + 50 * seed, nw, win_len=(L, L), p_n=p_n)
        wins = _equal(wins, L)
        smp = _pinned(wins) if pin else ac.Dna5Sample.from_windows(wins)
        work.append((ac.Jobs([(km, smp)]), oracle.count_myers(16, km, wins), pin))
    c = ac.ApproxCounter(0)
    try:
        for i in range(calls):
            jobs, exp, pin = work[i % len(work)]
            got = c.count_jobs(16, jobs)
            assert c.stage_mode() == (3 if pin else 2), (i, c.stage_mode())
            assert np.array_equal(got[0], exp), i
    finally:
        c.close()


def test_device_pack_rotating_inputs_bit_exact():
    code = "from tests.test_gpu_device_pack import pinned_rotation; pinned_rotation(28); print('OK')"
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, PYTHONPATH=ROOT), capture_output=True,
                       text=True, timeout=200, cwd=ROOT)
    assert r.returncode == 0 and "OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])


def test_device_pack_policy_small_call_host_large_call_device():
    """The default policy (no hook): a pinned call under 2^16 windows is packed by the host pool (stage
    mode 2, faster there: DESIGN.md 4d), one of 2^16 windows or more by the kernel (mode 3)."""
    code = ("import numpy as np, approx_counter_amd as ac, oracle\n"
            "from tests import cases\n"
            "km, w = cases.planted_case(9600, 16, 200, 3000, win_len=(100, 100), p_n=0.01)\n"
            "w = [(x + 'A' * 100)[:100] for x in w]\n"
            "big = w * 23\n"  # 69,000 windows
            "c = ac.ApproxCounter(0)\n"
            "g = c.count_jobs(16, ac.Jobs([(km, ac.Dna5Sample.from_windows(w).pinned())]))\n"
            "assert c.stage_mode() == 2, c.stage_mode()\n"
            "e = oracle.count_myers(16, km, w)\n"
            "assert np.array_equal(g[0], e)\n"
            "g = c.count_jobs(16, ac.Jobs([(km, ac.Dna5Sample.from_windows(big).pinned())]))\n"
            "assert c.stage_mode() == 3, c.stage_mode()\n"
            "assert np.array_equal(g[0], 23 * e)\n"
            "c.close(); print('OK')\n")
    env = dict(os.environ, PYTHONPATH=ROOT)
    env.pop("AC_DEVICE_PACK", None)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=200, cwd=ROOT)
    assert r.returncode == 0 and "OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])


def test_device_pack_off_is_the_host_path():
    """AC_DEVICE_PACK=0: the same pinned samples are packed by the host pool (stage mode 2)."""
    code = ("import numpy as np, approx_counter_amd as ac, oracle\n"
            "from tests import cases\n"
            "km, w = cases.planted_case(9500, 16, 300, 2000, win_len=(100, 100), p_n=0.01)\n"
            "w = [(x + 'A' * 100)[:100] for x in w]\n"
            "c = ac.ApproxCounter(0)\n"
            "g = c.count_jobs(16, ac.Jobs([(km, ac.Dna5Sample.from_windows(w).pinned())]))\n"
            "assert c.stage_mode() == 2, c.stage_mode()\n"
            "assert np.array_equal(g[0], oracle.count_myers(16, km, w))\n"
            "c.close(); print('OK')\n")
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, PYTHONPATH=ROOT, AC_DEVICE_PACK="0"),
                       capture_output=True, text=True, timeout=200, cwd=ROOT)
    assert r.returncode == 0 and "OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])
