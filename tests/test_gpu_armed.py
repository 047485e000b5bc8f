"""Armed launches (ABI 5; opt-in: AC_ARM_US > 0): a synchronous ac_error_count_jobs
call whose shape repeats the previous call's enqueues the NEXT call's staged count kernel behind its
own; the next call of that shape takes it over, anything else cancels it, and it gives up by itself
after AC_ARM_US microseconds without a call.  Every path -- taken over, expired, cancelled, and the
race between an expiry and a call -- must give the oracle's counts (errorCount,
approx_counter.cpp:531-601).  Each test runs in a child process with AC_ARM_US set (read once per
process)."""
import os
import subprocess
import sys
import time

import numpy as np
import pytest

import approx_counter_amd as ac
import oracle
from tests import cases

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def same_shape_workloads(n_work=3, nw=1200, n_k=300, L=(100, 101), seed=70):
    """Workloads of one shape (two ends: n_k candidates each, nw windows of L[0] / L[1] bases) and
    different data: other k-mers, other windows, N in some windows (inside their inline records),
    one with an N-only window -- so a kernel counting a stale slot or a stale generation shows."""
    work = []
    for w in range(n_work):
        jobs, exp = [], []
        for j, ln in enumerate(L):
            km, wins = cases.planted_case(seed + 10 * w + j, 16, n_k, nw, win_len=(ln, ln), p_n=0.01 * (w % 2))
            wins = [(x + "A" * ln)[:ln] for x in wins]
            if w == 2:
                wins[nw // 2] = "N" * ln
            jobs.append((km, ac.Dna5Sample.from_windows(wins)))
            exp.append(oracle.count_myers(16, km, wins))
        work.append((ac.Jobs(jobs), exp))
    return work


def _check(got, exp, tag):
    for g, e in zip(got, exp):
        assert np.array_equal(g, e), tag


def armed_taken_over():
    """Back-to-back calls of one shape: from the third call on each call's kernel was enqueued by
    the call before (taken over), with the data of three workloads rotating through the two
    slots -- bit-exact every time, and the early-launch mode reported."""
    work = same_shape_workloads()
    with ac.ApproxCounter(0) as c:
        for i in range(40):
            jobs, exp = work[i % len(work)]
            _check(c.count_jobs(16, jobs), exp, i)
            assert c.stage_mode() == 2
        enq, taken, expired, cancelled = c.arm_stats()
        assert enq >= 38 and taken >= 30, (enq, taken, expired, cancelled)
        c.idle()
        assert c.arm_stats()[3] == cancelled + 1  # the last call's armed launch, cancelled


def armed_expires():
    """A call that comes after the armed launch gave up (AC_ARM_US, default 100 us) launches its
    own kernel: counted the same."""
    work = same_shape_workloads(n_work=2, nw=800, n_k=200, seed=90)
    with ac.ApproxCounter(0) as c:
        for i in range(12):
            if i >= 2:
                time.sleep(0.003)  # well past the idle limit
            jobs, exp = work[i % 2]
            _check(c.count_jobs(16, jobs), exp, i)
        enq, taken, expired, _ = c.arm_stats()
        assert expired >= 5 and taken == 0, c.arm_stats()


def armed_cancelled():
    """An armed launch is cancelled by a call of another shape, by any other entry point (device
    count, exact count, submit) and by ac_idle; every result stays exact and nothing waits on the
    cancelled kernel."""
    import torch

    work = same_shape_workloads(n_work=2, nw=600, n_k=150, seed=110)
    a = cases.planted_case(131, 16, 90, 700, win_len=(90, 120), p_n=0.01)  # another shape (ragged)
    ja = ac.Jobs([(a[0], ac.Dna5Sample.from_windows(a[1]))])
    ea = oracle.count_myers(16, *a)
    with ac.ApproxCounter(0) as c:
        def arm():
            for i in range(3):
                jobs, exp = work[i % 2]
                _check(c.count_jobs(16, jobs), exp, ("arm", i))
            assert c.arm_stats()[0] >= 1
        arm()
        _check(c.count_jobs(16, ja), [ea], "other shape")
        arm()
        got = c.count(16, a[0], ac.pack_windows(a[1]))  # the one-call device path
        assert np.array_equal(got, ea)
        arm()
        got, _, _ = c.exact_count(16, ac.pack_windows(a[1]), 1.0, (), 10**6)  # the exact count
        assert len(got) > 0
        arm()
        d_counts = torch.zeros(sum(len(e) for e in work[0][1]), dtype=torch.int32, device="cuda")
        stream = torch.cuda.current_stream()
        c.submit_jobs(16, work[0][0], d_counts, stream=stream.cuda_stream)
        stream.synchronize()
        got = d_counts.cpu().numpy().astype(np.uint32)
        _check(np.split(got, [len(work[0][1][0])]), work[0][1], "submit")
        arm()
        c.idle()
        t = time.perf_counter()
        torch.cuda.synchronize()
        assert time.perf_counter() - t < 0.05
        cancelled = c.arm_stats()[3]
        assert cancelled >= 4, c.arm_stats()
        _check(c.count_jobs(16, work[1][0]), work[1][1], "after idle")


def _child(code, us="100"):
    env = dict(os.environ, AC_ARM_US=us, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", code + "; print('OK')"], env=env, capture_output=True, text=True,
                       timeout=200, cwd=ROOT)
    assert r.returncode == 0 and "OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])
    return r.stdout


def test_armed_launch_taken_over_rotating_data():
    _child("from tests.test_gpu_armed import armed_taken_over; armed_taken_over()")


def test_armed_launch_expires_then_call_runs_its_own():
    _child("from tests.test_gpu_armed import armed_expires; armed_expires()")


def test_armed_launch_cancelled_by_other_shapes_and_entry_points():
    _child("from tests.test_gpu_armed import armed_cancelled; armed_cancelled()")


def armed_race(calls=300):
    """Calls of one shape with the idle limit set so short (AC_ARM_US in the environment) that the
    armed kernel gives up while the call is publishing: the handshake decides, and either way the
    counts are exact."""
    work = same_shape_workloads(n_work=3, nw=400, n_k=128, seed=150)
    with ac.ApproxCounter(0) as c:
        for i in range(calls):
            jobs, exp = work[i % len(work)]
            _check(c.count_jobs(16, jobs), exp, i)
            if i % 7 == 3:
                time.sleep(float(os.environ.get("AC_ARM_US", "5")) * 1e-6)
        print("STATS", c.arm_stats())


@pytest.mark.parametrize("us", ["2", "8", "30"])
def test_armed_launch_expiry_race_is_exact(us):
    out = _child("from tests.test_gpu_armed import armed_race; armed_race()", us)
    stats = eval(out.split("STATS", 1)[1].splitlines()[0])
    assert stats[0] >= 250 and stats[1] + stats[2] >= 250, stats


def armed_off():
    w = same_shape_workloads(n_work=2, nw=300, n_k=64, seed=170)
    with ac.ApproxCounter(0) as c:
        for i in range(6):
            _check(c.count_jobs(16, w[i % 2][0]), w[i % 2][1], i)
        print("STATS", c.arm_stats())


@pytest.mark.parametrize("us", ["0", None])
def test_armed_launch_off_by_default_and_with_zero(us):
    """The default (no AC_ARM_US) and AC_ARM_US=0 never arm."""
    env = dict(os.environ, PYTHONPATH=ROOT)
    env.pop("AC_ARM_US", None)
    if us is not None:
        env["AC_ARM_US"] = us
    r = subprocess.run([sys.executable, "-c", "from tests.test_gpu_armed import armed_off; armed_off(); print('OK')"],
                       env=env, capture_output=True, text=True, timeout=200, cwd=ROOT)
    assert r.returncode == 0 and "OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])
    assert "STATS (0, 0, 0, 0)" in r.stdout
