"""The exact path bench.py times, at the size it times it, against the oracle.

bench.py's `value` is `ac_error_count_jobs` on cfg2 (k=16, 2 x 10k windows of
100 / 101 bases, 0.1 % N, 500 candidates per end, seed 1): the early launch
(`ac_stage_mode() == 2`: the host pool packs a cfg2 call, on ordinary or pinned memory; a pinned
call of >= 2^16 windows, such as one rank's cfg4 shard, is packed by the kernel's copier workgroups
themselves, `== 3`), i.e. `wm2_count_kernel<2, STAGED, EQ>` staging its own inputs.  Its N > 1 steps go through
`ac_error_count_jobs_submit` on one rank's shard.  Both are checked here over
EVERY candidate and window against `oracle.count_myers` (errorCount,
approx_counter.cpp:531-601), on the very workload objects bench.py builds
(`bench.build_workload`), so the timed path and the checked path are one."""
import argparse

import numpy as np
import pytest

import approx_counter_amd as ac
import bench
import oracle

pytestmark = pytest.mark.gpu
THREADS = 16
ENDS = ("start", "end")


def _bench_args(config, **over):
    a = argparse.Namespace(**{"read_len": 400, "seed": 1, **bench.CONFIGS[config], **over})
    a.read_len = max(a.read_len, 2 * a.sl)
    return a


def _expected(k, wl):
    return [oracle.count_myers(k, wl[e]["kmers"], wl[e]["windows"], THREADS) for e in ENDS]


def _samples(wl, where):
    smp = [ac.Dna5Sample.from_windows(wl[e]["windows"]) for e in ENDS]
    return [x.pinned() for x in smp] if where == "pinned" else smp


@pytest.mark.parametrize("where", ["pinned", "heap"])
def test_bench_cfg2_stage_bit_exact(where):
    """cfg2 as bench.py times it: the synchronous early launch, 6 calls on one context (both
    staging slots, three times each), then the submit form the N > 1 steps use; on the sample in
    pinned memory (device packing, bench --sample pinned, the default) and in ordinary memory."""
    mode = 2  # (cfg2's 20k windows are host-packed on pinned memory too: the default policy)
    import torch

    args = _bench_args("cfg2")
    wl, units = bench.build_workload(args, 0, 1)
    assert [wl[e]["kmers"].size for e in ENDS] == [500, 500]
    assert [len(wl[e]["windows"]) for e in ENDS] == [10_000, 10_000]
    assert units == sum(500 * sum(int(w.size) for w in wl[e]["windows"]) for e in ENDS)
    exp = _expected(16, wl)
    jobs = ac.Jobs([(wl[e]["kmers"], smp) for e, smp in zip(ENDS, _samples(wl, where))])
    with ac.ApproxCounter(0) as c:
        for i in range(6):
            got = c.count_jobs(16, jobs)
            assert c.stage_mode() == mode, c.stage_mode()  # the early launch, as timed
            for e, g, x in zip(ENDS, got, exp):
                assert np.array_equal(g, x), (i, e)
        out = torch.full((jobs.n_counts,), -1, dtype=torch.int32, device="cuda")
        st = torch.cuda.current_stream()
        for _ in range(3):
            c.submit_jobs(16, jobs, out, stream=st.cuda_stream)
        c.check(stream=st.cuda_stream)
        assert c.stage_mode() == mode
        got = out.cpu().numpy().view(np.uint32).astype(np.uint64)
        assert np.array_equal(got, np.concatenate(exp))


@pytest.mark.parametrize("where", ["pinned", "heap"])
@pytest.mark.parametrize("rank", [0, 7])
def test_bench_cfg4_rank_shard_submit_bit_exact(rank, where):
    """One rank's 1/8 shard of cfg4 (strong scaling, 2 x 125k windows) through
    ac_error_count_jobs_submit, as bench.py's N = 8 step issues it, over every
    candidate of both ends against the oracle on the shard's own windows."""
    import torch

    args = _bench_args("cfg4")
    wl, _ = bench.build_workload(args, rank, 8)
    assert all(abs(len(wl[e]["windows"]) - 125_000) < 100 for e in ENDS)
    exp = _expected(16, wl)
    jobs = ac.Jobs([(wl[e]["kmers"], smp) for e, smp in zip(ENDS, _samples(wl, where))])
    with ac.ApproxCounter(0) as c:
        out = torch.full((jobs.n_counts,), -1, dtype=torch.int32, device="cuda")
        st = torch.cuda.current_stream()
        for _ in range(2):
            c.submit_jobs(16, jobs, out, stream=st.cuda_stream)
        c.check(stream=st.cuda_stream)
        assert c.stage_mode() == (3 if where == "pinned" else 2)  # (250k windows: device-packed when pinned)
        got = out.cpu().numpy().view(np.uint32).astype(np.uint64)
        assert np.array_equal(got, np.concatenate(exp))
        sync = c.count_jobs(16, jobs)
        for g, x in zip(sync, exp):
            assert np.array_equal(g, x)


def test_bench_line_reports_the_pool_that_ran():
    """bench.py's host_pool record is read after the first stage call made the pool, so a pool sized
    by AC_HOST_THREADS is reported as such (the shard projection's line said 16 for a
    2-thread pool), and config.stage names the launch as issued first in the call."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    # (a 1-participant pool -- an 8-rank node's share -- still host-packs cfg2 on pinned memory: the
    # device-pack policy is by call size only)
    for threads, sample, dp, path, text in ((3, "heap", "", "early-launch", "issued first in the call"),
                                            (3, "pinned", "", "early-launch", "issued first in the call"),
                                            (1, "pinned", "", "early-launch", "issued first in the call"),
                                            (3, "pinned", "1", "early-launch-device-pack", "the host packs nothing")):
        r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "3", "--warmup", "1",
                            "--no-cpu-baseline", "--no-pipelined", "--no-kernel-leg", "--no-exact", "--sample", sample],
                           env=dict(os.environ, AC_HOST_THREADS=str(threads), AC_DEVICE_PACK=dp),
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
        assert line["host_pool"]["participants"] == threads
        assert line["config"]["stage_path"] == path and text in line["config"]["stage"]
        assert "armed_launch" not in line and "cgroup_cpu" in line
