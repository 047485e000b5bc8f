"""The N > 1 product path with the HIP kernel on every rank: two processes
(gloo, world size 2) share this box's GPU, each counts its contiguous window
shard of both read ends with ac_error_count_jobs_submit (device counts), the
count vectors are summed across ranks, and both ranks hold exactly the oracle's
counts (strong scaling: one sample sharded; approx_counter.cpp:567-597 is the
loop being split)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from tests import cases

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, k, parts, out):
    import torch
    import torch.distributed as dist

    import approx_counter_amd as ac
    from approx_counter_amd.shard import shard_bounds

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = []
        for km, wins in parts:
            c = shard_bounds([len(w) for w in wins], world)
            mine.append((km, ac.Dna5Sample.from_windows(wins[c[rank]:c[rank + 1]])))
        jobs = ac.Jobs(mine)
        with ac.ApproxCounter(0) as counter:
            d = torch.zeros(jobs.n_counts, dtype=torch.int32, device="cuda")
            st = torch.cuda.current_stream()
            counter.submit_jobs(k, jobs, d, stream=st.cuda_stream)
            counter.check(stream=st.cuda_stream)
            host = d.cpu().to(torch.int64)
        dist.all_reduce(host)  # gloo here; RCCL over xGMI in bench.py
        out[rank] = host.tolist()
    finally:
        dist.destroy_process_group()


def test_two_ranks_hip_strong_shards_equal_oracle():
    import oracle

    k = 16
    a = cases.planted_case(5151, k, 300, 900, win_len=(100, 100), p_n=0.01)
    b = cases.planted_case(5152, k, 200, 900, win_len=(101, 101), p_n=0.01)
    exp = [int(x) for x in oracle.count_myers(k, *a)] + [int(x) for x in oracle.count_myers(k, *b)]
    ctx = mp.get_context("spawn")
    with ctx.Manager() as mgr:
        out = mgr.dict()
        port = _free_port()
        procs = [ctx.Process(target=_worker, args=(r, 2, port, k, [a, b], out)) for r in range(2)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(240)
            assert p.exitcode == 0
        for r in range(2):
            assert out[r] == exp, r
