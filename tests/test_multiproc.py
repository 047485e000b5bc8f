"""The N > 1 path on CPU: window shards + sum all-reduce with gloo (world size 2
and 3) give exactly the single-process counts.  The per-shard counter here is
the oracle (tests only); on GPUs it is the HIP kernel (bench.py, CLI -g)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from approx_counter_amd.shard import shard_bounds
from tests import cases


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, k, kmers, windows, out):
    import torch.distributed as dist

    import oracle
    from approx_counter_amd.shard import sharded_count

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        got = sharded_count(k, kmers, windows, lambda kk, km, ws: oracle.count_myers(kk, km, ws, 1), rank, world)
        out[rank] = got.tolist()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_sharded_count_equals_single(world):
    import oracle

    kmers, wins = cases.planted_case(77, 16, 40, 90, win_len=(0, 160), p_n=0.02)
    exp = oracle.count_myers(16, kmers, wins, 1)
    ctx = mp.get_context("spawn")
    with ctx.Manager() as mgr:
        out = mgr.dict()
        port = _free_port()
        procs = [ctx.Process(target=_worker, args=(r, world, port, 16, kmers, wins, out)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(120)
            assert p.exitcode == 0
        for r in range(world):
            assert out[r] == [int(x) for x in exp], r


def test_shard_bounds_balance_and_cover():
    rng = np.random.default_rng(0)
    for n_shards in (1, 2, 3, 8):
        for n in (0, 1, 5, 1000):
            lens = rng.integers(0, 200, size=n)
            c = shard_bounds(lens, n_shards)
            assert c[0] == 0 and c[-1] == n and all(a <= b for a, b in zip(c, c[1:]))
            if n >= 100 and lens.sum():
                sums = [lens[c[g]:c[g + 1]].sum() for g in range(n_shards)]
                assert max(sums) - min(sums) <= 2 * lens.max()
