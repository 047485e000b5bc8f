"""Window sharding for multi-GPU counts.

Windows are independent units and counts are integer sums, so the candidate x
window grid splits into contiguous window ranges (balanced by total bases, the
unit of work), one per rank; every rank counts all candidates over its range
and one sum all-reduce of the count vector combines them (RCCL over xGMI on
GPUs, gloo in the CPU tests).  The same balancing is used by the CLI's -g
option (csrc/host/adaptfinder.cpp, error_count).
"""
from __future__ import annotations

from typing import Callable, Sequence

import numpy as np


def shard_bounds(lengths: Sequence[int], n_shards: int) -> list:
    """Cut points c[0]=0 <= ... <= c[n]=len(lengths): shard g = windows [c[g], c[g+1]),
    each holding about 1/n of the total bases (the CLI's rule: cut after the window
    at which the running sum first reaches g/n of the total)."""
    n = len(lengths)
    total = int(np.sum(lengths, dtype=np.int64)) if n else 0
    cuts = [0] + [n] * n_shards
    acc, g = 0, 1
    for i, L in enumerate(lengths):
        if g >= n_shards:
            break
        acc += int(L)
        while g < n_shards and acc * n_shards >= total * g:
            cuts[g] = i + 1
            g += 1
    return cuts


def sharded_count(k: int, kmers, windows, count_fn: Callable, rank: int, world: int, device="cpu"):
    """Count this rank's shard with `count_fn(k, kmers, windows) -> uint64 counts`, then
    sum over ranks with torch.distributed (the default process group).  Returns the
    full count vector (identical on every rank)."""
    import torch
    import torch.distributed as dist

    lengths = [len(w) for w in windows]
    c = shard_bounds(lengths, world)
    part = np.asarray(count_fn(k, kmers, windows[c[rank]:c[rank + 1]]), dtype=np.int64)
    t = torch.from_numpy(part).to(device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().numpy().astype(np.uint64)
