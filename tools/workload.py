"""Benchmark workload: synthetic reads -> sampled windows -> top-`lim` candidates.

Vectorized (numpy) host stages used only to SET UP bench.py's input (they are
outside the timed approximate-count stage): sampling with sn >= reads
(approx_counter.cpp:415-476), exact k-mer count with the low-complexity and N
filters (487-519, float32 DUST score 214-234) and get_most_frequent's
CompareCount order (275-305, 396-405).  tests/test_workload.py checks them
against oracle.host_ref on the config-1 fixture.
"""
from __future__ import annotations

import numpy as np

from tools.synth import make_reads, make_windows_fast

_LUT = np.full(256, 4, dtype=np.uint8)
for _c, _v in ((b"A", 0), (b"C", 1), (b"G", 2), (b"T", 3), (b"U", 3)):
    _LUT[_c[0]] = _v
    _LUT[_c.lower()[0]] = _v


def windows_from_reads(reads, sl: int, bottom: bool):
    """Dna5 windows of every read with len >= 2*sl (sn >= #reads)."""
    out = []
    for r in reads:
        a = _LUT[np.frombuffer(r, dtype=np.uint8)]
        if a.size >= 2 * sl:
            out.append(a[a.size - 1 - sl:] if bottom else a[:sl])
    return out


def complexity_f32(kmers: np.ndarray, k: int) -> np.ndarray:
    """getComplexity (247-267) for an array of k-mers, float32."""
    counts = np.zeros((kmers.size, 16), dtype=np.int64)
    v = kmers.copy()
    rows = np.arange(kmers.size)
    for _ in range(k - 1):
        np.add.at(counts, (rows, (v & np.uint64(15)).astype(np.int64)), 1)
        v >>= np.uint64(2)
    s = (counts * (counts - 1)).sum(axis=1)
    with np.errstate(divide="ignore", invalid="ignore"):
        return s.astype(np.float32) / np.float32(2 * (k - 2))


def adjust_threshold(c_old: float, k_old: int, k_new: int) -> np.float32:
    return np.float32(np.float32(c_old) * np.float32(((k_new - 1) ** 2) / ((k_old - 1) ** 2)))


def exact_topk(windows, k: int, limit: int, lc_param: float = 1.0):
    """count_kmers + get_most_frequent: list of (kmer, count), CompareCount order."""
    vals = []
    for w in windows:
        n = w.size - k + 1
        if n <= 0:
            continue
        idx = np.arange(n)[:, None] + np.arange(k)[None, :]
        sub = w[idx]
        ok = (sub < 4).all(axis=1)
        sub = sub[ok].astype(np.uint64)
        shifts = (2 * (k - 1 - np.arange(k))).astype(np.uint64)
        vals.append((sub << shifts[None, :]).sum(axis=1, dtype=np.uint64))
    if not vals:
        return []
    allv = np.concatenate(vals)
    uniq, cnt = np.unique(allv, return_counts=True)
    lc = adjust_threshold(lc_param, 16, k)
    comp = complexity_f32(uniq, k)
    keep = ~(comp >= lc)
    uniq, cnt, comp = uniq[keep], cnt[keep], comp[keep]
    # CompareCount: count desc, complexity asc, value desc  (lexsort: last key primary)
    order = np.lexsort((np.iinfo(np.uint64).max - uniq, comp, -cnt))
    top = order[:limit]
    return [(int(uniq[i]), int(cnt[i])) for i in top]


def build(n_reads: int = 10_000, read_len: int = 400, k: int = 16, sl: int = 100, lim: int = 500,
          seed: int = 1, shard: int = 0, n_shards: int = 1):
    """Config-2-shaped workload.  With n_shards > 1 (weak scaling), shard r gets its own
    n_reads reads (seed + r) carrying the same adapters; candidates are the top-`lim` of
    shard 0's sample for every shard, so all ranks count the same candidate vector."""
    reads0, adapters = make_reads(n_reads, read_len=read_len, seed=seed)
    reads = reads0 if shard == 0 else make_reads(n_reads, read_len=read_len, seed=seed + 7919 * shard,
                                                  adapter_seed=seed)[0]
    out = {}
    for end, bottom in (("start", False), ("end", True)):
        cand = exact_topk(windows_from_reads(reads0, sl, bottom), k, lim)
        out[end] = {"kmers": np.array([km for km, _ in cand], dtype=np.uint64),
                    "windows": windows_from_reads(reads, sl, bottom)}
    return out, adapters


def build_fast(n_reads: int = 1_000_000, k: int = 16, sl: int = 100, lim: int = 500, seed: int = 1,
               cand_windows: int = 20_000):
    """The 1M-read (cfg4) workload, vectorised: each end's windows as one (n, L) Dna5
    array (make_windows_fast: substitution-only adapter copies, 0.1 % N); candidates =
    the top-`lim` of an exact count over the first `cand_windows` windows of that end
    (the full-sample exact count is outside the approximate-count stage and would
    dominate set-up time).  Identical on every rank for a given seed, so ranks can
    take their shard of one sample (strong scaling)."""
    out = {}
    for end, L, bottom, sd in (("start", sl, False, seed * 2), ("end", sl + 1, True, seed * 2 + 1)):
        w, _ = make_windows_fast(n_reads, L, seed=sd, at_end=bottom)
        cand = exact_topk(list(w[:cand_windows]), k, lim)
        out[end] = {"kmers": np.array([km for km, _ in cand], dtype=np.uint64), "windows": w}
    return out
