"""Pure-Python restatement of approx_counter's host stages (test infrastructure).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Each function cites the
reference lines it restates; the float arithmetic of the low-complexity filter
and of the ranking tie-break is done in IEEE single precision (numpy.float32)
exactly as the C++ does with ``float``.  Used to generate and check the golden
fixtures under tests/golden/ and to check the product's C++ host pipeline.
"""
from __future__ import annotations

import os

import numpy as np

from . import count_myers, encode_dna5, int2dna


def read_fasta(path):
    """Minimal FASTA/FASTQ reader (SeqAn readRecords, approx_counter.cpp:824-825)."""
    ids, seqs = [], []
    with open(path, "rb") as fh:
        data = fh.read().decode()
    lines = data.splitlines()
    if lines and lines[0].startswith("@"):
        for i in range(0, len(lines) - 3, 4):
            ids.append(lines[i][1:])
            seqs.append(lines[i + 1].strip())
        return ids, seqs
    cur = None
    for ln in lines:
        if ln.startswith(">"):
            if cur is not None:
                seqs.append("".join(cur))
            ids.append(ln[1:])
            cur = []
        elif cur is not None:
            cur.append(ln.strip())
    if cur is not None:
        seqs.append("".join(cur))
    return ids, seqs


def sample_all(seqs, sl: int, bottom: bool):
    """sampleSequences (415-476) when sn >= number of eligible reads: every read
    of length >= 2*sl contributes prefix(sl) (466) or suffix from len-1-sl,
    i.e. sl+1 bases (463).  Order is irrelevant downstream."""
    out = []
    for s in seqs:
        if len(s) >= 2 * sl:
            out.append(s[len(s) - 1 - sl:] if bottom else s[:sl])
    return out


def adjust_threshold(c_old: float, k_old: int, k_new: int) -> np.float32:
    """approx_counter.cpp:183-186 (double ratio cast to float, float product)."""
    ratio = np.float32(float((k_new - 2 + 1) ** 2) / float((k_old - 2 + 1) ** 2))
    return np.float32(np.float32(c_old) * ratio)


def get_complexity(kmer: int, k: int) -> np.float32:
    """approx_counter.cpp:247-267 (DUST-like dimer score, float)."""
    counts = [0] * 16
    for _ in range(k - 1):
        counts[kmer & 15] += 1
        kmer >>= 2
    total = sum(v * (v - 1) for v in counts)
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.float32(np.float32(total) / np.float32(2 * (k - 2)))


def have_low_complexity(kmer: int, k: int, threshold) -> bool:
    """approx_counter.cpp:214-234."""
    return bool(get_complexity(kmer, k) >= np.float32(threshold))


def count_kmers(windows, k: int, threshold, forbidden=frozenset()):
    """count_kmers (487-519): exact k-mer counts of N-free, non-low-complexity,
    non-forbidden k-mers; returns (counter dict, number of k-mers with N)."""
    counter = {}
    had_n = 0
    lc_cache = {}
    thr = np.float32(threshold)
    for w in windows:
        codes = encode_dna5(w)
        for i in range(0, len(codes) - k + 1):
            win = codes[i:i + k]
            if (win >= 4).any():
                had_n += 1
                continue
            v = 0
            for c in win:
                v = (v << 2) | int(c)
            lc = lc_cache.get(v)
            if lc is None:
                lc = bool(get_complexity(v, k) >= thr)
                lc_cache[v] = lc
            if not lc and v not in forbidden:
                counter[v] = counter.get(v, 0) + 1
    return counter, had_n


def rank_key(k: int):
    """CompareCount (275-305): count desc, complexity asc, k-mer value desc."""
    def key(item):
        kmer, count = item
        return (-count, float(get_complexity(kmer, k)), -kmer)
    return key


def get_most_frequent(counter: dict, limit: int, k: int):
    """get_most_frequent (396-405)."""
    items = sorted(counter.items(), key=rank_key(k))
    return items[:limit]


def get_solid_kmers(counter: dict, solid: int, k: int):
    """get_solid_kmers (372-388).  The reference sorts by count only with an
    unstable std::sort, so tie order is unspecified there; CompareCount order
    is used here (and in the product) to make it deterministic."""
    return [kv for kv in sorted(counter.items(), key=rank_key(k)) if kv[1] >= solid]


def export_lines(pairs, k: int) -> str:
    """exportCounter (158-174): ``KMER\\tCOUNT\\n`` per entry."""
    return "".join(f"{int2dna(km, k)}\t{c}\n" for km, c in pairs)


def run_end(seqs, k, sl, limit, lc_param=1.0, bottom=False, forbidden=frozenset(), solid=0,
            approx=None):
    """One end of one run (main 858-933) with full sampling.  ``approx`` is a
    callable (k, kmers, windows) -> counts; defaults to the Myers oracle."""
    lc = adjust_threshold(lc_param, 16, k)
    windows = sample_all(seqs, sl, bottom)
    counter, _ = count_kmers(windows, k, lc, forbidden)
    if solid:
        first_n = get_solid_kmers(counter, solid, k)
    else:
        first_n = get_most_frequent(counter, limit, k)
    kmers = [km for km, _ in first_n]
    approx = approx or (lambda kk, km, ws: count_myers(kk, km, ws))
    counts = approx(k, kmers, windows) if kmers else []
    error_counter = {km: int(c) for km, c in zip(kmers, counts)}
    return first_n, get_most_frequent(error_counter, limit, k), windows


# ---- vectorised restatements for full-size samples (cfg4: 10^6 windows, cfg5: k = 22) ----------
# The same functions as count_kmers / get_most_frequent / get_solid_kmers above, on equal windows held
# as one (n, L) array of Dna5 ordinals, in numpy: tests/test_host_full_scale.py checks them against
# the loop restatements at small sizes, then the CLI's host stages (libac_host.so) against them at
# the BASELINE sample sizes.

_DIMER_TABLE = None
_SQ2 = ((np.arange(1 << 16) & 255) ** 2 + (np.arange(1 << 16) >> 8) ** 2).astype(np.int64)  # two byte lanes squared


def _dimer_table():
    """Dimer counts of every 8-base block (16 bits, 7 overlapping dimers): two uint64 words per
    block, one byte lane per dimer value (lanes 0-7 in the first word, 8-15 in the second)."""
    global _DIMER_TABLE
    if _DIMER_TABLE is None:
        v = np.arange(1 << 16, dtype=np.uint64)
        lo = np.zeros(v.size, np.uint64)
        hi = np.zeros(v.size, np.uint64)
        for i in range(7):
            d = (v >> np.uint64(2 * i)) & np.uint64(15)
            lane = np.uint64(1) << ((d & np.uint64(7)) * np.uint64(8))
            low = d < np.uint64(8)
            lo += np.where(low, lane, np.uint64(0))
            hi += np.where(low, np.uint64(0), lane)
        _DIMER_TABLE = (lo, hi)
    return _DIMER_TABLE


def complexity_dense(kmers, k: int) -> np.ndarray:
    """getComplexity (247-267) of every k-mer of a uint64 array, float32.  The k-1 dimers of a k-mer
    (dimer i = bits 2i..2i+3, as the reference reads them) are counted in 16 byte lanes of two uint64
    words (a count is at most k-1 <= 31): whole blocks of 7 dimers through a table of 8-base blocks,
    the rest one dimer at a time; then sum c(c-1) / (2(k-2)) in single precision like the C++."""
    kmers = np.asarray(kmers, dtype=np.uint64)
    out = np.empty(kmers.size, np.float32)
    tlo, thi = _dimer_table()
    one = np.uint64(1)

    def part(s0, s1):
        x = kmers[s0:s1]
        lo = np.zeros(x.size, np.uint64)
        hi = np.zeros(x.size, np.uint64)
        i = 0
        while i + 7 <= k - 1:  # dimers i .. i+6: bases i .. i+7
            blk = ((x >> np.uint64(2 * i)) & np.uint64(0xffff)).astype(np.intp)
            lo += tlo[blk]
            hi += thi[blk]
            i += 7
        for j in range(i, k - 1):
            d = (x >> np.uint64(2 * j)) & np.uint64(15)
            lane = one << ((d & np.uint64(7)) * np.uint64(8))
            low = d < np.uint64(8)
            lo += np.where(low, lane, np.uint64(0))
            hi += np.where(low, np.uint64(0), lane)
        # sum c(c-1) = sum c^2 - (k-1): the squares of two byte lanes at a time through a table
        sq = np.zeros(x.size, np.int64)
        for word in (lo, hi):
            for b in range(4):
                sq += _SQ2[((word >> np.uint64(16 * b)) & np.uint64(0xffff)).astype(np.intp)]
        with np.errstate(divide="ignore", invalid="ignore"):
            out[s0:s1] = (sq - (k - 1)).astype(np.float32) / np.float32(2 * (k - 2))

    step = 1 << 20
    spans = [(s0, min(kmers.size, s0 + step)) for s0 in range(0, kmers.size, step)]
    if len(spans) > 1:  # (numpy releases the GIL in these loops: chunks on a few threads)
        from concurrent.futures import ThreadPoolExecutor

        with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
            list(ex.map(lambda sp: part(*sp), spans))
    else:
        for sp in spans:
            part(*sp)
    return out


def count_kmers_dense(win2d, k: int, threshold, forbidden=()):
    """count_kmers (487-519) over equal windows (an (n, L) uint8 array of Dna5 ordinals): the distinct
    kept k-mers in ascending order, their counts, and the number of k-mer positions skipped for an N.
    Kept = N-free, not getComplexity >= threshold (float32), not forbidden."""
    w = np.ascontiguousarray(win2d, dtype=np.uint8)
    n, L = w.shape
    npos = L - k + 1
    if n == 0 or npos <= 0:
        return np.zeros(0, np.uint64), np.zeros(0, np.uint64), 0
    rows = 1 << 15

    def block(r):
        x = w[r:r + rows]
        isn = x >= 4
        cs = np.concatenate([np.zeros((x.shape[0], 1), np.int32), np.cumsum(isn, axis=1, dtype=np.int32)], axis=1)
        has_n = (cs[:, k:k + npos] - cs[:, :npos]) > 0
        key = np.zeros((x.shape[0], npos), np.uint64)
        c = (x & 3).astype(np.uint64)
        for j in range(k):
            key = (key << np.uint64(2)) | c[:, j:j + npos]
        return key[~has_n], int(has_n.sum())

    from concurrent.futures import ThreadPoolExecutor  # (numpy releases the GIL: row blocks on a few threads)

    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        res = list(ex.map(block, range(0, n, rows)))
    keys = [r[0] for r in res]
    had_n = sum(r[1] for r in res)
    del res
    allk = np.concatenate(keys)
    del keys
    uk, cnt = np.unique(allk, return_counts=True)
    del allk
    keep = ~(complexity_dense(uk, k) >= np.float32(threshold))  # (k = 2: 0/0 is NaN, never low-complexity)
    if len(forbidden):
        keep &= ~np.isin(uk, np.asarray(sorted(forbidden), np.uint64))
    return uk[keep], cnt[keep].astype(np.uint64), had_n


def rank_dense(kmers, counts, limit: int, solid: int, k: int):
    """get_most_frequent (396-405) / get_solid_kmers (372-388) with CompareCount (275-305): count
    descending, getComplexity ascending, k-mer value descending; the first `limit`, or with
    solid > 0 every entry of count >= solid.  Only the entries that can place are sorted: those
    whose count reaches the limit-th largest count."""
    kmers = np.asarray(kmers, np.uint64)
    counts = np.asarray(counts, np.uint64)
    if solid:
        sel = counts >= np.uint64(solid)
    else:
        if kmers.size == 0 or limit == 0:
            return []
        m = min(limit, kmers.size)
        cut = np.partition(counts, counts.size - m)[counts.size - m]
        sel = counts >= cut
    km, ct = kmers[sel], counts[sel]
    order = np.lexsort((~km, complexity_dense(km, k), -ct.astype(np.int64)))
    if not solid:
        order = order[:limit]
    return [(int(a), int(b)) for a, b in zip(km[order], ct[order])]
