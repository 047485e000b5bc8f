"""Pure-Python restatement of approx_counter's host stages (test infrastructure).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Each function cites the
reference lines it restates; the float arithmetic of the low-complexity filter
and of the ranking tie-break is done in IEEE single precision (numpy.float32)
exactly as the C++ does with ``float``.  Used to generate and check the golden
fixtures under tests/golden/ and to check the product's C++ host pipeline.
"""
from __future__ import annotations

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
