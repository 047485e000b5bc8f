"""Seeded synthetic nanopore-like reads.

Used by bench.py and by the golden-fixture generator; not part of the product.
Reads: ``n_reads`` reads of ``read_len`` iid uniform ACGT bases, a fraction
``p_n`` replaced by N.  Two random 28-bp adapters are drawn from the seed;
60 % of reads get the start adapter at offset U[0,5), 60 % get the end adapter
ending U[0,5) before the 3' end.  Each planted copy receives 0/1/2 random edits
(p = 0.5/0.3/0.2; substitution/insertion/deletion equiprobable).  The read
length stays ``read_len`` (planted copies overwrite bases; an insertion or
deletion in a copy is absorbed by trimming/padding the flank), so every read is
eligible for sampling whenever ``read_len >= 2*sl``.
"""
from __future__ import annotations

import numpy as np

ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)


def _edit(rng, seq: np.ndarray) -> np.ndarray:
    n_ed = rng.choice(3, p=[0.5, 0.3, 0.2])
    s = seq.copy()
    for _ in range(n_ed):
        op = rng.integers(3)
        if op == 0:
            i = rng.integers(len(s))
            s[i] = ACGT[rng.integers(4)]
        elif op == 1:
            i = rng.integers(len(s) + 1)
            s = np.insert(s, i, ACGT[rng.integers(4)])
        elif len(s) > 1:
            i = rng.integers(len(s))
            s = np.delete(s, i)
    return s


def make_reads(n_reads: int, read_len: int = 400, seed: int = 1, p_n: float = 0.001,
               adapters: bool = True, adapter_len: int = 28, p_adapter: float = 0.6,
               adapter_seed=None):
    """Return (list of read byte strings, (start_adapter, end_adapter)).
    ``adapter_seed`` (default: ``seed``) draws the adapters from another seed so
    that shards generated with different seeds share one adapter pair."""
    rng = np.random.default_rng(seed)
    if adapter_seed is None or adapter_seed == seed:
        arng = rng
        reads = ACGT[rng.integers(0, 4, size=(n_reads, read_len))]
    else:
        arng = np.random.default_rng(adapter_seed)
        arng.integers(0, 4, size=(n_reads, read_len))  # keep the adapter draw aligned with `seed`
        reads = ACGT[rng.integers(0, 4, size=(n_reads, read_len))]
    if p_n > 0:
        reads[rng.random(size=reads.shape) < p_n] = ord("N")
    if arng is not rng:
        arng.random(size=reads.shape)
    a_start = ACGT[arng.integers(0, 4, size=adapter_len)]
    a_end = ACGT[arng.integers(0, 4, size=adapter_len)]
    if adapters:
        for r in range(n_reads):
            if rng.random() < p_adapter:
                cp = _edit(rng, a_start)
                off = int(rng.integers(0, 5))
                n = min(len(cp), read_len - off)
                reads[r, off:off + n] = cp[:n]
            if rng.random() < p_adapter:
                cp = _edit(rng, a_end)
                gap = int(rng.integers(0, 5))
                end = read_len - gap
                n = min(len(cp), end)
                reads[r, end - n:end] = cp[len(cp) - n:]
    return [bytes(row) for row in reads], (bytes(a_start), bytes(a_end))


def write_fasta(path: str, reads, width: int = 0) -> None:
    with open(path, "wb") as fh:
        for i, r in enumerate(reads):
            fh.write(b">read_%d\n" % i)
            if width:
                for j in range(0, len(r), width):
                    fh.write(r[j:j + width] + b"\n")
            else:
                fh.write(r + b"\n")


def make_windows_fast(n: int, length: int, seed: int = 1, p_n: float = 0.001, adapter_len: int = 28,
                      p_adapter: float = 0.6, max_subs: int = 2, at_end: bool = False):
    """Vectorised equal-length windows for the 1M-window scale tests (Dna5 ordinals,
    shape (n, length)).  Like make_reads' read ends but with substitution-only
    adapter copies (0..max_subs per copy) so no per-read Python loop is needed."""
    rng = np.random.default_rng(seed)
    w = rng.integers(0, 4, size=(n, length), dtype=np.uint8)
    adapter = rng.integers(0, 4, size=adapter_len, dtype=np.uint8)
    rows = np.nonzero(rng.random(n) < p_adapter)[0]
    off = rng.integers(0, 5, size=rows.size)
    cols = (length - adapter_len - off)[:, None] + np.arange(adapter_len) if at_end else \
        off[:, None] + np.arange(adapter_len)
    cp = np.broadcast_to(adapter, (rows.size, adapter_len)).copy()
    for _ in range(max_subs):
        hit = rng.random(rows.size) < 0.4
        pos = rng.integers(0, adapter_len, size=rows.size)
        cp[hit, pos[hit]] = rng.integers(0, 4, size=int(hit.sum()), dtype=np.uint8)
    w[rows[:, None], cols] = cp
    w[rng.random(size=w.shape) < p_n] = 4
    return w, adapter
