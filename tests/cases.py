"""Seeded (k, kmers, windows) cases shared by the oracle and the GPU parity tests."""
from __future__ import annotations

import random

ALPH = "ACGT"


def rand_seq(rng, n, p_n=0.0):
    return "".join("N" if (p_n and rng.random() < p_n) else rng.choice(ALPH) for _ in range(n))


def mutate(rng, s, n_edits):
    s = list(s)
    for _ in range(n_edits):
        op = rng.randrange(3)
        if op == 0 and s:
            s[rng.randrange(len(s))] = rng.choice(ALPH)
        elif op == 1:
            s.insert(rng.randrange(len(s) + 1), rng.choice(ALPH))
        elif s:
            del s[rng.randrange(len(s))]
    return "".join(s)


def kmer_value(s):
    v = 0
    for ch in s:
        v = (v << 2) | ALPH.index(ch)
    return v


def kmer_string(v, k):
    return "".join(ALPH[(v >> (2 * (k - 1 - i))) & 3] for i in range(k))


def planted_case(seed, k, n_kmers, n_windows, win_len=(20, 120), p_n=0.01, p_plant=0.7,
                 max_edits=3):
    """Random candidates and windows; most windows carry a candidate with 0..max_edits
    edits planted at the start, the end or the middle (edges stress end indels)."""
    rng = random.Random(seed)
    kmers = [kmer_value(rand_seq(rng, k)) for _ in range(n_kmers)]
    windows = []
    for _ in range(n_windows):
        L = rng.randint(*win_len)
        w = rand_seq(rng, L, p_n)
        if kmers and rng.random() < p_plant:
            pl = mutate(rng, kmer_string(rng.choice(kmers), k), rng.randint(0, max_edits))
            where = rng.randrange(3)
            if where == 0:
                w = pl + w[len(pl):]
            elif where == 1:
                w = w[: max(0, len(w) - len(pl))] + pl
            else:
                p = rng.randrange(len(w) + 1)
                w = w[:p] + pl + w[p + len(pl):]
        windows.append(w)
    return kmers, windows


def edge_cases():
    """Hand-built edge cases: (name, k, kmers, windows)."""
    k16 = [kmer_value("ACGTACGTTGCAAGCT"), kmer_value("A" * 16), kmer_value("T" * 16)]
    out = [
        ("no_windows", 16, k16, []),
        ("empty_windows", 16, k16, ["", "", ""]),
        ("shorter_than_k", 16, k16, ["ACGTACGTTGCAAG", "ACG", "A" * 13, "A" * 14, "A" * 15]),
        ("exactly_k", 16, k16, ["ACGTACGTTGCAAGCT", "A" * 16, "T" * 15 + "A"]),
        ("all_n", 16, k16, ["N" * 100, "N" * 16]),
        ("n_inside", 16, k16, ["ACGTACGTNGCAAGCT", "ACGTACGTTGCAAGCN", "NCGTACGTTGCAAGCT",
                               "ACGTANNTTGCAAGCT", "AAAAAAAANAAAAAAAA"]),
        ("lowercase_iupac", 16, k16, ["acgtacgttgcaagct", "ACGTRYKMTGCAAGCT"]),
        ("long_window", 16, k16, ["ACGT" * 300 + "ACGTACGTTGCAAGCT"]),
        ("duplicate_kmers", 16, k16 + k16, ["ACGTACGTTGCAAGCT", "AAAAAAAAAAAAAAAAAAAA"]),
        ("k32", 32, [kmer_value("ACGT" * 8), kmer_value("A" * 32)],
         ["ACGT" * 8, "ACGT" * 7 + "ACG", "TTACGT" * 10, "A" * 31]),
        ("k2", 2, [kmer_value("AC"), kmer_value("GG")], ["A", "T", "AC", "GT", "", "N"]),
        ("k3", 3, [kmer_value("ACG"), kmer_value("TTT")], ["A", "AC", "ACG", "TT", "NNN", "CCCC"]),
        ("k4_many", 4, [kmer_value(a + b + c + d) for a in ALPH for b in ALPH for c in ALPH for d in ALPH],
         ["ACGTTGCA", "AAAA", "N", "GATTACA", "CCCCCCCCCCCCCCCCCCCCCCCCCCCCCCCCC"]),
    ]
    return out
