"""CPU oracle for the approximate-count stage of qbonenfant/approx_counter.

TEST INFRASTRUCTURE ONLY: imported by tests/, ``__graft_entry__.smoke()`` and
bench.py's ``cpu_baseline`` leg, never by the product package.

PARITY UNPINNED: the reference ships no tests or fixtures and cannot be built
here (SeqAn 2.4.0+ is absent).  The C library restates
``errorCount`` (approx_counter.cpp:531-601) three ways (see ac_oracle.h); the
Python module :mod:`oracle.host_ref` restates the host stages around it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libac_oracle.so")
_lib = None

DNA5 = {"A": 0, "C": 1, "G": 2, "T": 3}


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        p8 = ctypes.POINTER(ctypes.c_uint8)
        p32 = ctypes.POINTER(ctypes.c_uint32)
        p64 = ctypes.POINTER(ctypes.c_uint64)
        u32 = ctypes.c_uint32
        common = [u32, p64, u32, p8, p64, p32, u32, p64]
        L.oracle_count_dp.argtypes = common
        L.oracle_count_myers.argtypes = common + [ctypes.c_int]
        L.oracle_count_scheme.argtypes = common + [p8, ctypes.c_int]
        L.oracle_distance_dp.argtypes = [ctypes.c_uint64, u32, p8, u32, ctypes.c_int]
        for f in (L.oracle_count_dp, L.oracle_count_myers, L.oracle_count_scheme, L.oracle_distance_dp):
            f.restype = ctypes.c_int
        _lib = L
    return _lib


def _ptr(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


def encode_dna5(seq) -> np.ndarray:
    """SeqAn Dna5 ordinals: A/a 0, C/c 1, G/g 2, T/t (U/u) 3, anything else 4."""
    if isinstance(seq, np.ndarray):
        return seq.astype(np.uint8)
    if isinstance(seq, str):
        seq = seq.encode()
    table = np.full(256, 4, dtype=np.uint8)
    for ch, v in ((b"A", 0), (b"C", 1), (b"G", 2), (b"T", 3), (b"U", 3)):
        table[ch[0]] = v
        table[ch.lower()[0]] = v
    return table[np.frombuffer(bytes(seq), dtype=np.uint8)]


def dna2int(seq: str) -> int:
    """approx_counter.cpp:55-62 (value = value << 2 | ord(c))."""
    v = 0
    for ch in seq:
        v = (v << 2) | DNA5[ch]
    return v


def int2dna(value: int, k: int) -> str:
    """approx_counter.cpp:70-78."""
    return "".join("ACGT"[(value >> (2 * (k - 1 - i))) & 3] for i in range(k))


def _flatten(windows):
    if isinstance(windows, np.ndarray) and windows.ndim == 2:  # equal-length windows, Dna5 ordinals
        n, L = windows.shape
        bases = np.ascontiguousarray(windows, dtype=np.uint8).reshape(-1)
        if bases.size == 0:
            bases = np.zeros(1, dtype=np.uint8)
        return bases, np.arange(n, dtype=np.uint64) * np.uint64(L), np.full(n, L, dtype=np.uint32)
    arrs = [encode_dna5(w) for w in windows]
    lengths = np.array([len(a) for a in arrs], dtype=np.uint32)
    offsets = np.zeros(len(arrs), dtype=np.uint64)
    if len(arrs):
        offsets[1:] = np.cumsum(lengths[:-1], dtype=np.uint64)
    bases = np.concatenate(arrs) if arrs else np.zeros(1, dtype=np.uint8)
    if bases.size == 0:
        bases = np.zeros(1, dtype=np.uint8)
    return np.ascontiguousarray(bases, dtype=np.uint8), offsets, lengths


def _call(fn, k, kmers, windows, *extra):
    kmers = np.ascontiguousarray(np.asarray(kmers, dtype=np.uint64))
    bases, offsets, lengths = _flatten(windows)
    counts = np.zeros(max(len(kmers), 1), dtype=np.uint64)
    kp = _ptr(kmers if len(kmers) else np.zeros(1, np.uint64), ctypes.c_uint64)
    rc = fn(k, kp, len(kmers), _ptr(bases, ctypes.c_uint8),
            _ptr(offsets if len(offsets) else np.zeros(1, np.uint64), ctypes.c_uint64),
            _ptr(lengths if len(lengths) else np.zeros(1, np.uint32), ctypes.c_uint32),
            len(lengths), _ptr(counts, ctypes.c_uint64), *extra)
    if rc != 0:
        raise ValueError(f"oracle rejected arguments (k={k})")
    return counts[: len(kmers)]


def count_dp(k, kmers, windows):
    """Sum over windows of max(0, 3 - d) by plain DP (model M1)."""
    return _call(lib().oracle_count_dp, k, kmers, windows)


def count_myers(k, kmers, windows, n_threads: int = 0):
    """Same as count_dp via Myers' bit-vector; OpenMP over candidates."""
    return _call(lib().oracle_count_myers, k, kmers, windows, n_threads)


def count_scheme(k, kmers, windows, strict: bool = False, return_levels: bool = False):
    """Literal SeqAn 2.4 find<0,2> EditDistance simulation (per-level bitfields)."""
    n = len(kmers) * len(windows)
    levels = np.zeros(max(n, 1), dtype=np.uint8)
    counts = _call(lib().oracle_count_scheme, k, kmers, windows,
                   _ptr(levels, ctypes.c_uint8), 1 if strict else 0)
    if return_levels:
        return counts, levels[:n].reshape(len(kmers), len(windows))
    return counts


def distance(kmer: int, k: int, window) -> int:
    t = encode_dna5(window)
    buf = np.ascontiguousarray(t if t.size else np.zeros(1, np.uint8))
    return lib().oracle_distance_dp(kmer, k, _ptr(buf, ctypes.c_uint8), int(t.size), 3)
