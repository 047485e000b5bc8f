"""The bench's vectorized workload builder matches the oracle's host restatement."""
import json
import os

import numpy as np

from oracle import host_ref
from tools import synth, workload

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "cfg1")


def test_exact_topk_matches_host_ref():
    p = json.load(open(os.path.join(GOLDEN, "params.json")))
    _, seqs = host_ref.read_fasta(os.path.join(GOLDEN, "reads.fa"))
    reads = [s.encode() for s in seqs]
    for end, bottom in (("start", False), ("end", True)):
        wins = workload.windows_from_reads(reads, p["sl"], bottom)
        got = workload.exact_topk(wins, p["k"], p["lim"], p["lc"])
        assert host_ref.export_lines(got, p["k"]) == open(os.path.join(GOLDEN, "exact_0." + end)).read()


def test_complexity_matches_scalar():
    rng = np.random.default_rng(3)
    for k in (4, 9, 16, 22, 32):
        km = rng.integers(0, 4 ** min(k, 31), size=200, dtype=np.uint64)
        vec = workload.complexity_f32(km, k)
        for a, b in zip(km, vec):
            assert host_ref.get_complexity(int(a), k) == b


def test_shards_share_adapters():
    r0, a0 = synth.make_reads(50, seed=1)
    r1, a1 = synth.make_reads(50, seed=99, adapter_seed=1)
    assert a0 == a1 and r0 != r1
