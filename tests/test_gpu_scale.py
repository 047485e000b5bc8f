"""BASELINE.json configurations 3-5 at full size on the GPU.

cfg3 (k=16, 100k reads, lim=2000) and cfg5 (k=22, sl=150, lim=1000): bit-exact
against the oracle over every candidate, both ends fused in one launch, through
the device-segment entry point and through the host-buffer stage.
cfg4 (k=16, 1M windows per end, lim=500): bit-exact against the oracle over
every candidate and window, plus the shard-accumulation identity."""
import numpy as np
import pytest

import approx_counter_amd as ac
import oracle
from tools import workload

pytestmark = pytest.mark.gpu
THREADS = 16


def fused_counts(counter, k, parts):
    import torch

    segs = [ac.DeviceSegment.upload(km, ac.pack_windows(w)) for km, w in parts]
    counter.count_device(k, segs)
    torch.cuda.synchronize()
    return [s.counts_numpy() for s in segs]


@pytest.mark.parametrize("cfg", [dict(k=16, sn=100_000, sl=100, lim=2000), dict(k=22, sn=100_000, sl=150, lim=1000)],
                         ids=["cfg3", "cfg5"])
def test_full_config_bit_exact(counter, cfg):
    wl, _ = workload.build(n_reads=cfg["sn"], read_len=400, k=cfg["k"], sl=cfg["sl"], lim=cfg["lim"], seed=3)
    parts = [(wl[e]["kmers"], wl[e]["windows"]) for e in ("start", "end")]
    assert all(km.size == cfg["lim"] for km, _ in parts)
    got = fused_counts(counter, cfg["k"], parts)
    staged = counter.count_jobs(cfg["k"], [(km, ac.Dna5Sample.from_windows(w)) for km, w in parts])
    for (km, w), g, s in zip(parts, got, staged):
        exp = oracle.count_myers(cfg["k"], km, w, THREADS)
        assert np.array_equal(g, exp)  # device segments, one fused launch
        assert np.array_equal(s, exp)  # the product stage: Dna5 host buffers -> host counts


def test_cfg4_full_parity_and_shards(counter):
    """cfg4 (k=16, 1M windows per end, 500 candidates): the product stage
    (ac_error_count_jobs, both ends fused) against the oracle over EVERY candidate
    and window (1.005e11 kmer*bp, ~25 s on 16 threads), and 8 window shards
    accumulated on the device equal to the whole (the multi-GPU identity)."""
    import torch

    k, n = 16, 1_000_000
    wl = workload.build_fast(n_reads=n, k=k, sl=100, lim=500, seed=11)
    parts = [(wl[e]["kmers"], wl[e]["windows"]) for e in ("start", "end")]
    assert all(km.size == 500 for km, _ in parts)
    got = counter.count_jobs(k, [(km, ac.Dna5Sample.from_windows(w)) for km, w in parts])
    for (km, w), g in zip(parts, got):
        assert np.array_equal(g, oracle.count_myers(k, km, w, THREADS))
        assert g.max() > n  # adapter k-mers occur in most windows
    for (km, w), g in zip(parts, got):
        bounds = np.linspace(0, n, 9).astype(int)
        acc = ac.DeviceSegment.upload(km, ac.pack_windows(w[bounds[0]:bounds[1]]))
        counter.count_device(k, [acc])
        for i in range(1, 8):
            s = ac.DeviceSegment.upload(km, ac.pack_windows(w[bounds[i]:bounds[i + 1]]))
            s.counts = acc.counts
            counter.count_device(k, [s], accumulate=True)
        torch.cuda.synchronize()
        assert np.array_equal(acc.counts_numpy(), g)


def test_cfg4_submit_in_parts_and_rank_shards(counter):
    """The N > 1 bench path at cfg4 scale: ac_error_count_jobs_submit cuts a large call
    into parts (2M windows: four; one rank's 1/8 shard of 250k windows: two), each packed
    and sent while the previous part counts, the parts adding into the zeroed device
    counts.  The whole call and the sum of the 8 rank shards (strong scaling, one submit
    per shard as bench.py's ranks do) both equal the synchronous stage, which equals the
    oracle (test above; here a candidate subset is re-checked against the oracle)."""
    import torch

    from approx_counter_amd.shard import shard_bounds

    k, n = 16, 1_000_000
    wl = workload.build_fast(n_reads=n, k=k, sl=100, lim=500, seed=12)
    ends = ("start", "end")
    smp = {e: ac.Dna5Sample.from_windows(wl[e]["windows"]) for e in ends}
    whole = counter.count_jobs(k, [(wl[e]["kmers"], smp[e]) for e in ends])
    st = torch.cuda.Stream()
    n_c = sum(wl[e]["kmers"].size for e in ends)
    d = torch.zeros(n_c, dtype=torch.int32, device="cuda")
    jobs = ac.Jobs([(wl[e]["kmers"], smp[e]) for e in ends])
    counter.submit_jobs(k, jobs, d, stream=st.cuda_stream)
    st.synchronize()
    counter.check(stream=st.cuda_stream)
    got = d.cpu().numpy().view(np.uint32).astype(np.uint64)
    assert np.array_equal(got, np.concatenate(whole))
    total = np.zeros(n_c, np.uint64)
    cuts = {e: shard_bounds(smp[e].length.tolist(), 8) for e in ends}
    for r in range(8):
        part = ac.Jobs([(wl[e]["kmers"], smp[e].subset(cuts[e][r], cuts[e][r + 1])) for e in ends])
        d.fill_(-1)
        counter.submit_jobs(k, part, d, stream=st.cuda_stream)
        st.synchronize()
        total += d.cpu().numpy().view(np.uint32).astype(np.uint64)
    counter.check(stream=st.cuda_stream)
    assert np.array_equal(total, np.concatenate(whole))
    sub = slice(0, 40)
    for e, g in zip(ends, whole):
        assert np.array_equal(g[sub], oracle.count_myers(k, wl[e]["kmers"][sub], wl[e]["windows"], THREADS))
