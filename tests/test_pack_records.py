"""The host packer of the stage (approx_counter_amd/csrc/host_pack.cpp) on the CPU: 2-bit codes
and N bitmap against the Python packer, and the inline N records of equal windows
(approx_counter_amd/csrc/nrec.h) decoded here independently -- count, positions, the overflow
code and the N-bitmap words an overflowed window keeps -- for the AVX-512, AVX2 and scalar
packers (tools/pack_records.cpp built with g++; the ISA forced at compile time).  Also the span
scan (image bases and the equal-length test) that lays the image out."""
import os
import struct
import subprocess

import numpy as np
import pytest

import approx_counter_amd as ac

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "approx_counter_amd", "csrc")


def _has_avx512():
    try:
        return "avx512bw" in open("/proc/cpuinfo").read()
    except OSError:
        return False


@pytest.fixture(scope="module", params=[2, 1, 0], ids=["avx512", "avx2", "scalar"])
def packer(request, tmp_path_factory):
    if request.param == 2 and not _has_avx512():
        pytest.skip("no AVX-512 on this host")
    exe = str(tmp_path_factory.mktemp("pack") / f"pack_records_{request.param}")
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", f"-DAC_PACK_ISA={request.param}", "-I" + CSRC,
                    os.path.join(ROOT, "tools", "pack_records.cpp"), os.path.join(CSRC, "host_pack.cpp"), "-o", exe],
                   check=True)
    return exe


def _run(exe, tmp_path, windows):
    lens = np.array([w.size for w in windows], np.uint32)
    src, dst = tmp_path / "in.bin", tmp_path / "out.bin"
    with open(src, "wb") as fh:
        fh.write(struct.pack("<I", len(windows)))
        fh.write(lens.tobytes())
        for w in windows:
            fh.write(np.asarray(w, np.uint8).tobytes())
    subprocess.run([exe, str(src), str(dst)], check=True, timeout=60)
    raw = open(dst, "rb").read()
    fp, fr, span, first, diff, nb = struct.unpack_from("<IIQIIQ", raw)
    o = struct.calcsize("<IIQIIQ")
    arr = np.frombuffer(raw, np.uint32, offset=o)
    nc, nm = nb // 16, nb // 32
    return dict(flags_plain=fp, flags_rec=fr, span=span, first=first, diff=diff, n_bases=nb,
                codes=arr[:nc], nmask=arr[nc:nc + nm], codes_rec=arr[nc + nm:2 * nc + nm], nmask_rec=arr[2 * nc + nm:])


def nrec_bits(L):  # nrec.h, restated
    S = (L + 31) & ~31
    pad = S - L
    R = 2 * min(pad, 16)
    pb = 7 if S <= 128 else 8
    return 0 if (L == 0 or L > 256 or R < 3 + pb) else R


def _windows(seed, n, L, n_counts):
    rng = np.random.default_rng(seed)
    w = rng.integers(0, 4, size=(n, L), dtype=np.uint8)
    for i in range(n):
        c = n_counts[i % len(n_counts)]
        pos = rng.choice(L, size=min(c, L), replace=False)
        w[i, pos] = rng.choice([4, 5, 78, 255], size=pos.size)
    return [row for row in w]


@pytest.mark.parametrize("L", [16, 40, 100, 101, 150, 151, 64, 200])
def test_records_and_codes(packer, tmp_path, L):
    wins = _windows(L, 300, L, [0, 1, 2, 0, 3, 4, 5, 7, 0, 1])
    got = _run(packer, tmp_path, wins)
    ref = ac.pack_windows(wins)  # the Python packer (no records)
    assert np.array_equal(got["codes"], ref.codes) and np.array_equal(got["nmask"], ref.nmask)
    assert got["first"] == L and got["diff"] == 0 and got["span"] == len(wins) * ((L + 31) & ~31)
    R = nrec_bits(L)
    S = (L + 31) & ~31
    pb = 7 if S <= 128 else 8
    cap = min(4, (R - 3) // pb) if R else 0
    n_over = sum(1 for w in wins if (w > 3).sum() > cap)
    assert got["flags_plain"] == 1  # some N, no records asked for
    assert got["flags_rec"] == (1 | (2 if n_over and R else 0))  # (no room: plain windows, no overflow)
    words = S // 16
    for i, w in enumerate(wins):
        cw = got["codes_rec"][i * words:(i + 1) * words]
        rec_word = int(cw[-1])
        npos = np.flatnonzero(w > 3)
        # every text base's code unchanged (the record sits in padding only)
        plain = got["codes"][i * words:(i + 1) * words]
        text_mask = [(1 << (2 * min(16, max(0, L - 16 * k)))) - 1 if L - 16 * k < 16 else 0xFFFFFFFF
                     for k in range(words)]
        assert all((int(a) & m) == (int(b) & m) for a, b, m in zip(cw, plain, text_mask)), i
        if not R:  # a plain window: codes, bitmap as without records
            assert np.array_equal(cw, plain), i
            assert np.array_equal(got["nmask_rec"][i * (S // 32):(i + 1) * (S // 32)],
                                  got["nmask"][i * (S // 32):(i + 1) * (S // 32)]), i
            continue
        c = rec_word >> 29
        nm_words = got["nmask_rec"][i * (S // 32):(i + 1) * (S // 32)]
        if npos.size > cap:
            assert c == 7, (i, c)
            assert np.array_equal(nm_words, got["nmask"][i * (S // 32):(i + 1) * (S // 32)]), i
        else:
            assert c == npos.size, (i, c, npos)
            dec = [(rec_word >> (29 - pb * (k + 1))) & ((1 << pb) - 1) for k in range(c)]
            assert dec == list(npos), (i, dec, list(npos))
            if c == 0:
                assert rec_word >> (32 - R) == 0, i


def test_span_scan_ragged_and_edges(packer, tmp_path):
    rng = np.random.default_rng(3)
    for lens in ([0, 0, 5], [33] * 40 + [32], list(rng.integers(0, 300, 77)), [100] * 17, [1]):
        wins = [rng.integers(0, 4, size=int(n), dtype=np.uint8) for n in lens]
        got = _run(packer, tmp_path, wins)
        assert got["span"] == sum((int(n) + 31) // 32 * 32 for n in lens)
        assert got["first"] == lens[0]
        assert (got["diff"] == 0) == (len(set(int(x) for x in lens)) == 1)
        ref = ac.pack_windows(wins)
        n = ref.codes.size
        assert np.array_equal(got["codes"][:n], ref.codes) and np.array_equal(got["nmask"][:ref.nmask.size], ref.nmask)
