"""The fused reader + packer (host_stages read_windows /
sample_windows): the CLI's default path keeps only each read's sampling
windows, packed while parsing.  Its sampled window images must equal, word
for word, those of the reference-shaped path (--host-exact: readRecords
approx_counter.cpp:819-825, sampleSequences 415-476, then packing) for the
same seed, and decode to the oracle's windows.  CPU only (--dump-sample stops
before any GPU work)."""
import os
import random
import subprocess
import zlib

import numpy as np
import pytest

from oracle import host_ref

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "approx_counter_amd", "bin", "adaptFinder")
CFG1 = os.path.join(ROOT, "tests", "golden", "cfg1")


def dump(tmp_path, inp, tag, extra):
    r = subprocess.run([CLI, str(inp), "--dump-sample", str(tmp_path / tag)] + [str(a) for a in extra],
                       cwd=tmp_path, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return sorted(p for p in os.listdir(tmp_path) if p.startswith(tag + "_"))


def load_image(path):
    b = open(path, "rb").read()
    n, n_bases = np.frombuffer(b[:16], np.uint64)
    n, n_bases = int(n), int(n_bases)
    o = 16
    start = np.frombuffer(b[o:o + 8 * n], np.uint64); o += 8 * n
    length = np.frombuffer(b[o:o + 4 * n], np.uint32); o += 4 * n
    codes = np.frombuffer(b[o:o + 4 * (n_bases // 16)], np.uint32); o += 4 * (n_bases // 16)
    nmask = np.frombuffer(b[o:o + 4 * (n_bases // 32)], np.uint32); o += 4 * (n_bases // 32)
    assert o == len(b)
    return start, length, codes, nmask


def decode(img):
    start, length, codes, nmask = img
    out = []
    for s, l in zip(start.tolist(), length.tolist()):
        w = []
        for b in range(s, s + l):
            if (int(nmask[b >> 5]) >> (b & 31)) & 1:
                w.append("N")
            else:
                w.append("ACGT"[(int(codes[b >> 4]) >> (2 * (b & 15))) & 3])
        out.append("".join(w))
    return out


def write_reads(path, seqs, fmt, width=0, crlf=False, lower=False):
    nl = "\r\n" if crlf else "\n"
    with open(path, "w", newline="") as fh:
        for i, s in enumerate(seqs):
            s = s.lower() if lower and i % 2 else s
            if fmt == "fq":
                fh.write(f"@r{i}{nl}{s}{nl}+{nl}{'I' * len(s)}{nl}")
            else:
                fh.write(f">r{i} some description{nl}")
                if width:
                    for j in range(0, len(s), width):
                        fh.write(s[j:j + width] + nl)
                    if not s:
                        fh.write(nl)
                else:
                    fh.write(s + nl)


def rand_reads(seed, n, sl):
    rng = random.Random(seed)
    out = []
    for i in range(n):
        L = rng.choice([0, 5, sl, 2 * sl - 1, 2 * sl, 2 * sl + 1, rng.randint(2 * sl, 6 * sl)])
        s = "".join(rng.choice("ACGTN" if rng.random() < 0.2 else "ACGT") for _ in range(L))
        out.append(s)
    return out


@pytest.mark.parametrize("fmt,width,crlf,lower", [("fa", 0, False, False), ("fa", 60, False, True),
                                                   ("fa", 37, True, False), ("fq", 0, False, True),
                                                   ("fq", 0, True, False)])
def test_fused_images_equal_host_path(tmp_path, fmt, width, crlf, lower):
    sl = 40
    seqs = rand_reads(zlib.crc32(f"{fmt}{width}{crlf}{lower}".encode()), 400, sl)
    inp = tmp_path / f"reads.{fmt}"
    write_reads(inp, seqs, fmt, width, crlf, lower)
    for sn, extra in ((150, ["-mr", 2]), (10**6, [])):
        args = ["-sl", sl, "-k", 8, "-sn", sn, "--seed", 11, "-v", 0] + extra
        a = dump(tmp_path, inp, f"fused{sn}", args)
        b = dump(tmp_path, inp, f"host{sn}", args + ["--host-exact"])
        assert len(a) == len(b) == 2 * (2 if extra else 1)
        for fa, fb in zip(a, b):
            assert open(tmp_path / fa, "rb").read() == open(tmp_path / fb, "rb").read(), fa
        if sn == 10**6:  # every eligible read sampled: the oracle's windows, in shuffled order
            for f in a:
                bottom = f.endswith(".end")
                got = sorted(decode(load_image(tmp_path / f)))
                exp = sorted(w.upper() for w in host_ref.sample_all(seqs, sl, bottom))
                assert got == exp, f


def test_cfg1_and_skip_end_quirk(tmp_path):
    inp = os.path.join(CFG1, "reads.fa")
    # verbose -se stops after the start windows; silent multi-run -se samples starts twice (approx_counter.cpp:943-951)
    for extra, n_files in ((["-se"], 1), (["-se", "-mr", 2, "-v", 0], 4)):
        args = ["-sl", 100, "-sn", 400, "--seed", 3] + extra
        a = dump(tmp_path, inp, "f" + str(len(extra)), args)
        b = dump(tmp_path, inp, "h" + str(len(extra)), args + ["--host-exact"])
        assert [x[1:] for x in a] == [x[1:] for x in b] and len(a) == n_files
        for fa, fb in zip(a, b):
            assert open(tmp_path / fa, "rb").read() == open(tmp_path / fb, "rb").read()


def test_empty_and_unreadable_input(tmp_path):
    (tmp_path / "empty.fa").write_text("")
    names = dump(tmp_path, tmp_path / "empty.fa", "e", ["-sl", 20, "-k", 4])
    for f in names:
        start, length, codes, nmask = load_image(tmp_path / f)
        assert len(start) == 0 and len(codes) == 2 and len(nmask) == 1
    r = subprocess.run([CLI, str(tmp_path / "missing.fa"), "--dump-sample", "x"], capture_output=True, timeout=60)
    assert r.returncode == -6  # uncaught like SeqAn's IOError (test_cli.py)


def chunked_env(threads, min_chunk=2048):
    env = dict(os.environ)
    env.update(AC_READ_THREADS=str(threads), AC_READ_MIN_CHUNK=str(min_chunk), AC_READ_DEBUG="1")
    return env


def dump_env(tmp_path, inp, tag, extra, env):
    r = subprocess.run([CLI, str(inp), "--dump-sample", str(tmp_path / tag), "-v", "0"] + [str(a) for a in extra],
                       cwd=tmp_path, capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr
    if env.get("AC_READ_THREADS", "1") != "1":
        assert "[reader] chunked parse" in r.stderr, r.stderr
    return sorted(p for p in os.listdir(tmp_path) if p.startswith(tag + "_"))


@pytest.mark.parametrize("fmt,width,crlf,at_quality", [("fa", 0, False, False), ("fa", 61, True, False),
                                                        ("fq", 0, False, False), ("fq", 0, True, True)])
def test_chunked_reader_equals_sequential(tmp_path, fmt, width, crlf, at_quality):
    """read_windows with several threads parses chunks that start at guessed
    record boundaries; the result must be the sequential parse's, including
    FASTQ whose quality lines start with '@' (false boundary candidates)."""
    sl = 30
    seqs = rand_reads(zlib.crc32(f"chunk{fmt}{width}{crlf}{at_quality}".encode()), 1500, sl)
    inp = tmp_path / f"reads.{fmt}"
    if fmt == "fq" and at_quality:
        nl = "\r\n" if crlf else "\n"
        with open(inp, "w", newline="") as fh:
            for i, s in enumerate(seqs):
                q = ("@" + "I" * (len(s) - 1)) if s and i % 3 else "I" * len(s)
                fh.write(f"@r{i}{nl}{s}{nl}+{nl}{q}{nl}")
    else:
        write_reads(inp, seqs, fmt, width, crlf)
    args = ["-sl", sl, "-k", 8, "-sn", 10**6, "--seed", 4]
    seq = dump_env(tmp_path, inp, "seq", args, chunked_env(1))
    for t in (2, 7, 16):
        par = dump_env(tmp_path, inp, f"par{t}", args, chunked_env(t))
        assert len(par) == len(seq) == 2
        for a, b in zip(par, seq):
            assert open(tmp_path / a, "rb").read() == open(tmp_path / b, "rb").read(), (t, a)


def test_chunked_reader_falls_back_on_a_false_boundary(tmp_path):
    """Quality lines "@x" followed by an empty-sequence record look like record
    starts to the boundary guess ('+' two lines below, equal lengths); a chunk
    that starts there misparses and the sequential parse is used instead."""
    # 40-byte units after a 36-byte first record: 4 of the 7 chunk starts of an 8-way split land on "@x" lines
    recs = "@pp\n" + "A" * 14 + "\n+\n" + "I" * 14 + "\n"
    recs += "".join(f"@r{i:04d}\nACGTACGTAC\n+\n@xxxxxxxxx\n@s{i:04d}\n+\n" for i in range(3000))
    (tmp_path / "tricky.fq").write_text(recs)
    args = ["-sl", 4, "-k", 4, "-sn", 10**6, "--seed", 2]
    r = subprocess.run([CLI, str(tmp_path / "tricky.fq"), "--dump-sample", str(tmp_path / "par"), "-v", "0"] +
                       [str(a) for a in args], cwd=tmp_path, capture_output=True, text=True, timeout=60,
                       env=chunked_env(8, min_chunk=512))
    assert r.returncode == 0, r.stderr
    assert "not confirmed" in r.stderr, r.stderr
    seq = dump_env(tmp_path, tmp_path / "tricky.fq", "seq", args, chunked_env(1))
    assert len(seq) == 2
    for e in ("start", "end"):
        assert open(tmp_path / f"par_0.{e}", "rb").read() == open(tmp_path / f"seq_0.{e}", "rb").read()
