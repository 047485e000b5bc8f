"""The drop-in CLI end to end on an MI355X: every file it writes equals the
golden fixtures (or the oracle pipeline), through the HIP count."""
import json
import os
import subprocess

import pytest

import oracle
from oracle import host_ref

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "approx_counter_amd", "bin", "adaptFinder")
CFG1 = os.path.join(ROOT, "tests", "golden", "cfg1")
P = json.load(open(os.path.join(CFG1, "params.json")))
BASE = [os.path.join(CFG1, "reads.fa"), "-k", P["k"], "-sn", P["n_reads"], "-sl", P["sl"], "-lim", P["lim"]]


def run(args, cwd):
    r = subprocess.run([CLI] + [str(a) for a in args], cwd=cwd, capture_output=True, text=True, timeout=300)
    return r


def golden(name):
    return open(os.path.join(CFG1, name)).read()


def test_cfg1_all_files(tmp_path):
    r = run(BASE + ["-e", "exact", "-o", "out.txt"], tmp_path)
    assert r.returncode == 0, r.stderr
    for name in ("exact_0.start", "exact_0.end", "out.txt_0.start", "out.txt_0.end"):
        assert open(tmp_path / name).read() == golden(name), name


def test_shards_and_multi_run(tmp_path):
    r = run(BASE + ["-g", 3, "-mr", 2, "-o", "o"], tmp_path)  # 3 window shards (wrapping onto this box's GPU)
    assert r.returncode == 0, r.stderr
    for run_id in (0, 1):
        for end in ("start", "end"):
            assert open(tmp_path / f"o_{run_id}.{end}").read() == golden(f"out.txt_0.{end}")


def test_skip_end_quirk(tmp_path):
    # verbose: the loop breaks after the start (approx_counter.cpp:943-948)
    r = run(BASE + ["-se", "-o", "a"], tmp_path)
    assert r.returncode == 0
    assert (tmp_path / "a_0.start").exists() and not (tmp_path / "a_0.end").exists()
    # silent multi-run (mr_v = 0): no break, the second pass re-samples STARTS into .end
    r = run(BASE + ["-se", "-v", 0, "-mr", 2, "-o", "b"], tmp_path)
    assert r.returncode == 0
    assert open(tmp_path / "b_0.end").read() == golden("out.txt_0.start")


def test_solid_mode(tmp_path):
    solid = 40
    r = run(BASE + ["-sk", solid, "-o", "s", "-e", "se"], tmp_path)
    assert r.returncode == 0, r.stderr
    _, seqs = host_ref.read_fasta(os.path.join(CFG1, "reads.fa"))
    for end, bottom in (("start", False), ("end", True)):
        exact, approx, _ = host_ref.run_end(seqs, P["k"], P["sl"], P["lim"], 1.0, bottom, solid=solid)
        assert open(tmp_path / f"se_0.{end}").read() == host_ref.export_lines(exact, P["k"])
        assert open(tmp_path / f"s_0.{end}").read() == host_ref.export_lines(approx, P["k"])


@pytest.mark.parametrize("extra", [
    [],
    ["-lc", "1.5", "-k", 12],
    ["-sk", 25],
    ["-lim", 2000, "-k", 8],
])
def test_gpu_exact_stage_equals_host_stage(tmp_path, extra):
    """The default (GPU exact count + selection, sample uploaded once) writes the same
    files as --host-exact (the reference's host stages, approx_counter.cpp:874-899),
    here with N symbols, forbidden k-mers and FASTQ input."""
    _, seqs = host_ref.read_fasta(os.path.join(CFG1, "reads.fa"))
    with open(tmp_path / "reads.fq", "w") as fh:
        for i, s in enumerate(seqs):
            if i % 7 == 0:
                s = s[:30] + "N" + s[31:]
            if i % 11 == 0:
                s = "A" * 40 + s[40:]  # low-complexity prefix for -lc
            fh.write(f"@r{i}\n{s}\n+\n{'I' * len(s)}\n")
    banned = golden("exact_0.start").splitlines()[2].split("\t")[0]
    (tmp_path / "fk.txt").write_text(banned + "\n")
    args = ["reads.fq", "-k", P["k"], "-sn", P["n_reads"], "-sl", P["sl"], "-lim", P["lim"], "-fk", "fk.txt"] + extra
    a = run(args + ["-e", "ge", "-o", "go"], tmp_path)
    b = run(args + ["-e", "he", "-o", "ho", "--host-exact"], tmp_path)
    assert a.returncode == 0 and b.returncode == 0, (a.stderr, b.stderr)
    assert "A total of" in a.stderr and a.stderr.count("WARNING") == b.stderr.count("WARNING")
    for end in ("start", "end"):
        assert open(tmp_path / f"ge_0.{end}").read() == open(tmp_path / f"he_0.{end}").read(), end
        assert open(tmp_path / f"go_0.{end}").read() == open(tmp_path / f"ho_0.{end}").read(), end
    found = [l for l in a.stdout.splitlines() if "Number of kmer found" in l]
    assert found and [l.split("]")[-1] for l in found] == \
        [l.split("]")[-1] for l in b.stdout.splitlines() if "Number of kmer found" in l]
