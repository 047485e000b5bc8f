"""The drop-in CLI (bin/adaptFinder) on CPU: argument handling, config
precedence, the exact-count file (written before the approximate count, as
approx_counter.cpp:906-916 does) and the loud failure without a GPU.  The full
run with the HIP count is in tests/test_gpu_cli.py."""
import json
import os
import shutil
import subprocess

import pytest

from oracle import host_ref
from tests import cases

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "approx_counter_amd", "bin", "adaptFinder")
CFG1 = os.path.join(ROOT, "tests", "golden", "cfg1")


def run(args, cwd):
    return subprocess.run([CLI] + [str(a) for a in args], cwd=cwd, capture_output=True, text=True, timeout=120)


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def test_help_and_usage_errors(tmp_path):
    r = run(["--help"], tmp_path)
    assert r.returncode == 0 and "--kmer_size" in r.stdout and "--skip_end" in r.stdout
    assert run([], tmp_path).returncode == 1                       # input filename is required
    assert run(["a.fa", "b.fa"], tmp_path).returncode == 1
    assert run(["a.fa", "-k", "abc"], tmp_path).returncode == 1    # INTEGER option
    assert run(["a.fa", "--no_such_option", "1"], tmp_path).returncode == 1


@pytest.mark.parametrize("args", [["-k", "1"], ["-k", "33"], ["-k", "20", "-sl", "10"]])
def test_invalid_k_aborts_like_reference(tmp_path, args):
    # approx_counter.cpp:781-787 throws std::invalid_argument uncaught -> abort
    r = run([os.path.join(CFG1, "reads.fa")] + args, tmp_path)
    assert r.returncode == -6 and "kmer size must be" in r.stderr


def test_unreadable_input_aborts(tmp_path):
    r = run([str(tmp_path / "missing.fa")], tmp_path)
    assert r.returncode == -6


def _params():
    return json.load(open(os.path.join(CFG1, "params.json")))


@pytest.mark.skipif(_has_gpu(), reason="checks the no-GPU failure path")
def test_exact_file_then_loud_gpu_failure(tmp_path):
    p = _params()
    r = run([os.path.join(CFG1, "reads.fa"), "-k", p["k"], "-sn", p["n_reads"], "-sl", p["sl"], "-lim", p["lim"],
             "-e", "exact", "-o", "out.txt", "--host-exact"], tmp_path)
    assert r.returncode == 1
    assert "no HIP device" in r.stderr
    assert open(tmp_path / "exact_0.start").read() == open(os.path.join(CFG1, "exact_0.start")).read()
    assert not (tmp_path / "out.txt_0.start").exists()


@pytest.mark.skipif(_has_gpu(), reason="checks the no-GPU failure path")
def test_gpu_exact_count_fails_loudly_without_gpu(tmp_path):
    # default: the exact count runs on the GPU too, so nothing is written and no host fallback is taken
    p = _params()
    r = run([os.path.join(CFG1, "reads.fa"), "-k", p["k"], "-sn", p["n_reads"], "-sl", p["sl"], "-lim", p["lim"],
             "-e", "exact", "-o", "out.txt"], tmp_path)
    assert r.returncode == 1
    assert "exact count failed" in r.stderr and "no HIP device" in r.stderr
    assert not (tmp_path / "exact_0.start").exists()
    assert not (tmp_path / "out.txt_0.start").exists()


@pytest.mark.skipif(_has_gpu(), reason="checks the no-GPU failure path")
def test_config_file_and_cli_precedence(tmp_path):
    p = _params()
    conf = tmp_path / "ac.conf"
    # config sets everything; the CLI overrides lim (approx_counter.cpp:744-755)
    conf.write_text(f"# comment\nk = {p['k']}\nsn={p['n_reads']}\nsl={p['sl']}\nlim=7\ne=fromconf\nv=0\n")
    r = run([os.path.join(CFG1, "reads.fa"), "-conf", conf, "-lim", p["lim"], "--host-exact"], tmp_path)
    assert r.returncode == 1
    assert open(tmp_path / "fromconf_0.start").read() == open(os.path.join(CFG1, "exact_0.start")).read()
    assert r.stdout == ""  # v=0 from the config silences the parameter dump


@pytest.mark.skipif(_has_gpu(), reason="checks the no-GPU failure path")
def test_forbidden_kmers_and_fastq(tmp_path):
    p = _params()
    golden = open(os.path.join(CFG1, "exact_0.start")).read().splitlines()
    banned = [golden[0].split("\t")[0], golden[3].split("\t")[0]]
    (tmp_path / "fk.txt").write_text("\n".join(banned) + "\nNNNN\n")
    # same reads as FASTQ
    ids, seqs = host_ref.read_fasta(os.path.join(CFG1, "reads.fa"))
    with open(tmp_path / "reads.fq", "w") as fh:
        for i, s in zip(ids, seqs):
            fh.write(f"@{i}\n{s}\n+\n{'I' * len(s)}\n")
    r = run([tmp_path / "reads.fq", "-k", p["k"], "-sn", p["n_reads"], "-sl", p["sl"], "-lim", p["lim"],
             "-e", "exact", "-fk", "fk.txt", "--host-exact"], tmp_path)
    assert r.returncode == 1
    got = open(tmp_path / "exact_0.start").read().splitlines()
    assert not any(g.split("\t")[0] in banned for g in got)
    # expected: the host restatement with the forbidden set
    exact, _ = host_ref.count_kmers(host_ref.sample_all(seqs, p["sl"], False), p["k"], 1.0,
                                    {cases.kmer_value(b) for b in banned})
    exp = host_ref.export_lines(host_ref.get_most_frequent(exact, p["lim"], p["k"]), p["k"])
    assert "\n".join(got) + "\n" == exp


def test_missing_forbidden_file_exits_1(tmp_path):
    r = run([os.path.join(CFG1, "reads.fa"), "-fk", "nope.txt"], tmp_path)
    assert r.returncode == 1 and "COULD NOT OPEN EXCLUDED KMER FILE" in r.stderr
