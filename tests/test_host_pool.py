"""The host work pool that packs the stage's windows (approx_counter_amd/csrc/host_pack.cpp):
every task of every run() runs exactly once, whether workers spin, sleep or arrive late
(CPU only; tools/pool_stress.cpp built with g++)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def stress(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("pool") / "pool_stress")
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-I" + os.path.join(ROOT, "approx_counter_amd", "csrc"),
                    os.path.join(ROOT, "tools", "pool_stress.cpp"),
                    os.path.join(ROOT, "approx_counter_amd", "csrc", "host_pack.cpp"), "-o", exe], check=True)
    return exe


@pytest.mark.parametrize("threads,spin_us,calls", [(8, 2000, 20000), (8, 20, 20000), (4, 0, 5000), (16, 5, 5000)])
def test_every_task_runs_once(stress, threads, spin_us, calls):
    env = dict(os.environ, AC_HOST_SPIN_US=str(spin_us))
    r = subprocess.run([stress, str(threads), str(calls)], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("ok:")
