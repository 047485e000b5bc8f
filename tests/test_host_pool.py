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


@pytest.mark.parametrize("threads,calls,callers,hogs,pin", [
    (8, 3000, 3, 0, 0),    # several contexts' threads sharing host_pool() (the run lock)
    (8, 2000, 2, 8, 1),    # pinned workers under neighbour load: workers descheduled mid-task
    (16, 1000, 4, 4, 1),
])
def test_concurrent_callers_under_load(stress, threads, calls, callers, hogs, pin):
    env = dict(os.environ, AC_HOST_SPIN_US="50")
    r = subprocess.run([stress, str(threads), str(calls), str(callers), str(hogs), str(pin)], env=env,
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("ok:"), r.stdout
