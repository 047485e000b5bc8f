"""bench.py's driver contract, checked on CPU: the default workload is BASELINE.json's
headline configuration (configs[1]) and the metric string is BASELINE.json's."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_metric_is_baselines():
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        base = json.load(f)
    assert bench.METRIC == base["metric"]


def test_default_workload_is_cfg2(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert (a.gpus, a.k, a.sn, a.sl, a.lim) == (1, 16, 10_000, 100, 500)
    assert a.scaling == "weak"  # every rank its own sn reads (per-GPU work fixed)
    assert a.steps > 0 and a.warmup >= 0


def test_config_overrides(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py", "--config", "cfg5", "--steps", "3", "--warmup", "1"])
    a = bench.parse()
    assert (a.k, a.sn, a.sl, a.lim, a.steps, a.warmup) == (22, 100_000, 150, 1000, 3, 1)
    assert a.read_len >= 2 * a.sl  # every read long enough for both ends


def test_cfg4_is_strong_scaling(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py", "--config", "cfg4"])
    a = bench.parse()
    assert (a.k, a.sn, a.sl, a.lim, a.scaling) == (16, 1_000_000, 100, 500, "strong")


def test_cpu_share_reports_nproc():
    n, quota = bench.cpu_share()
    assert n == len(os.sched_getaffinity(0))
    assert quota is None or quota > 0


def test_stage_text_says_what_runs():
    """config.stage describes the timed step as it runs: the count launch is issued first in each
    call (the armed launch, which enqueued it during the previous step, was removed in ABI 6)."""
    for world in (1, 2):
        t = bench.stage_text("early-launch", world)
        assert "issued first in the call" in t
        assert "armed" not in t and "previous step" not in t
    assert "DMA" in bench.stage_text("dma", 1)
    assert bench.stage_text("early-launch", 2).endswith("RCCL all-reduce -> counts D2H")
