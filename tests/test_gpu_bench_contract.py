"""bench.py's output contract on the GPU: one JSON line with the driver's keys, the headline metric string of
BASELINE.json for C3, and the roofline / cpu_baseline objects (run on the fast C1 config and on a one-step C3)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config", "roofline"}


def _line(args, timeout=300):
    r = subprocess.run([sys.executable, "bench.py"] + args, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def _check(d, steps, warmup):
    assert KEYS <= set(d), KEYS - set(d)
    assert d["n_gpus"] == 1 and d["steps"] == steps and d["warmup"] == warmup
    assert d["higher_is_better"] is True and d["unit"] == "restarts/s" and d["dtype"] == "f64"
    assert d["value"] > 0 and d["ms_per_step"] > 0
    assert "workload" in d["config"]
    rf = d["roofline"]
    assert {"bound", "achieved", "peak", "unit", "frac", "traffic"} <= set(rf)
    if rf["achieved"] is not None and rf["peak"]:
        assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-9


def test_bench_c1_line():
    d = _line(["--config", "C1", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"])
    _check(d, 2, 1)


def test_bench_c3_line_has_the_headline_metric_and_cpu_baseline():
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        metric = json.load(f)["metric"]
    d = _line(["--steps", "1", "--warmup", "0", "--cpu-iters", "2"], timeout=600)
    _check(d, 1, 0)
    assert d["metric"] == metric
    assert d["roofline"]["bound"] == "mfma" and d["roofline"]["unit"] == "TFLOP/s"
    cb = d["cpu_baseline"]
    assert {"value", "unit", "cores", "kind", "sample"} <= set(cb) and cb["value"] > 0 and cb["cores"] >= 1
