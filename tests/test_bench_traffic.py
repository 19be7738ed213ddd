"""bench.py's HBM-traffic attribution: counter bytes from a committed PMC
profile are attached to a bench line only when the profile was taken on the same kernel source AND the same workload,
and never when they fall below the line's algorithmic bytes (every algorithmic byte crosses HBM at least once).
CPU only: no GPU call."""
import glob
import json
import os
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402

C3 = {"config": "C3", "stop_rule": "ref_compat", "maxiter": 10000, "restarts": 200}
FIXED = {"config": "C3", "stop_rule": "fixed", "maxiter": 1000, "restarts": 200}


def _kernels():
    return {"wta": {"avg_ms": 1.5, "algo_bytes_per_launch": 1.8e9}, "ahtw": {"avg_ms": 1.4, "algo_bytes_per_launch": 1.4e9}}


def test_traffic_below_algorithmic_bytes_is_rejected():
    roof, k = {"traffic": None}, _kernels()
    bench.attach_traffic(roof, k, "wta", {"wta": 1.35e9, "ahtw": 2.9e9}, "profiles/x/pmc_traffic.json")
    assert roof["traffic"] is None and "wta" in roof["traffic_rejected"]
    assert "traffic_bytes_per_launch" not in k["wta"]
    assert k["ahtw"]["traffic_bytes_per_launch"] == 2.9e9


def test_traffic_attached_when_consistent():
    roof, k = {"traffic": None}, _kernels()
    bench.attach_traffic(roof, k, "wta", {"wta": 2.5e9}, "p")
    assert roof["traffic"] == 2.5e9 and "traffic_rejected" not in roof
    assert roof["traffic"] >= k["wta"]["algo_bytes_per_launch"]


@pytest.fixture
def fake_root(tmp_path, monkeypatch):
    from nmfconsensus_amd.build import source_sha256
    sha = source_sha256()
    d = tmp_path / "profiles" / "r99"
    d.mkdir(parents=True)
    row = {"launches": 10, "hbm_bytes_per_launch": 2.0e9}
    (d / "pmc_traffic.json").write_text(json.dumps({"k_wta2": row, "k_ahtw4": row, "source_sha256": sha,
                                                    "workload": C3}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    return tmp_path


def test_profile_keyed_on_workload(fake_root):
    got = bench.pmc_profile_for(C3)
    assert got is not None and got[0]["wta"] == 2.0e9
    assert bench.pmc_profile_for(FIXED) is None                              # another stop rule / maxiter
    assert bench.pmc_profile_for(dict(C3, restarts=25)) is None              # another restart count
    assert bench.pmc_profile_for(dict(C3, config="C4")) is None


def test_profile_without_workload_is_the_default_line(tmp_path, monkeypatch):
    from nmfconsensus_amd.build import source_sha256
    d = tmp_path / "profiles" / "old"
    d.mkdir(parents=True)
    (d / "pmc_traffic.json").write_text(json.dumps({"k_wta2": {"launches": 1, "hbm_bytes_per_launch": 1.0},
                                                    "source_sha256": source_sha256()}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.pmc_profile_for(C3) is not None
    assert bench.pmc_profile_for(FIXED) is None


def test_committed_lines_traffic_not_below_algorithmic():
    """Every bench line committed from round 6 on: roofline.traffic (and each kernel's traffic) >= its algorithmic
    bytes per launch whenever both are present."""
    files = glob.glob(os.path.join(ROOT, "profiles", "r06", "**", "*.json"), recursive=True)
    for f in files:
        try:
            d = json.load(open(f))
        except (ValueError, UnicodeDecodeError):
            continue
        roof = d.get("roofline") if isinstance(d, dict) else None
        if not roof:
            continue
        if roof.get("traffic") is not None and roof.get("algo_bytes_per_launch"):
            assert roof["traffic"] >= roof["algo_bytes_per_launch"], f
        for name, kr in (roof.get("kernels") or {}).items():
            if kr.get("traffic_bytes_per_launch") is not None and kr.get("algo_bytes_per_launch"):
                assert kr["traffic_bytes_per_launch"] >= kr["algo_bytes_per_launch"], (f, name)
