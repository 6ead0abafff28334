"""bench.py's PMC-summary staleness check (CPU only): traffic figures from profiles/pmc_*.json are
used only when the summary's stamp matches the current kernel sources and the benched workload."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_source_hash_stable():
    assert bench.source_hash() == bench.source_hash() and len(bench.source_hash()) == 16


def test_pmc_summary_stale_detection(tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    monkeypatch.setattr(bench, "source_hash", lambda: "abc")
    assert bench.pmc_summary(2, 3) == (None, "no PMC summary in profiles/")
    kern = {"mcpt_dev::k_trace(mcpt_dev::TraceArgs)": {"hbm_bytes_per_launch": 1000}}
    (prof / "pmc_r09.json").write_text(json.dumps({"stamp": {"source_hash": "abc", "config": 2, "slots": 3},
                                                   "kernels": kern}))
    d, why = bench.pmc_summary(2, 3)
    assert why is None and bench.pmc_traffic(d, ("mcpt_dev::k_trace(",)) == 1000
    assert "3 slots" in bench.pmc_summary(2, 4)[1]
    monkeypatch.setattr(bench, "source_hash", lambda: "def")
    d, why = bench.pmc_summary(2, 3)
    assert "sources changed" in why
    (prof / "pmc_r10.json").write_text(json.dumps({"kernels": kern}))  # unstamped (round-1 format)
    assert bench.pmc_summary(2, 3)[1] is not None
