"""bench.py host logic (CPU only): the PMC-summary staleness check, the roofline derivation, the
frame / slot layout and the CPU-baseline thread count.  Traffic and counter figures from
profiles/pmc*_r*.json are used only when the summary's stamp matches the current kernel sources
and the benched workload (config, path slots, step kind)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_source_hash_stable():
    assert bench.source_hash() == bench.source_hash() and len(bench.source_hash()) == 16


def _stamp(h="abc", config=2, slots=3, step="frame"):
    return {"source_hash": h, "config": config, "slots": slots, "step": step}


def test_pmc_summary_stale_detection(tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    monkeypatch.setattr(bench, "source_hash", lambda: "abc")
    assert bench.pmc_summary(2, 3) == (None, "no pmc summary in profiles/")
    kern = {"void mcpt_dev::k_trace<2, 8>(mcpt_dev::TraceArgs)": {"hbm_bytes_per_launch": 1000}}
    (prof / "pmc_r09.json").write_text(json.dumps({"stamp": _stamp(), "kernels": kern}))
    d, why = bench.pmc_summary(2, 3)
    assert why is None and bench.pmc_traffic(d, ("mcpt_dev::k_trace<",)) == 1000
    assert "3 slots" in bench.pmc_summary(2, 4)[1]
    # a summary of the round-2 per-iteration steps is stale for the per-frame bench
    (prof / "pmc_r10.json").write_text(json.dumps({"stamp": _stamp(step="iteration"), "kernels": kern}))
    assert "iteration steps" in bench.pmc_summary(2, 3)[1]
    (prof / "pmc_r11.json").write_text(json.dumps({"stamp": _stamp(), "kernels": kern}))
    monkeypatch.setattr(bench, "source_hash", lambda: "def")
    d, why = bench.pmc_summary(2, 3)
    assert "sources changed" in why
    (prof / "pmc_r12.json").write_text(json.dumps({"kernels": kern}))  # unstamped (round-1 format)
    assert bench.pmc_summary(2, 3)[1] is not None
    # pmcdetail summaries are looked up separately (not mistaken for pmc_r*.json)
    (prof / "pmcdetail_r12.json").write_text(json.dumps({"stamp": _stamp(h="def"), "kernels": {
        "void mcpt_dev::k_trace<2, 8>(mcpt_dev::TraceArgs)": {"ratios": {"valu_busy": 0.7}}}}))
    d, why = bench.pmc_summary(2, 3, "pmcdetail")
    assert why is None and bench.pmc_detail(d, ("mcpt_dev::k_trace<",)) == {"valu_busy": 0.7}
    # other configs read their own summaries (pmc_c<config>_rNN.json), never config 2's
    assert bench.pmc_summary(3, 32) == (None, "no pmc summary in profiles/")
    (prof / "pmc_c3_r12.json").write_text(json.dumps({"stamp": _stamp(h="def", config=3, slots=32), "kernels": kern}))
    d, why = bench.pmc_summary(3, 32)
    assert why is None and d["stamp"]["config"] == 3
    assert bench.pmc_summary(5, 16)[0] is None
    # a launch's traffic depends on the spp (the path mix): config 5's 64-spp summary is stale for its
    # 4096-spp frame; summaries stamped before spp was recorded are not judged on it
    st5 = dict(_stamp(h="def", config=5, slots=24), spp=bench.stamp_spp(5, "--config 5 --steps 1 --spp 64"))
    assert st5["spp"] == 64 and bench.stamp_spp(5, "--config 5") == 4096
    (prof / "pmc_c5_r12.json").write_text(json.dumps({"stamp": st5, "kernels": kern}))
    assert bench.pmc_summary(5, 24, spp=64)[1] is None
    assert "taken at 64 spp" in bench.pmc_summary(5, 24, spp=4096)[1]
    assert bench.pmc_summary(3, 32, spp=999)[1] is None
    # a variant pass (a knob set: pmc_r13occoff.json) is never taken for the product's line, and a
    # summary stamped with knobs other than the run's is stale (neutral knobs aside)
    (prof / "pmc_r13.json").write_text(json.dumps({"stamp": dict(_stamp(h="def"), knobs={}), "kernels": kern}))
    (prof / "pmc_r13occoff.json").write_text(json.dumps({"stamp": dict(_stamp(h="def"), knobs={"MCPT_OCC_G": "0"}),
                                                         "kernels": {}}))
    d, why = bench.pmc_summary(2, 3)
    assert why is None and d["kernels"] == kern
    monkeypatch.setenv("MCPT_DIST_TIMEOUT_S", "30")  # neutral
    assert bench.pmc_summary(2, 3)[1] is None
    monkeypatch.setenv("MCPT_OCC_G", "0")
    assert "taken with knobs {}" in bench.pmc_summary(2, 3)[1]


class _St:
    def __init__(self, **kw):
        for k in bench.Acc.KEYS:
            setattr(self, k, 0)
        for k, v in kw.items():
            setattr(self, k, v)


def test_roofline_fields_never_exceed_one_and_bound_is_derived(tmp_path, monkeypatch):
    """achieved = HBM-resident algorithmic bytes (per-ray state), cache-served BVH bytes apart;
    bound = the most utilised resource, 'latency' when nothing reaches half its roof."""
    prof = tmp_path / "profiles"
    prof.mkdir()
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    monkeypatch.setattr(bench, "source_hash", lambda: "abc")
    # config-2-like frame: 10 launches of 6 M extension + 4.6 M any-hit rays at 0.72 ms
    st = _St(iterations=10, extend_rays=60_000_000, shadow_rays=23_000_000, vis_rays=23_000_000,
             ext_nodes=550_000_000, ext_tests=115_000_000, ext_hits=50_000_000,
             any_nodes=600_000_000, any_tests=110_000_000)
    r = bench.roofline(st, 7.2, 4.4, 2, 3)
    assert r["frac"] <= 1 and r["cache_served"]["l2_frac"] <= 1
    assert r["algorithmic_bytes_per_launch"] == (65 * 6_000_000 + 33 * 4_600_000)
    assert r["bound"] == "latency" and r["pmc_stale"]  # no PMC summary: HBM judged by the state bytes
    kern = {"void mcpt_dev::k_trace<2, 8>(mcpt_dev::TraceArgs)": {"hbm_bytes_per_launch": 420_000_000},
            "void mcpt_dev::k_shade<false>(mcpt_dev::ShadeArgs)": {"hbm_bytes_per_launch": 700_000_000},
            "void mcpt_dev::k_material<false>(mcpt_dev::ShadeArgs)": {"hbm_bytes_per_launch": 900_000_000}}
    (prof / "pmc_r03.json").write_text(json.dumps({"stamp": _stamp(), "kernels": kern}))
    (prof / "pmcdetail_r03.json").write_text(json.dumps({"stamp": _stamp(), "kernels": {
        "void mcpt_dev::k_trace<2, 8>(mcpt_dev::TraceArgs)": {
            "ratios": {"valu_busy": 0.78, "wait_frac": 0.57, "lane_util": 0.5}}}}))
    r = bench.roofline(st, 7.2, 4.4, 2, 3)
    assert r["traffic"] == 420_000_000 and abs(r["traffic_frac"] - 420e6 / 0.72e-3 / 8e12) < 1e-4
    # the VALU is judged by its useful share, busy x lane utilisation: 0.39, so no
    # resource reaches half its roof here
    assert r["counters"]["valu_useful"] == 0.39 and r["utilisation"]["valu"] == 0.39 and r["bound"] == "latency"
    assert "wait on memory 0.57" in r["binding"] and "busy 0.78 x lane utilisation 0.50" in r["binding"]
    (prof / "pmcdetail_r03.json").write_text(json.dumps({"stamp": _stamp(), "kernels": {
        "void mcpt_dev::k_trace<2, 8>(mcpt_dev::TraceArgs)": {"ratios": {"valu_busy": 0.9, "lane_util": 0.8}},
        "void mcpt_dev::k_shade<false>(mcpt_dev::ShadeArgs)": {"ratios": {"valu_busy": 0.7, "lane_util": 0.5}},
        "void mcpt_dev::k_material<false>(mcpt_dev::ShadeArgs)": {"ratios": {"valu_busy": 0.8, "lane_util": 0.75}}}}))
    r = bench.roofline(st, 7.2, 4.4, 2, 3)
    assert r["bound"] == "valu" and r["utilisation"]["valu"] == 0.72
    assert r["shade_stages"]["counters"]["k_shade"]["valu_useful"] == 0.35
    assert r["shade_stages"]["counters"]["k_material"]["valu_useful"] == 0.6
    assert r["shade_stages"]["traffic"] == 1_600_000_000
    for k in ("frac", "traffic_frac"):
        assert r[k] <= 1


def test_extend_shade_roofline(tmp_path, monkeypatch):
    """The metric's own fraction (extend + shade as a whole step): SURVEY 8(d) state bytes and the
    PMC summary's HBM bytes of k_trace + k_shade + k_material per frame over the frame time."""
    prof = tmp_path / "profiles"
    prof.mkdir()
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    monkeypatch.setattr(bench, "source_hash", lambda: "abc")
    # two frames of 64 iterations: 2.7 G rays per frame
    st = _St(iterations=128, extend_rays=2 * 1_250_000_000, shadow_rays=2 * 730_000_000, vis_rays=2 * 720_000_000)
    r = bench.extend_shade(st, 0.2886, 2, 2, 3)
    state = 367 * 730_000_000 + 49 * 520_000_000 + 65 * 1_250_000_000 + 33 * 1_450_000_000
    assert r["state_bytes_per_frame"] == state and abs(r["state_frac"] - state / 0.2886 / 8e12) < 1e-4
    assert r["iterations_per_frame"] == 64 and r["pmc_stale"] and "traffic_frac" not in r
    kern = {"void mcpt_dev::k_trace<2, 8>(mcpt_dev::TraceArgs)": {"hbm_bytes_per_launch": 1_970_000_000},
            "void mcpt_dev::k_shade<false>(mcpt_dev::ShadeArgs)": {"hbm_bytes_per_launch": 2_650_000_000},
            "void mcpt_dev::k_material<false>(mcpt_dev::ShadeArgs)": {"hbm_bytes_per_launch": 7_140_000_000}}
    (prof / "pmc_r04.json").write_text(json.dumps({"stamp": _stamp(), "kernels": kern}))
    r = bench.extend_shade(st, 0.2886, 2, 2, 3)
    assert r["traffic_bytes_per_frame"] == int(11_760_000_000 * 64)
    assert abs(r["traffic_frac"] - 11.76e9 * 64 / 0.2886 / 8e12) < 1e-4  # round 3's 0.33
    assert r["traffic_frac"] <= 1 and r["state_frac"] <= 1


def test_frame_and_slots_layout():
    import mcpt

    rc2, rc4 = mcpt.CONFIGS[2], mcpt.CONFIGS[4]
    assert bench.frame_size(rc2, 1, "weak") == (1920, 1080) and bench.frame_size(rc2, 8, "weak") == (1920, 8640)
    assert bench.frame_size(rc4, 8, "strong") == (3840, 2160)
    assert bench.BENCH_SLOTS[2] == 24 and set(bench.BENCH_SLOTS) == set(mcpt.CONFIGS)
    assert all(1 <= s <= 256 for s in bench.BENCH_SLOTS.values())  # mcpt_set_path_slots' range
    a = bench.parse(["--gpus", "4", "--config", "4", "--scaling", "strong"])
    assert (a.gpus, a.config, a.scaling, a.slots, a.steps) == (4, 4, "strong", None, 5)


def test_cpu_baseline_threads(monkeypatch):
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    assert bench.cpu_threads() == min(3, len(os.sched_getaffinity(0)))
    monkeypatch.delenv("OMP_NUM_THREADS")
    assert bench.cpu_threads() == len(os.sched_getaffinity(0))


def test_pmc_lookup_skips_the_counting_instantiation():
    """The bench's extra counting frame launches k_trace<W, S, true>; its traffic and counters
    must not be added to (or stand in for) the timed frames' k_trace<W, S, false>."""
    import bench

    s = {"kernels": {"void mcpt_dev::k_trace<2, 8, false>(mcpt_dev::TraceArgs)": {"hbm_bytes_per_launch": 100, "ratios": {"a": 1}},
                     "void mcpt_dev::k_trace<2, 8, true>(mcpt_dev::TraceArgs)": {"hbm_bytes_per_launch": 120, "ratios": {"a": 2}},
                     "void mcpt_dev::k_material<true>(mcpt_dev::ShadeArgs)": {"hbm_bytes_per_launch": 7}}}
    assert bench.pmc_traffic(s, ("mcpt_dev::k_trace<",)) == 100
    assert bench.pmc_detail(s, ("mcpt_dev::k_trace<",)) == {"a": 1}
    assert bench.pmc_traffic(s, ("mcpt_dev::k_material<",)) == 7  # quality mode's <true> is a timed kernel


def test_knobs_are_stamped_and_judged():
    """Every MCPT_* variable is stamped into the line; one that changes the measured kernels, their
    launch or the layout marks the line as not the product."""
    a = bench.parse([])
    assert bench.product_check(a, bench.knobs({})) == (True, [])
    kn = bench.knobs({"MCPT_CULL": "0", "PATH": "/bin", "MCPT_BVH_THREADS": "4"})
    assert kn == {"MCPT_BVH_THREADS": "4", "MCPT_CULL": "0"}
    ok, why = bench.product_check(a, kn)
    assert not ok and len(why) == 1 and why[0].startswith("MCPT_CULL=0")
    ok, why = bench.product_check(a, bench.knobs({"MCPT_TRACE_WAVES": "20", "MCPT_NEW_THING": "1"}))
    assert not ok and any("launch geometry" in w for w in why) and any("unknown knob" in w for w in why)
    assert not bench.product_check(bench.parse(["--spp", "64"]), {})[0]
    assert not bench.product_check(bench.parse(["--slots", "16"]), {})[0]
    assert bench.product_check(bench.parse(["--slots", "24"]), {})[0]  # the config's own
    # every knob the library reads through getenv is classified
    import re

    src = ""
    for root, _, files in os.walk(os.path.join(REPO, "mc-path-tracer_amd", "csrc")):
        for f in files:
            src += open(os.path.join(root, f)).read()
    read = set(re.findall(r'getenv\("(MCPT_[A-Z0-9_]+)"', src)) | set(re.findall(r'env_u32\("(MCPT_[A-Z0-9_]+)"', src))
    assert read and read <= set(bench.NON_PRODUCT_KNOBS) | bench.NEUTRAL_KNOBS, read - set(bench.NON_PRODUCT_KNOBS)
