"""Summarise the SQ / TCC counter passes of tools/pmc_trace.sh (gpurun_out/pmct_<label>/p*/) into
profiles/pmcdetail_<tag>.json: per kernel, the counters summed over its dispatches and the ratios
bench.py's roofline reports (VALU busy, wait fraction, lane utilisation, L2 hit rate).

  valu_busy  = SQ_ACTIVE_INST_VALU * 4 / (SIMDs * GRBM_GUI_ACTIVE / XCDs)  (4 cycles per wave64 op)
  wait_frac  = SQ_WAIT_ANY / SQ_WAVE_CYCLES           (share of wave cycles parked at s_waitcnt)
  lane_util  = SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU)
  l2_hit     = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
  salu_per_valu = SQ_INSTS_SALU / SQ_INSTS_VALU
Usage: PMC_CONFIG=2 python tools/pmc_detail.py <tag> <label> [gpurun_out]
"""
import collections
import csv
import glob
import json
import os
import sys

tag, label = sys.argv[1], sys.argv[2]
src = sys.argv[3] if len(sys.argv) > 3 else "gpurun_out"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

SIMDS, XCDS = 1024, 8  # MI355X: 256 CUs x 4 SIMDs, 8 XCDs
acc = collections.defaultdict(lambda: collections.defaultdict(float))
ndisp = collections.defaultdict(lambda: collections.defaultdict(int))
for f in glob.glob(os.path.join(src, f"pmct_{label}", "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k, c = r["Kernel_Name"], r["Counter_Name"]
        acc[k][c] += float(r["Counter_Value"])
        ndisp[k][c] += 1
out_k = {}
for k, m in acc.items():
    if not any(x in k for x in ("k_trace", "k_shade", "k_material")):
        continue
    r = {}
    if m.get("GRBM_GUI_ACTIVE") and "SQ_ACTIVE_INST_VALU" in m:
        r["valu_busy"] = round(m["SQ_ACTIVE_INST_VALU"] * 4 / (SIMDS * m["GRBM_GUI_ACTIVE"] / XCDS), 4)
    if m.get("SQ_WAVE_CYCLES") and "SQ_WAIT_ANY" in m:
        r["wait_frac"] = round(m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"], 4)
    if m.get("SQ_ACTIVE_INST_VALU") and "SQ_THREAD_CYCLES_VALU" in m:
        r["lane_util"] = round(m["SQ_THREAD_CYCLES_VALU"] / (64 * m["SQ_ACTIVE_INST_VALU"]), 4)
    if m.get("TCC_HIT_sum", 0) + m.get("TCC_MISS_sum", 0) > 0:
        r["l2_hit"] = round(m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"]), 4)
    if m.get("SQ_INSTS_VALU") and "SQ_INSTS_SALU" in m:
        r["salu_per_valu"] = round(m["SQ_INSTS_SALU"] / m["SQ_INSTS_VALU"], 4)
    out_k[k] = {"dispatches": max(ndisp[k].values()), "counters_summed": dict(m), "ratios": r}
cfg = int(os.environ.get("PMC_CONFIG", "2"))
out = {"round": tag, "stamp": {"source_hash": bench.source_hash(), "config": cfg,
                               "slots": int(os.environ.get("PMC_SLOTS", str(bench.BENCH_SLOTS[cfg]))),
                               "step": bench.STEP, "spp": bench.stamp_spp(cfg, os.environ.get("PMC_ARGS", "")),
                               "knobs": bench.knobs()},
       "source": f"tools/gpu/run.sh pmc ({label}): rocprofv3 --pmc passes (one counter group each) over "
                 f"'python3 {os.environ.get('PROG', 'bench.py')}'",
       "formulas": __doc__.split("\n\n")[1].strip(), "kernels": out_k}
name = os.environ.get("PMC_NAME", f"pmcdetail_{tag}")
json.dump(out, open(os.path.join(REPO, "profiles", f"{name}.json"), "w"), indent=1)
for k, v in out_k.items():
    print(k[:60], v["ratios"])
