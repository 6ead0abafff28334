"""Summarise rocprofv3 output (gpurun_out/prof_*) into profiles/ (committed evidence).

HBM traffic per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 B: on gfx950 FETCH_SIZE counts
exactly half the bytes of wide (16 B/lane) coalesced reads (MI355X_MICROARCH.md, HBM section);
the path-state streams are dwordx4 per lane.  FETCH/WRITE are collected in separate --pmc passes.
Usage: python tools/pmc.py <round-tag> [gpurun_out]
"""
import collections
import csv
import json
import os
import shutil
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
src = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = os.path.join(REPO, "profiles")
os.makedirs(dst, exist_ok=True)


def find(sub, suffix):
    # the newest match: gpurun merges a call's gpurun_out/ into the local one, so older runs'
    # files can sit beside the current ones
    d = os.path.join(src, sub)
    hits = [os.path.join(root, f) for root, _, files in os.walk(d) for f in files if f.endswith(suffix)]
    return max(hits, key=os.path.getmtime) if hits else None


stats = find("prof_kt", "kernel_stats.csv")
if stats:
    shutil.copy(stats, os.path.join(dst, os.environ.get("STATS_NAME", f"kernel_stats_{tag}") + ".csv"))
pmc = collections.defaultdict(dict)
for sub, ctr in (("prof_fetch", "FETCH_SIZE"), ("prof_write", "WRITE_SIZE")):
    f = find(sub, "counter_collection.csv")
    if not f:
        continue
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == ctr:
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        pmc[k][ctr + "_KB_avg"] = sum(v) / len(v)
        pmc[k]["launches"] = len(v)
dur = {}
if stats:
    for r in csv.DictReader(open(stats)):
        dur[r["Name"]] = float(r["AverageNs"])
sys.path.insert(0, REPO)
import bench  # noqa: E402  (source_hash only)

# The profiled commands run bench.py's defaults (config 2, BENCH_SLOTS, whole-frame steps) unless
# PMC_CONFIG / PMC_SLOTS say otherwise; bench.py uses the traffic only when this stamp matches its run.
cfg = int(os.environ.get("PMC_CONFIG", "2"))
stamp = {"source_hash": bench.source_hash(), "config": cfg,
         "slots": int(os.environ.get("PMC_SLOTS", str(bench.BENCH_SLOTS[cfg]))), "step": bench.STEP,
         "spp": bench.stamp_spp(cfg, os.environ.get("PMC_ARGS", "")),
         # the MCPT_* knobs the profiled runs had (set them here too when summarising elsewhere)
         "knobs": bench.knobs()}
out = {"round": tag, "stamp": stamp,
       "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) on "
       f"'python3 bench.py {os.environ.get('PMC_ARGS', '--no-cpu-baseline')}'; durations from --kernel-trace --stats",
       "correction": "hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE reads half of 16 B/lane streams)",
       "kernels": {}}
for k, v in pmc.items():
    if "FETCH_SIZE_KB_avg" in v and "WRITE_SIZE_KB_avg" in v:
        b = (2 * v["FETCH_SIZE_KB_avg"] + v["WRITE_SIZE_KB_avg"]) * 1024
        v["hbm_bytes_per_launch"] = int(b)
        if k in dur:
            v["avg_ns"] = dur[k]
            v["hbm_GBps"] = round(b / dur[k], 1)
    out["kernels"][k] = v
name = os.environ.get("PMC_NAME", f"pmc_{tag}")  # e.g. pmc_c5_r03 for another config's evidence
json.dump(out, open(os.path.join(dst, f"{name}.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
