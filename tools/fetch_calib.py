"""Join tools/hbm/fetch_calib's known byte counts with its FETCH_SIZE / WRITE_SIZE passes into
profiles/fetch_calib_<tag>.json: per access pattern, counter bytes / logical bytes and counter
bytes / distinct-line bytes, i.e. the correction a traffic figure of that pattern needs.
Usage: python tools/fetch_calib.py <tag> [gpurun_out]   (expects <out>/calib.jsonl, <out>/calib_fetch/,
<out>/calib_write/ from tools/gpu_r03.sh)"""
import csv
import json
import os
import sys

tag = sys.argv[1]
src = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(sub, name):
    vals = {}
    for root, _, files in os.walk(os.path.join(src, sub)):
        for f in files:
            if f.endswith("counter_collection.csv"):
                for r in csv.DictReader(open(os.path.join(root, f))):
                    if r["Counter_Name"] == name:
                        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
                        vals[k] = vals.get(k, 0.0) + float(r["Counter_Value"])
    return vals


known = [json.loads(l) for l in open(os.path.join(src, "calib.jsonl")) if l.startswith("{")]
fetch, write = counters("calib_fetch", "FETCH_SIZE"), counters("calib_write", "WRITE_SIZE")
rows = {}
for k in known:
    name = k["kernel"]
    rd = name.startswith("k_rd")
    kb = (fetch if rd else write).get(name)
    if kb is None:
        continue
    b = kb * 1024.0
    rows[name] = {"counter": "FETCH_SIZE" if rd else "WRITE_SIZE", "counter_bytes": b, "logical_bytes": k["logical"],
                  "line_bytes": k["lines"], "counter_over_logical": round(b / k["logical"], 4),
                  "counter_over_lines": round(b / k["lines"], 4)}
out = {"round": tag, "source": "tools/hbm/fetch_calib.hip under rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE "
       "(separate passes); 2 GiB buffers, each pattern one dispatch", "patterns": rows}
json.dump(out, open(os.path.join(REPO, "profiles", f"fetch_calib_{tag}.json"), "w"), indent=1)
for k, v in rows.items():
    print(f"{k:16s} {v['counter']:10s} counter/logical {v['counter_over_logical']:7.3f}  counter/lines {v['counter_over_lines']:6.3f}")
