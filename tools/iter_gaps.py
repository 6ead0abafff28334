"""Per-iteration timeline of a rocprofv3 kernel trace (CSV) of tools/rank_frames.py: for each frame
(k_clear starts one), the iterations (k_shade ... k_accumulate), each kernel's duration and the idle
gaps between consecutive kernels, summed; prints a summary as JSON.

  python tools/iter_gaps.py gpurun_out/rk/**/rk_kernel_trace.csv"""
import csv
import glob
import json
import sys


def main(path):
    f = sorted(glob.glob(path, recursive=True))[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    frames, cur = [], None
    for r in rows:
        n = r["Kernel_Name"]
        if "k_clear" in n:
            cur = []
            frames.append(cur)
        if cur is not None and "mcpt_dev::" in n:
            cur.append((n, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    out = []
    for fr in frames:
        if not fr:
            continue
        t0, t1 = fr[0][1], fr[-1][2]
        busy = {}
        gap = 0
        iters = 0
        for i, (n, s, e) in enumerate(fr):
            k = n.split("(")[0].replace("void ", "").replace("mcpt_dev::", "")
            k = k.split("<")[0]
            busy[k] = busy.get(k, 0) + (e - s)
            if i:
                gap += max(0, s - fr[i - 1][2])
            if "k_accumulate" in n:
                iters += 1
        out.append({"span_ms": round((t1 - t0) / 1e6, 3), "iterations": iters, "gap_ms": round(gap / 1e6, 3),
                    "kernel_ms": {k: round(v / 1e6, 3) for k, v in sorted(busy.items(), key=lambda kv: -kv[1])}})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
