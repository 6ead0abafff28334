"""Attribution of the shading kernels' HBM bytes (diagnostic builds):
per library variant, FETCH/WRITE per k_material / k_shade launch and per shadow ray.
usage: python tools/diag_attr.py <variant>... (reads gpurun_out/attr_<v>/)"""
import collections, csv, glob, json, os, sys
for v in sys.argv[1:]:
    d = os.path.join("gpurun_out", f"attr_{v}")
    tot = collections.defaultdict(float)
    n = collections.defaultdict(int)
    for kind in ("fetch", "write"):
        for f in glob.glob(os.path.join(d, kind, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                for name in ("k_material", "k_shade", "k_trace"):
                    if name in k:
                        tot[(name, kind)] += float(r["Counter_Value"])
                        n[(name, kind)] += 1
    b = [l for l in open(os.path.join(d, "bench.log")) if l.startswith('{"metric"')]
    rk = json.loads(b[-1])["config"]["rays_per_step_rank0"] if b else {}
    sh = rk.get("shadow", 0) or 1
    out = [v]
    for name in ("k_material", "k_shade", "k_trace"):
        rd = 2 * tot[(name, "fetch")] * 1024
        wr = tot[(name, "write")] * 1024
        out.append(f"{name}: read {rd / 1e9:.2f} GB ({rd / sh:.0f} B/shadow ray) write {wr / 1e9:.2f} GB ({wr / sh:.0f} B)")
    print(" | ".join(out), "| rays", rk)
