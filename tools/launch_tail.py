"""Per-launch fixed cost of k_trace (round 6): one frame rendered one iteration
at a time, k_trace's event time against the rays it traversed in each iteration, fitted as
ms = a + b * rays over the iterations with rays.  The intercept a is what a launch costs beyond its
rays -- dispatch, the partition scan and the tail in which the launch's last rays finish on a
nearly idle device -- and a x launches is the frame's share of it.  Layouts: the one-GPU frame at
the bench's slots, and rank 0 of the N = 8 strong split (compact path state, 64-px tiles, the
strong split's slots), as bench.py runs them.

Usage: python tools/launch_tail.py [--config 2] [--out f.json]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mc-path-tracer_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import mcpt
    from mcpt import parallel

    import bench

    rc = mcpt.CONFIGS[args.config]
    W, H = rc.width, rc.height
    scene = mcpt.build_config_scene(args.config)
    pt = mcpt.PathTracer(0, mcpt.default_config(spp=rc.spp, max_depth=rc.max_depth))
    pt.upload_scene(scene)
    pt.set_camera(mcpt.config_camera(rc))
    base = bench.BENCH_SLOTS[args.config]
    res = {"what": __doc__.split("\n\n")[0].replace("\n", " "), "config": args.config, "layouts": []}
    for world in (1, 8):
        if world == 1:
            pt.set_compact_paths(False)
            pt.set_path_slots(base)
            pt.resize(W, H)
            pt.set_tiles(None)
            slots = base
        else:
            slots = parallel.strong_slots(base, world, W, H, rc.spp, 64)
            pt.set_compact_paths(True)
            pt.set_path_slots(1)
            pt.resize(W, H, 64, 64)
            pt.set_tiles(parallel.tiles_for_rank(0, world, W, H, 64))
            pt.set_path_slots(slots)
        for rep in range(2):  # the first pass warms up the layout
            pt.clear()
            rays, ms = [], []
            prev = pt.ray_counts()
            for _ in range(400):
                st = pt.iterate(1)
                cur = pt.ray_counts()
                rays.append(cur["extension_traversed"] + cur["any_hit_traversed"]
                            - prev["extension_traversed"] - prev["any_hit_traversed"])
                ms.append(st.ms_extend)
                prev = cur
                if st.live_paths == 0:
                    break
        r = np.array(rays, np.float64)
        m = np.array(ms, np.float64)
        k = r > 0
        b, a = np.polyfit(r[k], m[k], 1)
        lay = {"world": world, "slots": slots, "launches": int(k.sum()), "k_trace_ms": round(float(m.sum()), 3),
               "rays": int(r.sum()), "fit_ms_per_launch": round(float(a), 4), "fit_ns_per_ray": round(float(b) * 1e6, 4),
               "fixed_share_ms": round(float(a) * int(k.sum()), 3),
               "per_launch": [[int(x), round(float(y), 4)] for x, y in zip(r, m)]}
        res["layouts"].append(lay)
        print(json.dumps({x: y for x, y in lay.items() if x != "per_launch"}), flush=True)
    pt.close()
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
