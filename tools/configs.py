"""Steady-state throughput of every BASELINE config on one GPU (all tiles of the full frame).

Prints one line per config: Mray/s over `--iters` wavefront iterations after `--warmup`,
per-kernel ms per iteration, rays per iteration and BVH size.  Configs 4/5 are the
8-GPU configs run here on a single device over the whole frame.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mc-path-tracer_amd"))
import mcpt  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--configs", default="1,2,3,4,5")
ap.add_argument("--warmup", type=int, default=20)
ap.add_argument("--iters", type=int, default=30)
ap.add_argument("--out", default=None)
ap.add_argument("--slots", default="auto", help="paths per pixel; auto = the measured best per config (AUTO_SLOTS)")
ap.add_argument("--full", default="1", help="configs also rendered as a whole frame to spp completion")
args = ap.parse_args()
# Path slots per config, measured (steady state, 1 GPU): C2 1/2/3/4 -> 7248/8095/8340/7520 Mray/s
# (full frame 0.481/0.419/0.396/0.400 s); C3 2/3 -> 5670/6146; C4 1/2/4 -> 4476/4852/4982;
# C5 1/2/4 -> 4548/4910/5011; C1 (65K pixels, 16 spp) renders all its samples at once with 16.
AUTO_SLOTS = {1: 16, 2: 3, 3: 3, 4: 4, 5: 4}
res = []
for c in [int(x) for x in args.configs.split(",")]:
    rc = mcpt.CONFIGS[c]
    t0 = time.time()
    scene = mcpt.build_config_scene(c)
    t_build = time.time() - t0
    a = scene.arrays()
    pt = mcpt.PathTracer(0, mcpt.default_config(spp=rc.spp, max_depth=rc.max_depth))
    pt.upload_scene(scene)
    pt.set_camera(mcpt.config_camera(rc))
    P = rc.width * rc.height
    S = AUTO_SLOTS.get(c, 1) if args.slots == "auto" else int(args.slots)
    pt.set_path_slots(S)
    pt.resize(rc.width, rc.height)
    pt.iterate(args.warmup)
    t1 = time.time()
    st = pt.iterate(args.iters)  # timed with the lean k_trace (no work counters)
    wall = time.time() - t1
    rays = st.extend_rays + st.shadow_rays + st.vis_rays
    # node / test counts from as many further, untimed iterations with the counting build (ADVICE r4:
    # its spilling k_trace must not be the one timed)
    pt.set_work_counters(True)
    wk = pt.iterate(args.iters)
    pt.set_work_counters(False)
    r = {"config": c, "W": rc.width, "H": rc.height, "spp": rc.spp, "depth": rc.max_depth,
         "tris": int(len(a["mat"])), "bvh_depth": scene.bvh_depth, "host_build_s": round(t_build, 2),
         "mray_s": round(rays / (st.ms_total * 1e-3) / 1e6, 1) if rays else None,  # None: finished in the warmup
         "mray_s_wall": round(rays / wall / 1e6, 1) if rays else None,
         "ms_trace": round(st.ms_extend / args.iters, 4), "ms_shade": round(st.ms_shade / args.iters, 4),
         "rays_per_iter": {"extend": st.extend_rays // args.iters, "shadow": st.shadow_rays // args.iters,
                           "vis": st.vis_rays // args.iters},
         "ext_nodes_per_ray": round(wk.ext_nodes / max(1, wk.extend_rays), 2),
         "any_nodes_per_ray": round(wk.any_nodes / max(1, wk.shadow_rays + wk.vis_rays), 2), "path_slots": S,
         "counts_from": "the next iterations, counting k_trace build, untimed"}
    if str(c) in args.full.split(","):
        pt.clear()
        t2 = time.time()
        fs = pt.render()
        dtf = time.time() - t2
        r["full_frame"] = {"seconds": round(dtf, 4), "iterations": fs.iterations,
                           "mray_s": round((fs.extend_rays + fs.shadow_rays + fs.vis_rays) / dtf / 1e6, 1)}
    print(json.dumps(r), flush=True)
    res.append(r)
    pt.close()
if args.out:
    json.dump(res, open(args.out, "w"), indent=1)
