"""GPU BVH builds (PLOC, linear BVH) vs the host SAH build: build time and the trace time of
the config's steady-state pipeline with each tree (extension + any-hit rays).
usage: python tools/gpu_bvh_bench.py [configs, default 2,3,5]"""
import json, os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mc-path-tracer_amd")]
import mcpt
out = []
for c in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "2,3,5").split(",")]:
    rc = mcpt.CONFIGS[c]
    t = time.time()
    s = mcpt.build_config_scene(c)  # host SAH (mcpt.DEFAULT_BVH) + env tables
    host_s = time.time() - t
    pt = mcpt.PathTracer(0, mcpt.default_config(spp=rc.spp, max_depth=rc.max_depth))
    pt.set_path_slots(3)
    r = {"config": c, "tris": int(len(s.arrays()["mat"])), "host_sah_build_s": round(host_s, 3)}
    for b in ("sah", "ploc", "lbvh"):
        gpu = False if b == "sah" else b
        pt.upload_scene(s, gpu_bvh=gpu)
        if gpu:
            pt.upload_scene(s, gpu_bvh=gpu)  # second build: warm
            r[f"gpu_{b}_build_ms"] = round(pt.last_build_ms, 2)
        pt.set_camera(mcpt.config_camera(rc)); pt.resize(rc.width, rc.height)
        pt.iterate(20)
        st = pt.iterate(20)  # timed with the lean k_trace
        r[f"trace_ms_{b}"] = round(st.ms_extend / 20, 4)
        pt.set_work_counters(True)  # node counts from 20 more, untimed iterations (counting build)
        wk = pt.iterate(20)
        pt.set_work_counters(False)
        r[f"nodes_per_ray_{b}"] = round((wk.ext_nodes + wk.any_nodes) / max(1, wk.rays), 2)
    print(json.dumps(r), flush=True)
    out.append(r)
    pt.close()
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
