"""Same rays, different BVHs: results must be identical (hits are BVH-independent: conservative
culling + (t, index) ties); compare trace time and steps per ray."""
import hashlib, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mc-path-tracer_amd")]
import numpy as np, mcpt
rc = mcpt.CONFIGS[2]
pt = mcpt.PathTracer(0, mcpt.default_config(spp=256, max_depth=5))
pt.upload_scene(mcpt.build_config_scene(2)); pt.set_camera(mcpt.config_camera(rc)); pt.resize(rc.width, rc.height)
pt.iterate(30)
ro, rd = pt.queue_rays()
for mp in (1, 2, 4, 8):
    s = mcpt.Scene(); s.make_proxy(2, mcpt.ASSET_DIR); s.build(mp)
    pt.upload_scene(s)
    ts, ta = [], []
    for i in range(3):
        r = pt.trace_closest(ro, rd, steps=True); ts.append(pt.last_stage_ms)
        v = pt.trace_any(ro, rd, steps=True); ta.append(pt.last_stage_ms)
    a = s.arrays()
    h = hashlib.md5(r[0].tobytes() + r[1].tobytes() + r[2].tobytes() + v[0].tobytes()).hexdigest()[:10]
    print(f"max_prims {mp}: nodes {len(a['nprims'])} depth {s.bvh_depth} [{h}] closest {min(ts):.3f} ms "
          f"steps {r[3].mean():.2f}  any {min(ta):.3f} ms steps {v[1].mean():.2f}", flush=True)
