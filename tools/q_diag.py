"""Per-config traversal sanity of a library build: a small frame, a few iterations, node /
triangle tests per ray and the trace time.  Usage: MCPT_LIB=... python tools/q_diag.py CID [W H]"""
import os
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mc-path-tracer_amd")]
import mcpt  # noqa: E402

cid = int(sys.argv[1])
W, H = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (320, 180)
rc = mcpt.CONFIGS[cid]
s = mcpt.build_config_scene(cid)
pt = mcpt.PathTracer(0, mcpt.default_config(spp=rc.spp, max_depth=rc.max_depth))
pt.upload_scene(s)
pt.set_camera(mcpt.config_camera(rc, W, H))
pt.resize(W, H)
for n in (1, 4):
    t0 = time.perf_counter()
    st = pt.iterate(n)
    dt = time.perf_counter() - t0
    e, a = max(st.extend_rays, 1), max(st.shadow_rays + st.vis_rays, 1)
    print(f"config {cid} {W}x{H} iters {n}: {dt*1e3:.1f} ms, ext {st.extend_rays} rays {st.ext_nodes/e:.2f} nodes "
          f"{st.ext_tests/e:.2f} tris, any {a} rays {st.any_nodes/a:.2f} nodes {st.any_tests/a:.2f} tris, "
          f"trace ms {st.ms_extend:.3f}", flush=True)
pt.close()
