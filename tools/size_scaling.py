"""Steady-state Mray/s of config 2's scene and camera at growing film heights (same view,
vertically supersampled): how much of a launch is fixed cost (ramp-up, drain)."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mc-path-tracer_amd")]
import mcpt
rc = mcpt.CONFIGS[2]
scene = mcpt.build_config_scene(2)
cam = mcpt.config_camera(rc, rc.width, rc.height)
for mult in [int(x) for x in os.environ.get("MULTS", "1,2,4").split(",")]:
    pt = mcpt.PathTracer(0, mcpt.default_config(spp=rc.spp, max_depth=rc.max_depth))
    pt.upload_scene(scene); pt.set_camera(cam); pt.resize(rc.width, rc.height * mult)
    pt.iterate(20)
    st = pt.iterate(30)
    rays = st.extend_rays + st.shadow_rays + st.vis_rays
    print(f"height x{mult}: {rays / (st.ms_total * 1e-3) / 1e6:.0f} Mray/s  trace {st.ms_extend / 30:.4f} ms  shade {st.ms_shade / 30:.4f} ms  rays/iter {rays / 30 / 1e6:.2f} M", flush=True)
    pt.close()
