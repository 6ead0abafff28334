"""Profiled program: steady-state config-2 wavefront iterations at the bench's path slots."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mc-path-tracer_amd")]
import mcpt
rc = mcpt.CONFIGS[2]
s = mcpt.build_config_scene(2)
pt = mcpt.PathTracer(0, mcpt.default_config(spp=256, max_depth=5))
pt.upload_scene(s); pt.set_camera(mcpt.config_camera(rc))
pt.set_path_slots(int(os.environ.get("SLOTS", "3")))
pt.resize(rc.width, rc.height)
pt.iterate(int(os.environ.get("ITERS", "12")))
print("ok")
