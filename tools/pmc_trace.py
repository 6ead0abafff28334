"""Profiled program: stage-run the steady-state config-2 extension rays (closest + any-hit)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mc-path-tracer_amd")]
import mcpt
rc = mcpt.CONFIGS[2]
s = mcpt.build_config_scene(2)
pt = mcpt.PathTracer(0, mcpt.default_config(spp=256, max_depth=5))
pt.upload_scene(s); pt.set_camera(mcpt.config_camera(rc)); pt.resize(rc.width, rc.height)
pt.iterate(30)
ro, rd = pt.queue_rays()
for i in range(2):
    pt.trace_closest(ro, rd)
    pt.trace_any(ro, rd)
print("rays", len(ro))
