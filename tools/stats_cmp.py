"""Traversal work counters of one config-2 run (iterations after a warmup), for comparing builds:
MCPT_LIB=<lib> python tools/stats_cmp.py"""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mc-path-tracer_amd")]
import mcpt
rc = mcpt.CONFIGS[2]
pt = mcpt.PathTracer(0, mcpt.default_config(spp=rc.spp, max_depth=rc.max_depth))
pt.upload_scene(mcpt.build_config_scene(2)); pt.set_camera(mcpt.config_camera(rc)); pt.resize(640, 360)
pt.iterate(10)
st = pt.iterate(5)
print(os.path.basename(os.environ.get("MCPT_LIB", "libmcpt.so")), {k: getattr(st, k) for k in
      ("extend_rays", "shadow_rays", "vis_rays", "ext_nodes", "ext_tests", "ext_hits", "any_nodes", "any_tests", "any_hits")})
