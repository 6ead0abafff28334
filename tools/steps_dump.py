"""Dump per-ray traversal steps of steady-state config-2 queue rays (for load-balance analysis)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mc-path-tracer_amd")]
import numpy as np, mcpt
rc = mcpt.CONFIGS[2]
pt = mcpt.PathTracer(0, mcpt.default_config(spp=256, max_depth=5))
pt.upload_scene(mcpt.build_config_scene(2)); pt.set_camera(mcpt.config_camera(rc)); pt.resize(rc.width, rc.height)
pt.iterate(30)
ro, rd = pt.queue_rays()
_, _, _, st = pt.trace_closest(ro, rd, steps=True)
_, sa = pt.trace_any(ro, rd, steps=True)
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(REPO, "gpurun_out", "steps.npz"), closest=st, any=sa)
print(len(st), st.mean(), sa.mean())
