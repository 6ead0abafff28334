import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mc-path-tracer_amd")]
import torch
import mcpt
rc = mcpt.CONFIGS[2]
s = mcpt.build_config_scene(2)
pt = mcpt.PathTracer(0, mcpt.default_config(spp=256, max_depth=5))
pt.upload_scene(s); pt.set_camera(mcpt.config_camera(rc)); pt.resize(rc.width, rc.height)
pt.iterate(30)
for i in range(3):
    st = pt.iterate(1)
    print("pipeline iter: shade %.3f extend %.3f shadow %.3f ms, ext %d any %d" % (st.ms_shade, st.ms_extend, st.ms_shadow, st.extend_rays, st.shadow_rays + st.vis_rays), flush=True)
ro, rd = pt.queue_rays()
for i in range(2):
    pt.trace_closest(ro, rd); print("stage_run warm: %.3f ms" % pt.last_stage_ms, flush=True)
big = torch.empty(2**28, dtype=torch.float32, device="cuda")
for i in range(2):
    big.fill_(float(i)); torch.cuda.synchronize()
    pt.trace_closest(ro, rd); print("stage_run after 1GB fill: %.3f ms" % pt.last_stage_ms, flush=True)
st = pt.iterate(1)
print("pipeline iter: shade %.3f extend %.3f shadow %.3f ms" % (st.ms_shade, st.ms_extend, st.ms_shadow))
st = pt.iterate(20)
print("pipeline x20: shade %.3f extend %.3f shadow %.3f ms" % (st.ms_shade/20, st.ms_extend/20, st.ms_shadow/20))
