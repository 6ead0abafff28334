#!/bin/bash
# time of the shading kernels without the env lookups (diagnostic builds; upper bounds of a deferral)
# variant library: the diag_NO_ENVB / diag_NO_ENVL builds of tools/experiments/diag_env_attribution.patch (see tools/gpu_attr.sh)
set -o pipefail
L=$PWD/mc-path-tracer_amd
KS_STEPS=2 bash tools/gpu_kstats.sh "MCPT_X=0" "MCPT_LIB=$L/libmcpt_diag_NO_ENVB.so" "MCPT_LIB=$L/libmcpt_diag_NO_ENVL.so" "MCPT_X=0" 2>&1 | grep -E "==|value|k_trace|k_material|k_shade"
timeout -k 10 120 python3 - <<'PY'
import sys; sys.path.insert(0, "mc-path-tracer_amd")
import mcpt
rc = mcpt.CONFIGS[2]
pt = mcpt.PathTracer(0, mcpt.default_config(spp=16, max_depth=rc.max_depth))
pt.upload_scene(mcpt.build_config_scene(2)); pt.set_camera(mcpt.config_camera(rc)); pt.resize(rc.width, rc.height)
st = pt.render()
print("any-hit rays", st.shadow_rays + st.vis_rays, "occluded", st.any_hits, "frac", st.any_hits / (st.shadow_rays + st.vis_rays))
PY
