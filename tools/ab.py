"""A/B traversal variants (separate libmcpt_*.so) on steady-state config-2 rays."""
import os, subprocess, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = r'''
import os, sys
sys.path[:0] = [os.path.join(%r, "mc-path-tracer_amd")]
import numpy as np, mcpt
rc = mcpt.CONFIGS[2]
s = mcpt.build_config_scene(2)
pt = mcpt.PathTracer(0, mcpt.default_config(spp=256, max_depth=5))
pt.upload_scene(s); pt.set_camera(mcpt.config_camera(rc)); pt.resize(rc.width, rc.height)
pt.iterate(30)
ro, rd = pt.queue_rays()
import hashlib
idx = np.lexsort(np.concatenate([ro, rd], 1).T[::-1])  # canonical order for the result hash only
ts = []
for i in range(3):
    r = pt.trace_closest(ro, rd); ts.append(pt.last_stage_ms)
h = hashlib.md5(b"".join(np.ascontiguousarray(x[idx]).tobytes() for x in r)).hexdigest()[:10]
ta = []
for i in range(3):
    va = pt.trace_any(ro, rd); ta.append(pt.last_stage_ms)
h += "/" + hashlib.md5(va[idx].tobytes()).hexdigest()[:6]
st = pt.iterate(20)
print("%%-24s [%%s] closest(stage) %%.3f any(stage) %%.3f | pipeline shade %%.3f trace %%.3f (+%%.3f) ms/iter" %% (
    os.environ.get("VARIANT"), h, min(ts), min(ta), st.ms_shade/20, st.ms_extend/20, st.ms_shadow/20), flush=True)
''' % REPO
# variant: "base", a libmcpt_<name>.so suffix, or env overrides on base: "K=V,K2=V2"
for v in sys.argv[1:]:
    extra = {}
    if "=" in v:
        extra = dict(kv.split("=", 1) for kv in v.split(","))
        lib = os.path.join(REPO, "mc-path-tracer_amd", "libmcpt.so")
    else:
        lib = os.path.join(REPO, "mc-path-tracer_amd", "libmcpt.so" if v == "base" else f"libmcpt_{v}.so")
    env = dict(os.environ, MCPT_LIB=lib, VARIANT=v)
    env.update(extra)
    subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=300)
