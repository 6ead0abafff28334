"""A/B of library variants on one BVH: tools/ab_tree.py <builder-kwargs-json> variant..."""
import json, os, subprocess, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
kw = sys.argv[1]
code = r'''
import os, sys, json
sys.path[:0] = [os.path.join(%r, "mc-path-tracer_amd")]
import mcpt
rc = mcpt.CONFIGS[2]
kw = json.loads(os.environ["TREE"])
pt = mcpt.PathTracer(0, mcpt.default_config(spp=256, max_depth=5))
pt.upload_scene(mcpt.build_config_scene(2, **kw)); pt.set_camera(mcpt.config_camera(rc)); pt.resize(rc.width, rc.height)
pt.iterate(30)
st = pt.iterate(30)
print("%%-10s %%-70s shade %%.4f trace %%.4f ms/iter" %% (os.environ["VARIANT"], kw, st.ms_shade / 30, st.ms_extend / 30), flush=True)
''' % REPO
for v in sys.argv[2:]:
    lib = os.path.join(REPO, "mc-path-tracer_amd", "libmcpt.so" if v == "base" else f"libmcpt_{v}.so")
    env = dict(os.environ, MCPT_LIB=lib, VARIANT=v, TREE=kw)
    subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=300)
