"""k_shade section profile on steady-state config-2 iterations (needs the -DMCPT_SHADE_PROF build:
tools/build_variant.sh sprof -DMCPT_SHADE_PROF; run with MCPT_LIB=.../libmcpt_sprof.so)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mc-path-tracer_amd")]
import mcpt
rc = mcpt.CONFIGS[2]
pt = mcpt.PathTracer(0, mcpt.default_config(spp=256, max_depth=5))
pt.upload_scene(mcpt.build_config_scene(2)); pt.set_camera(mcpt.config_camera(rc)); pt.set_path_slots(int(os.environ.get("SLOTS", "3"))); pt.resize(rc.width, rc.height)
pt.iterate(30)
pt.trace_profile(reset=True)
N = 10
st = pt.iterate(N)
p = list(pt.trace_profile().values())
names = ["shade:logic", "shade:gen", "shade:push", "mat:hit_record", "mat:continuation", "mat:light_sample",
         "mat:brdf_sample", "mat:occ_lookup", "mat:whole kernel", "mat:push+stores"]
sw, mw = p[11], p[10]
print(f"k_shade waves/launch {sw / N:.0f}  k_material waves/launch {mw / N:.0f}  ms/iter (both) {st.ms_shade / N:.4f}")
for i, n in enumerate(names):
    w = sw if i < 3 else mw
    print(f"  {n:20s} cycles/wave {p[i] / w:9.1f}")
